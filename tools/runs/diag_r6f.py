"""Round 6 diagnostic: where the dead-tile test's dK mismatches sit (d = 96, k = 16, N = 100), and which shape
parameter triggers them."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "code-structure-aware-transformer_amd"))
import numpy as np
import torch
import csa_amd.ops  # noqa
from test_sbm_gpu import _rand_case, _run_module, _dead_tile_masks
from oracle import closed_form

for shape in [(6, 2, 100, 96, 16), (6, 2, 100, 64, 16), (6, 2, 100, 96, 10), (6, 2, 150, 96, 16), (6, 2, 128, 96, 16)]:
    B, H, N, d, k = shape
    Q, K, V, _, u, dX, dsp, params = _rand_case(B, H, N, d, k, seed=97 + N)
    mask = _dead_tile_masks(B, N)
    X, sp, graph, dQ, dK, dV, grads = _run_module(Q, K, V, mask, u, dX, dsp, params, k)
    ref, rg = closed_form.sbm_fwd_bwd(Q, K, V, mask, params, u, k, dX, dsp, graph_override=graph)
    for name, t, key in (("dQ", dQ, "Q"), ("dK", dK, "K"), ("dV", dV, "V")):
        r = rg[key]
        bad = (t - r).abs() > (1e-5 + 1e-4 * r.abs())
        n = int(bad.sum())
        msg = f"{shape} {name}: {n} bad, max abs err {float((t - r).abs().max()):.3g}, max |ref| {float(r.abs().max()):.3g}"
        if n:
            idx = bad.nonzero()
            bs = sorted(set(idx[:, 0].tolist())); hs = sorted(set(idx[:, 1].tolist())); ks = sorted(set(idx[:, 2].tolist()))
            msg += f" b={bs} h={hs} rows={ks[:12]}{'...' if len(ks) > 12 else ''} cols={sorted(set(idx[:, 3].tolist()))[:8]}"
            i = tuple(idx[0].tolist())
            msg += f" e.g. got {float(t[i]):.6g} want {float(r[i]):.6g}"
        print(msg, flush=True)
