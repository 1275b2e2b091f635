"""Hypothesis property tests: random shapes N <= 150, random key padding, random
uniforms and random AST relations, HIP path vs the pinned oracle. Sampled masks must match
(away from fp32 ties), everything else within the north_star fp32 tolerance rtol 1e-4 / atol 1e-5."""
import numpy as np
import pytest
import torch
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs GPU")]
RTOL, ATOL = 1e-4, 1e-5
SETTINGS = dict(max_examples=20, deadline=None, derandomize=True,
                suppress_health_check=[HealthCheck.too_slow, HealthCheck.data_too_large])


@settings(**SETTINGS)
@given(B=st.integers(1, 2), H=st.sampled_from([1, 2, 8]), N=st.integers(1, 150), d=st.sampled_from([64, 96]),
       k=st.integers(2, 16), seed=st.integers(0, 2 ** 31 - 1), pad=st.booleans(), eval_p=st.floats(0.0, 1.0))
def test_sbm_random_shapes_match_oracle(B, H, N, d, k, seed, pad, eval_p):
    """SBMAttention fwd + bwd (eval, host-supplied uniforms): random N, heads, head dim, clusters and
    key-padding lengths (including fully padded rows' neighbours) vs the fp64 closed form."""
    from test_sbm_gpu import _rand_case, _run_module

    from oracle import closed_form
    Q, K, V, mask, u, dX, dsp, params = _rand_case(B, H, N, d, k, seed=seed, pad=pad)
    if eval_p < 0.2:  # stretch the uniforms toward the clamp edges 0.01 / 0.99
        u = u.pow(4.0) if eval_p < 0.1 else 1.0 - u.pow(4.0)
    X, sp, graph, dQ, dK, dV, grads = _run_module(Q, K, V, mask, u, dX, dsp, params, k)
    ref, rg = closed_form.sbm_fwd_bwd(Q, K, V, mask, params, u, k, dX, dsp, graph_override=graph)
    near = torch.abs(u - ref["expA"].clamp(0.01, 0.99)) < 1e-6
    assert bool(torch.all(near[graph != ref["graph"].float()])), "graph flips away from fp32 ties"
    np.testing.assert_allclose(X.numpy(), ref["X"].numpy(), rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(sp.numpy(), ref["sparsity"].numpy(), rtol=1e-6)
    for name, t, key in (("dQ", dQ, "Q"), ("dK", dK, "K"), ("dV", dV, "V")):
        np.testing.assert_allclose(t.numpy(), rg[key].numpy(), rtol=RTOL, atol=ATOL, err_msg=name)
    for pn, gv in grads.items():
        if not pn.startswith("orth_clusters"):
            np.testing.assert_allclose(gv.numpy(), rg[pn].numpy(), rtol=RTOL, atol=ATOL, err_msg=pn)


@settings(**SETTINGS)
@given(n=st.integers(1, 20000), seed=st.integers(0, 2 ** 31 - 1), lo=st.floats(0.0, 0.5), hi=st.floats(0.5, 1.0))
def test_ste_sample_bit_exact_random(n, seed, lo, hi):
    """STE.py:10-15 as u < clamp(p, lo, hi): bit-exact for any p (including outside [0, 1]) and u."""
    g = torch.Generator().manual_seed(seed)
    p = torch.rand(n, generator=g) * 1.4 - 0.2
    u = torch.rand(n, generator=g)
    A = torch.ops.csa.ste_sample(p.cuda(), u.cuda(), lo, hi).cpu()
    assert torch.equal(A, (u < p.clamp(lo, hi)).float())


@settings(**SETTINGS)
@given(B=st.integers(1, 3), N=st.integers(1, 150), dk=st.sampled_from([16, 32, 64]), seed=st.integers(0, 2 ** 31 - 1),
       compact=st.booleans())
def test_rel_attn_random_asts_match_oracle(B, N, dk, seed, compact):
    """DisentangledAttn.rel_attn fwd + bwd over random synthetic ASTs of random size (relation planes from
    the native builder, fully masked sibling rows included) vs the fp64 oracle."""
    from csa_amd import rel_ops
    from csa_amd.data import synthetic_batch
    from oracle import cse_ref
    H, L = 8, 150
    sb = synthetic_batch(B, max_size=N, seed=seed % 100000, min_nodes=1, max_nodes=N)
    g = torch.Generator().manual_seed(seed)
    q, k, v, dO = (torch.randn(B, H, N, dk, generator=g) for _ in range(4))
    lq, lk = (torch.randn(1, H, L, dk, generator=g) for _ in range(2))
    refrel, refmask = cse_ref.build_rel_mask(*(torch.from_numpy(sb[n]) for n in ("L", "T", "L_mask", "T_mask")))
    if compact:
        rel = torch.from_numpy(np.stack([sb["L"], sb["T"]], 1).astype(np.uint8))
        mask = torch.from_numpy(np.stack([sb["L_mask"], sb["T_mask"]], 1).astype(np.uint8))
    else:
        rel, mask = refrel, refmask
    tg = [x.cuda().requires_grad_(True) for x in (q, k, v, lq, lk)]
    o = rel_ops.rel_attn(*tg, rel.cuda(), mask.cuda())
    (o * dO.cuda()).sum().backward()
    tr = [x.double().requires_grad_(True) for x in (q, k, v, lq, lk)]
    oref = cse_ref.rel_attn(*tr, refrel, refmask)
    (oref * dO.double()).sum().backward()
    np.testing.assert_allclose(o.detach().cpu().numpy(), oref.detach().numpy(), rtol=RTOL, atol=ATOL)
    for name, a, b in zip(("dq", "dk", "dv", "dlq", "dlk"), tg, tr):
        ref = b.grad.numpy()
        atol = ATOL * max(1.0, float(np.abs(ref).max()) / 100) if name in ("dlq", "dlk") else ATOL
        np.testing.assert_allclose(a.grad.cpu().numpy(), ref, rtol=RTOL, atol=atol, err_msg=name)
