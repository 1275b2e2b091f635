"""Regenerable inputs of the large golden fixtures (tools/gen_golden.py writes only their outputs).

Everything here is numpy PCG64, whose streams are stable across numpy versions and machines, so the
GPU tests rebuild exactly the inputs the reference saw when the fixture was generated. Used by
tools/gen_golden.py (in this container, next to the reference) and by tests/ (on the GPU box).
"""
import numpy as np

JAVA = dict(src_vocab_size=10000, tgt_vocab_size=20000, hidden_size=512, num_heads=8, num_layers=4, sbm_layers=4,
            use_pegen="pegen", dim_feed_forward=2048, dropout=0.2, pe_dim=128, pegen_dim=512, sbm_enc_dim=768,
            clusters=[10, 10, 10, 10], full_att=False)  # config/java.py via module/csa_trans.py:67-158
JAVA_B, JAVA_N, JAVA_SEED = 2, 150, 81
JAVA_OUT_COL_STRIDE = 16  # the fixture keeps out[:, :, ::16] (20000-wide log-probabilities)
JAVA_GRAD_KEYS = ("SBM.transformer_0.mha.attn.", "SBM.transformer_3.mha.attn.", "pegen.layers.0.self_attn.l_linear.0",
                  "pegen.layers.3.self_attn.t_linear.1", "pegen.L_q", "pegen.T_q", "SBM.out.bias",
                  "SBM.pe_expand.bias", "generator.linear.bias", "pegen.layers.2.self_attn.linear_layers.0.bias")
PYTHON = dict(src_vocab_size=10000, tgt_vocab_size=20000, hidden_size=512, num_heads=8, num_layers=4, sbm_layers=4,
              use_pegen="pegen", dim_feed_forward=2048, dropout=0.2, pe_dim=256, pegen_dim=512, sbm_enc_dim=512,
              clusters=[10, 10, 10, 10], full_att=False)  # config/python.py via module/csa_trans.py:67-158
PY_B, PY_N, PY_SEED = 2, 150, 83
TIE_MARGIN = 5e-4  # STE uniforms closer than this to clamp(expA) are moved off the tie (see nudge_uniforms)


def fill_params_deterministic(model, seed):
    """Every parameter <- N(0,1) * 0.5/sqrt(fan_in) from PCG64 in sorted-name order."""
    import torch
    rng = np.random.default_rng(seed)
    named = dict(model.named_parameters())
    with torch.no_grad():
        for k in sorted(named):
            p = named[k]
            fan = p.shape[-1] if p.dim() > 1 else 1
            p.copy_(torch.from_numpy((rng.standard_normal(p.shape) * (0.5 / np.sqrt(fan))).astype(np.float32)))


def java_uniforms(layer, B=JAVA_B, H=8, N=JAVA_N, seed=JAVA_SEED):
    """Host-supplied STE uniforms of SBM layer `layer` before tie nudging, (B,H,N,N) fp32."""
    return np.random.default_rng([seed, 1000 + layer]).random((B, H, N, N), dtype=np.float32)


def python_uniforms(layer):
    """java_uniforms for the config/python.py fixture (csatrans_python)."""
    return java_uniforms(layer, B=PY_B, N=PY_N, seed=PY_SEED)


def e64(z, key):
    """The fixture's fp64-oracle value of `key` (float64): the reference's fp32 value plus the stored
    difference z['e64:' + key] = fp64 - fp32 (tools/gen_golden.py:csatrans_dims_case)."""
    return z[key].astype(np.float64) + z["e64:" + key].astype(np.float64)


def apply_nudges(u, idx, val):
    """Replace u.flat[idx] by val (the generator's tie nudges); returns a new array."""
    u = u.copy()
    u.reshape(-1)[idx] = val
    return u


def nudge_uniforms(u, p, margin=TIE_MARGIN):
    """Move every draw within `margin` of the clamped probability p = clamp(expA, .01, .99) to the
    same side at distance `margin`, so the sampled edge (u < p) cannot flip between two fp32
    evaluations of expA that differ in the last bits. Returns (u', flat indices, new values)."""
    d = u - p
    idx = np.flatnonzero(np.abs(d) < margin)
    flat = u.reshape(-1).copy()
    pf, df = p.reshape(-1), d.reshape(-1)
    new = np.where(df[idx] < 0, pf[idx] - margin, pf[idx] + margin).astype(np.float32)
    new = np.clip(new, 0.0, np.nextafter(np.float32(1.0), np.float32(0.0)))
    flat[idx] = new
    return flat.reshape(u.shape), idx.astype(np.int64), new


def rel_inputs(B, H, N, dk, L, seed):
    """q, k, v (B,H,N,dk), lq, lk (1,H,L,dk), dO (B,H,N,dk) fp32 from PCG64."""
    rng = np.random.default_rng(seed)
    f = lambda *s: rng.standard_normal(s, dtype=np.float32)
    return f(B, H, N, dk), f(B, H, N, dk), f(B, H, N, dk), f(1, H, L, dk), f(1, H, L, dk), f(B, H, N, dk)


def fill_dict_deterministic(shapes, seed):
    """fill_params_deterministic over a {name: shape} dict (the oracle's parameter dict): same draws in the
    same sorted-name order as over a model's named_parameters()."""
    import torch
    rng = np.random.default_rng(seed)
    out = {}
    for k in sorted(shapes):
        s = tuple(shapes[k])
        fan = s[-1] if len(s) > 1 else 1
        out[k] = torch.from_numpy((rng.standard_normal(s) * (0.5 / np.sqrt(fan))).astype(np.float32))
    return out
