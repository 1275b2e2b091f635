"""Pin the oracle (oracle/) to golden vectors produced by the reference itself (tools/gen_golden.py)."""
import numpy as np
import pytest
import torch

from oracle import closed_form, cse_ref, philox, sbm_ref

SBM_CASES = ["sbm_n37", "sbm_n1", "sbm_n7_d96_k16", "sbm_n64_noncontig", "sbm_n150", "sbm_n33_d96"]


def t(x, grad=False):
    return torch.from_numpy(np.ascontiguousarray(x)).requires_grad_(grad)


def sbm_params(z, grad=True):
    return {k[2:]: t(v, grad) for k, v in z.items() if k.startswith("p:")}


def test_bernoulli_equivalence_recorded(golden):
    assert bool(golden("bernoulli_equivalence")["ok"][0])


@pytest.mark.parametrize("case", SBM_CASES)
def test_sbm_oracle_matches_reference(golden, case):
    z = golden(case)
    B, H, N, d, k = z["meta"]
    Q, K, V = t(z["Q"], True), t(z["K"], True), t(z["V"], True)
    params = sbm_params(z)
    X, sp, graph, attn = sbm_ref.sbm_attention(Q, K, V, t(z["mask"]), params, t(z["u"]), int(k))
    assert np.array_equal(graph.detach().numpy().astype(np.uint8), z["graph"])
    np.testing.assert_allclose(X.detach().numpy(), z["X"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(attn.detach().numpy(), z["attn"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(sp.detach().numpy(), z["sparsity"], rtol=0, atol=0)
    ((X * t(z["dX"])).sum() + (sp * t(z["dsparsity"])).sum()).backward()
    for name, g in (("dQ", Q.grad), ("dK", K.grad), ("dV", V.grad)):
        np.testing.assert_allclose(g.numpy(), z[name], rtol=1e-4, atol=1e-5, err_msg=name)
    for pk, p in params.items():
        np.testing.assert_allclose(p.grad.numpy(), z["g:" + pk], rtol=1e-4, atol=1e-5, err_msg=pk)


@pytest.mark.parametrize("case", ["sbm_n37_mapgrad", "sbm_n33_d96_mapgrad"])
def test_sbm_oracle_map_gradients(golden, case):
    """Upstream gradients of the returned graph and attn maps (sbm_attn.py:66) flow like the reference's."""
    z = golden(case)
    B, H, N, d, k = z["meta"]
    Q, K, V = t(z["Q"], True), t(z["K"], True), t(z["V"], True)
    params = sbm_params(z)
    X, sp, graph, attn = sbm_ref.sbm_attention(Q, K, V, t(z["mask"]), params, t(z["u"]), int(k))
    assert np.array_equal(graph.detach().numpy().astype(np.uint8), z["graph"])
    loss = ((X * t(z["dX"])).sum() + (sp * t(z["dsparsity"])).sum() + (graph * t(z["dgraph"])).sum()
            + (attn * t(z["dattn"])).sum())
    loss.backward()
    for name, g in (("dQ", Q.grad), ("dK", K.grad), ("dV", V.grad)):
        np.testing.assert_allclose(g.numpy(), z[name], rtol=1e-4, atol=1e-5, err_msg=name)
    for pk, p in params.items():
        np.testing.assert_allclose(p.grad.numpy(), z["g:" + pk], rtol=1e-4, atol=1e-5, err_msg=pk)


@pytest.mark.parametrize("case", SBM_CASES)
def test_sampler_bit_exact_on_reference_expA(golden, case):
    """STE.py:10-15: A = u < clamp(expA, .01, .99) — bit-exact given the reference's own expA."""
    z = golden(case)
    A = sbm_ref.STESample.apply(t(z["expA"]), t(z["u"]))
    assert np.array_equal(A.numpy().astype(np.uint8), z["graph"])


@pytest.mark.parametrize("case", SBM_CASES)
def test_closed_form_matches_reference(golden, case):
    """The fp64 closed form (the kernels' spec) vs the reference autograd, at the kernel tolerance."""
    z = golden(case)
    B, H, N, d, k = z["meta"]
    params = {k_[2:]: t(v) for k_, v in z.items() if k_.startswith("p:")}
    out, g = closed_form.sbm_fwd_bwd(t(z["Q"]), t(z["K"]), t(z["V"]), t(z["mask"]), params, t(z["u"]), int(k),
                                     t(z["dX"]), t(z["dsparsity"]), graph_override=t(z["graph"].astype(np.float32)))
    np.testing.assert_allclose(out["X"].numpy(), z["X"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["attn"].numpy(), z["attn"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["expA"].numpy(), z["expA"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(g["Q"].numpy(), z["dQ"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(g["K"].numpy(), z["dK"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(g["V"].numpy(), z["dV"], rtol=1e-4, atol=1e-5)
    for pk in params:
        np.testing.assert_allclose(g[pk].numpy(), z["g:" + pk], rtol=1e-4, atol=1e-5, err_msg=pk)


@pytest.mark.parametrize("case", ["full_n37", "full_n150", "full_n37_mapgrad"])
def test_full_attention_oracle(golden, case):
    z = golden(case)
    Q, K, V = t(z["Q"], True), t(z["K"], True), t(z["V"], True)
    X, sp, graph, attn = sbm_ref.full_attention(Q, K, V, t(z["mask"]))
    np.testing.assert_allclose(X.detach().numpy(), z["X"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(attn.detach().numpy(), z["attn"], rtol=1e-5, atol=1e-6)
    loss = (X * t(z["dX"])).sum()
    if "dattn" in z:
        loss = loss + (attn * t(z["dattn"])).sum()
    loss.backward()
    for name, gg in (("dQ", Q.grad), ("dK", K.grad), ("dV", V.grad)):
        np.testing.assert_allclose(gg.numpy(), z[name], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("case", ["attn_layer_n29", "attn_layer_full_n29"])
def test_attention_layer_oracle(golden, case):
    z = golden(case)
    B, N, dim, H, k, full = z["meta"]
    params = {k_[2:]: t(v, True) for k_, v in z.items() if k_.startswith("p:")}
    X = t(z["X"], True)
    out, sp, graph, attn = sbm_ref.attention_layer(X, t(z["mask"]), params, t(z["u"]), int(H), int(dim // H), int(k),
                                                   full_att=bool(full))
    np.testing.assert_allclose(out.detach().numpy(), z["out"], rtol=1e-5, atol=1e-6)
    loss = (out * t(z["dout"])).sum()
    if sp is not None:
        loss = loss + (sp * t(z["dsparsity"])).sum()
    loss.backward()
    np.testing.assert_allclose(X.grad.numpy(), z["dX"], rtol=1e-4, atol=1e-5)
    for pk, p in params.items():
        np.testing.assert_allclose(p.grad.numpy(), z["g:" + pk], rtol=1e-4, atol=1e-5, err_msg=pk)


@pytest.mark.parametrize("case", ["rel_attn_n37", "rel_attn_n150", "rel_attn_n20_dk64"])
def test_rel_attn_oracle(golden, case):
    z = golden(case)
    rel, mask = cse_ref.build_rel_mask(t(z["L"]), t(z["T"]), t(z["L_mask"]), t(z["T_mask"]))
    q, k, v, lq, lk = (t(z[n], True) for n in ("q", "k", "v", "lq", "lk"))
    o = cse_ref.rel_attn(q, k, v, lq, lk, rel, mask)
    np.testing.assert_allclose(o.detach().numpy(), z["out"], rtol=1e-5, atol=1e-6)
    (o * t(z["dO"])).sum().backward()
    for n, x in (("dq", q), ("dk", k), ("dv", v), ("dlq", lq), ("dlk", lk)):
        np.testing.assert_allclose(x.grad.numpy(), z[n], rtol=1e-4, atol=1e-5, err_msg=n)


def test_disentangled_oracle(golden):
    z = golden("disentangled_n23")
    rel, mask = cse_ref.build_rel_mask(t(z["L"]), t(z["T"]), t(z["L_mask"]), t(z["T_mask"]))
    params = {k_[2:]: t(v, True) for k_, v in z.items() if k_.startswith("p:")}
    x, rq = t(z["x"], True), t(z["rel_q"], True)
    out, none = cse_ref.disentangled_attn(x, params, rq, rel, mask)
    assert none is None
    np.testing.assert_allclose(out.detach().numpy(), z["out"], rtol=1e-5, atol=1e-6)
    (out * t(z["dout"])).sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), z["dx"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(rq.grad.numpy(), z["drel_q"], rtol=1e-4, atol=1e-5)
    for pk, p in params.items():
        np.testing.assert_allclose(p.grad.numpy(), z["g:" + pk], rtol=1e-4, atol=1e-5, err_msg=pk)


# Random123 kat_vectors, philox4x32 with 10 rounds: (counter, key) -> output
PHILOX_KAT = [
    ((0x00000000, 0x00000000, 0x00000000, 0x00000000), (0x00000000, 0x00000000),
     (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF), (0xFFFFFFFF, 0xFFFFFFFF),
     (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,out", PHILOX_KAT)
def test_philox_round_function_known_answers(ctr, key, out):
    """The oracle's Philox (the kernels' train-mode random streams run 7 rounds of it) against the
    published 10-round known-answer vectors."""
    got = philox.philox4x32(*ctr, *key, rounds=10)
    assert tuple(int(v) for v in got) == out


def test_philox_stream_layout():
    """Draw layouts: 16-bit halves in word order, distinct streams, keep thresholds of fp32 p."""
    u = philox.attn_uniforms(1, 2, 5, 40, seed=(7 << 32) | 3, offset=9, stream=philox.RNG_STE)
    assert u.shape == (1, 2, 5, 40) and u.max() < 65536
    w = philox.philox4x32(0, 0, 0, (philox.RNG_STE << 28) ^ 9, 3, 7)
    assert int(u[0, 0, 0, 0]) == int(w[0]) & 0xFFFF        # key 0 = register 0, half 0: word x low
    assert int(u[0, 0, 0, 1]) == int(w[0]) >> 16            # key 1 = register 1: word x high
    assert int(u[0, 0, 0, 8]) == int(w[2]) & 0xFFFF        # key 8 = register 4: word z low
    assert int(u[0, 0, 0, 4]) != int(u[0, 0, 0, 0])         # key 4 = half 1: its own counter
    d = philox.attn_uniforms(1, 2, 5, 40, seed=(7 << 32) | 3, offset=9, stream=philox.RNG_ATTN_DROP)
    assert not np.array_equal(u, d)
    assert philox.keep_threshold(0.2) == 13108 and philox.keep_threshold(0.0) == 0
    k = philox.proj_keep(2, 2, 64, 64, seed=123, offset=0, p=0.25, layer=0, is_k=0)
    assert abs(k.mean() - 0.75) < 0.02


def test_csatrans_oracle_matches_reference_tiny(golden):
    """oracle/csatrans_ref.py (the whole model restated over a parameter dict; bench.py's config-1 CPU
    baseline) vs the reference CSATrans: same state_dict keys, forward log-probabilities, sparsity,
    loss and parameter gradients (tests/golden/csatrans_tiny.npz)."""
    import golden_inputs as gi
    from oracle import csatrans_ref
    z = golden("csatrans_tiny")
    cfg = csatrans_ref.config(**TINY_CFG)
    shapes = csatrans_ref.param_shapes(cfg)
    ref_keys = [k for k in z["state_keys"] if "orth_clusters" not in k and not k.endswith("pos_emb.pe")]
    assert sorted(shapes) == sorted(ref_keys)
    params = {k: v.requires_grad_(True) for k, v in gi.fill_dict_deterministic(shapes, 71).items()}
    f = lambda k, dt: torch.from_numpy(z[k]).to(dt)
    model = csatrans_ref.Model(cfg, params, training=False)
    out, sp = model.forward(f("src_seq", torch.int64), f("tgt_seq", torch.int64), f("L", torch.int64),
                            f("T", torch.int64), f("L_mask", torch.bool), f("T_mask", torch.bool),
                            u_list=[f("u0", torch.float32), f("u1", torch.float32)])
    loss = csatrans_ref.label_smoothing(out, f("target", torch.int64))
    np.testing.assert_allclose(out.detach().numpy(), z["out"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(sp.item(), z["sparsity"][0], rtol=1e-6)
    np.testing.assert_allclose(loss.item(), z["loss"][0], rtol=1e-6)
    (loss + 1e-2 * sp).backward()
    n = 0
    for k in z:
        if k.startswith("g:"):
            np.testing.assert_allclose(params[k[2:]].grad.numpy(), z[k], rtol=1e-4, atol=1e-6, err_msg=k)
            n += 1
    assert n >= 10


TINY_CFG = dict(src_vocab_size=50, tgt_vocab_size=60, hidden_size=64, num_heads=8, num_layers=1, sbm_layers=2,
                use_pegen="pegen", dim_feed_forward=128, dropout=0.2, pe_dim=32, pegen_dim=128, sbm_enc_dim=512,
                clusters=[10, 12], full_att=False)
