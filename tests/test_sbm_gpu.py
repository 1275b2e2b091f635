"""GPU parity: fused SBM / dense attention kernels vs the reference's golden vectors and the oracle."""
import numpy as np
import pytest
import torch

from conftest import has_gpu
from oracle import closed_form

pytestmark = pytest.mark.gpu

SBM_CASES = ["sbm_n37", "sbm_n1", "sbm_n7_d96_k16", "sbm_n64_noncontig", "sbm_n150", "sbm_n33_d96"]
RTOL, ATOL = 1e-4, 1e-5  # north_star fp32 tolerance


def dev(x, grad=False):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda().requires_grad_(grad)


def make_module(z, k):
    from csa_amd.module.sbm_attn import SBMAttention
    B, H, N, d, _ = z["meta"]
    m = SBMAttention({"attention_dropout": 0.2, "head_dim": int(d), "num_head": int(H), "num_clusters": [int(k)]}, 0)
    sd = {kk[2:]: torch.from_numpy(v) for kk, v in z.items() if kk.startswith("p:")}
    m.load_state_dict(sd, strict=False)
    return m.cuda().eval()


def flips_allowed(graph_ours, z):
    """Sampled masks must be bit-exact, except where u is within fp32 rounding of the clamped expA."""
    diff = graph_ours != z["graph"]
    if not diff.any():
        return 0
    p = np.clip(z["expA"], 0.01, 0.99)
    near = np.abs(z["u"] - p) < 1e-6
    assert np.all(near[diff]), f"{int(diff.sum())} graph flips, {int((diff & ~near).sum())} not at a near-tie"
    return int(diff.sum())


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
@pytest.mark.parametrize("case", SBM_CASES)
def test_sbm_forward_backward_matches_reference(golden, case):
    z = golden(case)
    B, H, N, d, k = (int(v) for v in z["meta"])
    m = make_module(z, k)
    Q, K, V = dev(z["Q"], True), dev(z["K"], True), dev(z["V"], True)
    m.uniforms = dev(z["u"])
    X, sp, graph, attn = m(Q, K, V, dev(z["mask"]))
    torch.cuda.synchronize()
    g = graph.detach().cpu().numpy().astype(np.uint8)
    nflip = flips_allowed(g, z)
    params = {kk[2:]: torch.from_numpy(v) for kk, v in z.items() if kk.startswith("p:")}
    ref, rg = closed_form.sbm_fwd_bwd(*(torch.from_numpy(z[n]) for n in ("Q", "K", "V", "mask")), params,
                                     torch.from_numpy(z["u"]), k, torch.from_numpy(z["dX"]),
                                     torch.from_numpy(z["dsparsity"]), graph_override=torch.from_numpy(g.astype(np.float32)))
    np.testing.assert_allclose(X.detach().cpu().numpy(), ref["X"].numpy(), rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(attn.detach().cpu().numpy(), ref["attn"].numpy(), rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(sp.detach().cpu().numpy(), ref["sparsity"].numpy(), rtol=1e-7, atol=0)
    if nflip == 0:  # directly against the reference's own outputs too
        np.testing.assert_allclose(X.detach().cpu().numpy(), z["X"], rtol=RTOL, atol=ATOL)
        np.testing.assert_array_equal(sp.detach().cpu().numpy(), z["sparsity"])
    ((X * dev(z["dX"])).sum() + (sp * dev(z["dsparsity"])).sum()).backward()
    for name, t, key in (("dQ", Q, "Q"), ("dK", K, "K"), ("dV", V, "V")):
        np.testing.assert_allclose(t.grad.cpu().numpy(), rg[key].numpy(), rtol=RTOL, atol=ATOL, err_msg=name)
        if nflip == 0:
            np.testing.assert_allclose(t.grad.cpu().numpy(), z[name], rtol=RTOL, atol=ATOL, err_msg=name + " (ref)")
    for pn, p in m.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), rg[pn].numpy(), rtol=RTOL, atol=ATOL, err_msg=pn)
        if nflip == 0:
            np.testing.assert_allclose(p.grad.cpu().numpy(), z["g:" + pn], rtol=RTOL, atol=ATOL, err_msg=pn + " (ref)")


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
@pytest.mark.parametrize("case", SBM_CASES)
def test_ste_sample_bit_exact(golden, case):
    """STE.py:10-15 on the reference's own expA and uniforms: bit-exact."""
    z = golden(case)
    A = torch.ops.csa.ste_sample(dev(z["expA"]), dev(z["u"]), 0.01, 0.99)
    np.testing.assert_array_equal(A.cpu().numpy().astype(np.uint8), z["graph"])


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
@pytest.mark.parametrize("case", ["full_n37", "full_n150"])
def test_full_attention_matches_reference(golden, case):
    from csa_amd.module.sbm_attn import FullAttention
    z = golden(case)
    B, H, N, d = (int(v) for v in z["meta"])
    m = FullAttention({"attention_dropout": 0.2, "head_dim": d, "num_head": H}, 0).cuda().eval()
    Q, K, V = dev(z["Q"], True), dev(z["K"], True), dev(z["V"], True)
    mask = dev(z["mask"])
    X, sp, graph, attn = m(Q, K, V, mask)
    assert sp is None and graph is mask
    np.testing.assert_allclose(X.detach().cpu().numpy(), z["X"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(attn.detach().cpu().numpy(), z["attn"], rtol=RTOL, atol=ATOL)
    (X * dev(z["dX"])).sum().backward()
    for name, t in (("dQ", Q), ("dK", K), ("dV", V)):
        np.testing.assert_allclose(t.grad.cpu().numpy(), z[name], rtol=RTOL, atol=ATOL, err_msg=name)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
@pytest.mark.parametrize("case", ["attn_layer_n29", "attn_layer_full_n29"])
def test_attention_layer_matches_reference(golden, case):
    """module/sbm_attn.py:90-140 Attention (W_q/W_k/W_v, strided split_heads views, ff)."""
    from csa_amd.module.sbm_attn import Attention
    z = golden(case)
    B, N, dim, H, k, full = (int(v) for v in z["meta"])
    cfg = {"attention_grad_checkpointing": False, "transformer_dim": dim, "head_dim": dim // H, "num_head": H,
           "attn_type": "sbm", "attention_dropout": 0.2, "num_clusters": [k]}
    m = Attention(cfg, 0, full_att=bool(full))
    m.load_state_dict({kk[2:]: torch.from_numpy(v) for kk, v in z.items() if kk.startswith("p:")}, strict=False)
    m = m.cuda().eval()
    if not full:
        m.attn.uniforms = dev(z["u"])
    X = dev(z["X"], True)
    out, sp, graph, attn = m([X, dev(z["mask"]), []])
    if not full:
        np.testing.assert_array_equal(graph.detach().cpu().numpy().astype(np.uint8), z["graph"])
    np.testing.assert_allclose(out.detach().cpu().numpy(), z["out"], rtol=RTOL, atol=ATOL)
    loss = (out * dev(z["dout"])).sum()
    if sp is not None:
        np.testing.assert_array_equal(sp.detach().cpu().numpy(), z["sparsity"])
        loss = loss + (sp * dev(z["dsparsity"])).sum()
    loss.backward()
    np.testing.assert_allclose(X.grad.cpu().numpy(), z["dX"], rtol=RTOL, atol=ATOL)
    for pn, p in m.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), z["g:" + pn], rtol=RTOL, atol=ATOL, err_msg=pn)

