"""GPU parity: CSE disentangled relation attention vs the reference's golden vectors."""
import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = pytest.mark.gpu
RTOL, ATOL = 1e-4, 1e-5


def dev(x, grad=False):
    return torch.from_numpy(np.ascontiguousarray(x)).cuda().requires_grad_(grad)


def ref_rel_mask(z):
    from oracle import cse_ref
    return cse_ref.build_rel_mask(*(torch.from_numpy(z[n]) for n in ("L", "T", "L_mask", "T_mask")))


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
@pytest.mark.parametrize("case", ["rel_attn_n37", "rel_attn_n150", "rel_attn_n20_dk64"])
@pytest.mark.parametrize("layout", ["reference", "compact"])
def test_rel_attn_matches_reference(golden, case, layout):
    from csa_amd import rel_ops
    z = golden(case)
    if layout == "reference":
        rel, mask = (t.cuda() for t in ref_rel_mask(z))
    else:  # zero-copy CSE planes: (B,2,N,N) uint8, heads 0-3 -> L, 4-7 -> T
        rel = dev(np.stack([z["L"], z["T"]], 1).astype(np.uint8))
        mask = dev(np.stack([z["L_mask"], z["T_mask"]], 1).astype(np.uint8))
    q, k, v, lq, lk = (dev(z[n], True) for n in ("q", "k", "v", "lq", "lk"))
    o = rel_ops.rel_attn(q, k, v, lq, lk, rel, mask)
    np.testing.assert_allclose(o.detach().cpu().numpy(), z["out"], rtol=RTOL, atol=ATOL)
    (o * dev(z["dO"])).sum().backward()
    for n, x in (("dq", q), ("dk", k), ("dv", v), ("dlq", lq), ("dlk", lk)):
        np.testing.assert_allclose(x.grad.cpu().numpy(), z[n], rtol=RTOL, atol=ATOL, err_msg=n)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_disentangled_attn_module_matches_reference(golden):
    from csa_amd.module.disentangled_attn import DisentangledAttn
    z = golden("disentangled_n23")
    B, N, d_model, L = (int(v) for v in z["meta"])
    m = DisentangledAttn(8, d_model, 0.2)
    m.load_state_dict({kk[2:]: torch.from_numpy(v) for kk, v in z.items() if kk.startswith("p:")})
    m = m.cuda().eval()
    rel, mask = (t.cuda() for t in ref_rel_mask(z))
    x, rq = dev(z["x"], True), dev(z["rel_q"], True)
    out, none = m(x, x, x, [rq], rel, mask)
    assert none is None
    np.testing.assert_allclose(out.detach().cpu().numpy(), z["out"], rtol=RTOL, atol=ATOL)
    (out * dev(z["dout"])).sum().backward()
    np.testing.assert_allclose(x.grad.cpu().numpy(), z["dx"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(rq.grad.cpu().numpy(), z["drel_q"], rtol=RTOL, atol=ATOL)
    for pn, p in m.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), z["g:" + pn], rtol=RTOL, atol=ATOL, err_msg=pn)
