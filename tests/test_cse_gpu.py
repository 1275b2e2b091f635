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


def _large_case(z):
    import golden_inputs as gi
    B, H, N, dk, L, seed = (int(v) for v in z["meta"])
    return gi.rel_inputs(B, H, N, dk, L, seed)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
@pytest.mark.parametrize("layout", ["reference", "compact"])
def test_rel_attn_production_head_size_matches_reference(golden, layout):
    """rel_attn at the CSE's production shape (d_k = pegen_dim/8 = 64, N = L = 150) vs the reference
    (tests/golden/rel_attn_n150_dk64.npz; inputs regenerated from PCG64, tests/golden_inputs.py)."""
    from csa_amd import rel_ops
    z = golden("rel_attn_n150_dk64")
    qn, kn, vn, lqn, lkn, dOn = _large_case(z)
    if layout == "reference":
        rel, mask = (t.cuda() for t in ref_rel_mask(z))
    else:
        rel = dev(np.stack([z["L"], z["T"]], 1).astype(np.uint8))
        mask = dev(np.stack([z["L_mask"], z["T_mask"]], 1).astype(np.uint8))
    q, k, v, lq, lk = (dev(a, True) for a in (qn, kn, vn, lqn, lkn))
    o = rel_ops.rel_attn(q, k, v, lq, lk, rel, mask)
    np.testing.assert_allclose(o.detach().cpu().numpy(), z["out"], rtol=RTOL, atol=ATOL)
    (o * dev(dOn)).sum().backward()
    for n, x in (("dq", q), ("dk", k), ("dv", v), ("dlq", lq), ("dlk", lk)):
        np.testing.assert_allclose(x.grad.cpu().numpy(), z[n], rtol=RTOL, atol=ATOL, err_msg=n)


def _run_rel(q, k, v, lq, lk, rel, mask, dO, schedule="auto", bf16=False):
    from csa_amd import rel_ops
    t = [x.cuda().requires_grad_(True) for x in (q, k, v, lq, lk)]
    o = rel_ops.rel_attn(*t, rel.cuda(), mask.cuda(), schedule=schedule, bf16=bf16)
    (o * dO.cuda()).sum().backward()
    torch.cuda.synchronize()
    return [o.detach().cpu()] + [x.grad.cpu() for x in t]


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_rel_attn_bf16_concurrent_schedule_bit_identical():
    """bf16 mode keeps the forking backward (k_rel_qstat + the key-side kernel on the caller's side stream beside
    the query-side one): "concurrent" and "in_order" give bitwise-identical outputs and gradients."""
    from csa_amd.data import synthetic_batch
    B, H, N, dk, L = 64, 8, 150, 64, 150
    sb = synthetic_batch(B, max_size=N, seed=6, min_nodes=60, max_nodes=N)
    g = torch.Generator().manual_seed(10)
    q, k, v, dO = (torch.randn(B, H, N, dk, generator=g) for _ in range(4))
    lq, lk = (torch.randn(1, H, L, dk, generator=g) for _ in range(2))
    rel = torch.from_numpy(np.stack([sb["L"], sb["T"]], 1).astype(np.uint8))
    mask = torch.from_numpy(np.stack([sb["L_mask"], sb["T_mask"]], 1).astype(np.uint8))
    r1 = _run_rel(q, k, v, lq, lk, rel, mask, dO, schedule="in_order", bf16=True)
    r2 = _run_rel(q, k, v, lq, lk, rel, mask, dO, schedule="concurrent", bf16=True)
    for a, b in zip(r1, r2):
        assert torch.equal(a, b)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_rel_attn_full_size_rows_match_oracle_and_deterministic():
    """The java train step's CSE shape (B=64 per GPU, H=8, N=L=150, d_k=64) in the compact layout:
    two runs are bitwise identical (fp32 takes the g-tile handoff, which runs its key and query halves in order
    whatever the schedule, so "in_order" vs "concurrent" here is a run-to-run determinism check; the forking
    path is compared in test_rel_attn_bf16_concurrent_schedule_bit_identical); out/dq/dk/dv of sampled batch rows
    match the fp64 oracle run on
    those rows alone (each row depends only on its AST); dlq/dlk (sums over the whole batch) match
    the fp64 oracle over all 64 rows."""
    from csa_amd.data import synthetic_batch
    from oracle import cse_ref
    B, H, N, dk, L = 64, 8, 150, 64, 150
    sb = synthetic_batch(B, max_size=N, seed=5, min_nodes=60, max_nodes=N)
    g = torch.Generator().manual_seed(9)
    q, k, v, dO = (torch.randn(B, H, N, dk, generator=g) for _ in range(4))
    lq, lk = (torch.randn(1, H, L, dk, generator=g) for _ in range(2))
    rel = torch.from_numpy(np.stack([sb["L"], sb["T"]], 1).astype(np.uint8))
    mask = torch.from_numpy(np.stack([sb["L_mask"], sb["T_mask"]], 1).astype(np.uint8))
    r1 = _run_rel(q, k, v, lq, lk, rel, mask, dO, schedule="in_order")
    r2 = _run_rel(q, k, v, lq, lk, rel, mask, dO, schedule="concurrent")
    for a, b in zip(r1, r2):
        assert torch.equal(a, b)
    refrel, refmask = cse_ref.build_rel_mask(*(torch.from_numpy(sb[n]) for n in ("L", "T", "L_mask", "T_mask")))
    t = [x.double().requires_grad_(True) for x in (q, k, v, lq, lk)]
    o = cse_ref.rel_attn(*t, refrel, refmask)
    (o * dO.double()).sum().backward()
    for b in (0, 17, 63):
        np.testing.assert_allclose(r1[0][b].numpy(), o[b].detach().numpy(), rtol=RTOL, atol=ATOL)
        for i, n in ((1, "dq"), (2, "dk"), (3, "dv")):
            np.testing.assert_allclose(r1[i][b].numpy(), t[i - 1].grad[b].numpy(), rtol=RTOL, atol=ATOL, err_msg=n)
    # dlq / dlk sum B*N terms per bin: fp32 accumulation error grows with the bin's population
    for i, n in ((4, "dlq"), (5, "dlk")):
        ref = t[i - 1].grad.numpy()
        np.testing.assert_allclose(r1[i].numpy(), ref, rtol=RTOL, atol=ATOL * max(1.0, np.abs(ref).max() / 100),
                                   err_msg=n)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
@pytest.mark.parametrize("N", [300, 1040])
def test_rel_attn_long_ast_tile_prep_matches_oracle(N):
    """The three relation-plane prep paths: N = 1040 > 1024 prepares one 32 x 32 tile per workgroup
    (k_rel_prep_t); N = 300 stages whole 32-row blocks in LDS in k_rel_prep's own launch (staged rows > 16 KB); at
    N <= 256 the same 32-row items run as one-wave workgroups of the logits launch, covered by every other test here
    (dword staging at N = 150, byte staging at N = 37 and 23). Random relation codes and masks in the compact
    (B,2,N,N) layout; outputs and gradients vs the fp64 oracle."""
    from oracle import cse_ref
    B, H, dk, L = 1, 8, 64, 150
    g = torch.Generator().manual_seed(21)
    Lr, Tr = (torch.randint(0, L, (B, N, N), generator=g, dtype=torch.int64) for _ in range(2))
    Lm, Tm = ((torch.rand(B, N, N, generator=g) < 0.3) for _ in range(2))
    q, k, v, dO = (torch.randn(B, H, N, dk, generator=g) for _ in range(4))
    lq, lk = (torch.randn(1, H, L, dk, generator=g) for _ in range(2))
    rel = torch.stack([Lr, Tr], 1).to(torch.uint8)
    mask = torch.stack([Lm, Tm], 1).to(torch.uint8)
    r = _run_rel(q, k, v, lq, lk, rel, mask, dO)
    refrel, refmask = cse_ref.build_rel_mask(Lr, Tr, Lm, Tm)
    t = [x.double().requires_grad_(True) for x in (q, k, v, lq, lk)]
    o = cse_ref.rel_attn(*t, refrel, refmask)
    (o * dO.double()).sum().backward()
    np.testing.assert_allclose(r[0].numpy(), o.detach().numpy(), rtol=RTOL, atol=ATOL)
    for i, n in ((1, "dq"), (2, "dk"), (3, "dv"), (4, "dlq"), (5, "dlk")):
        ref = t[i - 1].grad.numpy()
        np.testing.assert_allclose(r[i].numpy(), ref, rtol=RTOL, atol=ATOL * max(1.0, np.abs(ref).max() / 100),
                                   err_msg=n)
