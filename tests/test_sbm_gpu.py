"""GPU parity: fused SBM / dense attention kernels vs the reference's golden vectors and the oracle."""
import numpy as np
import pytest
import torch

from conftest import has_gpu
from csa_amd._lib import CSA_SCHED_CONCURRENT, CSA_SCHED_IN_ORDER
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


def _sbm_vs_oracle(z, Qn, Kn, u, k):
    """Forward + backward of the module with host-supplied uniforms against the closed-form oracle."""
    m = make_module(z, k)
    Q, K, V = dev(Qn, True), dev(Kn, True), dev(z["V"], True)
    m.uniforms = dev(u)
    X, sp, graph, attn = m(Q, K, V, dev(z["mask"]))
    g = graph.detach().cpu().numpy().astype(np.uint8)
    params = {kk[2:]: torch.from_numpy(v) for kk, v in z.items() if kk.startswith("p:")}
    ref, rg = closed_form.sbm_fwd_bwd(torch.from_numpy(Qn), torch.from_numpy(Kn), torch.from_numpy(z["V"]),
                                     torch.from_numpy(z["mask"]), params, torch.from_numpy(u), k, torch.from_numpy(z["dX"]),
                                     torch.from_numpy(z["dsparsity"]), graph_override=torch.from_numpy(g.astype(np.float32)))
    np.testing.assert_allclose(X.detach().cpu().numpy(), ref["X"].numpy(), rtol=RTOL, atol=ATOL)
    ((X * dev(z["dX"])).sum() + (sp * dev(z["dsparsity"])).sum()).backward()
    for name, t, key in (("dQ", Q, "Q"), ("dK", K, "K"), ("dV", V, "V")):
        np.testing.assert_allclose(t.grad.cpu().numpy(), rg[key].numpy(), rtol=RTOL, atol=ATOL, err_msg=name)
    for pn, p in m.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), rg[pn].numpy(), rtol=RTOL, atol=ATOL, err_msg=pn)
    return g, X.detach().cpu().numpy()


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_sbm_rows_without_edges_match_oracle(golden):
    """Query rows that sample no key (u = 1 never samples; host-supplied uniforms) in three of the five query
    blocks, the last, partial one included: their attn row and X row are zero (F.normalize's clamp), and
    every element of theirs is W_NO_EDGE in the backward's one-plane tiles."""
    z = golden("sbm_n150")
    k = int(z["meta"][4])
    u = z["u"].copy()
    rows = [3, 40, 41, 77, 149]
    u[:, :, rows, :] = 1.0
    g, X = _sbm_vs_oracle(z, z["Q"], z["K"], u, k)
    assert not g[:, :, rows, :].any() and not X[:, :, rows, :].any()


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_sbm_degenerate_normaliser_rows_match_oracle(golden):
    """A query row whose sampled keys carry almost no softmax mass (n = sum_j P A < eps = 1e-12, so
    F.normalize divides by eps, not n) has rho = gamma != 0: ds = (A dM - rho) P / sqrt(d) on every key, the
    case where the one-plane backward handoff (W_NO_EDGE) also stores P in the tile's second plane. Built by
    giving query row i and key j one dominant score (Q_i = K_j = t 1, t bisected so that n ~ 1e-13) and
    leaving key j unsampled (u = 1) while every other key of the row is sampled (u = 0)."""
    z = golden("sbm_n150")
    B, H, N, d, k = (int(v) for v in z["meta"])
    Qn, Kn, u = z["Q"].copy(), z["K"].copy(), z["u"].copy()
    i, j = 40, 77
    valid = z["mask"] == 0  # (B, N): keys that take part (sbm_attn.py:61)
    assert valid[:, j].all()

    def mass(t):  # the largest n over (b, h) of row i when Q_i = K_j = t 1 (float64)
        q, kk = Qn.astype(np.float64), Kn.astype(np.float64)
        q[:, :, i, :], kk[:, :, j, :] = t, t
        s = np.einsum("bhd,bhnd->bhn", q[:, :, i, :], kk) / np.sqrt(d)
        s = np.where(valid[:, None, :], s, -np.inf)
        p = np.exp(s - s.max(-1, keepdims=True))
        p /= p.sum(-1, keepdims=True)
        p[:, :, j] = 0.0
        return p.sum(-1)

    lo, hi = 0.5, 6.0  # n(t) falls as t grows
    for _ in range(60):
        mid = 0.5 * (lo + hi)
        lo, hi = (mid, hi) if mass(mid).max() > 1e-13 else (lo, mid)
    t = hi
    n = mass(t)
    assert n.max() <= 1e-13 and n.min() > 1e-18
    Qn[:, :, i, :], Kn[:, :, j, :] = t, t
    u[:, :, i, :] = 0.0
    u[:, :, i, j] = 1.0
    g, X = _sbm_vs_oracle(z, Qn, Kn, u, k)
    assert not g[:, :, i, j].any() and g[:, :, i, :].sum() == B * H * (N - 1) and np.abs(X[:, :, i, :]).max() > 0


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
@pytest.mark.parametrize("case", ["sbm_n37_mapgrad", "sbm_n33_d96_mapgrad"])
def test_sbm_map_gradients_match_reference(golden, case):
    """Gradients through the returned graph and attn maps (sbm_attn.py:66; ABI v4 dattn) as the reference's.
    A graph flip at a near-tie (flips_allowed) is pinned by re-running the CPU oracle with u nudged to the
    GPU's side of the tie."""
    from oracle import sbm_ref
    z = golden(case)
    B, H, N, d, k = (int(v) for v in z["meta"])
    m = make_module(z, k)
    Q, K, V = dev(z["Q"], True), dev(z["K"], True), dev(z["V"], True)
    m.uniforms = dev(z["u"])
    X, sp, graph, attn = m(Q, K, V, dev(z["mask"]))
    g = graph.detach().cpu().numpy().astype(np.uint8)
    nflip = flips_allowed(g, z)
    loss = ((X * dev(z["dX"])).sum() + (sp * dev(z["dsparsity"])).sum() + (graph * dev(z["dgraph"])).sum()
            + (attn * dev(z["dattn"])).sum())
    loss.backward()
    if nflip == 0:
        ref = {n: z[n] for n in ("dQ", "dK", "dV")}
        ref.update({pn: z["g:" + pn] for pn, _ in m.named_parameters()})
    else:
        u = z["u"].copy()
        u[g != z["graph"]] = np.where(g[g != z["graph"]] == 1, 0.0, 1.0)  # force the GPU's samples
        tq, tk, tv = (torch.from_numpy(z[n]).requires_grad_(True) for n in ("Q", "K", "V"))
        params = {kk[2:]: torch.from_numpy(v).requires_grad_(True) for kk, v in z.items() if kk.startswith("p:")}
        Xr, spr, gr, ar = sbm_ref.sbm_attention(tq, tk, tv, torch.from_numpy(z["mask"]), params, torch.from_numpy(u), k)
        ((Xr * torch.from_numpy(z["dX"])).sum() + (spr * torch.from_numpy(z["dsparsity"])).sum()
         + (gr * torch.from_numpy(z["dgraph"])).sum() + (ar * torch.from_numpy(z["dattn"])).sum()).backward()
        ref = {"dQ": tq.grad.numpy(), "dK": tk.grad.numpy(), "dV": tv.grad.numpy()}
        ref.update({pn: params[pn].grad.numpy() for pn in params})
    for name, t in (("dQ", Q), ("dK", K), ("dV", V)):
        np.testing.assert_allclose(t.grad.cpu().numpy(), ref[name], rtol=RTOL, atol=ATOL, err_msg=name)
    for pn, p in m.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), ref[pn], rtol=RTOL, atol=ATOL, err_msg=pn)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_full_attention_attn_gradient_matches_reference(golden):
    from csa_amd.module.sbm_attn import FullAttention
    z = golden("full_n37_mapgrad")
    B, H, N, d = (int(v) for v in z["meta"])
    m = FullAttention({"attention_dropout": 0.2, "head_dim": d, "num_head": H}, 0).cuda().eval()
    Q, K, V = dev(z["Q"], True), dev(z["K"], True), dev(z["V"], True)
    X, sp, graph, attn = m(Q, K, V, dev(z["mask"]))
    ((X * dev(z["dX"])).sum() + (attn * dev(z["dattn"])).sum()).backward()
    for name, t in (("dQ", Q), ("dK", K), ("dV", V)):
        np.testing.assert_allclose(t.grad.cpu().numpy(), z[name], rtol=RTOL, atol=ATOL, err_msg=name)


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



def _rand_case(B, H, N, d, k, seed, pad=True):
    g = torch.Generator().manual_seed(seed)
    Q, K, V = (torch.randn(B, H, N, d, generator=g) for _ in range(3))
    mask = torch.zeros(B, N)
    if pad:
        for b in range(B):
            n = int(torch.randint(max(1, N // 3), N + 1, (1,), generator=g))
            mask[b, n:] = 1.0
    u = torch.rand(B, H, N, N, generator=g)
    dX = torch.randn(B, H, N, d, generator=g)
    dsp = torch.full((H,), 3.125e-4)
    params = {"layer.weight": torch.nn.init.orthogonal_(torch.empty(H * k, d), generator=g)}
    for i in (0, 3, 6):
        params[f"proj.{i}.weight"] = torch.nn.init.xavier_uniform_(torch.empty(d, d), generator=g)
        params[f"proj.{i}.bias"] = 0.1 * torch.randn(d, generator=g)
    return Q, K, V, mask, u, dX, dsp, params


def _run_module(Q, K, V, mask, u, dX, dsp, params, k, training=False):
    from csa_amd.module.sbm_attn import SBMAttention
    B, H, N, d = Q.shape
    m = SBMAttention({"attention_dropout": 0.2, "head_dim": d, "num_head": H, "num_clusters": [k]}, 0)
    m.load_state_dict(params, strict=False)
    m = m.cuda().train(training)
    q, kk, v = (t.cuda().requires_grad_(True) for t in (Q, K, V))
    if u is not None:
        m.uniforms = u.cuda()
    X, sp, graph, attn = m(q, kk, v, mask.cuda())
    torch.autograd.backward([X, sp], [dX.cuda(), dsp.cuda()])
    grads = {n: p.grad.detach().cpu() for n, p in m.named_parameters()}
    return X.detach().cpu(), sp.detach().cpu(), graph.detach().cpu(), q.grad.cpu(), kk.grad.cpu(), v.grad.cpu(), grads


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
@pytest.mark.parametrize("shape", [(2, 2, 45, 64, 5), (2, 2, 200, 64, 64), (1, 2, 70, 64, 128), (1, 3, 150, 96, 20),
                                   (1, 2, 33, 64, 32), (1, 1, 1024, 64, 16), (1, 1, 1024, 64, 32),
                                   (1, 1, 1024, 64, 64), (1, 1, 1024, 64, 128)])
def test_sbm_shapes_vs_oracle(shape):
    """Shapes beyond the golden set (small k, k up to 128 = config-5 sweep, N > 150 up to the
    config-5 long-AST N = 1024) vs the pinned oracle."""
    B, H, N, d, k = shape
    Q, K, V, mask, u, dX, dsp, params = _rand_case(B, H, N, d, k, seed=sum(shape))
    X, sp, graph, dQ, dK, dV, grads = _run_module(Q, K, V, mask, u, dX, dsp, params, k)
    ref, rg = closed_form.sbm_fwd_bwd(Q, K, V, mask, params, u, k, dX, dsp, graph_override=graph)
    near = (torch.abs(u - ref["expA"].clamp(0.01, 0.99)) < 1e-6)
    assert bool(torch.all(near[graph != ref["graph"].float()])), "graph flips away from fp32 ties"
    np.testing.assert_allclose(X.numpy(), ref["X"].numpy(), rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(sp.numpy(), ref["sparsity"].numpy(), rtol=1e-6)
    for name, t, key in (("dQ", dQ, "Q"), ("dK", dK, "K"), ("dV", dV, "V")):
        np.testing.assert_allclose(t.numpy(), rg[key].numpy(), rtol=RTOL, atol=ATOL, err_msg=name)
    for pn, gv in grads.items():
        if pn.startswith("orth_clusters"):
            continue
        np.testing.assert_allclose(gv.numpy(), rg[pn].numpy(), rtol=RTOL, atol=ATOL, err_msg=pn)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_sbm_full_size_rows_match_oracle_and_deterministic():
    """BASELINE config 2 size (B=256, H=8, N=150, d=64, k=10): per-AST outputs/grads depend only on that
    AST, so sampled batch rows are checked against the oracle run on those rows alone; the batch-reduced
    parameter gradients against the fp64 oracle over the whole batch; and two runs are bitwise identical
    (fixed-order reductions, integer atomics only)."""
    B, H, N, d, k = 256, 8, 150, 64, 10
    Q, K, V, mask, u, dX, dsp, params = _rand_case(B, H, N, d, k, seed=7)
    r1 = _run_module(Q, K, V, mask, u, dX, dsp, params, k)
    r2 = _run_module(Q, K, V, mask, u, dX, dsp, params, k)
    for a, b in zip(r1[:6], r2[:6]):
        assert torch.equal(a, b)
    for n in r1[6]:
        assert torch.equal(r1[6][n], r2[6][n]), n
    X, sp, graph, dQ, dK, dV, _ = r1
    for b in (0, 131, 255):
        sl = slice(b, b + 1)
        ref, rg = closed_form.sbm_fwd_bwd(Q[sl], K[sl], V[sl], mask[sl], params, u[sl], k, dX[sl], dsp,
                                         graph_override=graph[sl])
        np.testing.assert_allclose(X[sl].numpy(), ref["X"].numpy(), rtol=RTOL, atol=ATOL)
        # the sparsity gradient scale is 1/(B N M) over the whole batch: rescale the oracle's dsp
        ref2, rg2 = closed_form.sbm_fwd_bwd(Q[sl], K[sl], V[sl], mask[sl], params, u[sl], k, dX[sl], dsp / B,
                                           graph_override=graph[sl])
        np.testing.assert_allclose(dV[sl].numpy(), rg2["V"].numpy(), rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(dQ[sl].numpy(), rg2["Q"].numpy(), rtol=RTOL, atol=ATOL)
        np.testing.assert_allclose(dK[sl].numpy(), rg2["K"].numpy(), rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(sp.numpy(), graph.sum((0, 2, 3)).numpy() / (B * N * N), rtol=1e-6)
    # the batch-reduced parameter gradients (dC, dW, db: sums over all 256 x 8 x 300 rows through the
    # per-workgroup slabs and k_reduce_slabs) against the fp64 closed form summed over 16-row chunks (each
    # chunk's sparsity gradient rescaled to the whole batch's 1 / (B N M))
    C = 16
    tot = None
    for b0 in range(0, B, C):
        sl = slice(b0, b0 + C)
        _, rg = closed_form.sbm_fwd_bwd(Q[sl], K[sl], V[sl], mask[sl], params, u[sl], k, dX[sl], dsp * C / B,
                                        graph_override=graph[sl])
        part = {n: rg[n] for n in params}
        tot = part if tot is None else {n: tot[n] + part[n] for n in params}
    for n, ref in tot.items():
        got = r1[6][n]
        np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=RTOL, atol=ATOL * max(1.0, float(ref.abs().max())),
                                   err_msg=n)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
@pytest.mark.parametrize("shape", [(64, 8, 150, 64, 10), (8, 8, 150, 96, 10)])
@pytest.mark.parametrize("with_dattn", [False, True])
def test_concurrent_backward_schedule_bit_identical(shape, with_dattn):
    """CSA_SCHED_CONCURRENT vs CSA_SCHED_IN_ORDER: the projection backward's key-block items (k_proj_bwd_s kind 1)
    on the caller's side stream beside k_attn_bwd_qg, its query-block items (kind 2) after it, against both kinds
    in ONE in-order launch (kind 3). Every workgroup gets the same items and slab either way, so every output and
    gradient is bitwise identical -- train mode with dropout and padded keys; without an upstream dattn (the
    training path: one-plane W_NO_EDGE handoff) and with one (the two-plane ds | G handoff)."""
    B, H, N, d, k = shape
    Q, K, V, mask, _, dX, dsp, params = _rand_case(B, H, N, d, k, seed=41 + d)
    cw = params["layer.weight"].cuda()
    pw = [params[f"proj.{i}.weight"].cuda() for i in (0, 3, 6)]
    pb = [params[f"proj.{i}.bias"].cuda() for i in (0, 3, 6)]
    q, kk, v, mk = Q.cuda(), K.cuda(), V.cuda(), mask.cuda()
    gen = torch.Generator().manual_seed(3)
    dattn = torch.randn(B, H, N, N, generator=gen).cuda() if with_dattn else None
    seed, offset = 0x5EED, 9
    X, sp, state = torch.ops.csa.sbm_fwd(q, kk, v, mk, cw, pw, pb, None, k, seed, offset, 0.2, 0.1, False)
    outs = []
    for mode in (CSA_SCHED_IN_ORDER, CSA_SCHED_CONCURRENT):
        g = torch.ops.csa.sbm_bwd(q, kk, v, mk, cw, pw, pb, k, 0.2, 0.1, seed, offset, False, state, X,
                                  dX.cuda(), dsp.cuda(), None, dattn=dattn, schedule=mode)
        torch.cuda.synchronize()
        outs.append([t.cpu() for t in g if isinstance(t, torch.Tensor)])
    assert len(outs[0]) == len(outs[1]) > 0
    for a, b in zip(*outs):
        assert torch.equal(a, b)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_forward_only_state_under_no_grad_gives_the_same_outputs():
    """Under torch.no_grad() / inference_mode the module's parameters still require grad, but no backward can
    run: the forward takes CSA_FLAG_FWD_ONLY (no saved MLP activations) and must return exactly the outputs of the
    grad-enabled forward."""
    from csa_amd import ops
    B, H, N, d, k = 4, 8, 150, 64, 10
    Q, K, V, mask, u, _, _, params = _rand_case(B, H, N, d, k, seed=19)
    cw = params["layer.weight"].cuda().requires_grad_()
    proj = []
    for i in (0, 3, 6):
        proj += [params[f"proj.{i}.weight"].cuda().requires_grad_(), params[f"proj.{i}.bias"].cuda().requires_grad_()]
    q, kk, v, mk, uu = (t.cuda() for t in (Q, K, V, mask, u))
    assert not ops._fwd_only(q, cw) and ops._fwd_only(q.detach())
    ref = ops.sbm_attention(q, kk, v, mk, cw, proj, k, uniforms=uu)
    for ctx in (torch.no_grad, torch.inference_mode):
        with ctx():
            assert ops._fwd_only(q, cw, *proj)
            got = ops.sbm_attention(q, kk, v, mk, cw, proj, k, uniforms=uu)
        for a, b in zip(ref, got):
            assert torch.equal(a.detach(), b)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_train_mode_dropout_statistics_and_determinism():
    """Train mode (in-kernel Philox sampling + dropout): same seed -> identical; keep-rate ~0.8;
    sampled-edge rate matches E[clamp(expA)]."""
    from csa_amd import ops
    B, H, N, d, k = 16, 8, 150, 64, 10
    Q, K, V, mask, u, dX, dsp, params = _rand_case(B, H, N, d, k, seed=11, pad=False)
    torch.manual_seed(5)
    r1 = _run_module(Q, K, V, mask, None, dX, dsp, params, k, training=True)
    torch.manual_seed(5)
    r2 = _run_module(Q, K, V, mask, None, dX, dsp, params, k, training=True)
    for a, b in zip(r1[:6], r2[:6]):
        assert torch.equal(a, b)
    ref, _ = closed_form.sbm_fwd_bwd(Q, K, V, mask, params, u, k, dX, dsp)
    # E[sparsity_h] = mean clamp(expA) (proj dropout perturbs expA slightly in train mode)
    np.testing.assert_allclose(r1[1].numpy(), ref["expA"].clamp(0.01, 0.99).mean((0, 2, 3)).numpy(), rtol=0.05)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
@pytest.mark.parametrize("shape", [(2, 2, 150, 64, 10), (1, 2, 45, 96, 5)])
def test_train_mode_matches_oracle_with_regenerated_masks(shape):
    """Train mode end to end: the oracle regenerates the kernels' Philox streams (oracle/philox.py) --
    attention dropout, both proj-dropout layers of the Q and K MLPs -- and the STE draws; the sampled
    graph must equal u16 < clamp(expA) * 65536 away from fp32 ties, and X / sparsity / every gradient
    must match the fp64 closed form run with those masks."""
    from oracle import philox
    B, H, N, d, k = shape
    Q, K, V, mask, _, dX, dsp, params = _rand_case(B, H, N, d, k, seed=3 * sum(shape))
    seed, offset, attn_p, proj_p = (0x1234567 << 32) | 0x89ABCDE, 77, 0.2, 0.1
    cw = params["layer.weight"].cuda()
    pw = [params[f"proj.{i}.weight"].cuda() for i in (0, 3, 6)]
    pb = [params[f"proj.{i}.bias"].cuda() for i in (0, 3, 6)]
    q, kk, v, mk = Q.cuda(), K.cuda(), V.cuda(), mask.cuda()
    X, sp, state = torch.ops.csa.sbm_fwd(q, kk, v, mk, cw, pw, pb, None, k, seed, offset, attn_p, proj_p, False)
    graph, _ = torch.ops.csa.sbm_maps(q, kk, v, mk, state, k, False)
    g = torch.ops.csa.sbm_bwd(q, kk, v, mk, cw, pw, pb, k, attn_p, proj_p, seed, offset, False, state, X,
                              dX.cuda(), dsp.cuda(), None)
    torch.cuda.synchronize()
    graph = graph.cpu()
    keep = philox.attn_keep(B, H, N, N, seed, offset, attn_p)
    ks = 1.0 / (1.0 - np.float32(proj_p))
    pk = {f"{s}{l}": torch.from_numpy(philox.proj_keep(B, H, N, d, seed, offset, proj_p, l, int(s == "k")) * ks)
          for s in "qk" for l in (0, 1)}
    assert 0.75 < keep.mean() < 0.85 and all(0.85 < float((t > 0).double().mean()) < 0.95 for t in pk.values())
    ref, rg = closed_form.sbm_fwd_bwd(Q, K, V, mask, params, None, k, dX, dsp,
                                     attn_keep=torch.from_numpy(keep / (1.0 - np.float32(attn_p))), proj_keep=pk,
                                     graph_override=graph)
    # STE draws: the GPU graph is the regenerated u16 draws against the oracle's expA (fp32 ties aside)
    u16 = philox.attn_uniforms(B, H, N, N, seed, offset, philox.RNG_STE)
    want = philox.ste_graph(ref["expA"].numpy(), u16)
    thr = np.clip(ref["expA"].numpy(), 0.01, 0.99) * 65536.0
    diff = want != graph.numpy().astype(bool)
    assert np.all(np.abs(u16[diff] - thr[diff]) < 0.5), f"{int(diff.sum())} graph flips away from ties"
    assert diff.mean() < 1e-4
    np.testing.assert_allclose(X.cpu().numpy(), ref["X"].numpy(), rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(sp.cpu().numpy(), ref["sparsity"].numpy(), rtol=1e-6)
    names = ["Q", "K", "V", "layer.weight", "proj.0.weight", "proj.0.bias", "proj.3.weight", "proj.3.bias",
             "proj.6.weight", "proj.6.bias"]
    for name, t in zip(names, g):
        np.testing.assert_allclose(t.cpu().numpy(), rg[name].numpy(), rtol=RTOL, atol=ATOL, err_msg=name)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_broadcast_upstream_gradient_is_materialised():
    """X.sum((0, 1, 2)) hands the backward a (B,H,N,d) gradient with strides (0, 0, 0, 1). The ABI reads an
    all-zero stride triple as "contiguous", so the op must materialise it: the gradients must equal those of
    an explicit contiguous ones() upstream gradient, bit for bit (SBM and CSE)."""
    from csa_amd import rel_ops
    from csa_amd.module.sbm_attn import SBMAttention
    B, H, N, d, k = 2, 8, 37, 64, 10
    Q, K, V, mask, u, _, _, params = _rand_case(B, H, N, d, k, seed=5)
    m = SBMAttention({"attention_dropout": 0.2, "head_dim": d, "num_head": H, "num_clusters": [k]}, 0)
    m.load_state_dict(params, strict=False)
    m = m.cuda().eval()
    outs = []
    for broadcast in (True, False):
        q, kk, v = (t.cuda().requires_grad_(True) for t in (Q, K, V))
        m.uniforms = u.cuda()
        X, sp, _, _ = m(q, kk, v, mask.cuda())
        if broadcast:
            X.sum((0, 1, 2)).sum().backward()
        else:
            X.backward(torch.ones(X.shape, device="cuda"))
        outs.append([q.grad.cpu(), kk.grad.cpu(), v.grad.cpu()] + [p.grad.cpu() for p in m.parameters()])
        m.zero_grad(set_to_none=True)
    for a, b in zip(*outs):
        assert torch.equal(a, b)
    g = torch.Generator().manual_seed(3)
    q, kk, v = (torch.randn(B, H, N, 64, generator=g) for _ in range(3))
    lq, lk = (torch.randn(1, H, 150, 64, generator=g) for _ in range(2))
    rel = torch.randint(0, 150, (B, 2, N, N), generator=g).to(torch.uint8)
    msk = (torch.rand(B, 2, N, N, generator=g) < 0.1).to(torch.uint8)
    outs = []
    for broadcast in (True, False):
        t = [x.cuda().requires_grad_(True) for x in (q, kk, v, lq, lk)]
        o = rel_ops.rel_attn(*t, rel.cuda(), msk.cuda())
        if broadcast:
            o.sum((0, 1, 2)).sum().backward()
        else:
            o.backward(torch.ones(o.shape, device="cuda"))
        outs.append([x.grad.cpu() for x in t])
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def _dead_tile_masks(B, N):
    """Key masks with whole 32-key tiles masked (padded ASTs): suffix padding at 1, 31, 64 and N valid keys, the
    first tile masked, a masked middle tile between live ones, and every key masked."""
    mask = torch.zeros(B, N)
    lens = [1, 31, 64, N]
    for b in range(min(B, 4)):
        mask[b, lens[b]:] = 1.0
    if B > 4:
        mask[4, :32] = 1.0  # the first key tile dead (the kernels still run it as live)
    if B > 5:
        mask[5, 32:64] = 1.0  # a dead tile between live ones
    if B > 6:
        mask[6, :] = 1.0  # every key masked: X rows of uniform attention over nothing (0/0 as the reference)
    return mask


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
@pytest.mark.parametrize("shape", [(6, 2, 150, 64, 10), (6, 2, 100, 96, 16), (6, 1, 300, 64, 64), (2, 1, 2080, 64, 10)])
def test_sbm_dead_key_tiles_match_oracle(shape):
    """Key tiles whose every key is masked run the light paths (forward: after the live tiles, expA, sampling and
    the graph's bit words only; k_attn_bwd_kv: a whole masked key block carries only the STE term into dT and stores
    no w tiles; k_attn_bwd_qg: no dQ products for a dead tile, its A bits from the forward's words). N = 2080 has 65
    key tiles, past the 64-tile dead-tile record: every tile runs the full path there. The sampled graph (padded
    positions included, sbm_attn.py:64), the sparsity, X, dQ / dK / dV and every parameter gradient -- dC and the MLP
    weights take the STE term of the dead tiles' edges -- against the fp64 closed form; two runs bitwise identical."""
    B, H, N, d, k = shape
    # (seed 97 + N at d = 96, k = 16 put one projection-MLP activation of an unpadded AST within fp32 rounding of
    # the ReLU kink: its K row's dK differs from the fp64 oracle by 1e-3 relative in every build, the round-start one
    # included -- a tie like the sampling ties above, not a dead-tile effect; profiles/r06_dead_tile_diag.txt)
    Q, K, V, _, u, dX, dsp, params = _rand_case(B, H, N, d, k, seed=101 + N)
    mask = _dead_tile_masks(B, N)
    r1 = _run_module(Q, K, V, mask, u, dX, dsp, params, k)
    r2 = _run_module(Q, K, V, mask, u, dX, dsp, params, k)
    for a, b in zip(r1[:6], r2[:6]):
        assert torch.equal(a, b)
    X, sp, graph, dQ, dK, dV, grads = r1
    ref, rg = closed_form.sbm_fwd_bwd(Q, K, V, mask, params, u, k, dX, dsp, graph_override=graph)
    near = (torch.abs(u - ref["expA"].clamp(0.01, 0.99)) < 1e-6)
    assert bool(torch.all(near[graph != ref["graph"].float()])), "graph flips away from fp32 ties"
    assert float(graph[:, :, :, 64:].sum()) > 0  # sampled edges at padded keys are kept (and counted)
    np.testing.assert_allclose(sp.numpy(), ref["sparsity"].numpy(), rtol=1e-6)
    live = mask.sum(1) < N  # rows with no valid key are 0/0 in the reference (NaN) -- compared where finite
    np.testing.assert_allclose(X[live].numpy(), ref["X"][live].numpy(), rtol=RTOL, atol=ATOL)
    for name, t, key in (("dQ", dQ, "Q"), ("dK", dK, "K"), ("dV", dV, "V")):
        np.testing.assert_allclose(t[live].numpy(), rg[key][live].numpy(), rtol=RTOL, atol=ATOL, err_msg=name)
    assert torch.all(dK[~live] == 0) and torch.all(dV[~live] == 0)
    if bool(live.all()):
        for pn, gv in grads.items():
            np.testing.assert_allclose(gv.numpy(), rg[pn].numpy(), rtol=RTOL, atol=ATOL, err_msg=pn)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_sbm_dead_key_tiles_parameter_gradients_match_oracle():
    """The STE-only gradient of fully masked key tiles into the cluster weights and the projection MLP (dC, dW, db)
    over a batch where most tiles are dead, against the fp64 closed form."""
    B, H, N, d, k = 6, 8, 150, 64, 10
    Q, K, V, _, u, dX, dsp, params = _rand_case(B, H, N, d, k, seed=1234)
    mask = _dead_tile_masks(B, N)
    X, sp, graph, dQ, dK, dV, grads = _run_module(Q, K, V, mask, u, dX, dsp, params, k)
    _, rg = closed_form.sbm_fwd_bwd(Q, K, V, mask, params, u, k, dX, dsp, graph_override=graph)
    for pn, gv in grads.items():
        np.testing.assert_allclose(gv.numpy(), rg[pn].numpy(), rtol=RTOL, atol=ATOL * max(1.0, float(rg[pn].abs().max())),
                                   err_msg=pn)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_train_mode_dead_key_tiles_match_oracle_with_regenerated_masks():
    """Train mode (in-kernel Philox draws) over dead key tiles: the light forward still draws the STE uniforms of
    every tile (not the keep bits of a dead tile, which nothing reads: its P is 0), so the graph equals the
    regenerated u16 < clamp(expA) 65536 and every gradient matches the closed form under the regenerated masks."""
    from oracle import philox
    B, H, N, d, k = 6, 2, 150, 64, 10
    Q, K, V, _, _, dX, dsp, params = _rand_case(B, H, N, d, k, seed=4321)
    mask = _dead_tile_masks(B, N)
    seed, offset, attn_p, proj_p = (0x2468ACE << 32) | 0x1357BDF, 5, 0.2, 0.1
    cw = params["layer.weight"].cuda()
    pw = [params[f"proj.{i}.weight"].cuda() for i in (0, 3, 6)]
    pb = [params[f"proj.{i}.bias"].cuda() for i in (0, 3, 6)]
    q, kk, v, mk = Q.cuda(), K.cuda(), V.cuda(), mask.cuda()
    X, sp, state = torch.ops.csa.sbm_fwd(q, kk, v, mk, cw, pw, pb, None, k, seed, offset, attn_p, proj_p, False)
    graph, _ = torch.ops.csa.sbm_maps(q, kk, v, mk, state, k, False)
    g = torch.ops.csa.sbm_bwd(q, kk, v, mk, cw, pw, pb, k, attn_p, proj_p, seed, offset, False, state, X,
                              dX.cuda(), dsp.cuda(), None)
    torch.cuda.synchronize()
    graph = graph.cpu()
    keep = philox.attn_keep(B, H, N, N, seed, offset, attn_p)
    ks = 1.0 / (1.0 - np.float32(proj_p))
    pk = {f"{s}{l}": torch.from_numpy(philox.proj_keep(B, H, N, d, seed, offset, proj_p, l, int(s == "k")) * ks)
          for s in "qk" for l in (0, 1)}
    ref, rg = closed_form.sbm_fwd_bwd(Q, K, V, mask, params, None, k, dX, dsp,
                                     attn_keep=torch.from_numpy(keep / (1.0 - np.float32(attn_p))), proj_keep=pk,
                                     graph_override=graph)
    u16 = philox.attn_uniforms(B, H, N, N, seed, offset, philox.RNG_STE)
    want = philox.ste_graph(ref["expA"].numpy(), u16)
    thr = np.clip(ref["expA"].numpy(), 0.01, 0.99) * 65536.0
    diff = want != graph.numpy().astype(bool)
    assert np.all(np.abs(u16[diff] - thr[diff]) < 0.5), f"{int(diff.sum())} graph flips away from ties"
    assert float(graph[:, :, :, 64:].sum()) > 0  # dead tiles sample too
    np.testing.assert_allclose(X.cpu().numpy(), ref["X"].numpy(), rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(sp.cpu().numpy(), ref["sparsity"].numpy(), rtol=1e-6)
    names = ["Q", "K", "V", "layer.weight", "proj.0.weight", "proj.0.bias", "proj.3.weight", "proj.3.bias",
             "proj.6.weight", "proj.6.bias"]
    for name, t in zip(names, g):
        np.testing.assert_allclose(t.cpu().numpy(), rg[name].numpy(), rtol=RTOL, atol=ATOL, err_msg=name)


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_map_gradient_path_over_dead_key_tiles_matches_training_path():
    """Upstream map gradients select the two-plane ds | G handoff with k_attn_rowprep's row constants; there a dead
    key block stores ds = 0 and its G tiles for the query side, where the training path stores no tile for it.
    Zero dgraph / dattn must give the training path's gradients (train mode, dropout, dead tiles)."""
    B, H, N, d, k = 6, 2, 150, 64, 10
    Q, K, V, _, _, dX, dsp, params = _rand_case(B, H, N, d, k, seed=777)
    mask = _dead_tile_masks(B, N)
    cw = params["layer.weight"].cuda()
    pw = [params[f"proj.{i}.weight"].cuda() for i in (0, 3, 6)]
    pb = [params[f"proj.{i}.bias"].cuda() for i in (0, 3, 6)]
    q, kk, v, mk = Q.cuda(), K.cuda(), V.cuda(), mask.cuda()
    seed, offset = 0xDEAD5EED, 3
    X, sp, state = torch.ops.csa.sbm_fwd(q, kk, v, mk, cw, pw, pb, None, k, seed, offset, 0.2, 0.1, False)
    g0 = torch.ops.csa.sbm_bwd(q, kk, v, mk, cw, pw, pb, k, 0.2, 0.1, seed, offset, False, state, X,
                               dX.cuda(), dsp.cuda(), None)
    zeros = torch.zeros(B, H, N, N, device="cuda")
    g1 = torch.ops.csa.sbm_bwd(q, kk, v, mk, cw, pw, pb, k, 0.2, 0.1, seed, offset, False, state, X,
                               dX.cuda(), dsp.cuda(), zeros, dattn=zeros)
    torch.cuda.synchronize()
    a = [t.cpu() for t in g0 if isinstance(t, torch.Tensor)]
    b = [t.cpu() for t in g1 if isinstance(t, torch.Tensor)]
    assert len(a) == len(b) > 0
    for i, (x, y) in enumerate(zip(a, b)):
        # the two paths sum gamma = rowsum(dX * X) in different orders: fp32 rounding apart
        np.testing.assert_allclose(y.numpy(), x.numpy(), rtol=1e-4, atol=1e-5 * max(1.0, float(x.abs().max())),
                                   err_msg=f"output {i}")


@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_full_attention_dead_key_tiles_match_oracle():
    """FullAttention (config 4) over dead key tiles: the same light paths without clusters -- X and dQ / dK / dV
    against the oracle's autograd (eval mode)."""
    from csa_amd.module.sbm_attn import FullAttention
    from oracle import sbm_ref
    B, H, N, d = 6, 2, 150, 64
    g = torch.Generator().manual_seed(55)
    Q, K, V, dX = (torch.randn(B, H, N, d, generator=g) for _ in range(4))
    mask = _dead_tile_masks(B, N)
    m = FullAttention({"attention_dropout": 0.2, "head_dim": d, "num_head": H}, 0).cuda().eval()
    q, kk, v = (t.cuda().requires_grad_(True) for t in (Q, K, V))
    X = m(q, kk, v, mask.cuda())[0]
    X.backward(dX.cuda())
    qr, kr, vr = (t.clone().double().requires_grad_(True) for t in (Q, K, V))
    Xr = sbm_ref.full_attention(qr, kr, vr, mask.double())
    Xr = Xr[0] if isinstance(Xr, tuple) else Xr
    Xr.backward(dX.double())
    np.testing.assert_allclose(X.detach().cpu().numpy(), Xr.detach().numpy(), rtol=RTOL, atol=ATOL)
    for name, a, r in (("dQ", q, qr), ("dK", kk, kr), ("dV", v, vr)):
        np.testing.assert_allclose(a.grad.cpu().numpy(), r.grad.numpy(), rtol=RTOL, atol=ATOL, err_msg=name)
