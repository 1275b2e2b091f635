"""Generate golden vectors by running the REFERENCE itself (this container only).

Imports /root/reference/module/{components,STE,sbm_attn,disentangled_attn}.py standalone
(SURVEY.md Appendix A recipe: a synthetic ``module`` package, no shims needed), drives the
reference's own ``torch.bernoulli`` with host-supplied uniforms (``u < p``; this script first
re-verifies that this is bit-identical to the real CPU draw), runs forward + backward on
seeded inputs, and writes small ``.npz`` fixtures to tests/golden/. The reference never
travels to the GPU box; only these fixtures do.

Run:  PYTHONDONTWRITEBYTECODE=1 python tools/gen_golden.py [large | dims | mapgrad | ast]
      (`large` = only the production-shape fixtures: rel_attn_n150_dk64, greedy_tiny, csatrans_java;
       `dims` = csatrans_java + csatrans_python with their fp64 error budgets)
"""
import importlib.util
import math
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden")
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "code-structure-aware-transformer_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))  # oracle/ (fp64 error budget)
from csa_amd.data import synthetic_batch  # noqa: E402
import golden_inputs as gi  # noqa: E402


def load_reference():
    pkg = types.ModuleType("module")
    pkg.__path__ = [f"{REF}/module"]
    sys.modules["module"] = pkg

    def load(n):
        s = importlib.util.spec_from_file_location(f"module.{n}", f"{REF}/module/{n}.py")
        m = importlib.util.module_from_spec(s)
        sys.modules[f"module.{n}"] = m
        s.loader.exec_module(m)
        return m

    comp = load("components")
    pkg._get_clones, pkg.transpose_for_scores = comp._get_clones, comp.transpose_for_scores
    return load("STE"), load("sbm_attn"), load("disentangled_attn")


STE, SA, DA = load_reference()
_real_bernoulli = torch.bernoulli


def verify_bernoulli_equivalence():
    """torch.bernoulli(p) == (torch.rand(p.shape) < p) under the same seed (CPU)."""
    ok = True
    for shape in [(1, 8, 150, 150), (7, 8, 150, 150), (3, 2, 37, 37)]:
        p = torch.rand(shape, generator=torch.Generator().manual_seed(5)).clamp(0.01, 0.99)
        torch.manual_seed(123)
        a = _real_bernoulli(p)
        torch.manual_seed(123)
        b = (torch.rand(p.shape) < p).float()
        ok &= bool(torch.equal(a, b))
    return ok


class HostUniforms:
    """Context manager: make the reference's torch.bernoulli consume the given uniforms."""

    def __init__(self, u):
        self.u = u

    def __enter__(self):
        torch.bernoulli = lambda p: (self.u < p).to(p.dtype)

    def __exit__(self, *a):
        torch.bernoulli = _real_bernoulli


def np32(t):
    return t.detach().cpu().numpy().astype(np.float32)


def sbm_case(name, B, H, N, d, k, pad_counts, seed, zero_row=None, noncontig=False, map_grads=False):
    g = torch.Generator().manual_seed(seed)
    torch.manual_seed(seed)
    mod = SA.SBMAttention({"attention_dropout": 0.2, "head_dim": d, "num_head": H, "num_clusters": [k]}, 0)
    for n_, p in mod.named_parameters():  # CSATrans init: xavier for dim>1, orthogonal clusters
        if p.dim() > 1:
            torch.nn.init.xavier_uniform_(p)
    torch.nn.init.orthogonal_(mod.layer.weight)
    mod.eval()
    if noncontig:  # (B,N,H*d) -> split_heads view, as Attention.forward produces
        base = lambda: torch.randn(B, N, H * d, generator=g).reshape(B, N, H, d).transpose(1, 2)
        Q, K, V = base(), base(), base()
    else:
        Q, K, V = (torch.randn(B, H, N, d, generator=g) for _ in range(3))
    Q.requires_grad_(True); K.requires_grad_(True); V.requires_grad_(True)
    mask = torch.zeros(B, N)
    for b, pc in enumerate(pad_counts):
        if pc:
            mask[b, N - pc:] = 1.0
    u = torch.rand(B, H, N, N, generator=g)
    if zero_row is not None:
        b, h, i = zero_row
        u[b, h, i, :] = 0.995  # > clamp ceiling 0.99 -> sampled graph row all-zero
    dX = torch.randn(B, H, N, d, generator=g)
    dsp = torch.full((H,), 3.125e-4) + 1e-4 * torch.randn(H, generator=g)
    with HostUniforms(u):
        X, sparsity, graph, attn = mod(Q, K, V, mask)
    # expA exactly as the reference computes it (sbm_attn.py:37-55), for the bit-exact sampler test
    with torch.no_grad():
        c = mod.layer.weight.reshape(H, k, -1)
        S = torch.softmax(torch.matmul(c, c.transpose(-1, -2)).reshape(H, k * k), -1).reshape(H, k, k).unsqueeze(0).repeat((B, 1, 1, 1))
        Qh = torch.sigmoid(torch.matmul(mod.proj(Q), c.transpose(-1, -2)))
        Kh = torch.sigmoid(torch.matmul(mod.proj(K), c.transpose(-1, -2)))
        expA = torch.matmul(Qh, torch.matmul(S, Kh.transpose(-1, -2)))
    loss = (X * dX).sum() + (sparsity * dsp).sum()
    extra = {}
    if map_grads:  # upstream gradients of the returned graph and attn maps too (sbm_attn.py:66)
        dgraph = 0.1 * torch.randn(B, H, N, N, generator=g)
        dattn = torch.randn(B, H, N, N, generator=g)
        loss = loss + (graph * dgraph).sum() + (attn * dattn).sum()
        extra = dict(dgraph=np32(dgraph), dattn=np32(dattn))
    loss.backward()
    out = dict(Q=np32(Q), K=np32(K), V=np32(V), mask=np32(mask), u=np32(u), dX=np32(dX), dsparsity=np32(dsp),
               X=np32(X), sparsity=np32(sparsity), graph=graph.detach().numpy().astype(np.uint8), attn=np32(attn),
               expA=np32(expA), dQ=np32(Q.grad), dK=np32(K.grad), dV=np32(V.grad),
               meta=np.array([B, H, N, d, k], np.int64), **extra)
    for n_, p in mod.named_parameters():
        out["p:" + n_] = np32(p)
        out["g:" + n_] = np32(p.grad)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **out)
    print(f"{name}: sparsity={sparsity.detach().numpy()} |X|={X.abs().max().item():.3g}")


def full_case(name, B, H, N, d, pad_counts, seed, map_grads=False):
    g = torch.Generator().manual_seed(seed)
    mod = SA.FullAttention({"attention_dropout": 0.2, "head_dim": d, "num_head": H}, 0).eval()
    Q, K, V = (torch.randn(B, H, N, d, generator=g).requires_grad_(True) for _ in range(3))
    mask = torch.zeros(B, N)
    for b, pc in enumerate(pad_counts):
        if pc:
            mask[b, N - pc:] = 1.0
    dX = torch.randn(B, H, N, d, generator=g)
    X, sp, graph, attn = mod(Q, K, V, mask)
    assert sp is None and graph is mask
    loss = (X * dX).sum()
    extra = {}
    if map_grads:  # upstream gradient of the returned attn map too (sbm_attn.py:87)
        dattn = torch.randn(B, H, N, N, generator=g)
        loss = loss + (attn * dattn).sum()
        extra = dict(dattn=np32(dattn))
    loss.backward()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), Q=np32(Q), K=np32(K), V=np32(V), mask=np32(mask),
                        dX=np32(dX), X=np32(X), attn=np32(attn), dQ=np32(Q.grad), dK=np32(K.grad),
                        dV=np32(V.grad), meta=np.array([B, H, N, d], np.int64), **extra)
    print(f"{name}: ok")


def attention_layer_case(name, B, N, dim, H, k, pad_counts, seed, full_att=False):
    g = torch.Generator().manual_seed(seed)
    torch.manual_seed(seed)
    cfg = {"attention_grad_checkpointing": False, "transformer_dim": dim, "head_dim": dim // H, "num_head": H,
           "attn_type": "sbm", "attention_dropout": 0.2, "num_clusters": [k]}
    mod = SA.Attention(cfg, 0, full_att=full_att)
    for n_, p in mod.named_parameters():
        if p.dim() > 1:
            torch.nn.init.xavier_uniform_(p)
    if not full_att:
        torch.nn.init.orthogonal_(mod.attn.layer.weight)
    mod.eval()
    X = torch.randn(B, N, dim, generator=g).requires_grad_(True)
    mask = torch.zeros(B, N, dtype=torch.bool)
    for b, pc in enumerate(pad_counts):
        if pc:
            mask[b, N - pc:] = True
    u = torch.rand(B, H, N, N, generator=g)
    dout = torch.randn(B, N, dim, generator=g)
    dsp = torch.full((H,), 3.125e-4)
    with HostUniforms(u):
        out, sparsity, graph, attn = mod([X, mask, []])
    loss = (out * dout).sum() + ((sparsity * dsp).sum() if sparsity is not None else 0)
    loss.backward()
    res = dict(X=np32(X), mask=mask.numpy(), u=np32(u), dout=np32(dout), dsparsity=np32(dsp), out=np32(out),
               attn=np32(attn), dX=np32(X.grad), meta=np.array([B, N, dim, H, k, int(full_att)], np.int64))
    if sparsity is not None:
        res["sparsity"] = np32(sparsity)
        res["graph"] = graph.detach().numpy().astype(np.uint8)
    for n_, p in mod.named_parameters():
        res["p:" + n_] = np32(p)
        res["g:" + n_] = np32(p.grad)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **res)
    print(f"{name}: ok")


def relations(B, N, seed, min_nodes=None):
    sb = synthetic_batch(B, max_size=N, seed=seed, min_nodes=min_nodes or max(1, N // 2), max_nodes=N)
    rel = np.concatenate([np.repeat(sb["L"][:, None], 4, 1), np.repeat(sb["T"][:, None], 4, 1)], 1).astype(np.int64)
    msk = np.concatenate([np.repeat(sb["L_mask"][:, None], 4, 1), np.repeat(sb["T_mask"][:, None], 4, 1)], 1)
    return sb, torch.from_numpy(rel), torch.from_numpy(msk)


def rel_attn_case(name, B, N, dk, L, seed):
    g = torch.Generator().manual_seed(seed)
    H = 8
    sb, rel, msk = relations(B, N, seed)
    q, k, v = (torch.randn(B, H, N, dk, generator=g).requires_grad_(True) for _ in range(3))
    lq, lk = (torch.randn(1, H, L, dk, generator=g).requires_grad_(True) for _ in range(2))
    dO = torch.randn(B, H, N, dk, generator=g)
    o = DA.DisentangledAttn.rel_attn(q, k, v, lq, lk, rel, msk)
    (o * dO).sum().backward()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), q=np32(q), k=np32(k), v=np32(v), lq=np32(lq), lk=np32(lk),
                        L=sb["L"], T=sb["T"], L_mask=sb["L_mask"], T_mask=sb["T_mask"], dO=np32(dO), out=np32(o),
                        dq=np32(q.grad), dk=np32(k.grad), dv=np32(v.grad), dlq=np32(lq.grad), dlk=np32(lk.grad),
                        meta=np.array([B, H, N, dk, L], np.int64))
    print(f"{name}: ok")


def disentangled_case(name, B, N, d_model, L, seed):
    g = torch.Generator().manual_seed(seed)
    torch.manual_seed(seed)
    H = 8
    mod = DA.DisentangledAttn(H, d_model, 0.2)
    for n_, p in mod.named_parameters():
        if p.dim() > 1:
            torch.nn.init.xavier_uniform_(p)
    mod.eval()
    sb, rel, msk = relations(B, N, seed)
    x = torch.randn(B, N, d_model, generator=g).requires_grad_(True)
    rel_q = torch.randn(2, L, d_model, generator=g).requires_grad_(True)
    dout = torch.randn(B, N, d_model, generator=g)
    out, none = mod(x, x, x, [rel_q], rel, msk)
    assert none is None
    (out * dout).sum().backward()
    res = dict(x=np32(x), rel_q=np32(rel_q), L=sb["L"], T=sb["T"], L_mask=sb["L_mask"], T_mask=sb["T_mask"],
               dout=np32(dout), out=np32(out), dx=np32(x.grad), drel_q=np32(rel_q.grad),
               meta=np.array([B, N, d_model, L], np.int64))
    for n_, p in mod.named_parameters():
        res["p:" + n_] = np32(p)
        res["g:" + n_] = np32(p.grad)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **res)
    print(f"{name}: ok")


def label_smoothing_case(name, seed, smoothing=0.0):
    """utils/label_smooth.py:15-40 (smoothing=0 as in every config; 0.1 for the general closed form) on
    log(softmax) outputs with padding."""
    s = importlib.util.spec_from_file_location("ref_label_smooth", f"{REF}/utils/label_smooth.py")
    m = importlib.util.module_from_spec(s)
    s.loader.exec_module(m)
    g = torch.Generator().manual_seed(seed)
    B, T, V = 3, 7, 50
    logits = torch.randn(B, T, V, generator=g).requires_grad_(True)
    x = torch.log(torch.softmax(logits, -1))
    target = torch.randint(4, V, (B, T), generator=g)
    target[0, 5:] = 0
    target[2, 3:] = 0
    crit = m.LabelSmoothing(padding_idx=0, smoothing=smoothing)
    loss = crit(x, target)
    loss.backward()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), logits=np32(logits), target=target.numpy(),
                        loss=np.array([loss.item()], np.float32), dlogits=np32(logits.grad))
    print(f"{name}: loss={loss.item():.5f}")


def generator_case(name, seed):
    """module/components.py:95-102 Generator in eval mode (dropout off): log(softmax(linear(x))), with
    one row whose softmax underflows (log -> -inf, NaN gradient row, as the reference computes it)."""
    comp = sys.modules["module.components"]
    g = torch.Generator().manual_seed(seed)
    B, T, D, V = 2, 5, 16, 1003
    gen = comp.Generator(V, D, 0.2).eval()
    with torch.no_grad():
        gen.linear.weight.copy_(torch.randn(V, D, generator=g) * 0.3)
        gen.linear.bias.copy_(torch.randn(V, generator=g) * 0.1)
    x = torch.randn(B, T, D, generator=g)
    x[1, 4] *= 400.0  # extreme logits: most probabilities underflow to 0 in fp32
    x.requires_grad_(True)
    out = gen(x)
    dout = torch.randn(B, T, V, generator=g)
    dout[0, :, :] = 0.0
    dout[0, torch.arange(T), torch.randint(0, V, (T,), generator=g)] = -0.25  # label-smoothing-like one-hot rows
    out.backward(dout)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), x=np32(x), weight=np32(gen.linear.weight),
                        bias=np32(gen.linear.bias), out=np32(out), dout=np32(dout), dx=np32(x.grad),
                        dweight=np32(gen.linear.weight.grad), dbias=np32(gen.linear.bias.grad))
    print(f"{name}: -inf entries {int(torch.isinf(out).sum())}, nan grads {int(torch.isnan(x.grad).sum())}")


def adamw_case(name, seed):
    """script/optimizer.py AdamW with correct_bias=False (script/train.py:80), 3 steps."""
    s = importlib.util.spec_from_file_location("ref_optimizer", f"{REF}/script/optimizer.py")
    m = importlib.util.module_from_spec(s)
    s.loader.exec_module(m)
    g = torch.Generator().manual_seed(seed)
    p0 = torch.randn(5, 4, generator=g)
    p1 = torch.randn(7, generator=g)
    grads = [(torch.randn(5, 4, generator=g), torch.randn(7, generator=g)) for _ in range(3)]
    a, b = torch.nn.Parameter(p0.clone()), torch.nn.Parameter(p1.clone())
    opt = m.AdamW([a, b], lr=1e-2, correct_bias=False)
    for ga, gb in grads:
        a.grad, b.grad = ga.clone(), gb.clone()
        opt.step()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), p0=np32(p0), p1=np32(p1),
                        g0=np.stack([np32(x[0]) for x in grads]), g1=np.stack([np32(x[1]) for x in grads]),
                        out0=np32(a), out1=np32(b))
    print(f"{name}: ok")


def load_full_reference_package():
    """SURVEY.md Appendix A, option 2: the whole `module` package with 3 in-process shims
    (torch 2.10 dropped T_co; torch_geometric and ipdb are not installed)."""
    import typing
    import torch.utils.data.dataset as tds
    if not hasattr(tds, "T_co"):
        tds.T_co = typing.TypeVar("T_co", covariant=True)
    tg = types.ModuleType("torch_geometric")
    tgd = types.ModuleType("torch_geometric.data")

    class Data:
        def __init__(self, **kw):
            self.__dict__.update(kw)

        def to(self, device):
            return self
    tgd.Data = Data
    tg.data = tgd
    sys.modules.setdefault("torch_geometric", tg)
    sys.modules.setdefault("torch_geometric.data", tgd)
    sys.modules.setdefault("ipdb", types.ModuleType("ipdb"))
    for k in [k for k in sys.modules if k == "module" or k.startswith("module.")]:
        del sys.modules[k]
    sys.path.insert(0, REF)
    import module as refmod  # noqa
    return refmod, Data


GRAD_KEYS = ("mha.attn.", "self_attn.l_linear.0", "self_attn.t_linear.1", "pegen.L_q", "pegen.T_q",
             "SBM.out.bias", "pe_expand.bias", "generator.linear.bias")


def fill_params_deterministic(model, seed):
    """Every parameter <- N(0,1) * 0.5/sqrt(fan_in) from numpy's PCG64 in sorted-key order (reproducible
    anywhere, so the fixture need not carry the weights; tests/test_model_gpu.py applies the same fill)."""
    rng = np.random.default_rng(seed)
    named = dict(model.named_parameters())
    with torch.no_grad():
        for k in sorted(named):
            p = named[k]
            fan = p.shape[-1] if p.dim() > 1 else 1
            p.copy_(torch.from_numpy((rng.standard_normal(p.shape) * (0.5 / np.sqrt(fan))).astype(np.float32)))


def csatrans_case(name, seed):
    """Tiny CSATrans (module/csa_trans.py) forward + loss + sw*sparsity backward, eval mode,
    host-supplied uniforms per SBM layer; saves the state_dict (checks key compatibility)."""
    refmod, Data = load_full_reference_package()
    s = importlib.util.spec_from_file_location("ref_label_smooth", f"{REF}/utils/label_smooth.py")
    ls = importlib.util.module_from_spec(s)
    s.loader.exec_module(ls)
    torch.manual_seed(seed)
    kw = dict(src_vocab_size=50, tgt_vocab_size=60, hidden_size=64, num_heads=8, num_layers=1, sbm_layers=2,
              use_pegen="pegen", dim_feed_forward=128, dropout=0.2, pe_dim=32, pegen_dim=128, sbm_enc_dim=512,
              clusters=[10, 12], full_att=False)
    model = refmod.CSATrans(**kw).eval()
    fill_params_deterministic(model, seed)
    B, N = 2, 20
    sb = synthetic_batch(B, max_size=N, seed=seed, min_nodes=12, max_nodes=N, src_vocab=50, tgt_vocab=60,
                         max_tgt_len=9)
    f = lambda a: torch.from_numpy(np.asarray(a))
    data = Data(src_seq=f(sb["src_seq"]), tgt_seq=f(sb["tgt_seq"]), L=f(sb["L"]).float(), T=f(sb["T"]).float(),
                L_mask=f(sb["L_mask"]), T_mask=f(sb["T_mask"]))
    g = torch.Generator().manual_seed(seed + 1)
    us = [torch.rand(B, 8, N, N, generator=g) for _ in range(2)]
    it = iter(us)
    torch.bernoulli = lambda p: (next(it) < p).to(p.dtype)
    try:
        out, sparsity, src_pe, graphs, attns = model(data)
    finally:
        torch.bernoulli = _real_bernoulli
    loss = ls.LabelSmoothing(padding_idx=0, smoothing=0.0)(out, f(sb["target"]))
    total = loss + 1e-2 * sparsity
    total.backward()
    res = {"src_seq": sb["src_seq"], "tgt_seq": sb["tgt_seq"], "target": sb["target"], "L": sb["L"], "T": sb["T"],
           "L_mask": sb["L_mask"], "T_mask": sb["T_mask"], "u0": np32(us[0]), "u1": np32(us[1]),
           "out": np32(out), "sparsity": np.array([sparsity.item()], np.float32),
           "loss": np.array([loss.item()], np.float32)}
    res["state_keys"] = np.array(sorted(model.state_dict().keys()))
    for k, p in model.named_parameters():
        if any(t in k for t in GRAD_KEYS):
            res["g:" + k] = np32(p.grad)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **res)
    print(f"{name}: loss={loss.item():.5f} sparsity={sparsity.item():.5f} keys={len(model.state_dict())}")


def rel_attn_large_case(name, B, N, dk, L, seed):
    """rel_attn at the production head size (d_k = pegen_dim/8 = 64, N = L = 150). Inputs are
    regenerated from PCG64 (tests/golden_inputs.py:rel_inputs), so only relations and outputs are stored."""
    H = 8
    sb, rel, msk = relations(B, N, seed)
    q, k, v, lq, lk, dO = (torch.from_numpy(a) for a in gi.rel_inputs(B, H, N, dk, L, seed))
    for t in (q, k, v, lq, lk):
        t.requires_grad_(True)
    o = DA.DisentangledAttn.rel_attn(q, k, v, lq, lk, rel, msk)
    (o * dO).sum().backward()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), L=sb["L"], T=sb["T"], L_mask=sb["L_mask"],
                        T_mask=sb["T_mask"], out=np32(o), dq=np32(q.grad), dk=np32(k.grad), dv=np32(v.grad),
                        dlq=np32(lq.grad), dlk=np32(lk.grad), meta=np.array([B, H, N, dk, L, seed], np.int64))
    print(f"{name}: ok")


def _java_batch(B, N, seed):
    return synthetic_batch(B, max_size=N, seed=seed, min_nodes=100, max_nodes=N)


def _oracle_fp64(model, dims, sb, us, B, N):
    """The pinned oracle CSATrans (oracle/csatrans_ref.py) in fp64 on the reference model's weights, batch and
    (nudged) STE uniforms: the error-budget baseline. Returns (log-probs, sparsity, loss, {name: grad})."""
    from oracle import csatrans_ref
    cfg = csatrans_ref.config(**dims)
    params = {k: p.detach().double().clone().requires_grad_(True) for k, p in model.named_parameters()
              if k in csatrans_ref.param_shapes(cfg)}
    om = csatrans_ref.Model(cfg, params, training=False)
    f = lambda k, dt: torch.from_numpy(np.asarray(sb[k])).to(dt)
    out, sp = om.forward(f("src_seq", torch.int64), f("tgt_seq", torch.int64), f("L", torch.int64), f("T", torch.int64),
                         f("L_mask", torch.bool), f("T_mask", torch.bool), u_list=[torch.from_numpy(u) for u in us])
    loss = csatrans_ref.label_smoothing(out, f("target", torch.int64))
    (loss + 1e-2 * sp).backward()
    return out.detach(), sp.detach(), loss.detach(), {k: p.grad for k, p in params.items()}


def csatrans_dims_case(name, dims, B, N, seed, uniforms, grad_keys):
    """CSATrans at production dims (config/java.py: sbm_enc_dim 768 -> SBM d=96, pe 128; config/python.py:
    sbm_enc_dim 512 -> SBM d=64, pe 256; both pegen 512 -> CSE d_k=64, N=150, 4 CSE + 4 SBM layers), eval
    mode, loss + sw*sparsity backward, then one reference AdamW step. Weights and STE uniforms are
    regenerated from PCG64 (tests/golden_inputs.py); the uniforms are moved off fp32 ties with the
    probability the reference's sampler actually sees, and only those moves are stored.

    Error budget: the same model, batch and uniforms through the oracle CSATrans in fp64; the fixture keeps
    fp64 - fp32(reference) as 'e64:<key>' for the log-prob columns, the loss and every stored gradient, so
    the GPU test can compare its own error against the reference's fp32 error on the same inputs."""
    refmod, Data = load_full_reference_package()
    s = importlib.util.spec_from_file_location("ref_label_smooth", f"{REF}/utils/label_smooth.py")
    ls = importlib.util.module_from_spec(s)
    s.loader.exec_module(ls)
    torch.manual_seed(seed)
    model = refmod.CSATrans(**dims).eval()
    gi.fill_params_deterministic(model, seed)
    sb = _java_batch(B, N, seed)
    f = lambda a: torch.from_numpy(np.asarray(a))
    data = Data(src_seq=f(sb["src_seq"]), tgt_seq=f(sb["tgt_seq"]), L=f(sb["L"]).float(), T=f(sb["T"]).float(),
                L_mask=f(sb["L_mask"]), T_mask=f(sb["T_mask"]))
    nudges, used = [], []

    def bern(p):
        layer = len(nudges)
        u, idx, val = gi.nudge_uniforms(uniforms(layer), p.detach().numpy())
        nudges.append((idx, val))
        used.append(u)
        return (torch.from_numpy(u) < p).to(p.dtype)

    torch.bernoulli = bern
    try:
        out, sparsity, src_pe, graphs, attns = model(data)
    finally:
        torch.bernoulli = _real_bernoulli
    assert len(nudges) == dims["sbm_layers"]
    loss = ls.LabelSmoothing(padding_idx=0, smoothing=0.0)(out, f(sb["target"]))
    (loss + 1e-2 * sparsity).backward()
    col = gi.JAVA_OUT_COL_STRIDE
    res = {"out_cols": np32(out[:, :, ::col]), "sparsity": np.array([sparsity.item()], np.float32),
           "loss": np.array([loss.item()], np.float32), "out_rowmax": np32(out.max(-1).values),
           "out_argmax": out.argmax(-1).numpy().astype(np.int32)}
    for i, (idx, val) in enumerate(nudges):
        res[f"nudge_idx{i}"], res[f"nudge_val{i}"] = idx, val
    res["state_keys"] = np.array(sorted(model.state_dict().keys()))
    for k, p in model.named_parameters():
        if any(k.startswith(t) for t in grad_keys):
            res["g:" + k] = np32(p.grad)
    # fp64 oracle on the same inputs (the graph is the same: every draw is >= TIE_MARGIN from its p)
    o64, sp64, loss64, g64 = _oracle_fp64(model, dims, sb, used, B, N)
    assert sp64.item() == pytest_approx(sparsity.item()), (sp64.item(), sparsity.item())
    res["e64:out_cols"] = (o64[:, :, ::col].numpy() - res["out_cols"].astype(np.float64)).astype(np.float32)
    res["e64:loss"] = np.array([loss64.item() - float(res["loss"][0])], np.float32)
    for k in [k for k in res if k.startswith("g:")]:
        res["e64:" + k] = (g64[k[2:]].numpy() - res[k].astype(np.float64)).astype(np.float32)
    # one optimizer step of the train step (script/train.py:80,110: the reference AdamW, lr 1e-4 from
    # config/java.py:49 and config/python.py, correct_bias=False; the GradScaler's power-of-two scale cancels)
    so = importlib.util.spec_from_file_location("ref_optimizer", f"{REF}/script/optimizer.py")
    om = importlib.util.module_from_spec(so)
    so.loader.exec_module(om)
    om.AdamW(model.parameters(), lr=1e-4, correct_bias=False).step()
    for k, p in model.named_parameters():
        if any(k.startswith(t) for t in grad_keys):
            res["p1:" + k] = np32(p)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), **res)
    rel = lambda k: float(np.abs(res["e64:" + k]).max() / max(np.abs(res[k]).max(), 1e-30))
    print(f"{name}: loss={loss.item():.5f} sparsity={sparsity.item():.5f} nudged={[len(n[0]) for n in nudges]}"
          f" grads={sum(k.startswith('g:') for k in res)} ref-fp32 vs fp64: out {rel('out_cols'):.2e},"
          f" worst grad {max(rel(k) for k in res if k.startswith('g:')):.2e}")


def pytest_approx(x, rel=1e-6):
    class _A:
        def __eq__(self, y):
            return abs(y - x) <= rel * max(abs(x), 1e-30)
    return _A()


def csatrans_java_case(name):
    csatrans_dims_case(name, gi.JAVA, gi.JAVA_B, gi.JAVA_N, gi.JAVA_SEED, gi.java_uniforms, gi.JAVA_GRAD_KEYS)


def csatrans_python_case(name):
    csatrans_dims_case(name, gi.PYTHON, gi.PY_B, gi.PY_N, gi.PY_SEED, gi.python_uniforms, gi.JAVA_GRAD_KEYS)


def greedy_tiny_case(name, seed, max_tgt_len=7):
    """GreedyGenerator (module/base_seq2seq.py:117-145) over the tiny CSATrans in eval mode: process_data,
    one encode, then max_tgt_len-1 decode + generator + argmax steps (script/train.py:271-282)."""
    refmod, Data = load_full_reference_package()
    from module.base_seq2seq import GreedyGenerator
    kw = dict(src_vocab_size=50, tgt_vocab_size=60, hidden_size=64, num_heads=8, num_layers=1, sbm_layers=2,
              use_pegen="pegen", dim_feed_forward=128, dropout=0.2, pe_dim=32, pegen_dim=128, sbm_enc_dim=512,
              clusters=[10, 12], full_att=False)
    torch.manual_seed(seed)
    model = refmod.CSATrans(**kw).eval()
    fill_params_deterministic(model, seed)
    B, N = 3, 20
    sb = synthetic_batch(B, max_size=N, seed=seed, min_nodes=12, max_nodes=N, src_vocab=50, tgt_vocab=60,
                         max_tgt_len=9)
    f = lambda a: torch.from_numpy(np.asarray(a))
    data = Data(src_seq=f(sb["src_seq"]), tgt_seq=None, L=f(sb["L"]).float(), T=f(sb["T"]).float(),
                L_mask=f(sb["L_mask"]), T_mask=f(sb["T_mask"]))
    g = torch.Generator().manual_seed(seed + 1)
    us = [torch.rand(B, 8, N, N, generator=g) for _ in range(2)]
    it = iter(us)
    with torch.no_grad():  # a spread-out generator so the greedy path is not one repeated token
        model.generator.linear.weight.mul_(8.0)
    steps = []
    hook = model.generator.register_forward_hook(lambda m, i, o: steps.append(o[:, -1, :].clone()))
    torch.bernoulli = lambda p: (next(it) < p).to(p.dtype)
    try:
        with torch.no_grad():
            ys = GreedyGenerator(model, max_tgt_len)(data)
    finally:
        torch.bernoulli = _real_bernoulli
        hook.remove()
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), src_seq=sb["src_seq"], L=sb["L"], T=sb["T"],
                        L_mask=sb["L_mask"], T_mask=sb["T_mask"], u0=np32(us[0]), u1=np32(us[1]),
                        ys=ys.numpy().astype(np.int64), step_logp=np32(torch.stack(steps)),
                        meta=np.array([seed, max_tgt_len], np.int64))
    print(f"{name}: ys={ys.tolist()}")


def ast_relations_case(name, seed, max_size=150):
    """F2 host data path pinned to the reference: random pre-order trees -> my_ast.Node trees ->
    MyAst.__sub_tree (the max_size truncation of __process_treesitter) -> MyAst.__get_matrices
    (my_ast.py:198-273) -> BaseASTDataSet.collect_fn's L/T encoding (dataset/base_data_set.py:33-36).
    Stores the parent arrays of the kept pre-order prefix and the collated uint8/bool planes."""
    refmod, Data = load_full_reference_package()
    import my_ast
    from dataset.base_data_set import BaseASTDataSet
    from csa_amd.data import random_tree
    rng = np.random.default_rng(seed)
    sizes = [1, 2, 3, 17, 60, 149, 150, 151, 230, 150, 90, 400]
    parents = np.full((len(sizes), max_size), -1, np.int32)
    n_nodes = np.zeros(len(sizes), np.int32)
    batch = []
    for b, n in enumerate(sizes):
        par, kids = random_tree(n, rng, max_children=int(rng.integers(2, 9)))
        nodes = [my_ast.Node(label=f"nont:n{v}", children=[]) for v in range(n)]
        for v in range(1, n):
            nodes[v].parent = nodes[par[v]]
        for v in range(n):
            for ci, c in enumerate(kids[v]):
                nodes[v].children.append(nodes[c])
                nodes[c].child_idx = ci
        my_ast.MyAst._MyAst__sub_tree(nodes[0], max_size)
        _, L, T, *_ = my_ast.MyAst._MyAst__get_matrices(nodes[0], "python", max_size)
        keep = min(n, max_size)
        parents[b, :keep] = par[:keep]
        n_nodes[b] = keep
        z = torch.zeros(1)
        batch.append(({"L": L, "T": T, "src_seq": z, "tgt_seq": z, "target": z, "num_node": keep, "adj": z,
                       "tree_pos": torch.zeros(keep, 2), "triplet": z}, None))
    data, _ = BaseASTDataSet.collect_fn(None, batch)
    np.savez_compressed(os.path.join(OUT, f"{name}.npz"), parents=parents, n_nodes=n_nodes,
                        L=data.L.numpy().astype(np.uint8), T=data.T.numpy().astype(np.uint8),
                        L_mask=data.L_mask.numpy(), T_mask=data.T_mask.numpy(), sizes=np.array(sizes, np.int64))
    print(f"{name}: {len(sizes)} trees, L range {int(data.L.min())}..{int(data.L.max())}")


def main():
    os.makedirs(OUT, exist_ok=True)
    torch.set_num_threads(8)
    eq = verify_bernoulli_equivalence()
    print("bernoulli == rand<p (CPU):", eq)
    assert eq, "host-uniform recipe does not reproduce torch.bernoulli"
    if sys.argv[1:] == ["ast"]:
        ast_relations_case("ast_relations", seed=91)
        return
    if sys.argv[1:] == ["mapgrad"]:  # only the round-2 map-gradient fixtures
        sbm_case("sbm_n37_mapgrad", B=2, H=2, N=37, d=64, k=10, pad_counts=[0, 7], seed=17, map_grads=True)
        sbm_case("sbm_n33_d96_mapgrad", B=1, H=2, N=33, d=96, k=10, pad_counts=[1], seed=18, map_grads=True)
        full_case("full_n37_mapgrad", B=2, H=2, N=37, d=64, pad_counts=[0, 5], seed=23, map_grads=True)
        return
    if sys.argv[1:] == ["dims"]:  # round 3: production-dims CSATrans with the fp64 error budget
        csatrans_java_case("csatrans_java")
        csatrans_python_case("csatrans_python")
        return
    if sys.argv[1:] == ["large"]:  # only the round-2 production-shape fixtures
        rel_attn_large_case("rel_attn_n150_dk64", B=1, N=150, dk=64, L=150, seed=44)
        greedy_tiny_case("greedy_tiny", seed=72)
        csatrans_java_case("csatrans_java")
        return
    np.savez(os.path.join(OUT, "bernoulli_equivalence.npz"), ok=np.array([eq]))
    sbm_case("sbm_n37", B=2, H=2, N=37, d=64, k=10, pad_counts=[0, 7], seed=11)
    sbm_case("sbm_n1", B=2, H=2, N=1, d=64, k=10, pad_counts=[0, 0], seed=12)
    sbm_case("sbm_n7_d96_k16", B=2, H=2, N=7, d=96, k=16, pad_counts=[2, 0], seed=13)
    sbm_case("sbm_n64_noncontig", B=2, H=2, N=64, d=64, k=10, pad_counts=[13, 0], seed=14, noncontig=True)
    sbm_case("sbm_n150", B=1, H=2, N=150, d=64, k=10, pad_counts=[30], seed=15, zero_row=(0, 1, 5))
    sbm_case("sbm_n33_d96", B=1, H=2, N=33, d=96, k=10, pad_counts=[1], seed=16)
    full_case("full_n37", B=2, H=2, N=37, d=64, pad_counts=[0, 5], seed=21)
    full_case("full_n150", B=1, H=2, N=150, d=64, pad_counts=[40], seed=22)
    attention_layer_case("attn_layer_n29", B=2, N=29, dim=128, H=2, k=10, pad_counts=[0, 4], seed=31)
    attention_layer_case("attn_layer_full_n29", B=2, N=29, dim=128, H=2, k=10, pad_counts=[3, 0], seed=32,
                         full_att=True)
    rel_attn_case("rel_attn_n37", B=2, N=37, dk=16, L=150, seed=41)
    rel_attn_case("rel_attn_n150", B=1, N=150, dk=16, L=150, seed=42)
    rel_attn_case("rel_attn_n20_dk64", B=1, N=20, dk=64, L=150, seed=43)
    disentangled_case("disentangled_n23", B=2, N=23, d_model=128, L=150, seed=51)
    label_smoothing_case("label_smoothing", seed=61)
    label_smoothing_case("label_smoothing_s01", seed=63, smoothing=0.1)
    generator_case("generator_v1003", seed=64)
    adamw_case("adamw_nobias", seed=62)
    csatrans_case("csatrans_tiny", seed=71)
    if True:
        sbm_case("sbm_n37_mapgrad", B=2, H=2, N=37, d=64, k=10, pad_counts=[0, 7], seed=17, map_grads=True)
        sbm_case("sbm_n33_d96_mapgrad", B=1, H=2, N=33, d=96, k=10, pad_counts=[1], seed=18, map_grads=True)
        full_case("full_n37_mapgrad", B=2, H=2, N=37, d=64, pad_counts=[0, 5], seed=23, map_grads=True)
        ast_relations_case("ast_relations", seed=91)
        rel_attn_large_case("rel_attn_n150_dk64", B=1, N=150, dk=64, L=150, seed=44)
        greedy_tiny_case("greedy_tiny", seed=72)
        csatrans_java_case("csatrans_java")
        csatrans_python_case("csatrans_python")


if __name__ == "__main__":
    main()
