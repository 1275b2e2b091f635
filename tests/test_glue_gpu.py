"""csa_bias_grad (csrc/csa_glue.hip) and the glue Linear vs torch's nn.Linear backward (fp32)."""
import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs GPU")]


@pytest.mark.parametrize("rows,cols", [(1, 1), (7, 3), (9600, 768), (3136, 20000), (255, 65), (100000, 4)])
def test_bias_grad_matches_column_sums(rows, cols):
    from csa_amd.glue import bias_grad
    g = torch.Generator().manual_seed(rows + cols)
    dy = torch.randn(rows, cols, generator=g, dtype=torch.float64)
    out = bias_grad(dy.float().cuda())
    ref = dy.sum(0)
    np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-5 * np.sqrt(rows))
    assert torch.equal(out, bias_grad(dy.float().cuda())), "deterministic"


def test_bias_grad_back_to_back_on_two_streams():
    """The one-launch path's per-stream arrival counters: many launches of different shapes queued back to
    back (no synchronisation between them) on the default stream and on a side stream at once, each sum
    checked. A counter not returned to 0 by its last workgroup would finish a later launch early."""
    from csa_amd.glue import bias_grad
    shapes = [(9600, 512), (300, 2048), (9600, 64), (1, 40), (2500, 130), (16384, 96)] * 3
    g = torch.Generator().manual_seed(11)
    dys = [torch.randn(r, c, generator=g) for r, c in shapes]
    side = torch.cuda.Stream()
    outs = []
    for i, dy in enumerate(dys):
        d = dy.cuda()
        st = side if i % 2 else torch.cuda.current_stream()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            outs.append(bias_grad(d))
            d.record_stream(st)
    torch.cuda.synchronize()
    for dy, out in zip(dys, outs):
        ref = dy.double().sum(0)
        np.testing.assert_allclose(out.cpu().numpy(), ref.numpy(), rtol=1e-4, atol=1e-5 * np.sqrt(dy.shape[0]))


def test_glue_linear_matches_nn_linear():
    from csa_amd.glue import Linear
    torch.manual_seed(3)
    ref = torch.nn.Linear(96, 40).cuda()
    mine = Linear(96, 40).cuda()
    mine.load_state_dict(ref.state_dict())
    x = torch.randn(4, 37, 96, device="cuda")
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    gy = torch.randn(4, 37, 40, device="cuda")
    ref(xa).backward(gy)
    mine(xb).backward(gy)
    for a, b in ((xa.grad, xb.grad), (ref.weight.grad, mine.weight.grad), (ref.bias.grad, mine.bias.grad)):
        np.testing.assert_allclose(b.cpu().numpy(), a.cpu().numpy(), rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("rows,cols", [(1, 4), (37, 512), (9600, 768), (130, 1024), (65, 100)])
def test_layernorm_matches_torch(rows, cols):
    from csa_amd.glue import LayerNorm
    torch.manual_seed(rows + cols)
    ref = torch.nn.LayerNorm(cols).cuda()
    with torch.no_grad():
        ref.weight.normal_()
        ref.bias.normal_()
    mine = LayerNorm(cols).cuda()
    mine.load_state_dict(ref.state_dict())
    x = (torch.randn(rows, cols, device="cuda") * 3 + 1)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    gy = torch.randn(rows, cols, device="cuda")
    ya, yb = ref(xa), mine(xb)
    np.testing.assert_allclose(yb.detach().cpu().numpy(), ya.detach().cpu().numpy(), rtol=1e-4, atol=1e-5)
    ya.backward(gy)
    yb.backward(gy)
    for a, b in ((xa.grad, xb.grad), (ref.weight.grad, mine.weight.grad), (ref.bias.grad, mine.bias.grad)):
        np.testing.assert_allclose(b.cpu().numpy(), a.cpu().numpy(), rtol=1e-4, atol=1e-4)


def _perm_view(x):
    """(B, T, E) batch-first tensor -> its (T, B, E) permuted view, as csa_trans.py hands the decoder."""
    return x.permute(1, 0, 2)


@pytest.mark.parametrize("train_dropout", [0.0, 0.2])
def test_glue_mha_matches_nn_mha(train_dropout):
    """Decoder self-attention (pad|future bool mask repeated per head, read back as view(B, H, T, S)
    exactly as torch does) and cross-attention (key padding mask) vs nn.MultiheadAttention, outputs and
    all gradients. With dropout the two draw the same SDPA Philox stream from the same seed."""
    from csa_amd.glue import MultiheadAttention
    from csa_amd.model import make_std_mask
    torch.manual_seed(5)
    B, T, S, E, H = 6, 11, 17, 64, 8
    ref_sa = torch.nn.MultiheadAttention(E, H, dropout=train_dropout).cuda()
    ref_ca = torch.nn.MultiheadAttention(E, H, dropout=train_dropout).cuda()
    sa = MultiheadAttention(E, H, dropout=train_dropout).cuda()
    ca = MultiheadAttention(E, H, dropout=train_dropout).cuda()
    with torch.no_grad():
        for m in (ref_sa, ref_ca):
            m.in_proj_bias.normal_()
            m.out_proj.bias.normal_()
    sa.load_state_dict(ref_sa.state_dict())
    ca.load_state_dict(ref_ca.state_dict())
    for m in (ref_sa, ref_ca, sa, ca):
        m.train(train_dropout > 0)
    tgt = torch.randint(1, 50, (B, T), device="cuda")
    tgt[:, 7:] = 0
    tgt[2, 4:] = 0
    tmask = make_std_mask(tgt, 0).repeat(H, 1, 1)
    src_pad = torch.zeros(B, S, dtype=torch.bool, device="cuda")
    src_pad[1, 9:] = True
    src_pad[4, 3:] = True
    x0 = torch.randn(B, T, E, device="cuda")
    m0 = torch.randn(B, S, E, device="cuda")
    gy = torch.randn(T, B, E, device="cuda")

    def run(mods, x, mem, contiguous):
        xs, ms = _perm_view(x), _perm_view(mem)
        if contiguous:
            xs, ms = xs.contiguous(), ms.contiguous()
        torch.manual_seed(11)
        h, _ = mods[0](xs, xs, xs, attn_mask=tmask, need_weights=False)
        y, _ = mods[1](h, ms, ms, key_padding_mask=src_pad, need_weights=False)
        y.backward(gy)
        return y

    for contiguous in (False, True):
        xa, xb = x0.clone().requires_grad_(True), x0.clone().requires_grad_(True)
        ma, mb = m0.clone().requires_grad_(True), m0.clone().requires_grad_(True)
        for m in (ref_sa, ref_ca, sa, ca):
            m.zero_grad(set_to_none=True)
        ya = run((ref_sa, ref_ca), xa, ma, contiguous)
        yb = run((sa, ca), xb, mb, contiguous)
        assert yb.shape == ya.shape == (T, B, E)
        np.testing.assert_allclose(yb.detach().cpu().numpy(), ya.detach().cpu().numpy(), rtol=1e-4, atol=1e-5)
        pairs = [(xa.grad, xb.grad), (ma.grad, mb.grad)]
        pairs += [(p.grad, q.grad) for r, g in ((ref_sa, sa), (ref_ca, ca))
                  for p, q in zip(r.parameters(), g.parameters())]
        for a, b in pairs:
            np.testing.assert_allclose(b.cpu().numpy(), a.cpu().numpy(), rtol=1e-4, atol=1e-4)


def test_glue_linear_layernorm_on_permuted_views():
    """Linear and LayerNorm on a (T, B, E) permuted view of batch-first memory run on that memory and
    return the same view layout; values and gradients as nn.Linear / nn.LayerNorm."""
    from csa_amd.glue import LayerNorm, Linear
    torch.manual_seed(9)
    ref_ln, ref_lin = torch.nn.LayerNorm(96).cuda(), torch.nn.Linear(96, 40).cuda()
    with torch.no_grad():
        ref_ln.weight.normal_()
        ref_ln.bias.normal_()
    ln, lin = LayerNorm(96).cuda(), Linear(96, 40).cuda()
    ln.load_state_dict(ref_ln.state_dict())
    lin.load_state_dict(ref_lin.state_dict())
    x = torch.randn(5, 23, 96, device="cuda") * 2 + 0.5
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    gy = torch.randn(23, 5, 40, device="cuda")
    ya = ref_lin(ref_ln(_perm_view(xa)))
    yb = lin(ln(_perm_view(xb)))
    assert yb.transpose(0, 1).is_contiguous(), "output keeps the batch-first memory"
    np.testing.assert_allclose(yb.detach().cpu().numpy(), ya.detach().cpu().numpy(), rtol=1e-4, atol=1e-5)
    ya.backward(gy)
    yb.backward(gy)
    for a, b in ((xa.grad, xb.grad), (ref_ln.weight.grad, ln.weight.grad), (ref_ln.bias.grad, ln.bias.grad),
                 (ref_lin.weight.grad, lin.weight.grad), (ref_lin.bias.grad, lin.bias.grad)):
        np.testing.assert_allclose(b.cpu().numpy(), a.cpu().numpy(), rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("shape,batch_major", [((64, 150, 512), False), ((49, 64, 512), True), ((3, 5, 7), False),
                                               ((1, 1, 1), False), ((11, 3, 12), True)])
def test_residual_dropout_matches_oracle(shape, batch_major):
    """csa_residual_dropout_fwd/_bwd vs the oracle keep mask (oracle/philox.py:res_keep over the memory
    order): y = x + keep * o / (1 - p) and d_o = keep * dy / (1 - p) bit-exact, dx = dy; eval mode is
    the identity dropout."""
    import sys
    import os
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle.philox import res_keep
    from csa_amd.glue import residual_dropout
    from csa_amd.ops import _draw_seed
    p = 0.2
    drop = torch.nn.Dropout(p).train()
    g = torch.Generator().manual_seed(sum(shape))
    mem = (shape[1], shape[0], shape[2]) if batch_major else shape
    x0, o0, gy0 = (torch.randn(*mem, generator=g) for _ in range(3))
    if batch_major:
        x0, o0, gy0 = (t.transpose(0, 1) for t in (x0, o0, gy0))
    x = x0.cuda().requires_grad_(True)
    o = o0.cuda().requires_grad_(True)
    if batch_major:  # (T, B, E) views of batch-first memory, as the decoder sees them
        x = x0.transpose(0, 1).contiguous().cuda().transpose(0, 1).detach().requires_grad_(True)
        o = o0.transpose(0, 1).contiguous().cuda().transpose(0, 1).detach().requires_grad_(True)
    torch.manual_seed(77)
    y = residual_dropout(x, o, drop)
    torch.manual_seed(77)
    seed = _draw_seed()
    n = x0.numel()
    to_mem = (lambda t: t.transpose(0, 1).contiguous()) if batch_major else (lambda t: t.contiguous())
    keep = torch.from_numpy(res_keep(n, seed, 0, p)).view(to_mem(x0).shape)
    scale = np.float32(1.0 / (1.0 - np.float32(p)))
    o_m, x_m = to_mem(o0), to_mem(x0)
    ref = x_m + torch.where(keep, o_m * float(scale), 0.0 * o_m)
    assert torch.equal(to_mem(y.detach().cpu()), ref)
    y.backward(gy0.cuda())
    gy_m = to_mem(gy0)
    assert torch.equal(to_mem(o.grad.cpu()), torch.where(keep, gy_m * float(scale), 0.0 * gy_m))
    assert torch.equal(x.grad.cpu(), gy0)
    assert 0.7 < keep.float().mean().item() < 0.9 or n < 100
    drop.eval()
    assert torch.equal(residual_dropout(x, o, drop).detach(), (x + o).detach())


@pytest.mark.parametrize("shape,batch_major,p", [((64, 150, 768), False, 0.2), ((49, 64, 2048), True, 0.2),
                                                 ((3, 5, 7), False, 0.2), ((9, 4, 16), True, 0.0)])
def test_gelu_dropout_matches_oracle(shape, batch_major, p):
    """csa_gelu_dropout_fwd/_bwd vs torch's exact GELU under the oracle keep mask
    (oracle/philox.py:ffn_keep over the memory order): y = keep * gelu(h) / (1 - p),
    dh = keep * dy / (1 - p) * gelu'(h) (torch autograd of gelu); fp32 tolerance 1e-5 (device erff vs the
    host's differ by an ulp or two)."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle.philox import ffn_keep
    from csa_amd.glue import gelu_dropout
    from csa_amd.ops import _draw_seed
    drop = torch.nn.Dropout(p).train()
    g = torch.Generator().manual_seed(sum(shape))
    mem = (shape[1], shape[0], shape[2]) if batch_major else shape
    h_mem, gy_mem = torch.randn(*mem, generator=g) * 3, torch.randn(*mem, generator=g)
    to_logical = (lambda t: t.transpose(0, 1)) if batch_major else (lambda t: t)
    to_mem = (lambda t: t.transpose(0, 1).contiguous()) if batch_major else (lambda t: t.contiguous())
    h = to_logical(h_mem.cuda()).detach().requires_grad_(True)
    torch.manual_seed(91)
    y = gelu_dropout(h, drop)
    torch.manual_seed(91)
    seed = _draw_seed() if p > 0 else 0
    keep = (torch.from_numpy(ffn_keep(h_mem.numel(), seed, 0, p)).view(mem) if p > 0
            else torch.ones(mem, dtype=torch.bool))
    scale = float(np.float32(1.0 / (1.0 - np.float32(p))))
    hr = h_mem.clone().requires_grad_(True)
    yr = torch.where(keep, torch.nn.functional.gelu(hr) * scale, 0.0 * hr)
    np.testing.assert_allclose(to_mem(y.detach().cpu()).numpy(), yr.detach().numpy(), rtol=1e-5, atol=1e-5)
    y.backward(to_logical(gy_mem.cuda()))
    yr.backward(gy_mem)
    np.testing.assert_allclose(to_mem(h.grad.cpu()).numpy(), hr.grad.numpy(), rtol=1e-5, atol=1e-5)
