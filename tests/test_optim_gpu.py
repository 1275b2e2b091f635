"""csa_adamw_step (csrc/csa_optim.hip) vs the reference AdamW (script/optimizer.py:49-106): the
reference's own golden trajectory (tests/golden/adamw_nobias.npz, made by tools/gen_golden.py from
the reference optimizer) and, for ragged / unaligned multi-tensor layouts with weight decay and bias
correction, the per-op CPU path of the same class (the reference's op order as foreach ops)."""
import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs GPU")]


def test_fused_adamw_matches_reference_golden(golden):
    from csa_amd.train import AdamW
    z = golden("adamw_nobias")
    a = torch.nn.Parameter(torch.from_numpy(z["p0"]).cuda())
    b = torch.nn.Parameter(torch.from_numpy(z["p1"]).cuda())
    opt = AdamW([a, b], lr=1e-2, correct_bias=False)
    for i in range(3):
        a.grad, b.grad = torch.from_numpy(z["g0"][i]).cuda(), torch.from_numpy(z["g1"][i]).cuda()
        opt.step()
    np.testing.assert_allclose(a.detach().cpu().numpy(), z["out0"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(b.detach().cpu().numpy(), z["out1"], rtol=1e-6, atol=1e-7)


@pytest.mark.parametrize("correct_bias,wd", [(False, 0.0), (True, 0.01)])
def test_fused_adamw_ragged_unaligned_matches_per_op_path(correct_bias, wd):
    from csa_amd.train import AdamW
    g = torch.Generator().manual_seed(5)
    sizes = [1, 3, 4, 4095, 4096, 4097, 10005, 3 * 4096 + 7]
    base = [torch.randn(n + 1, generator=g) for n in sizes]
    # even-indexed tensors are offset by one element inside their storage: 4-B aligned only, so the
    # scalar path runs next to the dwordx4 path
    cpu = [torch.nn.Parameter(t[1:].clone() if i % 2 == 0 else t[:-1].clone()) for i, t in enumerate(base)]
    gpu = [torch.nn.Parameter(t.cuda()[1:] if i % 2 == 0 else t.cuda()[:-1]) for i, t in enumerate(base)]
    o_cpu = AdamW(cpu, lr=3e-3, weight_decay=wd, correct_bias=correct_bias)
    o_gpu = AdamW(gpu, lr=3e-3, weight_decay=wd, correct_bias=correct_bias)
    for step in range(4):
        for pc, pg in zip(cpu, gpu):
            gr = torch.randn(pc.shape, generator=g) * (10.0 ** (step - 2))
            pc.grad, pg.grad = gr.clone(), gr.cuda()
        o_cpu.step()
        o_gpu.step()
    for pc, pg in zip(cpu, gpu):
        np.testing.assert_allclose(pg.detach().cpu().numpy(), pc.detach().numpy(), rtol=1e-5, atol=1e-7)
        for key in ("exp_avg", "exp_avg_sq"):
            np.testing.assert_allclose(o_gpu.state[pg][key].cpu().numpy(), o_cpu.state[pc][key].numpy(),
                                       rtol=1e-5, atol=1e-12)


def test_fused_adamw_under_gradscaler_unscales_and_skips_on_inf():
    """script/train.py:109-111 (GradScaler.scale(loss).backward(); step; update) with the device-side
    unscale / skip path: same parameters as unscaled grads through the per-op CPU path; an inf
    gradient leaves parameters and moments untouched and halves the scale, with no host sync."""
    from csa_amd.train import AdamW
    g = torch.Generator().manual_seed(11)
    w0 = torch.randn(300, 7, generator=g)
    x = torch.randn(64, 300, generator=g)
    pg = torch.nn.Parameter(w0.cuda())
    pc = torch.nn.Parameter(w0.clone())
    og, oc = AdamW([pg], lr=1e-3, correct_bias=False), AdamW([pc], lr=1e-3, correct_bias=False)
    scaler = torch.amp.GradScaler("cuda", init_scale=2.0 ** 16)
    for step in range(3):
        og.zero_grad(set_to_none=True)
        oc.zero_grad(set_to_none=True)
        scaler.scale((x.cuda() @ pg).square().mean()).backward()
        (x @ pc).square().mean().backward()
        scaler.step(og)
        scaler.update()
        oc.step()
    np.testing.assert_allclose(pg.detach().cpu().numpy(), pc.detach().numpy(), rtol=1e-5, atol=1e-7)
    before = pg.detach().clone()
    m_before = og.state[pg]["exp_avg"].clone()
    og.zero_grad(set_to_none=True)
    scale = scaler.get_scale()
    scaler.scale((x.cuda() @ pg).square().mean() * float("inf")).backward()
    scaler.step(og)
    scaler.update()
    assert torch.equal(pg.detach(), before) and torch.equal(og.state[pg]["exp_avg"], m_before)
    assert scaler.get_scale() == scale * 0.5


def test_fused_adamw_two_param_groups_cache_per_group():
    """A decay / no-decay split (two param groups): each group keeps its own chunk tables and
    descriptors, so after the first step no table is rebuilt or re-sent; results match the per-op
    CPU path."""
    from csa_amd.train import AdamW
    g = torch.Generator().manual_seed(8)
    shapes = [(300, 7), (5000,), (64, 64), (9,)]
    base = [torch.randn(s, generator=g) for s in shapes]
    cpu = [torch.nn.Parameter(t.clone()) for t in base]
    gpu = [torch.nn.Parameter(t.cuda()) for t in base]
    groups = lambda ps: [{"params": ps[:2], "weight_decay": 0.01}, {"params": ps[2:], "weight_decay": 0.0}]
    o_cpu = AdamW(groups(cpu), lr=2e-3, correct_bias=False)
    o_gpu = AdamW(groups(gpu), lr=2e-3, correct_bias=False)
    seen = None
    for step in range(3):
        for pc, pg in zip(cpu, gpu):
            gr = torch.randn(pc.shape, generator=g)
            if pg.grad is None:
                pc.grad, pg.grad = gr.clone(), gr.cuda()
            else:  # grads stay in place (zero_grad(set_to_none=False) semantics): descriptors reused
                pc.grad.copy_(gr)
                pg.grad.copy_(gr.cuda())
        o_cpu.step()
        o_gpu.step()
        now = {k: (id(e["desc"]), id(e["owner"])) for k, e in o_gpu._tables.items()}
        assert len(now) == 2
        if seen is not None:
            assert now == seen
        seen = now
    for pc, pg in zip(cpu, gpu):
        np.testing.assert_allclose(pg.detach().cpu().numpy(), pc.detach().numpy(), rtol=1e-5, atol=1e-7)
