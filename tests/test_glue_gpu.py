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
