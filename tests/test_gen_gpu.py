"""Generator head (module/components.py:95-102) on the HIP kernels (csrc/csa_gen.hip) vs the reference:
the reference Generator's own fixture (eval; incl. an underflowed row: -inf log-probabilities and its
NaN gradient row, as torch computes log(softmax)), and train-mode dropout against the reference op
chain under the kernel's regenerated Philox keep mask (oracle/philox.py:gen_keep)."""
import numpy as np
import pytest
import torch

from conftest import has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs GPU")]
RTOL, ATOL = 1e-4, 1e-5  # north_star fp32 tolerance (sums over V = 20000 terms: ~1e-5 rounding)


def test_generator_matches_reference_golden(golden):
    from csa_amd.model import Generator
    z = golden("generator_v1003")
    V, D = z["weight"].shape
    gen = Generator(V, D, 0.2).cuda().eval()
    with torch.no_grad():
        gen.linear.weight.copy_(torch.from_numpy(z["weight"]))
        gen.linear.bias.copy_(torch.from_numpy(z["bias"]))
    x = torch.from_numpy(z["x"]).cuda().requires_grad_(True)
    out = gen(x)
    out.backward(torch.from_numpy(z["dout"]).cuda())
    o = out.detach().cpu().numpy()
    assert np.array_equal(np.isinf(o), np.isinf(z["out"])), "-inf pattern of log(softmax)"
    np.testing.assert_allclose(o, z["out"], rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(x.grad.cpu().numpy(), z["dx"], rtol=1e-4, atol=1e-5)  # NaN == NaN
    np.testing.assert_allclose(gen.linear.weight.grad.cpu().numpy(), z["dweight"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(gen.linear.bias.grad.cpu().numpy(), z["dbias"], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize("rows,V,p", [(37, 20000, 0.2), (5, 1003, 0.5), (3, 7, 0.2), (64, 4096, 0.0)])
def test_train_mode_matches_reference_chain_under_regenerated_mask(rows, V, p, monkeypatch):
    from csa_amd import gen_ops
    from oracle import philox
    seed = 0x1234_5678_9ABC_DEF0
    monkeypatch.setattr(gen_ops, "_draw_seed", lambda: seed)
    g = torch.Generator().manual_seed(rows + V)
    z = torch.randn(rows, V, generator=g) * 3.0
    dout = torch.randn(rows, V, generator=g)
    zg = z.cuda().requires_grad_(True)
    out = gen_ops.gen_log_softmax(zg, p)
    out.backward(dout.cuda())
    keep = torch.from_numpy(philox.gen_keep(rows, V, seed, 0, p)) if p > 0 else torch.ones(rows, V, dtype=torch.bool)
    if p > 0:
        frac = keep.float().mean().item()
        assert abs(frac - (1 - p)) < 6 * np.sqrt(p * (1 - p) / keep.numel()) + 1e-3
    zc = z.clone().requires_grad_(True)
    ref = torch.log(torch.softmax(zc * keep.float() / (1.0 - p), -1))  # nn.Dropout then components.py:101-102
    ref.backward(dout)
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), rtol=RTOL, atol=ATOL)
    np.testing.assert_allclose(zg.grad.cpu().numpy(), zc.grad.numpy(), rtol=RTOL, atol=ATOL)
