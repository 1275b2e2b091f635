"""End-to-end: the caller model (csa_amd.model.CSATrans) on the HIP kernels vs the REFERENCE CSATrans
(module/csa_trans.py) on identical weights, inputs and uniforms (tests/golden/csatrans_tiny.npz)."""
import numpy as np
import pytest
import torch

from conftest import has_gpu

TINY = dict(src_vocab_size=50, tgt_vocab_size=60, hidden_size=64, num_heads=8, num_layers=1, sbm_layers=2,
            use_pegen="pegen", dim_feed_forward=128, dropout=0.2, pe_dim=32, pegen_dim=128, sbm_enc_dim=512,
            clusters=[10, 12], full_att=False)


def fill_params_deterministic(model, seed):
    """Same fill as tools/gen_golden.py (numpy PCG64, sorted parameter names)."""
    rng = np.random.default_rng(seed)
    named = dict(model.named_parameters())
    with torch.no_grad():
        for k in sorted(named):
            p = named[k]
            fan = p.shape[-1] if p.dim() > 1 else 1
            p.copy_(torch.from_numpy((rng.standard_normal(p.shape) * (0.5 / np.sqrt(fan))).astype(np.float32)))


def test_state_dict_keys_match_reference(golden):
    """Reference checkpoints load into the MI355X model unchanged (module/csa_trans.py:176-177)."""
    from csa_amd.model import CSATrans
    z = golden("csatrans_tiny")
    m = CSATrans(**TINY)
    assert sorted(m.state_dict().keys()) == list(z["state_keys"])


@pytest.mark.gpu
@pytest.mark.skipif(not has_gpu(), reason="needs GPU")
def test_csatrans_forward_backward_matches_reference(golden):
    from csa_amd.data import synthetic_batch  # noqa: F401
    from csa_amd.model import CSATrans, batch_to_device, label_smoothing_loss
    z = golden("csatrans_tiny")
    m = CSATrans(**TINY)
    fill_params_deterministic(m, 71)
    m = m.cuda().eval()
    for i in range(2):
        getattr(m.SBM, f"transformer_{i}").mha.attn.uniforms = torch.from_numpy(z[f"u{i}"]).cuda()
    x, y = batch_to_device({k: z[k] for k in ("src_seq", "tgt_seq", "target", "L", "T", "L_mask", "T_mask")},
                           torch.device("cuda"))
    out, sparsity, pe, graphs, attns = m(x)
    loss = label_smoothing_loss(out, y)
    np.testing.assert_allclose(out.detach().cpu().numpy(), z["out"], rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(sparsity.item(), z["sparsity"][0], rtol=1e-6)
    np.testing.assert_allclose(loss.item(), z["loss"][0], rtol=1e-5)
    (loss + 1e-2 * sparsity).backward()
    named = dict(m.named_parameters())
    checked = 0
    for k in z:
        if k.startswith("g:"):
            np.testing.assert_allclose(named[k[2:]].grad.cpu().numpy(), z[k], rtol=1e-3, atol=2e-5, err_msg=k)
            checked += 1
    assert checked >= 10
