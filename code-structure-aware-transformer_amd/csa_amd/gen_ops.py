"""Generator head (module/components.py:95-102): log(softmax(dropout(logits))) as one HIP kernel per
direction (csrc/csa_gen.hip, csa_gen_logsoftmax_fwd / _bwd). GPU only: no CPU fallback."""
import ctypes

import torch

from ._lib import check, lib, on_device
from .ops import _draw_seed, _require_gpu, _stream


class GenLogSoftmax(torch.autograd.Function):
    """logits (..., V) fp32 -> logp (..., V); dropout p applied to the logits first (train mode)."""

    @staticmethod
    def forward(ctx, logits, p):
        _require_gpu(logits)
        if logits.dtype != torch.float32:
            raise RuntimeError("csa_gen_logsoftmax: fp32 logits expected")
        z = logits.contiguous()
        V = z.shape[-1]
        rows = z.numel() // V if V else 0
        out = torch.empty_like(z)
        seed = _draw_seed() if p > 0.0 else 0
        with on_device(z.device):
            check(lib().csa_gen_logsoftmax_fwd(ctypes.c_void_p(z.data_ptr()), ctypes.c_void_p(out.data_ptr()), rows, V,
                                               p, seed, 0, _stream(z.device)), "csa_gen_logsoftmax_fwd")
        ctx.save_for_backward(out)
        ctx.cfg = (rows, V, p, seed)
        return out

    @staticmethod
    def backward(ctx, g):
        (logp,) = ctx.saved_tensors
        rows, V, p, seed = ctx.cfg
        g = g.contiguous()
        dz = torch.empty_like(logp)
        with on_device(g.device):
            check(lib().csa_gen_logsoftmax_bwd(ctypes.c_void_p(g.data_ptr()), ctypes.c_void_p(logp.data_ptr()),
                                               ctypes.c_void_p(dz.data_ptr()), rows, V, p, seed, 0, _stream(g.device)),
                  "csa_gen_logsoftmax_bwd")
        return dz, None


def gen_log_softmax(logits, p):
    return GenLogSoftmax.apply(logits, float(p))
