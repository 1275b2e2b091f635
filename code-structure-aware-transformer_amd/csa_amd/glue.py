"""Encoder/decoder glue of the train step: nn.Linear whose bias gradient is
csa_bias_grad (csrc/csa_glue.hip) instead of torch's generic strided reduction. Forward and the
two GEMMs of the backward stay on hipBLASLt. Same parameters and state_dict keys as nn.Linear."""
import ctypes

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._lib import check, lib


def bias_grad(gy2: torch.Tensor) -> torch.Tensor:
    """(rows, cols) contiguous fp32 on the GPU -> (cols,) column sums (deterministic order)."""
    rows, cols = gy2.shape
    db = torch.empty(cols, device=gy2.device, dtype=torch.float32)
    L = lib()
    ws = torch.empty(max(1, L.csa_bias_grad_workspace_bytes(rows, cols)), dtype=torch.uint8, device=gy2.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(gy2.device).cuda_stream)
    check(L.csa_bias_grad(ctypes.c_void_p(gy2.data_ptr()), ctypes.c_void_p(db.data_ptr()), rows, cols, 0,
                          ctypes.c_void_p(ws.data_ptr()), stream), "csa_bias_grad")
    return db


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy2 = gy.reshape(-1, gy.shape[-1])
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = gy @ w
        if ctx.needs_input_grad[1]:
            dw = gy2.t() @ x.reshape(-1, x.shape[-1])
        if ctx.needs_input_grad[2]:
            g = gy2 if gy2.is_contiguous() and gy2.dtype == torch.float32 else gy2.float().contiguous()
            db = bias_grad(g).to(gy.dtype)
        return dx, dw, db


def linear(x, w, b=None):
    if b is None or not x.is_cuda or x.dtype != torch.float32:
        return F.linear(x, w, b)
    return _LinearFn.apply(x, w, b)


class Linear(nn.Linear):
    def forward(self, x):
        return linear(x, self.weight, self.bias)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        L = lib()
        cols = x.shape[-1]
        x2 = x.reshape(-1, cols)
        y = torch.empty_like(x2)
        stats = torch.empty(x2.shape[0], 2, device=x.device, dtype=torch.float32)
        stream = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        check(L.csa_layernorm_fwd(p(x2), p(w), p(b), p(y), p(stats), x2.shape[0], cols, eps, stream),
              "csa_layernorm_fwd")
        ctx.save_for_backward(x2, w, stats)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, gy):
        x2, w, stats = ctx.saved_tensors
        L = lib()
        rows, cols = x2.shape
        gy2 = gy.reshape(rows, cols).contiguous()
        dx = torch.empty_like(x2)
        dw = torch.empty(cols, device=x2.device, dtype=torch.float32)
        db = torch.empty_like(dw)
        ws = torch.empty(max(1, L.csa_layernorm_bwd_workspace_bytes(rows, cols)), dtype=torch.uint8,
                         device=x2.device)
        stream = ctypes.c_void_p(torch.cuda.current_stream(x2.device).cuda_stream)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        check(L.csa_layernorm_bwd(p(gy2), p(x2), p(stats), p(w), p(dx), p(dw), p(db), rows, cols, p(ws), stream),
              "csa_layernorm_bwd")
        return dx.view(gy.shape), dw, db, None


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm (same parameters / state_dict keys) on csa_layernorm_fwd/_bwd (csrc/csa_glue.hip)
    for fp32 CUDA inputs over one normalised dim with affine weights; anything else takes torch's."""

    def forward(self, x):
        if (x.is_cuda and x.dtype == torch.float32 and len(self.normalized_shape) == 1 and self.weight is not None
                and self.bias is not None and lib().csa_layernorm_supported(x.shape[-1])
                and x.is_contiguous()):
            return _LayerNormFn.apply(x, self.weight, self.bias, float(self.eps))
        return super().forward(x)
