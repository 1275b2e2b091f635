"""SampleGraphSparseGraph — drop-in for module/STE.py:8-19 (HIP sampler + STE backward)."""
import torch

from .. import ops

__all__ = ["SampleGraphSparseGraph"]


class SampleGraphSparseGraph(torch.autograd.Function):
    """forward: A = bernoulli(clamp(p, 0.01, 0.99)) (STE.py:10-15), drawn as u < clamp(p) with
    u = torch.rand (torch's global generator) on the GPU; backward: hardtanh(A * grad) (STE.py:17-19).
    ``apply(p, u)`` additionally accepts host-supplied uniforms (bit-exact parity mode)."""

    @staticmethod
    def forward(ctx, input, u=None):
        if u is None:
            u = torch.rand(input.shape, device=input.device, dtype=torch.float32)
        A = torch.ops.csa.ste_sample(input, u, 0.01, 0.99)
        ctx.save_for_backward(A)
        return A

    @staticmethod
    def backward(ctx, grad_output):
        (A,) = ctx.saved_tensors
        return torch.ops.csa.ste_backward(A, grad_output), None
