"""Autograd for DisentangledAttn.rel_attn (module/disentangled_attn.py:44-65) over torch.ops.csa.rel_attn_{fwd,bwd}
(C++ implementations in csrc/csa_torch.cpp, calling the C ABI)."""

import torch

from .ops import lib, packed_qkv, schedule_code, shim


def _planes(rel: torch.Tensor, mask: torch.Tensor, H: int):
    """Relation/mask planes as uint8 + (batch stride, head stride, head group).

    Accepts the reference layout (B,H,N,N) int64 / bool (module/csa_trans.py:206-211) or the compact
    CSE layout (B,2,N,N) uint8 planes (parent L, sibling T) shared by heads [0,H/2) and [H/2,H)."""
    if rel.dim() != 4:
        raise ValueError("rel must be (B,H,N,N) or (B,2,N,N)")
    rel = rel if rel.dtype == torch.uint8 else rel.to(torch.uint8)
    mask = mask if mask.dtype == torch.uint8 else mask.to(torch.uint8)
    rel, mask = rel.contiguous(), mask.contiguous()
    if rel.shape[1] == 2 and H != 2:
        group = H // 2
    elif rel.shape[1] == H:
        group = 0
    else:
        raise ValueError(f"rel has {rel.shape[1]} planes for {H} heads")
    return rel, mask, group


# fake (meta) implementations of the C++ ops csa::rel_attn_fwd / rel_attn_bwd (schemas: csa_amd.ops._SCHEMAS,
# implementations: csrc/csa_torch.cpp). rel_attn_fwd returns [out (B,H,N,d), row_stats (B,H,N,2), state]; for
# d_k = 64 out is a (B,H,N,d) view of (B,N,H,d) memory. rel_attn_bwd returns [dq, dk, dv, dlq, dlk], or with
# packed (d_k = 64) [P (B,N,3,H,d), dlq, dlk], P the gradient of the fused QKV projection (ops.packed_qkv).
@torch.library.register_fake("csa::rel_attn_fwd")
def _(q, k, v, lq, lk, rel, mask, group, bf16=False):
    B, H, N, d = q.shape
    return [q.new_empty(B, N, H, d).transpose(1, 2) if d == 64 else q.new_empty(B, H, N, d), q.new_empty(B, H, N, 2),
            q.new_empty(lib().csa_rel_attn_state_bytes(B, H, N, lq.shape[1], d), dtype=torch.uint8)]


@torch.library.register_fake("csa::rel_attn_bwd")
def _(q, k, v, lq, lk, rel, mask, group, out, lse, state, dout, bf16=False, packed=False, schedule=0):
    B, H, N, d = q.shape
    if packed:
        return [q.new_empty(B, N, 3, H, d), torch.empty_like(lq), torch.empty_like(lk)]
    return [torch.empty_like(q), torch.empty_like(k), torch.empty_like(v), torch.empty_like(lq), torch.empty_like(lk)]


class RelAttnFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, lq, lk, rel, mask, group, bf16=False, schedule=0):
        shim()
        out, lse, state = torch.ops.csa.rel_attn_fwd(q, k, v, lq, lk, rel, mask, group, bf16)
        ctx.save_for_backward(q, k, v, lq, lk, rel, mask, out, lse, state)
        ctx.group, ctx.bf16, ctx.schedule = group, bf16, schedule
        ctx.packed = q.shape[-1] == 64 and packed_qkv(q, k, v)
        return out

    @staticmethod
    def backward(ctx, dout):
        q, k, v, lq, lk, rel, mask, out, lse, state = ctx.saved_tensors
        g = torch.ops.csa.rel_attn_bwd(q, k, v, lq, lk, rel, mask, ctx.group, out, lse, state, dout, ctx.bf16,
                                       ctx.packed, ctx.schedule)
        if ctx.packed:  # head-major views of the packed gradient (split_heads3's backward takes it whole)
            dq, dk, dv = (g[0][:, :, i].transpose(1, 2) for i in range(3))
            dlq, dlk = g[1], g[2]
        else:
            dq, dk, dv, dlq, dlk = g
        return dq, dk, dv, dlq, dlk, None, None, None, None, None


def rel_attn(q, k, v, lq, lk, rel, mask, bf16=False, schedule="auto"):
    """DisentangledAttn.rel_attn (module/disentangled_attn.py:44-65) on the GPU.

    q,k,v (B,H,N,d) (strided views fine); lq,lk (1,H,L,d) or (H,L,d); rel/mask (B,H,N,N) (reference
    int64/bool layout) or (B,2,N,N) uint8 planes shared by head halves (compact CSE layout).
    schedule: the backward's "auto" | "in_order" | "concurrent" (CSA_SCHED_*; bitwise-identical results). Only
    bf16 mode forks: the fp32 fused backward hands its key half's g tiles to the query half and runs in order."""
    H = q.shape[1]
    rel, mask, group = _planes(rel, mask, H)
    if lq.dim() == 4:  # (1,H,L,d): a view (select's backward would zero-fill a (1,H,L,d) gradient)
        lq, lk = lq.squeeze(0), lk.squeeze(0)
    return RelAttnFunction.apply(q, k, v, lq, lk, rel, mask, group, bool(bf16), schedule_code(schedule))
