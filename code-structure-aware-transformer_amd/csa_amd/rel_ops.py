"""torch.ops.csa.rel_attn_{fwd,bwd} + autograd for DisentangledAttn.rel_attn
(module/disentangled_attn.py:44-65) over the C ABI."""
import ctypes
from typing import List

import torch

from ._lib import CSA_DTYPE_BF16, CSA_DTYPE_F32, RelAttnArgs, RelAttnBwdArgs, check, lib
from .ops import _bhnd, _require_gpu, _stream, head_major_out, packed_grads, packed_qkv, schedule_code, set_side_lane


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


def _fwd_args(q, k, v, lq, lk, rel, mask, group, out, lse, state, bf16=False):
    B, H, N, d = q.shape
    a = RelAttnArgs()
    a.B, a.H, a.N, a.L, a.d = B, H, N, lq.shape[1], d
    a.q, (a.q_sb, a.q_sh, a.q_sn) = q.data_ptr(), q.stride()[:3]
    a.k, (a.k_sb, a.k_sh, a.k_sn) = k.data_ptr(), k.stride()[:3]
    a.v, (a.v_sb, a.v_sh, a.v_sn) = v.data_ptr(), v.stride()[:3]
    a.lq, a.lk = lq.data_ptr(), lk.data_ptr()
    a.rel, a.rel_sb, a.rel_sh = rel.data_ptr(), rel.stride(0), rel.stride(1)
    a.mask, a.mask_sb, a.mask_sh = mask.data_ptr(), mask.stride(0), mask.stride(1)
    a.rel_head_group = group
    a.dtype = CSA_DTYPE_BF16 if bf16 else CSA_DTYPE_F32
    a.out, a.row_stats, a.state = out.data_ptr(), lse.data_ptr(), state.data_ptr()
    a.o_sb, a.o_sh, a.o_sn = out.stride()[:3]
    return a


@torch.library.custom_op("csa::rel_attn_fwd", mutates_args=())
def rel_attn_fwd_op(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, lq: torch.Tensor, lk: torch.Tensor,
                    rel: torch.Tensor, mask: torch.Tensor, group: int, bf16: bool = False) -> List[torch.Tensor]:
    """Returns [out (B,H,N,d), row_stats (B,H,N,2), state (uint8)]; bf16 = CSA_DTYPE_BF16 (d_k = 64).
    d_k = 64: out is a (B,H,N,d) view of (B,N,H,d) memory (the module's permute + view is then free)."""
    _require_gpu(q, k, v, lq, lk, rel, mask)
    q, k, v = _bhnd(q), _bhnd(k), _bhnd(v)
    lq, lk = lq.float().contiguous(), lk.float().contiguous()
    B, H, N, d = q.shape
    L = lq.shape[1]
    out = head_major_out(B, H, N, d, q.device) if d == 64 else torch.empty(B, H, N, d, device=q.device)
    lse = torch.empty(B, H, N, 2, device=q.device, dtype=torch.float32)  # (row max, 1/row sum)
    state = torch.empty(lib().csa_rel_attn_state_bytes(B, H, N, L, d), device=q.device, dtype=torch.uint8)
    a = _fwd_args(q, k, v, lq, lk, rel, mask, group, out, lse, state, bf16)
    check(lib().csa_rel_attn_fwd(ctypes.byref(a), _stream(q.device)), "csa_rel_attn_fwd")
    return [out, lse, state]


@rel_attn_fwd_op.register_fake
def _(q, k, v, lq, lk, rel, mask, group, bf16=False):
    B, H, N, d = q.shape
    return [q.new_empty(B, N, H, d).transpose(1, 2) if d == 64 else q.new_empty(B, H, N, d), q.new_empty(B, H, N, 2),
            q.new_empty(lib().csa_rel_attn_state_bytes(B, H, N, lq.shape[1], d), dtype=torch.uint8)]


@torch.library.custom_op("csa::rel_attn_bwd", mutates_args=())
def rel_attn_bwd_op(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, lq: torch.Tensor, lk: torch.Tensor,
                    rel: torch.Tensor, mask: torch.Tensor, group: int, out: torch.Tensor, lse: torch.Tensor,
                    state: torch.Tensor, dout: torch.Tensor, bf16: bool = False,
                    packed: bool = False, schedule: int = 0) -> List[torch.Tensor]:
    """Returns [dq, dk, dv, dlq (H,L,d), dlk (H,L,d)]; packed (d_k = 64): [dq, dk, dv] is ONE packed
    (B, N, 3, H, d) tensor, the gradient of the fused QKV projection (ops.packed_qkv)."""
    q, k, v = _bhnd(q), _bhnd(k), _bhnd(v)
    lq, lk = lq.float().contiguous(), lk.float().contiguous()
    B, H, N, d = q.shape
    dout = _bhnd(dout) if d == 64 else dout.float().contiguous()
    L = lq.shape[1]
    a = _fwd_args(q, k, v, lq, lk, rel, mask, group, out, lse, state, bf16)
    if packed:
        P, (dq, dk, dv) = packed_grads(B, H, N, d, q.device)
    else:
        dq, dk, dv = (torch.empty(B, H, N, d, device=q.device, dtype=torch.float32) for _ in range(3))
    dlq, dlk = torch.empty_like(lq), torch.empty_like(lk)
    ws = torch.empty(lib().csa_rel_attn_bwd_workspace_bytes(B, H, N, L, d), device=q.device, dtype=torch.uint8)
    b = RelAttnBwdArgs()
    b.fwd = ctypes.pointer(a)
    b.dout, b.dq, b.dk, b.dv = dout.data_ptr(), dq.data_ptr(), dk.data_ptr(), dv.data_ptr()
    b.do_sb, b.do_sh, b.do_sn = dout.stride()[:3]
    if packed:
        b.dq_sb, b.dq_sh, b.dq_sn = dq.stride()[:3]
        b.dk_sb, b.dk_sh, b.dk_sn = dk.stride()[:3]
        b.dv_sb, b.dv_sh, b.dv_sn = dv.stride()[:3]
    b.dlq, b.dlk, b.workspace = dlq.data_ptr(), dlk.data_ptr(), ws.data_ptr()
    set_side_lane(b, q.device, schedule)
    check(lib().csa_rel_attn_bwd(ctypes.byref(b), _stream(q.device)), "csa_rel_attn_bwd")
    return [P, dlq, dlk] if packed else [dq, dk, dv, dlq, dlk]


@rel_attn_bwd_op.register_fake
def _(q, k, v, lq, lk, rel, mask, group, out, lse, state, dout, bf16=False, packed=False, schedule=0):
    B, H, N, d = q.shape
    if packed:
        return [q.new_empty(B, N, 3, H, d), torch.empty_like(lq), torch.empty_like(lk)]
    return [torch.empty_like(q), torch.empty_like(k), torch.empty_like(v), torch.empty_like(lq), torch.empty_like(lk)]


class RelAttnFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, q, k, v, lq, lk, rel, mask, group, bf16=False, schedule=0):
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
    schedule: the backward's "auto" | "in_order" | "concurrent" (CSA_SCHED_*; bitwise-identical results)."""
    H = q.shape[1]
    rel, mask, group = _planes(rel, mask, H)
    if lq.dim() == 4:
        lq, lk = lq[0], lk[0]
    return RelAttnFunction.apply(q, k, v, lq, lk, rel, mask, group, bool(bf16), schedule_code(schedule))
