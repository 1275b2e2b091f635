"""torch custom ops (``torch.ops.csa.*``) over the C ABI, plus their autograd wrappers.

Layering (top to bottom):
  csa_amd.module.*            drop-in nn.Modules with the reference's names/signatures/state_dict keys
  SBMAttentionFunction etc.   torch.autograd.Function: saves what the backward needs
  torch.ops.csa.*             torch.library custom ops: validate, allocate outputs/state/workspace
                              with the torch caching allocator, pass raw pointers + the current
                              HIP stream to ...
  libcsa_hip.so               extern "C" entry points (include/csa_hip.h) -> gfx950 kernels

There is no CPU path: every op raises on a non-CUDA tensor or when the library is absent.
"""
import ctypes
import math
import os
from typing import List, Optional, Tuple

import torch

from . import _lib
from ._lib import CSA_DTYPE_BF16, CSA_DTYPE_F32, CSA_FLAG_DENSE, SCHEDULES, SbmBwdArgs, SbmFwdArgs, check, lib

__all__ = ["sbm_attention", "dense_attention", "ste_sample", "ste_backward", "rel_attn", "SBMAttentionFunction"]


# Optional per-stage event profiling (bench.py): csa_prof structs owned by the caller.
_PROF = {"fwd": None, "bwd": None}


def set_stage_profiler(fwd_prof=None, bwd_prof=None):
    """Install caller-owned csa_prof structs (ctypes) that the next sbm fwd/bwd calls record into."""
    _PROF["fwd"], _PROF["bwd"] = fwd_prof, bwd_prof


def _ptr(t: Optional[torch.Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("csa ops run only on the GPU (HIP); got a tensor on " + str(t.device))


def _bhnd(t: torch.Tensor) -> torch.Tensor:
    """(B,H,N,d) fp32 view usable by the kernels: last dim contiguous, 16-B aligned, strides % 4 == 0.
    Non-contiguous split_heads views (sbm_attn.py:137-140) pass through without a copy. A zero leading
    stride (a broadcast, e.g. the gradient of X.sum((0, 1, 2))) is materialised: the ABI reads an all-zero
    stride triple as "contiguous", and the kernels' row arithmetic assumes distinct rows."""
    if t.dtype != torch.float32:
        t = t.float()
    ok = (t.stride(3) == 1 and t.data_ptr() % 16 == 0 and all(s % 4 == 0 and s > 0 for s in t.stride()[:3]))
    return t if ok else t.contiguous()


# ---------------------------------------------------------------------------------------
# Backward schedule + the caller-owned side lane (ABI v5: the library owns no streams or events)
# ---------------------------------------------------------------------------------------
_SIDE = {}  # device index -> (torch.cuda.Stream, fork hipEvent_t, join hipEvent_t)
# debugging override of every module's bwd_schedule: CSA_BWD_CONCUR=0 -> in_order, 1 -> concurrent
_SCHED_OVERRIDE = {"0": "in_order", "1": "concurrent"}.get(os.environ.get("CSA_BWD_CONCUR", ""))


def _hip_event(device):
    hip = ctypes.CDLL("libamdhip64.so.7")
    hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
    e = ctypes.c_void_p()
    with torch.cuda.device(device):
        if hip.hipEventCreateWithFlags(ctypes.byref(e), 0x2) != 0:  # hipEventDisableTiming
            raise RuntimeError("hipEventCreateWithFlags failed")
    return e.value


def side_lane(device):
    """(side stream, fork event, join event) raw handles of `device`, created once per device and owned
    here (Python), handed to every backward that may run its two halves side by side."""
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    ent = _SIDE.get(idx)
    if ent is None:
        s = torch.cuda.Stream(device=idx)
        ent = _SIDE[idx] = (s, _hip_event(idx), _hip_event(idx))
    return ent[0].cuda_stream, ent[1], ent[2]


def schedule_code(schedule: str) -> int:
    """"auto" | "in_order" | "concurrent" -> CSA_SCHED_* (the CSA_BWD_CONCUR override wins)."""
    s = _SCHED_OVERRIDE or schedule
    if s not in SCHEDULES:
        raise ValueError(f"bwd schedule must be one of {sorted(SCHEDULES)}, got {schedule!r}")
    return SCHEDULES[s]


def set_side_lane(args, device, schedule: int):
    """Fill the ABI v5 schedule / side-lane fields of a bwd args struct."""
    args.schedule = schedule
    if schedule != SCHEDULES["in_order"]:
        args.side_stream, args.side_fork, args.side_join = side_lane(device)


def packed_qkv(Q, K, V) -> bool:
    """Q, K, V are the three head-major views of one packed (B, N, 3, H, d) projection output
    (glue.split_heads3): same storage, K / V offset by H*d / 2*H*d elements."""
    if not (Q.shape == K.shape == V.shape and Q.stride() == K.stride() == V.stride() and Q.dim() == 4):
        return False
    B, H, N, d = Q.shape
    if Q.stride() != (N * 3 * H * d, d, 3 * H * d, 1) or Q.dtype != torch.float32:
        return False
    st = Q.untyped_storage().data_ptr()
    return (K.untyped_storage().data_ptr() == st and V.untyped_storage().data_ptr() == st
            and K.storage_offset() == Q.storage_offset() + H * d and V.storage_offset() == Q.storage_offset() + 2 * H * d)


def packed_grads(B, H, N, d, device):
    """A packed (B, N, 3, H, d) gradient buffer and its three head-major (B, H, N, d) views."""
    P = torch.empty(B, N, 3, H, d, device=device, dtype=torch.float32)
    return P, [P[:, :, i].transpose(1, 2) for i in range(3)]


def head_major_out(B, H, N, d, device):
    """(B, H, N, d) view of a (B, N, H, d) buffer: combine_heads (sbm_attn.py:143-146,
    disentangled_attn.py:63) of it is a free view."""
    return torch.empty(B, N, H, d, device=device, dtype=torch.float32).transpose(1, 2)


def _fwd_struct(Q, K, V, mask, cluster_w, pw, pb, u, seed, offset, attn_p, proj_p, dense, X, sp, state, k,
                bf16=False):
    B, H, N, d = Q.shape
    M = K.shape[2]
    a = SbmFwdArgs()
    a.B, a.H, a.N, a.M, a.d, a.k = B, H, N, M, d, (0 if dense else k)
    a.Q, (a.q_sb, a.q_sh, a.q_sn) = Q.data_ptr(), Q.stride()[:3]
    a.K, (a.k_sb, a.k_sh, a.k_sn) = K.data_ptr(), K.stride()[:3]
    a.V, (a.v_sb, a.v_sh, a.v_sn) = V.data_ptr(), V.stride()[:3]
    if mask is not None:
        a.key_mask, a.mask_sb = mask.data_ptr(), mask.stride(0)
    if not dense:
        a.cluster_w = cluster_w.data_ptr()
        for i in range(3):
            a.proj_w[i] = pw[i].data_ptr()
            a.proj_b[i] = pb[i].data_ptr()
        a.sparsity = sp.data_ptr()
    if u is not None:
        a.uniforms = u.data_ptr()
    a.seed, a.offset = seed & (2 ** 64 - 1), offset & (2 ** 64 - 1)
    a.attn_dropout, a.proj_dropout = attn_p, proj_p
    a.flags = CSA_FLAG_DENSE if dense else 0
    a.dtype = CSA_DTYPE_BF16 if bf16 else CSA_DTYPE_F32
    a.X = X.data_ptr()
    if X.dim() == 4:
        a.x_sb, a.x_sh, a.x_sn = X.stride()[:3]
    a.state = state.data_ptr()
    return a


def _prep(Q, K, V, mask, cluster_w, pw, pb, u):
    _require_gpu(Q, K, V)
    Q, K, V = _bhnd(Q), _bhnd(K), _bhnd(V)
    if mask is not None:
        mask = mask.to(device=Q.device, dtype=torch.float32).contiguous()
    if u is not None:
        u = u.to(device=Q.device, dtype=torch.float32).contiguous()
    cw = None if cluster_w is None else cluster_w.float().contiguous()
    pw = [w.float().contiguous() for w in pw] if pw else []
    pb = [b.float().contiguous() for b in pb] if pb else []
    return Q, K, V, mask, cw, pw, pb, u


# ---------------------------------------------------------------------------------------
# torch.library custom ops
# ---------------------------------------------------------------------------------------
@torch.library.custom_op("csa::sbm_fwd", mutates_args=())
def sbm_fwd_op(Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, mask: Optional[torch.Tensor],
               cluster_w: Optional[torch.Tensor], proj_w: List[torch.Tensor], proj_b: List[torch.Tensor],
               uniforms: Optional[torch.Tensor], k: int, seed: int, offset: int, attn_p: float, proj_p: float,
               dense: bool, bf16: bool = False) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Forward of SBMAttention (module/sbm_attn.py:32-66) or FullAttention (:77-87, dense=True).
    Returns (X (B,H,N,d), sparsity (H,) [empty if dense], state (uint8, saved for backward)).
    bf16=True: the N^2 contractions on bf16 MFMA (CSA_DTYPE_BF16; fp32 storage, fp32 expA / sampling)."""
    Q, K, V, mask, cw, pw, pb, u = _prep(Q, K, V, mask, cluster_w, proj_w, proj_b, uniforms)
    B, H, N, d = Q.shape
    M = K.shape[2]
    L = lib()
    flags = CSA_FLAG_DENSE if dense else 0
    if not L.csa_sbm_supported(d, k, flags):
        raise RuntimeError(f"csa::sbm_fwd: unsupported head_dim={d} / num_clusters={k}")
    X = head_major_out(B, H, N, d, Q.device)
    sp = torch.empty(0 if dense else H, device=Q.device, dtype=torch.float32)
    state = torch.empty(L.csa_sbm_state_bytes(B, H, N, M, d, k, flags), device=Q.device, dtype=torch.uint8)
    a = _fwd_struct(Q, K, V, mask, cw, pw, pb, u, seed, offset, attn_p, proj_p, dense, X, sp, state, k, bf16)
    if _PROF["fwd"] is not None:
        a.prof = ctypes.pointer(_PROF["fwd"])
    check(L.csa_sbm_fwd(ctypes.byref(a), _stream(Q.device)), "csa_sbm_fwd")
    return X, sp, state


@sbm_fwd_op.register_fake
def _(Q, K, V, mask, cluster_w, proj_w, proj_b, uniforms, k, seed, offset, attn_p, proj_p, dense, bf16=False):
    B, H, N, d = Q.shape
    return (Q.new_empty(B, N, H, d).transpose(1, 2), Q.new_empty(0 if dense else H),
            Q.new_empty(lib().csa_sbm_state_bytes(B, H, N, K.shape[2], d, k, CSA_FLAG_DENSE if dense else 0),
                        dtype=torch.uint8))


@torch.library.custom_op("csa::sbm_maps", mutates_args=())
def sbm_maps_op(Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, mask: Optional[torch.Tensor],
                state: torch.Tensor, k: int, dense: bool) -> Tuple[torch.Tensor, torch.Tensor]:
    """The (graph, attn) maps SBMAttention returns (sbm_attn.py:57,62), from a forward's state."""
    Q, K, V, mask, _, _, _, _ = _prep(Q, K, V, mask, None, None, None, None)
    B, H, N, d = Q.shape
    M = K.shape[2]
    graph = torch.empty(B, H, N, M, device=Q.device, dtype=torch.float32)
    attn = torch.empty_like(graph)
    a = _fwd_struct(Q, K, V, mask, None, [], [], None, 0, 0, 0.0, 0.0, True, graph, None, state, k)
    a.flags = CSA_FLAG_DENSE if dense else 0
    a.k = 0 if dense else k
    a.X = Q.data_ptr()  # unused by maps; must be a valid aligned pointer for validation
    a.x_sb = a.x_sh = a.x_sn = 0
    if not dense:  # validation of non-dense args needs these non-null (unused by the maps kernel)
        a.cluster_w = a.Q
        a.sparsity = a.Q
        for i in range(3):
            a.proj_w[i] = a.Q
            a.proj_b[i] = a.Q
    check(lib().csa_sbm_maps(ctypes.byref(a), _ptr(graph), _ptr(attn), _stream(Q.device)), "csa_sbm_maps")
    return graph, attn


@sbm_maps_op.register_fake
def _(Q, K, V, mask, state, k, dense):
    B, H, N, d = Q.shape
    g = Q.new_empty(B, H, N, K.shape[2])
    return g, torch.empty_like(g)


@torch.library.custom_op("csa::sbm_bwd", mutates_args=())
def sbm_bwd_op(Q: torch.Tensor, K: torch.Tensor, V: torch.Tensor, mask: Optional[torch.Tensor],
               cluster_w: Optional[torch.Tensor], proj_w: List[torch.Tensor], proj_b: List[torch.Tensor],
               k: int, attn_p: float, proj_p: float, seed: int, offset: int, dense: bool, state: torch.Tensor,
               X: torch.Tensor, dX: torch.Tensor, dsparsity: Optional[torch.Tensor],
               dgraph: Optional[torch.Tensor], bf16: bool = False, packed: bool = False,
               dattn: Optional[torch.Tensor] = None, schedule: int = 0) -> List[torch.Tensor]:
    """Backward of csa::sbm_fwd. Returns [dQ, dK, dV] (+ [dcluster_w, dW0, db0, dW1, db1, dW2, db2] if not dense).
    dgraph / dattn: upstream gradients of the returned graph / attn maps (sbm_attn.py:66), or None.
    packed: [dQ, dK, dV] is replaced by ONE packed (B, N, 3, H, d) tensor (the gradient of a fused QKV
    projection, written in place by the kernels; see packed_qkv)."""
    Q, K, V, mask, cw, pw, pb, _ = _prep(Q, K, V, mask, cluster_w, proj_w, proj_b, None)
    B, H, N, d = Q.shape
    M = K.shape[2]
    L = lib()
    flags = CSA_FLAG_DENSE if dense else 0
    sp = torch.empty(0 if dense else H, device=Q.device, dtype=torch.float32)
    a = _fwd_struct(Q, K, V, mask, cw, pw, pb, None, seed, offset, attn_p, proj_p, dense, X, sp, state, k, bf16)
    dX = _bhnd(dX)  # strided (e.g. the combine_heads view's gradient) without a copy
    if packed:
        P, (dQ, dK, dV) = packed_grads(B, H, N, d, Q.device)
        outs = [P]
    else:
        dQ = torch.empty(B, H, N, d, device=Q.device, dtype=torch.float32)
        dK = torch.empty(B, H, M, d, device=Q.device, dtype=torch.float32)
        dV = torch.empty_like(dK)
        outs = [dQ, dK, dV]
    b = SbmBwdArgs()
    b.fwd = ctypes.pointer(a)
    b.dX, b.dQ, b.dK, b.dV = dX.data_ptr(), dQ.data_ptr(), dK.data_ptr(), dV.data_ptr()
    b.dx_sb, b.dx_sh, b.dx_sn = dX.stride()[:3]
    b.dq_sb, b.dq_sh, b.dq_sn = dQ.stride()[:3]
    b.dk_sb, b.dk_sh, b.dk_sn = dK.stride()[:3]
    b.dv_sb, b.dv_sh, b.dv_sn = dV.stride()[:3]
    keep = []
    ws = None
    if dattn is not None or not dense:
        ws = torch.empty(L.csa_sbm_bwd_workspace_bytes(B, H, N, M, d, k, flags), device=Q.device, dtype=torch.uint8)
        b.workspace = ws.data_ptr()
        keep.append(ws)
    if dattn is not None:
        dattn = dattn.float().contiguous()
        b.dattn = dattn.data_ptr()
    if not dense:
        if dsparsity is not None:
            dsparsity = dsparsity.float().contiguous()
            b.dsparsity = dsparsity.data_ptr()
        if dgraph is not None:
            dgraph = dgraph.float().contiguous()
            b.dgraph = dgraph.data_ptr()
        dC = torch.empty_like(cw)
        b.dcluster_w = dC.data_ptr()
        outs.append(dC)
        for i in range(3):
            dw, db = torch.empty_like(pw[i]), torch.empty_like(pb[i])
            b.dproj_w[i], b.dproj_b[i] = dw.data_ptr(), db.data_ptr()
            outs += [dw, db]
    if _PROF["bwd"] is not None:
        b.prof = ctypes.pointer(_PROF["bwd"])
    set_side_lane(b, Q.device, schedule)
    check(L.csa_sbm_bwd(ctypes.byref(b), _stream(Q.device)), "csa_sbm_bwd")
    return outs


@sbm_bwd_op.register_fake
def _(Q, K, V, mask, cluster_w, proj_w, proj_b, k, attn_p, proj_p, seed, offset, dense, state, X, dX, dsparsity,
      dgraph, bf16=False, packed=False, dattn=None, schedule=0):
    B, H, N, d = Q.shape
    outs = [Q.new_empty(B, N, 3, H, d)] if packed else [torch.empty_like(Q), torch.empty_like(K), torch.empty_like(V)]
    if not dense:
        outs.append(torch.empty_like(cluster_w))
        for i in range(3):
            outs += [torch.empty_like(proj_w[i]), torch.empty_like(proj_b[i])]
    return outs


@torch.library.custom_op("csa::ste_sample", mutates_args=())
def ste_sample_op(p: torch.Tensor, u: torch.Tensor, lo: float, hi: float) -> torch.Tensor:
    """STE.py:10-15: A = (u < clamp(p, lo, hi)) as fp32 {0,1}."""
    _require_gpu(p, u)
    p = p.float().contiguous()
    u = u.float().contiguous()
    A = torch.empty_like(p)
    check(lib().csa_ste_sample(_ptr(p), _ptr(u), _ptr(A), p.numel(), lo, hi, _stream(p.device)), "csa_ste_sample")
    return A


@ste_sample_op.register_fake
def _(p, u, lo, hi):
    return torch.empty_like(p)


@torch.library.custom_op("csa::ste_backward", mutates_args=())
def ste_backward_op(A: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
    """STE.py:17-19: hardtanh(A * grad)."""
    _require_gpu(A, g)
    A = A.float().contiguous()
    g = g.float().contiguous()
    out = torch.empty_like(g)
    check(lib().csa_ste_backward(_ptr(A), _ptr(g), _ptr(out), g.numel(), _stream(g.device)), "csa_ste_backward")
    return out


@ste_backward_op.register_fake
def _(A, g):
    return torch.empty_like(g)


# ---------------------------------------------------------------------------------------
# autograd
# ---------------------------------------------------------------------------------------
def _draw_seed():
    # one 64-bit Philox key per call from torch's global CPU generator (seeded by torch.manual_seed)
    return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())


class SBMAttentionFunction(torch.autograd.Function):
    """Differentiable fused SBM / dense attention. Inputs after ctx: see sbm_attention()."""

    @staticmethod
    def forward(ctx, Q, K, V, mask, cluster_w, w0, b0, w1, b1, w2, b2, uniforms, k, attn_p, proj_p, dense,
                want_maps, bf16=False, schedule=0):
        seed = _draw_seed()
        pw = [] if dense else [w0, w1, w2]
        pb = [] if dense else [b0, b1, b2]
        X, sp, state = torch.ops.csa.sbm_fwd(Q, K, V, mask, None if dense else cluster_w, pw, pb, uniforms, k, seed, 0,
                                            attn_p, proj_p, dense, bf16)
        graph = attn = None
        if want_maps:
            graph, attn = torch.ops.csa.sbm_maps(Q, K, V, mask, state, k, dense)
        ctx.save_for_backward(Q, K, V, mask, cluster_w, w0, b0, w1, b1, w2, b2, state, X)
        ctx.cfg = (k, attn_p, proj_p, seed, dense, bf16, schedule)
        ctx.packed = packed_qkv(Q, K, V)
        ctx.set_materialize_grads(False)
        return X, (sp if not dense else None), graph, attn

    @staticmethod
    def backward(ctx, dX, dsp, dgraph, dattn):
        Q, K, V, mask, cluster_w, w0, b0, w1, b1, w2, b2, state, X = ctx.saved_tensors
        k, attn_p, proj_p, seed, dense, bf16, schedule = ctx.cfg
        if dX is None:
            dX = torch.zeros_like(X)
        pw = [] if dense else [w0, w1, w2]
        pb = [] if dense else [b0, b1, b2]
        g = torch.ops.csa.sbm_bwd(Q, K, V, mask, None if dense else cluster_w, pw, pb, k, attn_p, proj_p, seed, 0,
                                  dense, state, X, dX, dsp, None if dense else dgraph, bf16, ctx.packed, dattn,
                                  schedule)
        if ctx.packed:  # the three head-major views of the packed gradient (split_heads3's backward takes it whole)
            dQ, dK, dV = (g[0][:, :, i].transpose(1, 2) for i in range(3))
            g = [None, None] + list(g)
        else:
            dQ, dK, dV = g[:3]
        if dense:
            return (dQ, dK, dV) + (None,) * 16
        dC, dw0, db0, dw1, db1, dw2, db2 = g[3:]
        return dQ, dK, dV, None, dC, dw0, db0, dw1, db1, dw2, db2, None, None, None, None, None, None, None, None


def sbm_attention(Q, K, V, mask, cluster_w, proj, k, uniforms=None, attn_p=0.0, proj_p=0.0, want_maps=True,
                  bf16=False, schedule="auto"):
    """Fused SBMAttention.forward (module/sbm_attn.py:32-66) -> (X, sparsity, graph, attn).

    proj: [w0, b0, w1, b1, w2, b2] (proj.0/.3/.6). uniforms: optional (B,H,N,M) host-supplied draws
    (bit-exact parity mode); otherwise in-kernel Philox. graph/attn are None when want_maps=False.
    bf16: bf16-MFMA attention contractions (the maps, if requested, are still computed in fp32).
    schedule: the backward's "auto" | "in_order" | "concurrent" (CSA_SCHED_*; bitwise-identical results)."""
    w0, b0, w1, b1, w2, b2 = proj
    return SBMAttentionFunction.apply(Q, K, V, mask, cluster_w, w0, b0, w1, b1, w2, b2, uniforms, int(k),
                                      float(attn_p), float(proj_p), False, bool(want_maps), bool(bf16),
                                      schedule_code(schedule))


def dense_attention(Q, K, V, mask, attn_p=0.0, want_maps=True, bf16=False, schedule="auto"):
    """Fused FullAttention.forward (module/sbm_attn.py:77-87) -> (X, None, graph(unused), attn)."""
    return SBMAttentionFunction.apply(Q, K, V, mask, None, None, None, None, None, None, None, None, 0,
                                      float(attn_p), 0.0, True, bool(want_maps), bool(bf16), schedule_code(schedule))


class _STEFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p, u):
        A = torch.ops.csa.ste_sample(p, u, 0.01, 0.99)
        ctx.save_for_backward(A)
        return A

    @staticmethod
    def backward(ctx, g):
        (A,) = ctx.saved_tensors
        return torch.ops.csa.ste_backward(A, g), None


def ste_sample(p, u=None):
    """SampleGraphSparseGraph (STE.py:8-19) on the GPU; u defaults to torch.rand (global generator)."""
    if u is None:
        u = torch.rand(p.shape, device=p.device, dtype=torch.float32)
    return _STEFunction.apply(p, u)


def ste_backward(A, g):
    return torch.ops.csa.ste_backward(A, g)


def rel_attn(*args, **kwargs):
    from .rel_ops import rel_attn as _r
    return _r(*args, **kwargs)
