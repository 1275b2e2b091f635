"""torch custom ops (``torch.ops.csa.*``) over the C ABI, plus their autograd wrappers.

Layering (top to bottom):
  csa_amd.module.*            drop-in nn.Modules with the reference's names/signatures/state_dict keys
  SBMAttentionFunction etc.   torch.autograd.Function: saves what the backward needs
  torch.ops.csa.*             hot-path ops (SBM, STE, CSE): schemas + fake implementations defined here,
                              GPU implementations in the C++ shim libcsa_torch.so (csrc/csa_torch.cpp,
                              TORCH_LIBRARY_IMPL): validate, allocate outputs/state/workspace with the torch
                              caching allocator, pass raw pointers + the current HIP stream to ...
  libcsa_hip.so               extern "C" entry points (include/csa_hip.h) -> gfx950 kernels

There is no CPU path: every op raises on a non-CUDA tensor or when the libraries are absent.
"""
import ctypes
import os
from typing import List, Optional, Tuple

import torch

from . import _lib
from ._lib import CSA_FLAG_DENSE, CSA_FLAG_FWD_ONLY, SCHEDULES, lib

__all__ = ["sbm_attention", "dense_attention", "ste_sample", "ste_backward", "rel_attn", "SBMAttentionFunction"]

SHIM_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "libcsa_torch.so")

# Schemas of the hot-path ops (implemented by csrc/csa_torch.cpp). Defined here so the package imports and
# traces (fake tensors) without the GPU libraries; the implementations register when the shim loads.
_SCHEMAS = {
    "sbm_fwd": "(Tensor Q, Tensor K, Tensor V, Tensor? mask, Tensor? cluster_w, Tensor[] proj_w, Tensor[] proj_b, "
               "Tensor? uniforms, int k, int seed, int offset, float attn_p, float proj_p, bool dense, "
               "bool bf16=False, bool fwd_only=False) -> (Tensor, Tensor, Tensor)",
    "sbm_maps": "(Tensor Q, Tensor K, Tensor V, Tensor? mask, Tensor state, int k, bool dense) -> (Tensor, Tensor)",
    "sbm_bwd": "(Tensor Q, Tensor K, Tensor V, Tensor? mask, Tensor? cluster_w, Tensor[] proj_w, Tensor[] proj_b, "
               "int k, float attn_p, float proj_p, int seed, int offset, bool dense, Tensor state, Tensor X, "
               "Tensor dX, Tensor? dsparsity, Tensor? dgraph, bool bf16=False, bool packed=False, "
               "Tensor? dattn=None, int schedule=0) -> Tensor[]",
    "ste_sample": "(Tensor p, Tensor u, float lo, float hi) -> Tensor",
    "ste_backward": "(Tensor A, Tensor g) -> Tensor",
    "rel_attn_fwd": "(Tensor q, Tensor k, Tensor v, Tensor lq, Tensor lk, Tensor rel, Tensor mask, int group, "
                    "bool bf16=False) -> Tensor[]",
    "rel_attn_bwd": "(Tensor q, Tensor k, Tensor v, Tensor lq, Tensor lk, Tensor rel, Tensor mask, int group, "
                    "Tensor out, Tensor lse, Tensor state, Tensor dout, bool bf16=False, bool packed=False, "
                    "int schedule=0) -> Tensor[]",
}
for _name, _schema in _SCHEMAS.items():
    torch.library.define("csa::" + _name, _schema)

_SHIM = None


def shim():
    """Load (once) the C ABI library (RTLD_GLOBAL) and then the C++ op shim, which registers the GPU
    implementations of _SCHEMAS; raises CsaError when either is absent (no fallback)."""
    global _SHIM
    if _SHIM is None:
        lib()
        if not os.path.exists(SHIM_PATH):
            raise _lib.CsaError(f"libcsa_torch.so not found at {SHIM_PATH}: run `python __graft_entry__.py build`")
        torch.ops.load_library(SHIM_PATH)
        S = ctypes.CDLL(SHIM_PATH)
        S.csa_torch_set_stage_profiler.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        S.csa_torch_set_stage_profiler.restype = None
        S.csa_torch_set_rel_profiler.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        S.csa_torch_set_rel_profiler.restype = None
        _SHIM = S
    return _SHIM


if os.path.exists(_lib.LIB_PATH) and os.path.exists(SHIM_PATH):
    shim()  # register the implementations at import (no GPU is touched); otherwise on first use


# Optional per-stage event profiling (bench.py): csa_prof structs owned by the caller (kept alive here).
_PROF = {"fwd": None, "bwd": None, "rel_fwd": None, "rel_bwd": None}


def set_stage_profiler(fwd_prof=None, bwd_prof=None):
    """Install caller-owned csa_prof structs (ctypes) that the next sbm fwd/bwd calls record into."""
    _PROF["fwd"], _PROF["bwd"] = fwd_prof, bwd_prof
    shim().csa_torch_set_stage_profiler(None if fwd_prof is None else ctypes.addressof(fwd_prof),
                                        None if bwd_prof is None else ctypes.addressof(bwd_prof))


def set_rel_profiler(fwd_prof=None, bwd_prof=None):
    """The same for the CSE relation attention's stages (ABI v9, _lib.REL_STAGES slots)."""
    _PROF["rel_fwd"], _PROF["rel_bwd"] = fwd_prof, bwd_prof
    shim().csa_torch_set_rel_profiler(None if fwd_prof is None else ctypes.addressof(fwd_prof),
                                      None if bwd_prof is None else ctypes.addressof(bwd_prof))


def _stream(device):
    """The current HIP stream of `device` as a ctypes handle (the Python-registered glue / generator ops)."""
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _require_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError("csa ops run only on the GPU (HIP); got a tensor on " + str(t.device))


# ---------------------------------------------------------------------------------------
# Backward schedule (ABI v5: the side lane is created and owned by the C++ shim, not the library)
# ---------------------------------------------------------------------------------------
# debugging override of every module's bwd_schedule: CSA_BWD_CONCUR=0 -> in_order, 1 -> concurrent
_SCHED_OVERRIDE = {"0": "in_order", "1": "concurrent"}.get(os.environ.get("CSA_BWD_CONCUR", ""))


def schedule_code(schedule: str) -> int:
    """"auto" | "in_order" | "concurrent" -> CSA_SCHED_* (CSA_BWD_CONCUR overrides "auto" only: an explicit
    schedule passed by the caller wins)."""
    s = (_SCHED_OVERRIDE or schedule) if schedule == "auto" else schedule
    if s not in SCHEDULES:
        raise ValueError(f"bwd schedule must be one of {sorted(SCHEDULES)}, got {schedule!r}")
    return SCHEDULES[s]


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


# ---------------------------------------------------------------------------------------
# fake (meta) implementations of the C++ ops
# ---------------------------------------------------------------------------------------
def _state_bytes(B, H, N, M, d, k, dense, fwd_only=False):
    return lib().csa_sbm_state_bytes(B, H, N, M, d, k, (CSA_FLAG_DENSE if dense else 0) |
                                     (CSA_FLAG_FWD_ONLY if fwd_only else 0))


@torch.library.register_fake("csa::sbm_fwd")
def _(Q, K, V, mask, cluster_w, proj_w, proj_b, uniforms, k, seed, offset, attn_p, proj_p, dense, bf16=False,
      fwd_only=False):
    B, H, N, d = Q.shape
    return (Q.new_empty(B, N, H, d).transpose(1, 2), Q.new_empty(0 if dense else H),
            Q.new_empty(_state_bytes(B, H, N, K.shape[2], d, k, dense, fwd_only), dtype=torch.uint8))


@torch.library.register_fake("csa::sbm_maps")
def _(Q, K, V, mask, state, k, dense):
    B, H, N, d = Q.shape
    g = Q.new_empty(B, H, N, K.shape[2])
    return g, torch.empty_like(g)


@torch.library.register_fake("csa::sbm_bwd")
def _(Q, K, V, mask, cluster_w, proj_w, proj_b, k, attn_p, proj_p, seed, offset, dense, state, X, dX, dsparsity,
      dgraph, bf16=False, packed=False, dattn=None, schedule=0):
    B, H, N, d = Q.shape
    outs = [Q.new_empty(B, N, 3, H, d)] if packed else [torch.empty_like(Q), torch.empty_like(K), torch.empty_like(V)]
    if not dense:
        outs.append(torch.empty_like(cluster_w))
        for i in range(3):
            outs += [torch.empty_like(proj_w[i]), torch.empty_like(proj_b[i])]
    return outs


@torch.library.register_fake("csa::ste_sample")
def _(p, u, lo, hi):
    return torch.empty_like(p)


@torch.library.register_fake("csa::ste_backward")
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
                want_maps, bf16=False, schedule=0, fwd_only=False):
        shim()
        seed = _draw_seed()
        pw = [] if dense else [w0, w1, w2]
        pb = [] if dense else [b0, b1, b2]
        # fwd_only (decided by the caller before apply: grad mode is always off in here): no backward will run
        # (eval under no_grad / inference_mode, or nothing requires grad), so the forward skips the activations
        # only the backward reads
        X, sp, state = torch.ops.csa.sbm_fwd(Q, K, V, mask, None if dense else cluster_w, pw, pb, uniforms, k, seed, 0,
                                            attn_p, proj_p, dense, bf16, fwd_only)
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
            return (dQ, dK, dV) + (None,) * 17
        dC, dw0, db0, dw1, db1, dw2, db2 = g[3:]
        return dQ, dK, dV, None, dC, dw0, db0, dw1, db1, dw2, db2, None, None, None, None, None, None, None, None, None


def _fwd_only(*inputs):
    """True when no backward can run through this call: grad mode off (no_grad / inference_mode) or no
    input requiring grad. Evaluated before Function.apply, where grad mode is still the caller's."""
    return not (torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in inputs))


def sbm_attention(Q, K, V, mask, cluster_w, proj, k, uniforms=None, attn_p=0.0, proj_p=0.0, want_maps=True,
                  bf16=False, schedule="auto"):
    """Fused SBMAttention.forward (module/sbm_attn.py:32-66) -> (X, sparsity, graph, attn).

    proj: [w0, b0, w1, b1, w2, b2] (proj.0/.3/.6). uniforms: optional (B,H,N,M) host-supplied draws
    (bit-exact parity mode); otherwise in-kernel Philox. graph/attn are None when want_maps=False.
    bf16: bf16-MFMA attention contractions (the maps, if requested, are still computed in fp32).
    schedule: the backward's "auto" | "in_order" | "concurrent" (CSA_SCHED_*; bitwise-identical results)."""
    w0, b0, w1, b1, w2, b2 = proj
    fwd_only = _fwd_only(Q, K, V, cluster_w, w0, b0, w1, b1, w2, b2)
    return SBMAttentionFunction.apply(Q, K, V, mask, cluster_w, w0, b0, w1, b1, w2, b2, uniforms, int(k),
                                      float(attn_p), float(proj_p), False, bool(want_maps), bool(bf16),
                                      schedule_code(schedule), fwd_only)


def dense_attention(Q, K, V, mask, attn_p=0.0, want_maps=True, bf16=False, schedule="auto"):
    """Fused FullAttention.forward (module/sbm_attn.py:77-87) -> (X, None, graph(unused), attn)."""
    return SBMAttentionFunction.apply(Q, K, V, mask, None, None, None, None, None, None, None, None, 0,
                                      float(attn_p), 0.0, True, bool(want_maps), bool(bf16), schedule_code(schedule),
                                      _fwd_only(Q, K, V))


class _STEFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p, u):
        shim()
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
    shim()
    return torch.ops.csa.ste_backward(A, g)


def rel_attn(*args, **kwargs):
    from .rel_ops import rel_attn as _r
    return _r(*args, **kwargs)
