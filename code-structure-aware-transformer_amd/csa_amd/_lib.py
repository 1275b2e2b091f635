"""ctypes binding of libcsa_hip.so (include/csa_hip.h). No torch types cross this boundary.

The shared library is built in-tree (csa_amd/build.py -> csa_amd/lib/libcsa_hip.so) and loaded
after torch so that it binds to the HIP runtime torch already loaded (same SONAME
libamdhip64.so.7). There is deliberately no fallback: if the library is missing, every op
raises.
"""
import contextlib
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CSA_HIP_LIB", os.path.join(_HERE, "lib", "libcsa_hip.so"))

CSA_ABI_VERSION = 9
CSA_FLAG_DENSE = 1
CSA_FLAG_FWD_ONLY = 2
CSA_FLAG_BF16_WS = 4  # ABI v8: bf16-mode backward workspace (no fp32 tile handoff)
CSA_SCHED_AUTO, CSA_SCHED_IN_ORDER, CSA_SCHED_CONCURRENT = 0, 1, 2
SCHEDULES = {"auto": CSA_SCHED_AUTO, "in_order": CSA_SCHED_IN_ORDER, "concurrent": CSA_SCHED_CONCURRENT}
CSA_DTYPE_F32, CSA_DTYPE_BF16 = 0, 1
STATUS = {0: "CSA_OK", 1: "CSA_INVALID_ARG", 2: "CSA_UNSUPPORTED_SHAPE", 3: "CSA_LAUNCH_FAILED"}

i64, u64, u32, f32, vp = ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_float, ctypes.c_void_p


CSA_STAGE_COUNT = 9
STAGES = {"prep": 0, "proj_fwd": 1, "attn_fwd": 2, "attn_bwd_q": 3, "attn_bwd_kv": 4, "proj_bwd": 5, "reduce": 6,
          "proj_bwd_k": 7, "attn_rowprep": 8}
# ABI v9: CSE relation-attention stages (csa_rel_attn_args.prof / csa_rel_attn_bwd_args.prof) and their kernels
REL_STAGES = {"logits": 0, "fwd": 1, "qstat": 2, "bwd_k": 3, "bwd_q": 4, "lgrad": 5}
REL_KERNEL_OF_STAGE = {"logits": "k_rel_logits", "fwd": "k_rel_fwd_f", "qstat": "k_rel_qstat", "bwd_k": "k_rel_bwd_kh",
                       "bwd_q": "k_rel_bwd_qg", "lgrad": "k_rel_lgrad"}
KERNEL_OF_STAGE = {"proj_fwd": "k_proj_fwd", "attn_fwd": "k_attn_fwd", "attn_bwd_q": "k_attn_bwd_qg",
                   "attn_bwd_kv": "k_attn_bwd_kv", "proj_bwd": "k_proj_bwd", "proj_bwd_k": "k_proj_bwd",
                   "attn_rowprep": "k_attn_rowprep"}


def on_device(device):
    """Makes `device` the calling thread's current device for one library call. The library runs on the device
    of the stream it is given, but PyTorch's default stream is the null handle, which HIP resolves to the
    thread's current device: a tensor on cuda:1 called while cuda:0 is current would otherwise launch on 0."""
    import torch
    if device.type != "cuda" or device.index is None or device.index == torch.cuda.current_device():
        return contextlib.nullcontext()
    return torch.cuda.device(device)


class CsaProf(ctypes.Structure):
    _fields_ = [("start", vp * CSA_STAGE_COUNT), ("stop", vp * CSA_STAGE_COUNT)]


class SbmFwdArgs(ctypes.Structure):
    _fields_ = [
        ("B", i64), ("H", i64), ("N", i64), ("M", i64), ("d", i64), ("k", i64),
        ("Q", vp), ("q_sb", i64), ("q_sh", i64), ("q_sn", i64),
        ("K", vp), ("k_sb", i64), ("k_sh", i64), ("k_sn", i64),
        ("V", vp), ("v_sb", i64), ("v_sh", i64), ("v_sn", i64),
        ("key_mask", vp), ("mask_sb", i64),
        ("cluster_w", vp),
        ("proj_w", vp * 3), ("proj_b", vp * 3),
        ("uniforms", vp),
        ("seed", u64), ("offset", u64),
        ("attn_dropout", f32), ("proj_dropout", f32),
        ("flags", u32), ("dtype", u32),
        ("X", vp), ("sparsity", vp), ("state", vp),
        ("prof", ctypes.POINTER(CsaProf)),
        ("x_sb", i64), ("x_sh", i64), ("x_sn", i64),  # ABI v3: 0,0,0 = (B,H,N,d) contiguous
    ]


class SbmBwdArgs(ctypes.Structure):
    _fields_ = [
        ("fwd", ctypes.POINTER(SbmFwdArgs)),
        ("dX", vp), ("dsparsity", vp), ("dgraph", vp),
        ("dQ", vp), ("dK", vp), ("dV", vp),
        ("dcluster_w", vp), ("dproj_w", vp * 3), ("dproj_b", vp * 3),
        ("workspace", vp),
        ("prof", ctypes.POINTER(CsaProf)),
        ("dx_sb", i64), ("dx_sh", i64), ("dx_sn", i64), ("dq_sb", i64), ("dq_sh", i64), ("dq_sn", i64),
        ("dk_sb", i64), ("dk_sh", i64), ("dk_sn", i64), ("dv_sb", i64), ("dv_sh", i64), ("dv_sn", i64),
        ("dattn", vp),  # ABI v4
        ("schedule", u32), ("side_stream", vp), ("side_fork", vp), ("side_join", vp),  # ABI v5
    ]


class RelAttnArgs(ctypes.Structure):
    _fields_ = [
        ("B", i64), ("H", i64), ("N", i64), ("L", i64), ("d", i64),
        ("q", vp), ("q_sb", i64), ("q_sh", i64), ("q_sn", i64),
        ("k", vp), ("k_sb", i64), ("k_sh", i64), ("k_sn", i64),
        ("v", vp), ("v_sb", i64), ("v_sh", i64), ("v_sn", i64),
        ("lq", vp), ("lk", vp),
        ("rel", vp), ("rel_sb", i64), ("rel_sh", i64),
        ("mask", vp), ("mask_sb", i64), ("mask_sh", i64),
        ("rel_head_group", i64), ("dtype", u32),
        ("out", vp), ("row_stats", vp),
        ("state", vp),
        ("o_sb", i64), ("o_sh", i64), ("o_sn", i64),  # ABI v3: 0,0,0 = contiguous
        ("prof", ctypes.POINTER(CsaProf)),  # ABI v9
    ]


class RelAttnBwdArgs(ctypes.Structure):
    _fields_ = [
        ("fwd", ctypes.POINTER(RelAttnArgs)),
        ("dout", vp),
        ("dq", vp), ("dk", vp), ("dv", vp),
        ("dlq", vp), ("dlk", vp),
        ("workspace", vp),
        ("do_sb", i64), ("do_sh", i64), ("do_sn", i64), ("dq_sb", i64), ("dq_sh", i64), ("dq_sn", i64),
        ("dk_sb", i64), ("dk_sh", i64), ("dk_sn", i64), ("dv_sb", i64), ("dv_sh", i64), ("dv_sn", i64),
        ("schedule", u32), ("side_stream", vp), ("side_fork", vp), ("side_join", vp),  # ABI v5
        ("prof", ctypes.POINTER(CsaProf)),  # ABI v9
    ]


class AdamwArgs(ctypes.Structure):
    _fields_ = [
        ("tensors", vp), ("chunk_tensor", vp), ("chunk_start", vp),
        ("ntensors", i64), ("nchunks", i64),
        ("beta1", f32), ("beta2", f32), ("one_minus_beta1", f32), ("one_minus_beta2", f32),
        ("eps", f32), ("step_size", f32), ("decay", f32),
        ("grad_scale", vp), ("found_inf", vp),
    ]


ADAMW_CHUNK = 4096  # CSA_ADAMW_CHUNK


class CsaError(RuntimeError):
    pass


_lib = None


def lib():
    """Load (once) and return the library; raises CsaError when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise CsaError(f"libcsa_hip.so not found at {LIB_PATH}: run `python __graft_entry__.py build` "
                       "(there is no CPU fallback for the hot path)")
    # RTLD_GLOBAL: the C++ op shim (libcsa_torch.so, csa_amd.ops) resolves its csa_* symbols against THIS
    # library at its own load time, so both always use one instance (also for a CSA_HIP_LIB variant build)
    L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    L.csa_abi_version.restype = ctypes.c_int
    L.csa_source_hash.restype = ctypes.c_char_p
    L.csa_status_str.restype = ctypes.c_char_p
    L.csa_status_str.argtypes = [ctypes.c_int]
    L.csa_last_error_str.restype = ctypes.c_char_p
    L.csa_sbm_supported.restype = ctypes.c_int
    L.csa_sbm_supported.argtypes = [i64, i64, u32]
    for fn in ("csa_sbm_state_bytes", "csa_sbm_bwd_workspace_bytes"):
        getattr(L, fn).restype = ctypes.c_size_t
        getattr(L, fn).argtypes = [i64] * 6 + [u32]
    for fn in ("csa_rel_attn_state_bytes", "csa_rel_attn_bwd_workspace_bytes"):
        getattr(L, fn).restype = ctypes.c_size_t
        getattr(L, fn).argtypes = [i64] * 5
    L.csa_sbm_fwd.restype = ctypes.c_int
    L.csa_sbm_fwd.argtypes = [ctypes.POINTER(SbmFwdArgs), vp]
    L.csa_sbm_maps.restype = ctypes.c_int
    L.csa_sbm_maps.argtypes = [ctypes.POINTER(SbmFwdArgs), vp, vp, vp]
    L.csa_sbm_bwd.restype = ctypes.c_int
    L.csa_sbm_bwd.argtypes = [ctypes.POINTER(SbmBwdArgs), vp]
    L.csa_dense_attn_fwd.restype = ctypes.c_int
    L.csa_dense_attn_fwd.argtypes = [ctypes.POINTER(SbmFwdArgs), vp]
    L.csa_dense_attn_bwd.restype = ctypes.c_int
    L.csa_dense_attn_bwd.argtypes = [ctypes.POINTER(SbmBwdArgs), vp]
    L.csa_ste_sample.restype = ctypes.c_int
    L.csa_ste_sample.argtypes = [vp, vp, vp, i64, f32, f32, vp]
    L.csa_ste_backward.restype = ctypes.c_int
    L.csa_ste_backward.argtypes = [vp, vp, vp, i64, vp]
    L.csa_rel_attn_fwd.restype = ctypes.c_int
    L.csa_rel_attn_fwd.argtypes = [ctypes.POINTER(RelAttnArgs), vp]
    L.csa_rel_attn_bwd.restype = ctypes.c_int
    L.csa_rel_attn_bwd.argtypes = [ctypes.POINTER(RelAttnBwdArgs), vp]
    L.csa_gen_logsoftmax_fwd.restype = ctypes.c_int
    L.csa_gen_logsoftmax_fwd.argtypes = [vp, vp, i64, i64, f32, u64, u64, vp]
    L.csa_gen_logsoftmax_bwd.restype = ctypes.c_int
    L.csa_gen_logsoftmax_bwd.argtypes = [vp, vp, vp, i64, i64, f32, u64, u64, vp]
    L.csa_bias_grad_workspace_bytes.restype = ctypes.c_size_t
    L.csa_bias_grad_workspace_bytes.argtypes = [i64, i64]
    L.csa_bias_grad.restype = ctypes.c_int
    L.csa_bias_grad.argtypes = [vp, vp, i64, i64, ctypes.c_int, vp, vp]
    L.csa_layernorm_supported.restype = ctypes.c_int
    L.csa_layernorm_supported.argtypes = [i64]
    L.csa_layernorm_bwd_workspace_bytes.restype = ctypes.c_size_t
    L.csa_layernorm_bwd_workspace_bytes.argtypes = [i64, i64]
    L.csa_layernorm_fwd.restype = ctypes.c_int
    L.csa_layernorm_fwd.argtypes = [vp, vp, vp, vp, vp, i64, i64, f32, vp]
    L.csa_layernorm_bwd.restype = ctypes.c_int
    L.csa_layernorm_bwd.argtypes = [vp, vp, vp, vp, vp, vp, vp, i64, i64, vp, vp]
    L.csa_residual_dropout_fwd.restype = ctypes.c_int
    L.csa_residual_dropout_fwd.argtypes = [vp, vp, vp, i64, f32, u64, u64, vp]
    L.csa_residual_dropout_bwd.restype = ctypes.c_int
    L.csa_residual_dropout_bwd.argtypes = [vp, vp, i64, f32, u64, u64, vp]
    L.csa_gelu_dropout_fwd.restype = ctypes.c_int
    L.csa_gelu_dropout_fwd.argtypes = [vp, vp, i64, f32, u64, u64, vp]
    L.csa_gelu_dropout_bwd.restype = ctypes.c_int
    L.csa_gelu_dropout_bwd.argtypes = [vp, vp, vp, i64, f32, u64, u64, vp]
    L.csa_ast_relations.restype = ctypes.c_int
    L.csa_ast_relations.argtypes = [vp, vp, i64, i64, vp, vp, vp, vp, ctypes.c_int]
    L.csa_collate_relations.restype = ctypes.c_int
    L.csa_collate_relations.argtypes = [vp, vp, i64, vp, vp, vp, vp, ctypes.c_int]
    L.csa_adamw_step.restype = ctypes.c_int
    L.csa_adamw_step.argtypes = [ctypes.POINTER(AdamwArgs), vp]
    if L.csa_abi_version() != CSA_ABI_VERSION:
        raise CsaError(f"ABI mismatch: library {L.csa_abi_version()} != binding {CSA_ABI_VERSION}")
    _lib = L
    return L


def loaded_source_hash():
    """sha256 of the sources the loaded library was built from (csa_source_hash())."""
    return lib().csa_source_hash().decode()


def check(status, what):
    if status != 0:
        L = lib()
        raise CsaError(f"{what} failed: {STATUS.get(status, status)}: {L.csa_last_error_str().decode()}")


EXPORTED_SYMBOLS = (
    "csa_abi_version", "csa_source_hash", "csa_status_str", "csa_last_error_str", "csa_sbm_supported", "csa_sbm_state_bytes",
    "csa_sbm_bwd_workspace_bytes", "csa_sbm_fwd", "csa_sbm_maps", "csa_sbm_bwd", "csa_dense_attn_fwd",
    "csa_dense_attn_bwd", "csa_ste_sample",
    "csa_ste_backward", "csa_rel_attn_state_bytes", "csa_rel_attn_bwd_workspace_bytes", "csa_rel_attn_fwd", "csa_rel_attn_bwd",
    "csa_adamw_step", "csa_gen_logsoftmax_fwd", "csa_gen_logsoftmax_bwd",
    "csa_bias_grad_workspace_bytes", "csa_bias_grad", "csa_ast_relations",
    "csa_layernorm_supported", "csa_layernorm_bwd_workspace_bytes", "csa_layernorm_fwd", "csa_layernorm_bwd",
    "csa_residual_dropout_fwd", "csa_residual_dropout_bwd", "csa_gelu_dropout_fwd", "csa_gelu_dropout_bwd",
    "csa_collate_relations",
)
