"""CPU-side checks of the C-ABI library: it loads, exports every symbol include/csa_hip.h declares,
and its host-side queries/validation behave (no GPU compute is launched)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "csa_hip.h")).read()
    return sorted(set(re.findall(r"\b(csa_[a-z_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    from csa_amd import _lib
    L = _lib.lib()
    syms = declared_symbols()
    assert len(syms) >= 14
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib.EXPORTED_SYMBOLS)


def test_abi_version_and_status_strings():
    from csa_amd import _lib
    L = _lib.lib()
    assert L.csa_abi_version() == _lib.CSA_ABI_VERSION
    assert L.csa_status_str(0) == b"CSA_OK"
    assert L.csa_status_str(2) == b"CSA_UNSUPPORTED_SHAPE"


def test_supported_shapes():
    from csa_amd import _lib
    L = _lib.lib()
    assert L.csa_sbm_supported(64, 10, 0) and L.csa_sbm_supported(96, 10, 0)
    assert L.csa_sbm_supported(64, 0, _lib.CSA_FLAG_DENSE)
    assert not L.csa_sbm_supported(48, 10, 0)
    assert L.csa_sbm_supported(64, 128, 0) and not L.csa_sbm_supported(64, 129, 0)
    assert not L.csa_sbm_supported(96, 33, 0)


def test_state_and_workspace_sizes_monotone():
    from csa_amd import _lib
    L = _lib.lib()
    a = L.csa_sbm_state_bytes(2, 8, 150, 150, 64, 10, 0)
    b = L.csa_sbm_state_bytes(4, 8, 150, 150, 64, 10, 0)
    assert 0 < a < b
    assert L.csa_sbm_bwd_workspace_bytes(256, 8, 150, 150, 64, 10, 0) > 0
    # CSA_FLAG_FWD_ONLY drops exactly the projection MLP's activation blocks (B H (NQB + NKB) 32-row items of
    # h1 | h2 | po | hat: (3 d + 32) x 32 fp32 each)
    f = L.csa_sbm_state_bytes(4, 8, 150, 150, 64, 10, _lib.CSA_FLAG_FWD_ONLY)
    assert b - f == 4 * 8 * 10 * (3 * 64 + 32) * 32 * 4
    # the backward workspace holds the ds / G tiles (dense: ds only) and the per-row constants
    dense = _lib.CSA_FLAG_DENSE
    assert L.csa_sbm_bwd_workspace_bytes(4, 8, 150, 150, 64, 0, dense) >= 4 * 8 * 25 * 1024 * 4 + 4 * 8 * 160 * 16
    # ABI v8: a bf16-mode backward recomputes on the query side: its workspace has no fp32 tile handoff (two
    # (B,H,NQB,NKB,32,32) planes with clusters, one without); the state is unaffected
    bf = _lib.CSA_FLAG_BF16_WS
    for (n, k, fl, planes) in ((1024, 16, 0, 2), (150, 10, 0, 2), (150, 0, dense, 1)):
        full = L.csa_sbm_bwd_workspace_bytes(2, 8, n, n, 64, k, fl)
        slim = L.csa_sbm_bwd_workspace_bytes(2, 8, n, n, 64, k, fl | bf)
        nb = (n + 31) // 32
        assert full - slim == planes * 2 * 8 * nb * nb * 1024 * 4
        assert L.csa_sbm_state_bytes(2, 8, n, n, 64, k, fl | bf) == L.csa_sbm_state_bytes(2, 8, n, n, 64, k, fl)


def test_invalid_args_rejected_without_gpu():
    from csa_amd import _lib
    L = _lib.lib()
    a = _lib.SbmFwdArgs()  # all zero -> INVALID_ARG before any HIP call
    assert L.csa_sbm_fwd(ctypes.byref(a), None) == 1
    assert b"B, H, N, M" in L.csa_last_error_str()
    assert L.csa_sbm_fwd(None, None) == 1
    assert L.csa_ste_sample(None, None, None, 4, 0.01, 0.99, None) == 1


def test_ops_refuse_cpu_tensors():
    import torch
    import csa_amd.ops  # noqa: F401
    x = torch.zeros(4)
    with pytest.raises(RuntimeError):
        torch.ops.csa.ste_sample(x, x, 0.01, 0.99)


def test_adamw_step_validates_without_gpu():
    from csa_amd import _lib
    L = _lib.lib()
    assert L.csa_adamw_step(None, None) == 1
    a = _lib.AdamwArgs(nchunks=0, beta1=0.9, beta2=0.999)  # nothing to update: OK, no launch
    assert L.csa_adamw_step(ctypes.byref(a), None) == 0
    a = _lib.AdamwArgs(nchunks=3, ntensors=1, beta1=0.9, beta2=0.999)  # null tables
    assert L.csa_adamw_step(ctypes.byref(a), None) == 1
    assert b"null tensor table" in L.csa_last_error_str()


def test_torch_shim_registers_gpu_implementations():
    """The C++ TORCH_LIBRARY_IMPL shim (csrc/csa_torch.cpp, libcsa_torch.so) is loaded by csa_amd.ops and
    registers a CUDA (HIP) kernel for every hot-path op schema; there is no CPU kernel (no fallback)."""
    import torch
    import csa_amd.ops as ops
    assert ops._SHIM is not None and os.path.exists(ops.SHIM_PATH)
    for name in ops._SCHEMAS:
        assert torch._C._dispatch_has_kernel_for_dispatch_key("csa::" + name, "CUDA"), name
        assert not torch._C._dispatch_has_kernel_for_dispatch_key("csa::" + name, "CPU"), name


def test_tuned_gemm_table_is_well_formed():
    """csa_amd/gemm_tuned_gfx950.csv (tools/tune_gemms.py, loaded by csa_amd.train.use_tuned_gemms): TunableOp's
    CSV with validator rows for gfx950 and one fp32 GEMM solution per shape of the java train step."""
    import csv

    from csa_amd.train import GEMM_TABLE
    rows = list(csv.reader(open(GEMM_TABLE)))
    val = {r[1]: r[2] for r in rows if r[0] == "Validator"}
    assert val["GCN_ARCH_NAME"].startswith("gfx950") and "PT_VERSION" in val
    ent = [r for r in rows if r[0] != "Validator"]
    assert len(ent) >= 30 and all(r[0].startswith("Gemm") and "float" in r[0] for r in ent)
    assert len({(r[0], r[1]) for r in ent}) == len(ent)
    # the 9600-row (64 ASTs x 150 nodes) encoder shapes of the train step are covered
    assert any("_9600_" in r[1] for r in ent)


def test_every_shim_op_guards_its_tensors_device():
    """The C++ op shim resolves PyTorch's current stream, whose default is the null handle; the library maps a
    null stream to the calling thread's current device, so every registered op must make its tensors' device
    current first (at::OptionalDeviceGuard), as codegen'd ATen ops do."""
    src = open(os.path.join(ROOT, "code-structure-aware-transformer_amd", "csrc", "csa_torch.cpp")).read()
    ops = re.findall(r'm\.impl\("(\w+)", &(\w+)\)', src)
    assert len(ops) >= 7
    for name, fn in ops:
        body = re.search(r"\b" + fn + r"\([^;{]*\)\s*\{(.*?)\n\}", src, re.S)
        assert body, fn
        head = body.group(1).split("\n")[1]
        assert "OptionalDeviceGuard" in head, f"{name}: first statement is not a device guard: {head.strip()}"


def test_python_ops_call_the_library_on_the_tensors_device():
    """The ctypes-bound glue / generator / optimizer ops wrap each library call in _lib.on_device."""
    pkg = os.path.join(ROOT, "code-structure-aware-transformer_amd", "csa_amd")
    for f in ("glue.py", "gen_ops.py", "train.py"):
        lines = open(os.path.join(pkg, f)).read().split("\n")
        calls = [i for i, ln in enumerate(lines) if re.match(r"\s*check\((L|lib\(\))\.csa_", ln)]
        assert calls, f
        for i in calls:
            assert "with on_device(" in lines[i - 1], f"{f}:{i + 1} library call outside on_device"
