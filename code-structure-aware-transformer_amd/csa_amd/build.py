"""Build libcsa_hip.so in-tree with hipcc for gfx950 (no torch extension toolchain involved).

The library carries the sha256 of the sources it was compiled from (csa_source_hash(), also written
next to it as libcsa_hip.so.sha256); build() recompiles whenever the tree's hash differs, so a
stale prebuilt binary is never reused, and smoke() asserts the loaded library matches the tree."""
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
OUT = os.path.join(HERE, "lib", "libcsa_hip.so")
SOURCES = ["csa_sbm.hip", "csa_rel.hip", "csa_optim.hip", "csa_gen.hip", "csa_glue.hip", "csa_host.cpp"]
# the C++ TORCH_LIBRARY shim (torch.ops.csa.* of the hot path): host code against the torch headers; its
# csa_* symbols resolve at load time to the libcsa_hip.so that csa_amd._lib loaded (RTLD_GLOBAL) first
SHIM = "csa_torch.cpp"
SHIM_OUT = os.path.join(HERE, "lib", "libcsa_torch.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wno-unused-result",
         "-Wno-unused-function"]


HEADER = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "csa_hip.h")


def _deps():
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    hdrs = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h")))
    return srcs, srcs + [os.path.join(CSRC, SHIM)] + hdrs + [HEADER]


def source_hash():
    """sha256 over (name, content) of every source and header the library is built from."""
    h = hashlib.sha256()
    for p in _deps()[1]:
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def built_hash():
    try:
        with open(OUT + ".sha256") as f:
            return f.read().strip()
    except OSError:
        return None


def shim_cmd():
    """hipcc line of libcsa_torch.so (host C++; torch's headers and HIP runtime; no kernels)."""
    import torch
    tdir = os.path.dirname(torch.__file__)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    return [HIPCC, "-O2", "-std=c++17", "-fPIC", "-shared", f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-DUSE_ROCM",
            "-I" + os.path.join(tdir, "include"), "-I" + os.path.join(tdir, "include", "torch", "csrc", "api", "include"),
            os.path.join(CSRC, SHIM), "-L" + os.path.join(tdir, "lib"), "-lc10", "-lc10_hip", "-ltorch", "-ltorch_cpu",
            "-ltorch_hip", "-o", SHIM_OUT + ".tmp"]


def shim_stamp(digest):
    """What libcsa_torch.so depends on: the sources, and the torch it is compiled and linked against (its
    headers, libraries and C++ ABI flag), so a torch upgrade rebuilds the shim even when csrc/ is unchanged."""
    import torch
    return f"{digest} torch={torch.__version__} cxx11abi={int(torch._C._GLIBCXX_USE_CXX11_ABI)}"


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def build(force=False, verbose=True):
    srcs, deps = _deps()
    digest = source_hash()
    stamp = shim_stamp(digest)
    lib_ok = not force and os.path.exists(OUT) and built_hash() == digest
    shim_ok = not force and os.path.exists(SHIM_OUT) and _read(SHIM_OUT + ".stamp") == stamp
    if lib_ok and shim_ok:
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    objs = []
    procs = []
    if not lib_ok:
        for s in srcs:
            o = os.path.join(os.path.dirname(OUT), os.path.basename(s) + ".o")
            cmd = [HIPCC] + FLAGS[:-3] + ["-c", "-fPIC", "-Wall", "-Wno-unused-result",
                                          f'-DCSA_SOURCE_HASH="{digest}"', "-o", o, s]
            cmd = [c for c in cmd if c != "-shared"]
            procs.append((subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT), cmd))
            objs.append(o)
    if not shim_ok:
        procs.append((subprocess.Popen(shim_cmd(), stdout=subprocess.PIPE, stderr=subprocess.STDOUT), shim_cmd()))
    for p, cmd in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out.decode())
            raise RuntimeError("hipcc failed: " + " ".join(cmd))
    if not shim_ok:
        os.replace(SHIM_OUT + ".tmp", SHIM_OUT)
        with open(SHIM_OUT + ".stamp", "w") as f:
            f.write(stamp + "\n")
    if not lib_ok:
        cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp"] + objs
        subprocess.check_call(cmd)
        os.replace(OUT + ".tmp", OUT)
        with open(OUT + ".sha256", "w") as f:
            f.write(digest + "\n")
    if verbose:
        print("built", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
