"""Dev tool: build an experimental copy of the library with extra -D flags (lib/libcsa_<name>.so).

usage: python tools/build_variant.py NAME -DFLAG [...]; load it with CSA_HIP_LIB=<path>. Only the
HIP sources are recompiled with the flags; the host objects of the last regular build are reused."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
from csa_amd import build as B  # noqa: E402

if __name__ == "__main__":
    name, defs = sys.argv[1], sys.argv[2:]
    B.build(verbose=False)
    lib = os.path.dirname(B.OUT)
    objs, procs = [], []
    for s in B.SOURCES:
        o = os.path.join(lib, os.path.basename(s) + ".o")
        if s.endswith(".hip"):
            o = os.path.join(lib, f"{name}_{os.path.basename(s)}.o")
            cmd = [B.HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "-fPIC", *defs,
                   f'-DCSA_SOURCE_HASH="variant-{name}"', "-o", o, os.path.join(B.CSRC, s)]
            procs.append(subprocess.Popen(cmd))
        objs.append(o)
    assert all(p.wait() == 0 for p in procs)
    out = os.path.join(lib, f"libcsa_{name}.so")
    subprocess.check_call([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs)
    print("built", out)
