"""Dev tool: build the library from the HIP sources of an earlier git revision (lib/libcsa_<name>.so) for a
same-box A/B against the working tree. The host objects of the last regular build are reused, so the
revision must have the same C ABI (csa_hip.h) as the tree.

usage: python tools/build_rev.py REV NAME [-DFLAG ...]; load it with CSA_HIP_LIB=<path>."""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
from csa_amd import build as B  # noqa: E402

if __name__ == "__main__":
    rev, name, defs = sys.argv[1], sys.argv[2], sys.argv[3:]
    B.build(verbose=False)
    lib = os.path.dirname(B.OUT)
    with tempfile.TemporaryDirectory() as tmp:
        arch = subprocess.run(["git", "-C", ROOT, "archive", rev, "code-structure-aware-transformer_amd/csrc",
                               "include"], check=True, capture_output=True).stdout
        subprocess.run(["tar", "-x", "-C", tmp], input=arch, check=True)
        csrc = os.path.join(tmp, "code-structure-aware-transformer_amd", "csrc")
        objs, procs = [], []
        for s in B.SOURCES:
            if s.endswith(".hip"):
                o = os.path.join(lib, f"{name}_{s}.o")
                cmd = [B.HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "-fPIC", *defs,
                       f'-DCSA_SOURCE_HASH="rev-{rev}"', "-o", o, os.path.join(csrc, s)]
                procs.append(subprocess.Popen(cmd))
            else:
                o = os.path.join(lib, os.path.basename(s) + ".o")
            objs.append(o)
        assert all(p.wait() == 0 for p in procs)
    out = os.path.join(lib, f"libcsa_{name}.so")
    subprocess.check_call([B.HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", out] + objs)
    for o in objs:
        if os.path.basename(o).startswith(name + "_"):
            os.remove(o)
    print("built", out)
