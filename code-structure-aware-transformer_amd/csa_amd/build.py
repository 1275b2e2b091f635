"""Build libcsa_hip.so in-tree with hipcc for gfx950 (no torch extension toolchain involved)."""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")
OUT = os.path.join(HERE, "lib", "libcsa_hip.so")
SOURCES = ["csa_sbm.hip", "csa_rel.hip", "csa_optim.hip", "csa_gen.hip", "csa_glue.hip", "csa_host.cpp"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC", "-Wall", "-Wno-unused-result",
         "-Wno-unused-function"]


def build(force=False, verbose=True):
    srcs = [os.path.join(CSRC, s) for s in SOURCES]
    deps = srcs + [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".h"))]
    deps.append(os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "csa_hip.h"))
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in deps):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    objs = []
    procs = []
    for s in srcs:
        o = os.path.join(os.path.dirname(OUT), os.path.basename(s) + ".o")
        cmd = [HIPCC] + FLAGS[:-3] + ["-c", "-fPIC", "-Wall", "-Wno-unused-result", "-o", o, s]
        cmd = [c for c in cmd if c != "-shared"]
        procs.append((subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT), cmd))
        objs.append(o)
    for p, cmd in procs:
        out, _ = p.communicate()
        if p.returncode != 0:
            sys.stderr.write(out.decode())
            raise RuntimeError("hipcc failed: " + " ".join(cmd))
    cmd = [HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", OUT + ".tmp"] + objs
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    if verbose:
        print("built", OUT)
    return OUT


if __name__ == "__main__":
    build(force="--force" in sys.argv)
