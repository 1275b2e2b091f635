"""Dev tool: csa_bias_grad timing (torch.cuda events, 200 calls) at the java train step's shapes.
usage: CSA_HIP_LIB=<lib> python tools/bench_bias_grad.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
import torch  # noqa: E402

from csa_amd.glue import bias_grad  # noqa: E402

out = {}
for rows, cols in ((9600, 512), (9600, 1536), (9600, 2048), (3136, 512), (3136, 2048), (3136, 1536)):
    dy = torch.randn(rows, cols, device="cuda")
    for _ in range(10):
        bias_grad(dy)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(200):
        bias_grad(dy)
    b.record()
    torch.cuda.synchronize()
    out[f"{rows}x{cols}"] = round(a.elapsed_time(b) / 200 * 1000, 2)
print(os.path.basename(os.environ.get("CSA_HIP_LIB", "libcsa_hip.so")), out)
