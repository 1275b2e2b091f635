"""CSE relation attention alone (the java train step's shape: B=64 per GPU, H=8, N=L=150, d_k=64,
compact planes): fwd+bwd timing with torch.cuda events; run under rocprofv3 --kernel-trace --stats
for the per-kernel split. usage: python tools/cse_bench.py [B] [steps] [auto|in_order|concurrent] Algorithmic work per AST: 3*H*8*N^2*d (276.5 MFLOP)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from csa_amd import rel_ops  # noqa: E402
from csa_amd.data import synthetic_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
schedule = sys.argv[3] if len(sys.argv) > 3 else "auto"  # the backward's schedule (rel_ops.rel_attn)
H, N, d, L = 8, 150, 64, 150
sb = synthetic_batch(B, N, seed=3)
dev = torch.device("cuda")
rel = torch.from_numpy(np.stack([sb["L"], sb["T"]], 1)).to(dev)
mask = torch.from_numpy(np.stack([sb["L_mask"], sb["T_mask"]], 1).astype(np.uint8)).to(dev)
q, k, v, dO = (torch.randn(B, H, N, d, device=dev) for _ in range(4))
lq, lk = (torch.randn(H, L, d, device=dev) for _ in range(2))
for t in (q, k, v, lq, lk):
    t.requires_grad_(True)


def step():
    # fresh gradients each step, as in the train step (zero_grad(set_to_none=True)): no .grad accumulation adds
    for t in (q, k, v, lq, lk):
        t.grad = None
    o = rel_ops.rel_attn(q, k, v, lq, lk, rel, mask, schedule=schedule)
    o.backward(dO)


for _ in range(3):
    step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    step()
torch.cuda.synchronize()
ms = (time.perf_counter() - t0) * 1000 / steps
fl = 3 * H * 8 * N * N * d * B
print(f"CSE rel_attn fwd+bwd B={B} ({schedule}): {ms:.3f} ms/layer, {fl / ms / 1e9:.1f} TF/s ({fl / ms / 1e9 / 157.3:.1%} of fp32 MFMA)")
