"""Dev tool: is the headline layer step GPU-bound? Times the host side of one SBM layer fwd+bwd step (enqueue only,
no synchronisation) against the synchronised wall time per step, same module / inputs as bench.py's headline.

usage (GPU box): python tools/cpu_overhead.py [steps]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))

import torch  # noqa: E402

from csa_amd.module.sbm_attn import SBMAttention  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
dev = torch.device("cuda:0")
B, H, N, d, k = 256, 8, 150, 64, 10
cfg = {"attention_dropout": 0.2, "head_dim": d, "num_head": H, "num_clusters": [k], "return_maps": False,
       "attn_precision": "fp32"}
torch.manual_seed(1234)
mod = SBMAttention(cfg, 0).to(dev)
mod.train(True)
Q, K, V = (torch.randn(B, H, N, d, device=dev).requires_grad_(True) for _ in range(3))
mask = torch.zeros(B, N, device=dev)
dX = torch.randn(B, H, N, d, device=dev)
dsp = torch.full((H,), 3.125e-4, device=dev)


def step():
    for t in (Q, K, V):
        t.grad = None
    for p in mod.parameters():
        p.grad = None
    X, sp, _, _ = mod(Q, K, V, mask)
    torch.autograd.backward([X, sp], [dX, dsp])


for _ in range(10):
    step()
torch.cuda.synchronize()
# host time per step while the device is busy: enqueue `steps` steps back to back, time only the host calls
t0 = time.perf_counter()
host = []
for _ in range(steps):
    a = time.perf_counter()
    step()
    host.append(time.perf_counter() - a)
t_enq = time.perf_counter() - t0
torch.cuda.synchronize()
t_wall = time.perf_counter() - t0
host.sort()
print(f"host per step: median {1e3 * host[len(host) // 2]:.3f} ms, mean {1e3 * t_enq / steps:.3f} ms; "
      f"wall per step {1e3 * t_wall / steps:.3f} ms -> "
      f"{'GPU-bound' if t_enq < 0.8 * t_wall else 'host-bound or close'} "
      f"(host/wall {t_enq / t_wall:.2f})")
