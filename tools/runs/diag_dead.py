"""Round 6 diagnostic: stage times of the headline layer (B=256, N=150) with every AST padded to the same length n
(32-key tiles past n fully masked), to price a dead key tile in each attention kernel."""
import os
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

dev = torch.device("cuda", 0)
for n in [int(x) for x in os.environ.get("DIAG_NS", "150,128,96,64,150,128,96,64").split(",")]:
    bench.padded_lengths = lambda B, N, rank, n=n: torch.full((B,), n, dtype=torch.long)
    L = bench.measure_layer(1, 0, dev, 10, 3, 256, 150, 64, 10, False, "fp32", False, "torch", padded=True)
    print(n, {k: round(v, 4) for k, v in L["stage_ms"].items()}, flush=True)
