"""Dev tool: run the CSATrans java train step (bench.py's train_step_bench) for rocprofv3 kernel stats.

usage: rocprofv3 --kernel-trace --stats -d DIR -o run -- python tools/prof_train.py [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    r = bench.train_step_bench(1, 0, torch.device("cuda:0"), steps, 3)
    print(r)
