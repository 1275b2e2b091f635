"""Dev tool: run the CSATrans java train step (bench.py's train_step_bench) for rocprofv3 kernel stats.

usage: rocprofv3 --kernel-trace --stats -d DIR -o run -- python tools/prof_train.py [steps] [gemm table | default]
(the train step runs on the tuned GEMM table, csa_amd.train.use_tuned_gemms, unless "default")"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    table = sys.argv[2] if len(sys.argv) > 2 else None
    from csa_amd.train import GEMM_TABLE, use_tuned_gemms
    if table != "default":
        print("tuned GEMM shapes:", use_tuned_gemms(path=table or GEMM_TABLE), flush=True)
    if os.environ.get("CSA_SDP") == "math":  # A/B: the decoder's SDPA on the math backend
        torch.backends.cuda.enable_flash_sdp(False)
        torch.backends.cuda.enable_mem_efficient_sdp(False)
    r = bench.train_step_bench(1, 0, torch.device("cuda:0"), steps, 3)
    print(r)
