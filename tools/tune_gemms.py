"""Dev tool (GPU): build csa_amd/gemm_tuned_gfx950.csv, the per-shape GEMM table that
csa_amd.train.use_tuned_gemms loads. Runs the config/java.py train step (64 ASTs per GPU) and the
config/python.py protocol legs (B=32) with PyTorch TunableOp searching every stock fp32 GEMM shape
they issue; the table is written to OUT when the process exits (TunableOp's own writer).

usage: python tools/tune_gemms.py OUT.csv [ms of timing per candidate solution, default 15]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from csa_amd.train import use_tuned_gemms  # noqa: E402

if __name__ == "__main__":
    out = os.path.abspath(sys.argv[1])
    if os.path.exists(out):
        os.remove(out)
    use_tuned_gemms(path=out, tune=True)
    if len(sys.argv) > 2:
        torch.cuda.tunable.set_max_tuning_duration(int(sys.argv[2]))
    dev = torch.device("cuda:0")
    print("java train step", bench.train_step_bench(1, 0, dev, 3, 1), flush=True)
    print("python protocol", bench.gpu_config1(dev, reps=2), flush=True)
    print("shapes", len(torch.cuda.tunable.get_results()), flush=True)
