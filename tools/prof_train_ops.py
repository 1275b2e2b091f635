"""Dev tool: which torch ops launch the small fill / elementwise kernels of the java train step.

Runs bench.py's train step (config/java.py, 64 ASTs, tuned GEMM table) under torch.profiler and prints, for
the GPU kernels whose names match the given substrings (default: FillFunctor, CUDAFunctor), their count per
step grouped by the calling Python frames (top of stack), plus the top ops by self device time.

usage: python tools/prof_train_ops.py [steps] [substring ...]
"""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    pats = sys.argv[2:] or ["FillFunctor", "CUDAFunctor"]
    from csa_amd.data import synthetic_batch
    from csa_amd.model import CONFIGS, CSATrans, batch_to_device, label_smoothing_loss
    from csa_amd.train import AdamW, GEMM_TABLE, make_train_step, use_tuned_gemms, wrap_ddp
    use_tuned_gemms(path=GEMM_TABLE)
    dev = torch.device("cuda")
    torch.manual_seed(2021)
    model = CSATrans(**CONFIGS["java"]).to(dev)
    ddp = wrap_ddp(model, dev)
    opt = AdamW(model.parameters(), lr=1e-4, correct_bias=False)
    scaler = torch.amp.GradScaler("cuda")
    step = make_train_step(ddp, opt, label_smoothing_loss, sw=1e-2, scaler=scaler)
    batch = batch_to_device(synthetic_batch(64, 150, seed=1), dev)
    for _ in range(3):
        step(*batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        for _ in range(steps):
            step(*batch)
        torch.cuda.synchronize()
    # CPU op -> the kernels it launched (FunctionEvent.kernels), keeping the innermost op that owns a match
    counts = collections.Counter()
    for e in prof.events():
        ks = [k for k in (getattr(e, "kernels", None) or []) if any(p in k.name for p in pats)]
        if not ks:
            continue
        chain, p = [e.name], e.cpu_parent
        while p is not None and len(chain) < 4:
            chain.append(p.name)
            p = p.cpu_parent
        stack = [s_ for s_ in (e.stack or []) if "csa_amd" in s_ or "bench" in s_ or "torch/nn" in s_]
        for k in ks:
            counts[(k.name[:40], " <- ".join(chain), " | ".join(stack[:2]))] += 1
    for (k, chain, stack), n in counts.most_common(40):
        print(f"{n / steps:6.1f}/step  {k:40s}  {chain}  [{stack}]")
    print(prof.key_averages().table(sort_by="self_cuda_time_total", row_limit=25))


if __name__ == "__main__":
    main()
