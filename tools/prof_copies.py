"""Dev tool: attribute the java train step's torch copy/fill kernels to Python call sites.

usage: python tools/prof_copies.py [steps] > out.txt   (GPU box)
Runs bench.train_step_bench's model for a few steps under torch.profiler (with_stack) and prints, for
aten::copy_/clone/contiguous/fill_/zero_/cat ops, the count per step, their device time and the first
stack frame inside this repository (or torch's autograd when the op runs in the backward)."""
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402


OPS = ("aten::copy_", "aten::clone", "aten::contiguous", "aten::fill_", "aten::zero_", "aten::cat",
       "aten::add", "aten::add_", "aten::mul", "aten::native_dropout", "aten::gelu", "aten::masked_fill")


def site(ev):
    for fr in ev.stack or []:
        if ROOT in fr and "tools/prof_copies.py" not in fr:
            return fr.replace(ROOT + "/", "")
    p = ev.cpu_parent
    while p is not None:
        if p.name.startswith("autograd::engine::evaluate_function"):
            return p.name.replace("autograd::engine::evaluate_function: ", "bwd:")
        p = p.cpu_parent
    return (ev.stack[0] if ev.stack else "<no stack: autograd engine>")[:120]


if __name__ == "__main__":
    from csa_amd.data import synthetic_batch
    from csa_amd.model import CONFIGS, CSATrans, batch_to_device, label_smoothing_loss
    from csa_amd.train import AdamW, make_train_step, wrap_ddp
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    dev = torch.device("cuda:0")
    torch.manual_seed(2021)
    model = CSATrans(**CONFIGS["java"]).to(dev)
    opt = AdamW(model.parameters(), lr=1e-4, correct_bias=False)
    step = make_train_step(wrap_ddp(model, dev), opt, label_smoothing_loss, sw=1e-2,
                           scaler=torch.amp.GradScaler("cuda"))
    batch = batch_to_device(synthetic_batch(64, 150, seed=1), dev)
    for _ in range(3):
        step(*batch)
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
                 record_shapes=True) as prof:
        for _ in range(steps):
            step(*batch)
        torch.cuda.synchronize()
    agg = collections.defaultdict(lambda: [0, 0.0, set()])
    for ev in prof.events():
        if ev.name not in OPS:
            continue
        key = (ev.name, site(ev))
        a = agg[key]
        a[0] += 1
        a[1] += ev.device_time_total
        a[2].add(str(ev.input_shapes)[:90])
    rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
    print(f"{'per step':>8} {'us/step':>9}  op / site / shapes")
    for (name, s), (n, t, shp) in rows[:60]:
        print(f"{n / steps:8.1f} {t / steps:9.1f}  {name}  {s}  {sorted(shp)[:3]}")
