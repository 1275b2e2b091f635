"""Dev tool (GPU): where the DDP wrapper's cost at world size 1 goes.

One process, a world-size-1 RCCL group, the java CSATrans train step (bench.py's train_step_bench setup, tuned GEMM
table) under several wrappers, alternated R times on the same box:
  plain       no DDP wrapper
  ddp         csa_amd.train.wrap_ddp(force=True) as bench.py's train_ddp_world1 leg (round-4 defaults)
  + any of the wrap_ddp switches named on the command line, e.g. "ddp:broadcast_buffers=0,static_graph=1"

usage: python tools/ddp_variants.py [R] [variant ...]     (variants: plain, ddp, ddp:<k=v,...>)
With CSA_DDP_PROF=<variant>, only that variant runs (for a rocprofv3 --kernel-trace capture of its steps)."""
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def parse(v):
    if v == "plain":
        return None
    kw = {}
    if ":" in v:
        for item in v.split(":", 1)[1].split(","):
            k, x = item.split("=")
            kw[k] = int(x) if x.isdigit() else x
    return kw


def run(variant, dev, steps=30, warmup=10):
    from csa_amd.data import synthetic_batch
    from csa_amd.model import CONFIGS, CSATrans, batch_to_device, label_smoothing_loss
    from csa_amd.train import AdamW, make_train_step, wrap_ddp
    torch.manual_seed(2021)
    model = CSATrans(**CONFIGS["java"]).to(dev)
    kw = parse(variant)
    net = model if kw is None else wrap_ddp(model, dev, force=True, **kw)
    opt = AdamW(model.parameters(), lr=1e-4, correct_bias=False)
    scaler = torch.amp.GradScaler("cuda")
    step = make_train_step(net, opt, label_smoothing_loss, sw=1e-2, scaler=scaler)
    batches = [batch_to_device(synthetic_batch(64, 150, seed=1 + i), dev) for i in range(3)]
    for i in range(warmup):
        step(*batches[i % 3])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses = [step(*batches[i % 3]) for i in range(steps)]
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1000 / steps
    return round(ms, 3), round(float(torch.stack(losses).mean()), 4)


def main():
    args = sys.argv[1:]
    rounds = int(args[0]) if args and args[0].isdigit() else 2
    variants = [a for a in args if not a.isdigit()] or ["plain", "ddp"]
    only = os.environ.get("CSA_DDP_PROF")
    if only:
        variants, rounds = [only], 1
    from csa_amd.train import use_tuned_gemms
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    print("tuned GEMM shapes:", use_tuned_gemms(True), flush=True)
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        for r in range(rounds):
            for v in variants:
                ms, loss = run(v, dev)
                print(json.dumps({"round": r, "variant": v, "ms_per_step": ms, "mean_loss": loss}), flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
