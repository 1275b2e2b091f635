"""Round 6: per-step times of the java train step legs (unwrapped, world-size-1 bucketed, torch DDP), to see whether
the legs' run-to-run spread comes from a few slow steps (HIP events around every step)."""
import os
import socket
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from csa_amd import train as T  # noqa: E402
from csa_amd.data import synthetic_batch  # noqa: E402
from csa_amd.model import CONFIGS, CSATrans, batch_to_device, label_smoothing_loss  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
T.use_tuned_gemms(True)
with socket.socket() as s_:
    s_.bind(("127.0.0.1", 0))
    port = s_.getsockname()[1]
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
for rnd in range(2):
    for impl, force in (("none", False), ("bucketed", True), ("torch", True)):
        torch.manual_seed(2021)
        model = CSATrans(**CONFIGS["java"]).to(dev)
        ddp = T.wrap_ddp(model, dev, force=force, impl=impl if force else "torch")
        opt = T.AdamW(model.parameters(), lr=1e-4, correct_bias=False)
        scaler = torch.amp.GradScaler("cuda")
        step = T.make_train_step(ddp, opt, label_smoothing_loss, sw=1e-2, scaler=scaler)
        batches = [batch_to_device(synthetic_batch(64, 150, seed=1 + i), dev) for i in range(3)]
        for i in range(20):
            step(*batches[i % 3])
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(51)]
        ev[0].record()
        for i in range(50):
            step(*batches[i % 3])
            ev[i + 1].record()
        torch.cuda.synchronize()
        ts = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(50))
        tot = ev[0].elapsed_time(ev[50])
        print(rnd, impl, f"mean {tot / 50:.3f} median {ts[25]:.3f} min {ts[0]:.3f} top5 {[round(t, 2) for t in ts[-5:]]}",
              flush=True)
        del ddp, model, opt, step
dist.destroy_process_group()
