"""Round 6: the java train step unwrapped, under the round-6 BucketedDataParallel (rank 0's layout, in-order issue)
and under the round-5 one (tools/runs/_bdp_r5.py), alternating on one box over a world-size-1 RCCL group."""
import os
import socket
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import bench  # noqa: E402
from csa_amd import train as T  # noqa: E402
import _bdp_r5  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
T.use_tuned_gemms(True)
with socket.socket() as s_:
    s_.bind(("127.0.0.1", 0))
    port = s_.getsockname()[1]
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
cur = T.BucketedDataParallel
for rnd in range(2):
    for name in ("unwrapped", "bucketed_r6", "bucketed_r5"):
        if name == "bucketed_r5":
            T.BucketedDataParallel = _bdp_r5.BucketedDataParallel
        else:
            T.BucketedDataParallel = cur
        r = bench.train_step_bench(1, 0, dev, 50, 20, force_ddp=name != "unwrapped", impl="bucketed")
        print(rnd, name, r["ms_per_step"], r["mean_loss"], flush=True)
dist.destroy_process_group()
