"""Dev tool (GPU): when does each gradient bucket become ready, and how much of an 8-rank all-reduce could the
backward hide.

One process, a world-size-1 RCCL group, the java CSATrans train step (bench.py's train_step_bench setup, tuned GEMM
table) under csa_amd.train.BucketedDataParallel with its event timeline on. For each bucket cap given (MB) it prints
the layout and, averaged over the recorded steps, every bucket's pack-completion time measured from the end of the
forward, and the end of the backward. It then projects the 8-rank exchange: each bucket's ring all-reduce takes
2 (N-1)/N x bytes / busbw on RCCL's one stream, starting when the bucket is packed and the previous bucket's
all-reduce has ended; "exposed" is how far the last all-reduce ends after the backward does (the step's added time),
for a range of bus bandwidths (the xGMI ring's per-rank rate is what an 8-GPU node measures; not measurable on a
one-GPU box).

usage: python tools/ddp_timeline.py [cap_mb ...]     (default: 64)"""
import json
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

BUSBW_GBS = (200, 300, 450, 600, 900)


def project(ready_ms, nbytes, bwd_end_ms, busbw_gbs, n=8):
    t_end = 0.0
    for r, nb in zip(ready_ms, nbytes):
        t_end = max(t_end, r) + 2 * (n - 1) / n * nb / (busbw_gbs * 1e9) * 1e3
    return t_end, max(0.0, t_end - bwd_end_ms)


def run(cap_mb, dev, steps=8, warmup=10):
    from csa_amd.data import synthetic_batch
    from csa_amd.model import CONFIGS, CSATrans, batch_to_device, label_smoothing_loss
    from csa_amd.train import AdamW, make_train_step, wrap_ddp
    torch.manual_seed(2021)
    model = CSATrans(**CONFIGS["java"]).to(dev)
    net = wrap_ddp(model, dev, force=True, bucket_cap_mb=cap_mb)
    opt = AdamW(model.parameters(), lr=1e-4, correct_bias=False)
    scaler = torch.amp.GradScaler("cuda")
    step = make_train_step(net, opt, label_smoothing_loss, sw=1e-2, scaler=scaler)
    batches = [batch_to_device(synthetic_batch(64, 150, seed=1 + i), dev) for i in range(3)]
    for i in range(warmup):
        step(*batches[i % 3])
    torch.cuda.synchronize()
    rows = []
    for i in range(steps):
        net.timeline = []
        step(*batches[i % 3])
        torch.cuda.synchronize()
        tl, net.timeline = net.timeline, None
        f0 = next(ev for tag, _, ev in tl if tag == "forward")
        packs = {b: f0.elapsed_time(ev) for tag, b, ev in tl if tag == "pack"}
        fin = next(f0.elapsed_time(ev) for tag, _, ev in tl if tag == "finish")
        rows.append((packs, fin))
    nb = len(net.bucket_table())
    ready = [sum(r[0][b] for r in rows) / steps for b in range(nb)]
    bwd_end = sum(r[1] for r in rows) / steps
    elem_bytes = model.parameters().__next__().element_size()
    nbytes = [e * elem_bytes for _, e, _ in net.bucket_table()]
    out = {"bucket_cap_mb": cap_mb, "buckets": [{"bucket": b, "MiB": round(nbytes[b] / 2 ** 20, 2),
                                                 "params": net.bucket_table()[b][2],
                                                 "ready_ms_after_forward": round(ready[b], 3)}
                                                for b in range(nb)],
           "backward_end_ms_after_forward": round(bwd_end, 3), "total_MiB": round(sum(nbytes) / 2 ** 20, 2),
           "projection_8_ranks": {}}
    for bw in BUSBW_GBS:
        end, exposed = project(ready, nbytes, bwd_end, bw)
        serial = 2 * 7 / 8 * sum(nbytes) / (bw * 1e9) * 1e3
        out["projection_8_ranks"][f"busbw_{bw}GBs"] = {"ring_ms_all_buckets": round(serial, 3),
                                                        "last_allreduce_end_ms": round(end, 3),
                                                        "exposed_ms": round(exposed, 3),
                                                        "hidden_frac": round(1 - exposed / serial, 3)}
    return out


def main():
    caps = [float(a) for a in sys.argv[1:]] or [64.0]
    from csa_amd.train import use_tuned_gemms
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    use_tuned_gemms(True)
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    try:
        for c in caps:
            print(json.dumps(run(c, dev)), flush=True)
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
