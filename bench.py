#!/usr/bin/env python
"""bench.py — SBM-attention fwd+bwd ASTs/s at L=150 (BASELINE.json configs[1]) on MI355X.

One "step" = one SBMAttention training pass (module/sbm_attn.py:32-66 forward + backward, train
mode: attention + proj dropout on, Bernoulli edge sampling from in-kernel Philox) over a batch of
256 synthetic 150-node ASTs with config/python.py dims (H=8, head_dim=64, k=10), inputs resident
in HBM. The upstream gradients are X's (dX ~ N(0,1)) and sparsity's (sw/32 per head), exactly
what the reference's train step feeds the layer (script/train.py:109).

Multi-GPU (torchrun, one process per GPU): each rank processes its own 256 ASTs (weak scaling)
and the layer's parameter gradients are all-reduced over RCCL (csa_amd.train's bucketed data-parallel
reducer, DDP semantics), the one exchange of script/train.py:83,109. value = ASTs processed by all
ranks / max-over-ranks wall time.

Printed JSON line (rank 0): contract fields + "roofline" for the dominant kernel (HIP events
recorded around that kernel's launch on its stream, every timed step; the dominant kernel and the
per-stage "stage_ms" come from an untimed pass with events around every stage, so the timed steps
carry only the two events of one kernel) + "cpu_baseline" (the oracle restatement of the reference
op sequence on the host CPU, rank 0 at N=1).
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "code-structure-aware-transformer_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "SBM-attn fwd+bwd ASTs/sec (L=150) + train samples/sec @1/2/4/8 GPU"
PEAK_F32_MFMA_TFLOPS = 157.3  # MI355X_MICROARCH.md: f32-input MFMA dense peak
PEAK_HBM_GBS = 8000.0
# ideal fused bytes per AST (fwd+bwd; Q,K,V,dX in, X, graph, dQ,dK,dV out) with fp32
# operands (the bf16 mode's own I/O: it takes and returns fp32 tensors) and with bf16 operands
IDEAL_BYTES_PER_AST_F32IO = 3.739e6
IDEAL_BYTES_PER_AST_BF16IO = 2.050e6


PMC_TABLE = os.path.join(ROOT, "code-structure-aware-transformer_amd", "csa_amd", "pmc_gfx950.json")
# the kernels of each profiled stage (csa_sbm.hip launch order)
STAGE_KERNELS = {"prep": ("k_prep",), "proj_fwd": ("k_proj_fwd_l",),
                 "attn_fwd": ("k_attn_fwd",), "attn_rowprep": ("k_attn_rowprep",), "attn_bwd_kv": ("k_attn_bwd_kv",),
                 "attn_bwd_q": ("k_attn_bwd_qg",), "proj_bwd": ("k_proj_bwd_s",),
                 "reduce": ("k_reduce_slabs", "k_cluster_grad")}  # (proj_bwd_k: k_proj_bwd_s as well)


def pmc_table():
    """The per-kernel HBM bytes / rocprof durations of the headline configuration (tools/pmc_traffic.py), shipped
    inside the package so the driver's run on the GPU box carries them."""
    if not os.path.exists(PMC_TABLE):
        return None
    with open(PMC_TABLE) as f:
        return json.load(f)


def traffic_evidence(table, B, stage_ms):
    """north_star's "achieved HBM GB/s against MI355X peak for the masking/softmax/sampling kernels": counter
    bytes per launch / the rocprof average duration of the same capture, per kernel, and the whole layer's
    counter bytes against the ideal fused traffic (3.739 MB per AST)."""
    ks = table["kernels"]
    by = {}
    for stage, names in STAGE_KERNELS.items():
        for n in names:
            t = ks.get(n)
            if not t or not t.get("rocprof_avg_ns"):
                continue
            gbs = t["bytes"] / (t["rocprof_avg_ns"] * 1e-9) / 1e9
            by[n] = {"stage": stage, "bytes": t["bytes"], "rocprof_avg_ms": round(t["rocprof_avg_ns"] * 1e-6, 4),
                     "GB_s": round(gbs, 1), "frac_of_hbm_peak": round(gbs / PEAK_HBM_GBS, 4)}
    total = sum(t["bytes"] for n, t in ks.items() if any(n in v for v in STAGE_KERNELS.values()))
    live = {s: round(sum(by[n]["bytes"] for n in names if n in by) / (stage_ms[s] * 1e-3) / 1e9, 1)
            for s, names in STAGE_KERNELS.items() if s in stage_ms and any(n in by for n in names)}
    return {"traffic_by_kernel": by, "traffic_GB_s_by_live_stage": live,
            "traffic_bytes_per_step": total, "ideal_bytes_per_step": round(IDEAL_BYTES_PER_AST_F32IO * B),
            "wasted_traffic_ratio": round(total / (IDEAL_BYTES_PER_AST_F32IO * B), 3),
            "pmc_table": os.path.relpath(PMC_TABLE, ROOT)}


def stage_flops_per_ast(H, N, M, D, k):
    """Algorithmic FLOPs per AST (one batch element, all heads) per kernel stage. The attention
    backward's algorithmic work (dP, dV, dK, dT | dQ, dQh) is split as its kernels do it: k_attn_bwd_kv computes
    dP = dX V^T (plus the S it recomputes, not counted) and dV, dK, dT; k_attn_bwd_qg dQ and dQh."""
    return {
        "proj_fwd": H * ((N + M) * (6 * D * D + 2 * k * D) + M * 2 * k * k),
        "attn_fwd": H * (4 * N * M * D + 2 * N * M * k),
        "attn_bwd_q": H * (2 * N * M * D + 2 * N * M * k),
        "attn_bwd_kv": H * (6 * N * M * D + 2 * N * M * k),
        "proj_bwd": H * ((N + M) * (12 * D * D + 4 * k * D) + M * 4 * k * k),
    }


class HipEvents:
    """hipEvent_t handles created through the HIP runtime torch already loaded."""

    def __init__(self):
        self.hip = ctypes.CDLL("libamdhip64.so.7")
        self.hip.hipEventCreate.argtypes = [ctypes.POINTER(ctypes.c_void_p)]
        self.hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
        self.hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
        self.made = []

    def create(self):
        e = ctypes.c_void_p()
        if self.hip.hipEventCreate(ctypes.byref(e)) != 0:
            raise RuntimeError("hipEventCreate failed")
        self.made.append(e)
        return e

    def elapsed_ms(self, a, b):
        ms = ctypes.c_float()
        if self.hip.hipEventElapsedTime(ctypes.byref(ms), a, b) != 0:
            # a stage that did not run (e.g. the projection stages of the dense ablation) left its
            # events unrecorded: clear the thread's HIP error so the next library call does not
            # report it as its own launch failure
            self.hip.hipGetLastError()
            return float("nan")
        return ms.value

    def destroy(self):
        for e in self.made:
            self.hip.hipEventDestroy(e)


def host_cpu_info():
    """What the CPU legs run on: the CPU model, the machine's logical CPUs (os.cpu_count()), the CPUs this
    process may run on (sched_getaffinity) and the cgroup CPU quota (cpu.max), when readable."""
    info = {"cpu": None, "machine_logical_cpus": os.cpu_count(), "affinity_cpus": None, "cgroup_cpu_quota": None}
    try:
        with open("/proc/cpuinfo") as fh:
            info["cpu"] = next(ln.split(":", 1)[1].strip() for ln in fh if ln.startswith("model name"))
    except (OSError, StopIteration):
        pass
    try:
        info["affinity_cpus"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, per = fh.read().split()[:2]
            if q != "max":
                info["cgroup_cpu_quota"] = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return info


def progress(msg):
    """One stderr line per bench leg, so a long default run is never silent for minutes."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def pick_threads(step, info):
    """Thread count for a CPU leg: os.cpu_count() as SURVEY 8(d) asks, unless the process is held to fewer
    CPUs by a cgroup CPU quota (the GPU box: os.cpu_count() = 256, quota 16): then the quota. Oversubscribing
    a quota only slows the baseline down -- measured on the box, one reduced-batch trial step took 0.06 s on
    16 threads and 18.8 s on 256 (SBM oracle), 0.24 s vs 104 s (CSATrans oracle): profiles/r03_bench_v1.json.
    Held by affinity or OMP_NUM_THREADS only (no quota): both counts are tried on one small trial step
    (`step`) and the faster is used."""
    machine = info["machine_logical_cpus"] or 1
    quota = info["cgroup_cpu_quota"]
    if quota and quota < machine:
        return max(1, int(quota)), {"thread_choice": f"cgroup CPU quota {quota:g} of {machine} logical CPUs"}
    cands = {machine}
    omp = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    held = min(x for x in (info["affinity_cpus"], omp, machine) if x)
    cands.add(max(1, int(held)))
    if len(cands) == 1:
        return cands.pop(), {}
    trial = {}
    for t in sorted(cands):
        torch.set_num_threads(t)
        t0 = time.perf_counter()
        step()
        trial[t] = round(time.perf_counter() - t0, 3)
    best = min(trial, key=trial.get)
    return best, {"thread_trial_s_per_step": trial}


def cpu_baseline(seconds, B=256, H=8, N=150, d=64, k=10):
    """Oracle (torch-CPU restatement of sbm_attn.py:32-66 + STE.py) fwd+bwd, train mode, timed on host cores,
    at the headline batch (B=256) unless a smaller B is passed."""
    from oracle import sbm_ref
    info = host_cpu_info()
    g = torch.Generator().manual_seed(0)
    Q, K, V = (torch.randn(B, H, N, d, generator=g).requires_grad_(True) for _ in range(3))
    params = {"layer.weight": torch.nn.init.orthogonal_(torch.empty(H * k, d)).requires_grad_(True)}
    for i in (0, 3, 6):
        params[f"proj.{i}.weight"] = torch.nn.init.xavier_uniform_(torch.empty(d, d)).requires_grad_(True)
        params[f"proj.{i}.bias"] = torch.zeros(d).requires_grad_(True)
    mask = torch.zeros(B, N)
    dX = torch.randn(B, H, N, d, generator=g)
    dsp = torch.full((H,), 3.125e-4)

    def step(nb=B):
        u = torch.rand(nb, H, N, N)  # == torch.bernoulli's draws
        keep = (torch.rand(nb, H, N, N) >= 0.2).float() / 0.8
        pk = {n: (torch.rand(nb, H, N, d) >= 0.2).float() / 0.8 for n in ("q0", "q1", "k0", "k1")}
        X, sp, graph, attn = sbm_ref.sbm_attention(Q[:nb], K[:nb], V[:nb], mask[:nb], params, u, k, attn_keep=keep,
                                                   proj_keep=pk)
        torch.autograd.backward([X, sp], [dX[:nb], dsp])

    step(min(B, 4))  # warm-up (allocator, thread pool)
    threads, trial = pick_threads(lambda: step(min(B, 8)), info)
    torch.set_num_threads(threads)
    n, t0 = 0, time.perf_counter()
    while True:
        step()
        n += 1
        el = time.perf_counter() - t0
        if el >= seconds and n >= 2:
            break
    return {"value": round(n * B / el, 2), "unit": "ASTs/s", "cores": threads, "kind": "port", **info, **trial,
            "sample": f"{n} oracle fwd+bwd steps of B={B} (H={H},N={N},d={d},k={k}, train mode) in {el:.1f}s "
                      f"on {threads} threads"}


def cpu_config1(reps=5, B=32, N=150):
    """BASELINE config 1: the csa_trans_time_memory.py:100-150 protocol on the host cores, restated on
    the oracle CSATrans (oracle/csatrans_ref.py, pinned to the reference's own CSATrans output):
    config/python.py dims, B synthetic 150-node ASTs, model.train() (dropouts and STE sampling from
    torch's CPU generator), three timings -- forward under no_grad; forward + out.mean().backward();
    LabelSmoothing + sw*sparsity forward + backward (script/train.py:107-109) -- 1 warm-up + `reps`
    timed passes each (the script runs 20 sweeps of the test loader; bounded here)."""
    from csa_amd.data import synthetic_batch
    from csa_amd.model import CONFIGS
    from oracle import csatrans_ref
    info = host_cpu_info()
    torch.manual_seed(0)
    cfg = csatrans_ref.config(**CONFIGS["python"])
    params = {k: v.requires_grad_(True) for k, v in csatrans_ref.init_params(cfg, seed=0).items()}
    model = csatrans_ref.Model(cfg, params, training=True)
    sb = synthetic_batch(B, N, seed=1)
    f = lambda k, dt: torch.as_tensor(sb[k]).to(dt)
    args = (f("src_seq", torch.int64), f("tgt_seq", torch.int64), f("L", torch.int64), f("T", torch.int64),
            f("L_mask", torch.bool), f("T_mask", torch.bool))
    tgt = f("target", torch.int64)

    def zero():
        for v in params.values():
            v.grad = None

    def fwd():
        with torch.no_grad():
            model.forward(*args)

    def fwd_bwd_mean():
        zero()
        out, _ = model.forward(*args)
        out.mean().backward()

    def train_loss():
        zero()
        out, sp = model.forward(*args)
        (csatrans_ref.label_smoothing(out, tgt) + 1e-2 * sp).backward()

    def fwd_small():  # thread-count trial on 4 of the batch's ASTs
        with torch.no_grad():
            model.forward(*(a[:4] for a in args))

    fwd_small()  # warm-up
    threads, trial = pick_threads(fwd_small, info)
    torch.set_num_threads(threads)
    res = {}
    for name, fn in (("fwd_no_grad", fwd), ("fwd_bwd_out_mean", fwd_bwd_mean), ("loss_sparsity_fwd_bwd", train_loss)):
        fn()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        res[name] = round(B * reps / (time.perf_counter() - t0), 2)
    return {"unit": "samples/s", "cores": threads, "kind": "port", **info, **trial, **res,
            "sample": f"oracle CSATrans config/python.py, B={B}, N={N}, train mode, 1 warm-up + {reps} timed passes "
                      f"each (the script runs 20 test-loader sweeps per leg)"}


def gpu_config1(dev, reps=10, B=32, N=150):
    """The same config-1 protocol on the MI355X path (csa_amd.model.CSATrans, config/python.py dims, B=32,
    train mode), beside cpu_config1: samples/s for fwd (no_grad), fwd + out.mean().backward() and
    loss + sw*sparsity fwd + bwd."""
    from csa_amd.data import synthetic_batch
    from csa_amd.model import CONFIGS, CSATrans, batch_to_device, label_smoothing_loss
    torch.manual_seed(0)
    model = CSATrans(**CONFIGS["python"]).to(dev).train()
    x, y = batch_to_device(synthetic_batch(B, N, seed=1), dev)

    def fwd():
        with torch.no_grad():
            model(x)

    def fwd_bwd_mean():
        model.zero_grad(set_to_none=True)
        model(x)[0].mean().backward()

    def train_loss():
        model.zero_grad(set_to_none=True)
        out, sp = model(x)[:2]
        (label_smoothing_loss(out, y) + 1e-2 * sp).backward()

    res, mem = {}, {}
    for name, fn in (("fwd_no_grad", fwd), ("fwd_bwd_out_mean", fwd_bwd_mean), ("loss_sparsity_fwd_bwd", train_loss)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        # csa_trans_time_memory.py:88-93,117,141-146: allocated_bytes.all.peak per timing pass
        torch.cuda.reset_peak_memory_stats(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        res[name] = round(B * reps / (time.perf_counter() - t0), 1)
        mem[name] = round(torch.cuda.max_memory_allocated(dev) / 2 ** 20, 1)
    return {"unit": "samples/s", "config": f"config/python.py CSATrans, B={B}, N={N}, train mode", **res,
            "peak_allocated_MiB": mem,
            "peak_note": "torch.cuda.max_memory_allocated over each leg's timed passes (parameters and grads included)"}


def train_step_bench(world, rank, dev, steps, warmup, config="java", per_gpu_batch=64, nbatches=3, force_ddp=False,
                     impl="torch"):
    """script/train.py:_update (config/java.py dims), data parallel over RCCL; returns samples/s over all ranks.
    force_ddp: wrap even at world size 1 (needs an initialised process group). impl: wrap_ddp's reducer
    ("bucketed" = csa_amd.train.BucketedDataParallel, "torch" = DistributedDataParallel)."""
    from csa_amd.data import synthetic_batch
    from csa_amd.model import CONFIGS, CSATrans, batch_to_device, label_smoothing_loss
    from csa_amd.train import AdamW, make_train_step, wrap_ddp
    torch.manual_seed(2021 + rank)  # set_seed(seed + rank), script/train.py:158
    model = CSATrans(**CONFIGS[config]).to(dev)
    ddp = wrap_ddp(model, dev, force=force_ddp, impl=impl)
    opt = AdamW(model.parameters(), lr=1e-4, correct_bias=False)
    scaler = torch.amp.GradScaler("cuda")
    step = make_train_step(ddp, opt, label_smoothing_loss, sw=1e-2, scaler=scaler)
    batches = [batch_to_device(synthetic_batch(per_gpu_batch, 150, seed=1 + 1000 * rank + i), dev)
               for i in range(nbatches)]
    for i in range(warmup):
        step(*batches[i % nbatches])
    losses = []
    # an event after every step (no host sync) for the per-step median beside the contract's mean: the legs' means
    # swing by several ms from run to run on a few long steps (profiles/r06_train_step_distribution.txt)
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)] if dev.type == "cuda" else None

    def timed(i):
        if evs is not None and i == 0:
            evs[0].record()
        losses.append(step(*batches[i % nbatches]))
        if evs is not None:
            evs[i + 1].record()

    el = timed_region(world, dev, steps, timed)
    med = None
    if evs is not None:
        per = sorted(evs[i].elapsed_time(evs[i + 1]) for i in range(steps))
        med = round(per[steps // 2], 3)
    mean_loss = float(torch.stack(losses).mean())
    nparam = sum(p.numel() for p in model.parameters())
    wrapped = world > 1 or force_ddp
    reducer = "BucketedDataParallel" if impl == "bucketed" else "torch DDP"
    return {"config": f"config/{config}.py CSATrans summary train step" + (f" ({reducer} over RCCL)" if wrapped else
                                                                           " (one GPU, no data-parallel wrapper)"),
            "per_gpu_batch": per_gpu_batch,
            "global_batch": per_gpu_batch * world, "steps": steps, "warmup": warmup,
            "ms_per_step": round(el * 1000 / steps, 3), "median_step_ms": med,
            "samples_per_s": round(world * per_gpu_batch * steps / el, 1),
            "params": nparam, "mean_loss": round(mean_loss, 4), "n_ranks": world,
            "exchange": (f"{reducer} gradient all-reduce over RCCL ({16 if impl == 'bucketed' else 64} MB buckets)"
                         if world > 1 else
                         f"{reducer} over a world-size-1 RCCL group (hooks + bucket packing, no peer)" if force_ddp
                         else "none (1 GPU, unwrapped)")}


def launch_ranks(nproc):
    """--gpus N > 1 without a torchrun environment: start N ranks with torch.distributed.run and exit
    with its status. This parent never touches the GPU (no HIP call happens before the children
    start), so each rank initialises its own device, as script/train.py's launcher does
    (torch.distributed.launch --nproc_per_node N, README.md:18)."""
    import socket
    import subprocess
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def init_ranks(args):
    """(world, rank, local, device) from the torchrun environment; RCCL ("nccl") on GPUs, gloo for the
    CPU launcher self-test. The world size is the process group's, and must equal --gpus."""
    env_world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if env_world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}")
    if args.device == "cpu":
        dev = torch.device("cpu")
        if env_world > 1:
            dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if env_world > 1:
            dist.init_process_group("nccl", device_id=dev)
    world = dist.get_world_size() if dist.is_initialized() else 1
    return world, rank, local, dev


def timed_region(world, dev, steps, step):
    """The contract's timed region: barrier + device sync on both sides of exactly `steps` steps;
    returns the max over ranks of the elapsed wall time (s)."""
    sync = torch.cuda.synchronize if dev.type == "cuda" else (lambda: None)
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for i in range(steps):
        step(i)
    sync()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el


def launcher_selftest(args, world, rank, dev):
    """--device cpu: exercises the launcher, the process group and the max-over-ranks timing on host
    CPUs (gloo) with a Linear under the bucketed data-parallel reducer; no kernel of this repo runs, so the
    line says so."""
    from csa_amd.train import BucketedDataParallel
    torch.manual_seed(rank)
    lin = torch.nn.Linear(64, 64)
    model = BucketedDataParallel(lin) if world > 1 else lin
    x = torch.randn(32, 64)

    def step(i):
        lin.zero_grad(set_to_none=True)
        model(x).square().mean().backward()

    for i in range(args.warmup):
        step(i)
    el = timed_region(world, dev, args.steps, step)
    return {"metric": "launcher self-test (data-parallel Linear on CPU/gloo; not the hot path)", "value": round(world * 32 *
            args.steps / el, 1), "unit": "samples/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(el * 1000 / args.steps, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "launcher self-test", "parallelism": f"dp{world}"}}


def stage_profilers():
    """(HipEvents, make_profs(n, stages, slots, fwd_stages), stage_times(profs, stages, slots, fwd_stages))."""
    from csa_amd._lib import CsaProf
    ev = HipEvents()

    def make_profs(n, stages, slots, fwd_stages):
        out = []
        for _ in range(n):
            pf, pb = CsaProf(), CsaProf()
            for name in stages:
                s_ = slots[name]
                tgt = pf if name in fwd_stages else pb
                tgt.start[s_], tgt.stop[s_] = ev.create().value, ev.create().value
            out.append((pf, pb))
        return out

    def stage_times(profs, stages, slots, fwd_stages):
        res = {}
        for name in stages:
            s_ = slots[name]
            vals = []
            for pf, pb in profs:
                tgt = pf if name in fwd_stages else pb
                if tgt.start[s_] and tgt.stop[s_]:
                    vals.append(ev.elapsed_ms(ctypes.c_void_p(tgt.start[s_]), ctypes.c_void_p(tgt.stop[s_])))
            vals = [v for v in vals if v == v and v > 0]
            if vals:
                res[name] = sum(vals) / len(vals)
        return res
    return ev, make_profs, stage_times


def padded_lengths(B, N, rank):
    """Config 2's padded batches: n_b ~ U[50, N] real nodes per AST (seeded per rank)."""
    gpad = torch.Generator().manual_seed(4321 + rank)
    return torch.randint(min(50, N), N + 1, (B,), generator=gpad)


def measure_layer(world, rank, dev, steps, warmup, B, N, d, k, dense, precision, eval_, reducer="torch", padded=False):
    """One SBMAttention (or FullAttention) fwd+bwd step on synthetic inputs resident in HBM: an untimed pass with
    HIP events around every stage (per-stage kernel times, the dominant stage), then the timed region with events
    only around the dominant kernel's launch (its live average launch duration). Returns the pieces of the line."""
    from csa_amd import ops
    from csa_amd._lib import STAGES, KERNEL_OF_STAGE
    from csa_amd.module.sbm_attn import FullAttention, SBMAttention
    H = 8
    torch.manual_seed(1234 + rank)
    cfg = {"attention_dropout": 0.2, "head_dim": d, "num_head": H, "num_clusters": [k], "return_maps": False,
           "attn_precision": precision}
    mod = (FullAttention(cfg, 0) if dense else SBMAttention(cfg, 0)).to(dev)
    for p in mod.parameters():
        if p.dim() > 1:
            torch.nn.init.xavier_uniform_(p)
    if not dense:
        torch.nn.init.orthogonal_(mod.layer.weight)
    mod.train(not eval_)
    model = mod
    if world > 1 and not dense:  # FullAttention has no parameters: no gradient exchange exists
        from csa_amd.train import wrap_ddp
        model = wrap_ddp(mod, dev, impl=reducer)  # in-order attention backward beside RCCL
    Q, K, V = (torch.randn(B, H, N, d, device=dev).requires_grad_(True) for _ in range(3))
    mask = torch.zeros(B, N, device=dev)
    if padded:
        nb = padded_lengths(B, N, rank)
        mask.copy_((torch.arange(N)[None, :] >= nb[:, None]).float())
    dX = torch.randn(B, H, N, d, device=dev)
    dsp = torch.full((H,), 3.125e-4, device=dev)

    def step(i=0):
        for t in (Q, K, V):
            t.grad = None
        for p in mod.parameters():
            p.grad = None
        X, sp, _, _ = model(Q, K, V, mask)
        if sp is None:
            torch.autograd.backward([X], [dX])
        else:
            torch.autograd.backward([X, sp], [dX, dsp])

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ev, make_profs_, stage_times_ = stage_profilers()
    fwd_stages = ("prep", "proj_fwd", "attn_fwd")
    make_profs = lambda n, stages: make_profs_(n, stages, STAGES, fwd_stages)  # noqa: E731
    stage_times = lambda profs, stages: stage_times_(profs, stages, STAGES, fwd_stages)  # noqa: E731

    # 1) untimed profiling pass: HIP events around every stage -> per-stage kernel times (diagnostic)
    nprof = max(3, min(steps, 10))
    profs = make_profs(nprof, list(STAGES))
    for i in range(nprof):
        ops.set_stage_profiler(*profs[i])
        step()
    ops.set_stage_profiler(None, None)
    torch.cuda.synchronize()
    stage_ms = stage_times(profs, list(STAGES))
    flops = stage_flops_per_ast(H, N, N, d, 0 if dense else k)
    if dense:
        flops = {"attn_fwd": H * 4 * N * N * d, "attn_bwd_q": H * 2 * N * N * d, "attn_bwd_kv": H * 6 * N * N * d}
    if "proj_bwd_k" in stage_ms:  # concurrent schedule: the projection backward's key / query items split
        flops["proj_bwd_k"] = H * (N * (12 * d * d + 4 * k * d) + N * 4 * k * k)
        flops["proj_bwd"] = H * N * (12 * d * d + 4 * k * d)
    timed = {s_: v for s_, v in stage_ms.items() if s_ in flops}
    # side-stream backward: a stage window that overlaps another backward stage's window is not one kernel's
    # launch alone on the device, so it cannot be the roofline kernel
    pb0 = profs[-1][1]
    win = {}
    base = None
    for name in ("attn_rowprep", "attn_bwd_kv", "attn_bwd_q", "proj_bwd_k", "proj_bwd", "reduce"):
        s_ = STAGES[name]
        if pb0.start[s_] and pb0.stop[s_]:
            if base is None:
                base = pb0.start[s_]
            win[name] = (ev.elapsed_ms(ctypes.c_void_p(base), ctypes.c_void_p(pb0.start[s_])),
                         ev.elapsed_ms(ctypes.c_void_p(base), ctypes.c_void_p(pb0.stop[s_])))
    over = {a for a in win for b_ in win if a != b_ and win[a][0] < win[b_][1] - 1e-4 and win[b_][0] < win[a][1] - 1e-4}
    cand = {s_: v for s_, v in timed.items() if s_ not in over}
    dom = max(cand, key=cand.get) if cand else None
    kernel_of = dict(KERNEL_OF_STAGE)
    if not dense and d in (64, 96) and k <= 16:
        kernel_of["proj_bwd"] = kernel_of["proj_bwd_k"] = "k_proj_bwd_s"  # the k <= 16 projection-backward variant

    # 2) timed region: events only around the dominant kernel (its live average launch duration)
    profs = make_profs(steps, [dom] if dom else [])

    def timed_step(i):
        ops.set_stage_profiler(*profs[i])
        step()

    elapsed = timed_region(world, dev, steps, timed_step)
    ops.set_stage_profiler(None, None)
    dom_ms = stage_times(profs, [dom]).get(dom) if dom else None
    ev.destroy()
    roofline = None
    if dom and dom_ms:
        ach = flops[dom] * B / (dom_ms * 1e-3) / 1e12
        roofline = {"bound": "mfma", "kernel": kernel_of[dom], "achieved": round(ach, 2),
                    "peak": PEAK_F32_MFMA_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / PEAK_F32_MFMA_TFLOPS, 4),
                    "traffic": None, "avg_launch_ms": round(dom_ms, 4),
                    "frac_basis": "live: HIP events on the kernel's stream around each of its launches in the timed "
                                  "steps (event timestamps include the launch's dispatch edge; frac_rocprof, when "
                                  "present, uses the committed rocprofv3 kernel-trace average)"}
    return {"mod": mod, "step": step, "mask": mask, "stage_ms": stage_ms, "flops": flops, "timed": timed,
            "over": over, "overlapped": bool(over), "dom": dom, "dom_ms": dom_ms, "kernel_of": kernel_of,
            "elapsed": elapsed, "roofline": roofline}


def rocprof_frac(table, leg, kernel, flops_per_launch):
    """frac_rocprof of a side leg's dominant kernel from the shipped rocprof table (tools/pmc_traffic.py legs)."""
    if not table:
        return {}
    t = (table.get("legs", {}).get(leg, {}) or {}).get(kernel)
    if not t or not t.get("rocprof_avg_ns"):
        return {}
    ach = flops_per_launch / (t["rocprof_avg_ns"] * 1e-9) / 1e12
    return {"frac_rocprof": round(ach / PEAK_F32_MFMA_TFLOPS, 4), "rocprof_avg_launch_ms": round(t["rocprof_avg_ns"] * 1e-6, 4),
            "pmc_table_matches_library": table.get("csa_source_hash") == _loaded_hash()}


def _loaded_hash():
    from csa_amd._lib import loaded_source_hash
    return loaded_source_hash()


def side_layer_leg(dev, steps, warmup, B, N, d, k, dense, table, leg):
    """A BASELINE config beside the headline (config 4 dense FullAttention, config 5 long ASTs): the same
    measurement as the headline (measure_layer) on one GPU; its own line fields, never `value`."""
    L = measure_layer(1, 0, dev, steps, warmup, B, N, d, k, dense, "fp32", False)
    ms = L["elapsed"] * 1000.0 / steps
    total = sum(L["flops"].values()) * B
    out = {"value": round(B * steps / L["elapsed"], 1), "unit": "ASTs/s", "ms_per_step": round(ms, 4),
           "batch": B, "seq_len": N, "head_dim": d, "clusters": 0 if dense else k, "steps": steps,
           "step_tflops": round(total / (ms * 1e-3) / 1e12, 2),
           "step_frac_of_f32_mfma_peak": round(total / (ms * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS, 4),
           "stage_ms": {s_: round(v, 4) for s_, v in L["stage_ms"].items()}}
    if L["roofline"]:
        r = dict(L["roofline"])
        r.pop("frac_basis", None)
        r.update(rocprof_frac(table, leg, r["kernel"], L["flops"][L["dom"]] * B))
        out["roofline"] = r
    del L
    torch.cuda.empty_cache()
    return out


CSE_FLOPS_PER_AST = 3 * 8 * 8 * 150 * 150 * 64  # 3 * H * 8 N^2 d_k (fwd + bwd) = 276.5 MFLOP


def cse_leg(dev, steps, warmup, table, B=64):
    """north_star's second kernel: the CSE relation attention (module/disentangled_attn.py:44-65) alone at the java
    train step's shape (B = 64 ASTs per GPU, H = 8, N = L = 150, d_k = 64, synthetic AST relation planes), fwd+bwd
    with fresh input gradients each step (the train step's zero_grad(set_to_none=True)). HIP events around every
    CSE stage in an untimed pass (ABI v9 CSA_REL_STAGE_*), then the timed steps with events around the dominant
    kernel only."""
    import numpy as np
    from csa_amd import ops, rel_ops
    from csa_amd._lib import REL_STAGES, REL_KERNEL_OF_STAGE
    from csa_amd.data import synthetic_batch
    H, N, d, Lr = 8, 150, 64, 150
    sb = synthetic_batch(B, N, seed=3)
    rel = torch.from_numpy(np.stack([sb["L"], sb["T"]], 1)).to(dev)
    msk = torch.from_numpy(np.stack([sb["L_mask"], sb["T_mask"]], 1).astype(np.uint8)).to(dev)
    g = torch.Generator(device=dev).manual_seed(77)
    q, k, v, dO = (torch.randn(B, H, N, d, device=dev, generator=g) for _ in range(4))
    lq, lk = (torch.randn(H, Lr, d, device=dev, generator=g) for _ in range(2))
    for t in (q, k, v, lq, lk):
        t.requires_grad_(True)

    def step(i=0):
        for t in (q, k, v, lq, lk):
            t.grad = None
        rel_ops.rel_attn(q, k, v, lq, lk, rel, msk).backward(dO)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ev, make_profs_, stage_times_ = stage_profilers()
    fwd_stages = ("logits", "fwd")
    stages = list(REL_STAGES)
    profs = make_profs_(max(3, min(steps, 10)), stages, REL_STAGES, fwd_stages)
    for pr in profs:
        ops.set_rel_profiler(*pr)
        step()
    ops.set_rel_profiler(None, None)
    torch.cuda.synchronize()
    stage_ms = stage_times_(profs, stages, REL_STAGES, fwd_stages)
    # algorithmic FLOP per stage and AST (12 products of 2 H N^2 d = 276.5 MFLOP with L = N), split as
    # the kernels compute them: logits c2p = Q LK^T, p2c = K LQ^T; forward Q K^T, P V; key side dP = dO V^T,
    # dv = P^T dO, dk = g^T Q + G_p2c^T LQ (S recomputed, not counted); query side dq = g K + G_c2p LK; lgrad
    # dlk = G_c2p^T Q, dlq = G_p2c^T K
    u, ul = 2 * H * N * N * d, 2 * H * N * Lr * d
    flops = {"logits": 2 * ul, "fwd": 2 * u, "bwd_k": 3 * u + ul, "bwd_q": u + ul, "lgrad": 2 * ul}
    dom = max((s_ for s_ in stage_ms if s_ in flops), key=stage_ms.get)
    profs = make_profs_(steps, [dom], REL_STAGES, fwd_stages)

    def timed_step(i):
        ops.set_rel_profiler(*profs[i])
        step()

    el = timed_region(1, dev, steps, timed_step)
    ops.set_rel_profiler(None, None)
    dom_ms = stage_times_(profs, [dom], REL_STAGES, fwd_stages).get(dom)
    ev.destroy()
    ms = el * 1000.0 / steps
    out = {"value": round(B * steps / el, 1), "unit": "ASTs/s", "ms_per_layer": round(ms, 4), "batch": B,
           "seq_len": N, "heads": H, "d_k": d, "steps": steps,
           "workload": "CSE DisentangledAttn.rel_attn fwd+bwd (config/java.py pegen_dim 512 / 8 heads), synthetic "
                       "AST relation planes",
           "layer_tflops": round(CSE_FLOPS_PER_AST * B / (ms * 1e-3) / 1e12, 2),
           "layer_frac_of_f32_mfma_peak": round(CSE_FLOPS_PER_AST * B / (ms * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS, 4),
           "stage_ms": {s_: round(v, 4) for s_, v in stage_ms.items()}}
    if dom_ms:
        ach = flops[dom] * B / (dom_ms * 1e-3) / 1e12
        r = {"bound": "mfma", "kernel": REL_KERNEL_OF_STAGE[dom], "achieved": round(ach, 2),
             "peak": PEAK_F32_MFMA_TFLOPS, "unit": "TFLOP/s", "frac": round(ach / PEAK_F32_MFMA_TFLOPS, 4),
             "avg_launch_ms": round(dom_ms, 4), "flops_per_ast": flops[dom]}
        r.update(rocprof_frac(table, "cse", r["kernel"], flops[dom] * B))
        out["roofline"] = r
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--seq-len", type=int, default=150, help="AST nodes N (config 5 long-AST stress: 1024)")
    ap.add_argument("--clusters", type=int, default=10, help="SBM clusters k (config 5 sweep: 16..128)")
    ap.add_argument("--head-dim", type=int, choices=(64, 96), default=64,
                    help="SBM head dim d (config/python.py: 64; config/java.py sbm_enc_dim 768 / 8 heads: 96)")
    ap.add_argument("--dense", action="store_true", help="FullAttention ablation (config/python_full_att.py)")
    ap.add_argument("--eval", action="store_true", help="eval mode (no dropout)")
    ap.add_argument("--precision", choices=("fp32", "bf16"), default="fp32",
                    help="operand precision of the attention contractions (fp32 = the reference's)")
    ap.add_argument("--no-bf16-leg", action="store_true", help="skip the bf16-mode side measurement")
    ap.add_argument("--no-padded-leg", action="store_true", help="skip the padded-mask (n_b ~ U[50,150]) leg")
    ap.add_argument("--padded", action="store_true",
                    help="the main measurement on padded batches (n_b ~ U[50, N], key mask on the padding; diagnostic)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cpu-config1", action="store_true", help="skip the config-1 CPU CSATrans protocol")
    ap.add_argument("--no-train", action="store_true", help="skip the full train-step measurement")
    ap.add_argument("--no-side-legs", action="store_true",
                    help="skip the CSE (java), dense (config 4) and long-AST (config 5) legs")
    ap.add_argument("--reducer", choices=("torch", "bucketed"), default="torch",
                    help="multi-GPU gradient reducer (csa_amd.train.wrap_ddp impl; bucketed is unverified over RCCL "
                         "with more than one rank)")
    ap.add_argument("--default-gemms", action="store_true",
                    help="train legs on hipBLASLt's default GEMM heuristic instead of the tuned table")
    ap.add_argument("--train-steps", type=int, default=50)
    ap.add_argument("--train-warmup", type=int, default=20)
    ap.add_argument("--device", choices=("cuda", "cpu"), default="cuda",
                    help="cpu = launcher self-test over gloo (no HIP kernels)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    # stdout carries exactly one line, the JSON result: RCCL prints a version banner on fd 1 when a communicator
    # comes up (the world-size-1 train legs), so fd 1 is kept for the result and everything else written to it
    # goes to stderr
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)

    def emit(obj):
        os.write(json_fd, (json.dumps(obj) + "\n").encode())

    world, rank, local, dev = init_ranks(args)
    if args.device == "cpu":
        out = launcher_selftest(args, world, rank, dev)
        if rank == 0:
            emit(out)
        if world > 1:
            dist.destroy_process_group()
        return

    from csa_amd._lib import loaded_source_hash

    B, H, N, d, k = args.batch, 8, args.seq_len, args.head_dim, args.clusters
    progress(f"SBM layer B={B} N={N} d={d} k={k}: warm-up")
    L = measure_layer(world, rank, dev, args.steps, args.warmup, B, N, d, k, args.dense, args.precision, args.eval,
                      reducer=args.reducer, padded=args.padded)
    mod, step, mask = L["mod"], L["step"], L["mask"]
    stage_ms, flops, timed, over, overlapped = L["stage_ms"], L["flops"], L["timed"], L["over"], L["overlapped"]
    dom, dom_ms, kernel_of, elapsed = L["dom"], L["dom_ms"], L["kernel_of"], L["elapsed"]
    ms_per_step = elapsed * 1000.0 / args.steps
    value = world * B * args.steps / elapsed
    roofline = L["roofline"]
    headline = (B, N, d, k, args.precision, args.dense, args.eval, args.padded) == (256, 150, 64, 10, "fp32", False, False, False)
    table = pmc_table() if headline else None
    if roofline and table:
        tr = table["kernels"].get(kernel_of[dom])
        if tr:  # HBM bytes per launch and rocprof duration from the shipped PMC table (tools/pmc_traffic.py)
            roofline["traffic"] = tr["bytes"]
            roofline["traffic_unit"] = ("bytes/launch (rocprofv3 2 x FETCH_SIZE + WRITE_SIZE, " +
                                        os.path.relpath(PMC_TABLE, ROOT) + ")")
            if tr.get("rocprof_avg_ns"):
                ach_r = flops[dom] * B / (tr["rocprof_avg_ns"] * 1e-9) / 1e12
                roofline["frac_rocprof"] = round(ach_r / PEAK_F32_MFMA_TFLOPS, 4)
                roofline["rocprof_avg_launch_ms"] = round(tr["rocprof_avg_ns"] * 1e-6, 4)
            roofline["pmc_table_matches_library"] = table["csa_source_hash"] == loaded_source_hash()
    total_flops = sum(flops.values()) * B
    out = {
        "metric": METRIC, "value": round(value, 1), "unit": "ASTs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32" if args.precision == "fp32" else "bf16 MFMA operands, f32 storage/accumulation",
        "data": f"synthetic (N(0,1) Q/K/V, {N}-node ASTs, " + ("padded: n_b ~ U[50, N] real nodes)" if args.padded else "no padding)"),
        "config": {"workload": "SBMAttention fwd+bwd (config/python.py dims) " + ("dense FullAttention" if args.dense
                   else "SBM") + ("" if N == 150 else f", long-AST stress N={N} k={k}"), "global_batch": B * world, "per_gpu_batch": B, "seq_len": N, "heads": H,
                   "head_dim": d, "clusters": 0 if args.dense else k, "mode": "eval" if args.eval else "train",
                   "parallelism": f"dp{world}",
                   "exchange": "none (FullAttention has no parameters)" if args.dense else
                   (f"gradient all-reduce over RCCL ({args.reducer} reducer)" if world > 1 else "none (1 GPU)")},
        "roofline": roofline,
        "step_tflops": round(total_flops / (ms_per_step * 1e-3) / 1e12, 2),
        "step_frac_of_f32_mfma_peak": round(total_flops / (ms_per_step * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS, 4),
        "stage_ms": {s: round(v, 4) for s, v in stage_ms.items()},  # untimed profiling pass, all stages
        # algorithmic FLOP / stage time / fp32 MFMA peak per compute stage (when the backward runs its two
        # attention kernels side by side -- B=64 shapes, DESIGN §3 -- their stage windows overlap)
        "stage_frac_of_f32_mfma_peak": {s: round(flops[s] * B / (v * 1e-3) / 1e12 / PEAK_F32_MFMA_TFLOPS, 3)
                                        for s, v in timed.items() if v > 0},
        "bwd_schedule": ("projection backward key-block items on a side stream beside k_attn_bwd_qg (overlapped "
                         "stage windows: " + ", ".join(sorted(over)) + ")") if overlapped else "in order",
    }
    if table:
        out.update(traffic_evidence(table, B, stage_ms))
    if args.precision == "fp32" and not args.no_bf16_leg and not args.dense and N <= 150:
        # the same layer with CSA_DTYPE_BF16 (north_star's bf16 variant): side measurement, same step
        progress("bf16-mode leg")
        mod.attn_precision = "bf16"
        for _ in range(args.warmup):
            step()
        el_bf = timed_region(world, dev, args.steps, lambda i: step())
        mod.attn_precision = "fp32"
        out["bf16_mode"] = {"value": round(world * B * args.steps / el_bf, 1), "unit": "ASTs/s",
                            "ms_per_step": round(el_bf * 1000.0 / args.steps, 4),
                            "note": "QK^T/PV/dP/dQ/dK/dV, the projection MLP and sigmoid(.C^T) (fwd+bwd) on bf16 MFMA; "
                                    "T = Kh S^T, expA, sampling and all elementwise fp32"}
        vb = out["bf16_mode"]["value"] / world  # per GPU
        out["bf16_mode"]["roofline"] = {
            "bound": "hbm", "unit": "GB/s", "peak": PEAK_HBM_GBS,
            "achieved": round(vb * IDEAL_BYTES_PER_AST_F32IO / 1e9, 1),
            "frac": round(vb * IDEAL_BYTES_PER_AST_F32IO / 1e9 / PEAK_HBM_GBS, 4),
            "ideal_bytes_per_ast": IDEAL_BYTES_PER_AST_F32IO,
            "frac_at_bf16_io": round(vb * IDEAL_BYTES_PER_AST_BF16IO / 1e9 / PEAK_HBM_GBS, 4),
            "note": "ideal fused bytes per AST x ASTs/s against 8 TB/s (SURVEY 8(d) config 2); frac with the "
                    "fp32 I/O the mode takes and returns, frac_at_bf16_io with 2.05 MB/AST bf16 I/O"}
    if not args.dense and N == 150 and not args.no_padded_leg:
        # config 2's real batches are padded: n_b ~ U[50, 150] nodes per AST, the rest key-masked (same layer, B)
        progress("padded-mask leg")
        nb = padded_lengths(B, N, rank)
        mask.copy_((torch.arange(N)[None, :] >= nb[:, None]).float())
        for _ in range(args.warmup):
            step()
        el_pad = timed_region(world, dev, args.steps, lambda i: step())
        mask.zero_()
        out["padded_mask"] = {"value": round(world * B * args.steps / el_pad, 1), "unit": "ASTs/s",
                              "ms_per_step": round(el_pad * 1000.0 / args.steps, 4),
                              "mean_nodes": round(float(nb.float().mean()), 2),
                              "note": "config 2 padded batches: n_b ~ U[50,150] real nodes per AST (seeded), key mask "
                                      "1 on the padding; fully masked 32-key tiles take the attention kernels' light "
                                      "paths (STE term only), the projection runs every row"}
    if world == 1 and headline and not args.no_side_legs:
        # BASELINE's other kernel configurations beside the headline, each with its dominant kernel's live roofline
        progress("CSE leg (java relation attention, B=64)")
        out["cse"] = cse_leg(dev, args.steps, args.warmup, table)
        progress("dense leg (config 4: FullAttention, B=256)")
        out["dense"] = side_layer_leg(dev, args.steps, args.warmup, 256, 150, 64, 0, True, table, "dense")
        out["dense"]["workload"] = "config 4: FullAttention fwd+bwd (config/python_full_att.py), train mode"
        out["long_ast"] = {"workload": "config 5: SBM fwd+bwd at N = 1024 (B = 16), k sweep, train mode"}
        for kk in (16, 32, 64, 128):
            progress(f"long-AST leg (config 5: N=1024, k={kk}, B=16)")
            out["long_ast"][f"k{kk}"] = side_layer_leg(dev, max(5, args.steps // 2), max(2, args.warmup // 2), 16,
                                                       1024, 64, kk, False, table, f"long_k{kk}")
    if not args.no_train:
        progress("train-step leg (config/java.py, 64 ASTs per GPU)")
        from csa_amd.train import GEMM_TABLE, use_tuned_gemms
        ntuned = use_tuned_gemms(not args.default_gemms)
        out["train"] = train_step_bench(world, rank, dev, args.train_steps, args.train_warmup, impl=args.reducer)
        out["train"]["gemms"] = (f"TunableOp table {os.path.basename(GEMM_TABLE)} ({ntuned} shapes)" if ntuned
                                 else "hipBLASLt default heuristic")
        if world == 1:
            # the same step under the data-parallel wrapper over a world-size-1 RCCL group: the reducer's own
            # cost on record (BucketedDataParallel, and torch DDP beside it for comparison)
            import socket
            with socket.socket() as s_:
                s_.bind(("127.0.0.1", 0))
                port = s_.getsockname()[1]
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
            try:
                out["train_ddp_world1"] = train_step_bench(1, rank, dev, args.train_steps, args.train_warmup,
                                                           force_ddp=True, impl="bucketed")
                out["train_torch_ddp_world1"] = train_step_bench(1, rank, dev, args.train_steps, args.train_warmup,
                                                                 force_ddp=True, impl="torch")
            finally:
                dist.destroy_process_group()
            progress("config-1 protocol on the GPU")
            out["config1_gpu"] = gpu_config1(dev)
            if ntuned:
                # the unwrapped step once more on hipBLASLt's default GEMM choice: what the table buys
                progress("train-step leg on default GEMMs")
                use_tuned_gemms(False)
                out["train_default_gemms"] = {k: v for k, v in train_step_bench(
                    world, rank, dev, args.train_steps, args.train_warmup).items()
                    if k in ("ms_per_step", "samples_per_s", "mean_loss")}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("CPU baseline (oracle SBM layer on host cores)")
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, B=B if N <= 150 else 1, N=N, k=k)
        if not args.no_cpu_config1:
            progress("config-1 protocol on host cores (oracle CSATrans)")
            out["cpu_config1"] = cpu_config1()
    if rank == 0:
        emit(out)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
