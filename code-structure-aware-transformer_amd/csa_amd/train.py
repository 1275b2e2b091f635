"""The data-parallel training step of script/train.py:103-116, on PyTorch-ROCm + RCCL.

    _update: model.train(); zero_grad; y_pred, sparsity, ... = model(x)
             loss = LabelSmoothing(y_pred, y); GradScaler.scale(loss + sw*sparsity).backward()
             scaler.step(AdamW); scaler.update()

Multi-GPU: one process per GPU (torchrun), data parallel over the "nccl" backend (= RCCL on ROCm,
xGMI between the GPUs of a node) as idist.auto_model's DistributedDataParallel does
(script/train.py:83,331), with this repo's bucketed reducer (BucketedDataParallel: one pack launch
per 16 MB bucket instead of DDP's per-parameter copies); each rank draws its own batches
(DistributedSampler semantics: per-rank shard) and seeds with seed + rank (script/train.py:158).
Gradients are averaged, so the global step equals the mean of the per-rank losses, exactly the
reference's semantics (LabelSmoothing divides by per-rank ntokens, utils/label_smooth.py:27,40).

The optimizer is the reference's HF-style AdamW (script/optimizer.py:49-106) with
correct_bias=False (script/train.py:80). On GPU every parameter is updated by ONE launch of the
HIP kernel csa_adamw_step (csrc/csa_optim.hip: 28 B of HBM traffic per parameter); CPU parameters
(the gloo DDP tests) take multi-tensor foreach ops with the same op order.
"""
import ctypes
import os

import torch
import torch.distributed as dist


class AdamW(torch.optim.Optimizer):
    """script/optimizer.py:10-106 (decoupled weight decay, optional bias correction): one csa_adamw_step
    launch for all CUDA parameters, foreach ops on CPU.

    Under torch.amp.GradScaler the optimizer takes the scaler's device-side `grad_scale` and
    `found_inf` (_step_supports_amp_scaling): the kernel unscales the gradients and skips the update
    on inf/NaN itself, so `scaler.step()` needs no host sync. The skip then happens on the device
    while the host-side step counter still advances; bias correction depends on that counter, so
    groups with correct_bias=True (not the reference's configuration, script/train.py:80) take the
    host-synchronised skip instead."""

    _step_supports_amp_scaling = True

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.0, correct_bias=True):
        if lr < 0.0 or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0 or eps < 0.0:
            raise ValueError("invalid AdamW hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      correct_bias=correct_bias))
        self._tables = {}  # param-group index -> device chunk tables + descriptors for csa_adamw_step

    def _chunk_tables(self, key, ps, grads, m, v):
        """Device tables for csa_adamw_step, cached per parameter group (`key`): chunk -> tensor and
        first chunk per tensor (rebuilt only when the group's sizes change), and the (param, grad,
        exp_avg, exp_avg_sq, numel) descriptors, re-sent only when a pointer changes (set_to_none grads
        may come back elsewhere) through a pinned non-blocking copy, so the step never waits for the
        device. Each group keeps its own entry, so a decay/no-decay split does not rebuild per step."""
        from ._lib import ADAMW_CHUNK
        dev = ps[0].device
        sizes = tuple(p.numel() for p in ps)
        ent = self._tables.get(key)
        if ent is None or ent["sizes"] != sizes:
            nchunk = [(n + ADAMW_CHUNK - 1) // ADAMW_CHUNK for n in sizes]
            start = torch.zeros(len(sizes), dtype=torch.int64)
            if len(sizes) > 1:
                start[1:] = torch.cumsum(torch.tensor(nchunk[:-1], dtype=torch.int64), 0)
            owner = torch.repeat_interleave(torch.arange(len(sizes), dtype=torch.int32),
                                            torch.tensor(nchunk, dtype=torch.int64))
            ent = {"sizes": sizes, "owner": owner.to(dev), "start": start.to(dev), "nchunks": sum(nchunk),
                   "ptrs": None, "desc": None}
            self._tables[key] = ent
        ptrs = tuple(x for q in zip(ps, grads, m, v) for x in (q[0].data_ptr(), q[1].data_ptr(),
                                                               q[2].data_ptr(), q[3].data_ptr()))
        if ent["ptrs"] != ptrs:
            host = torch.tensor([x for i in range(len(ps)) for x in (*ptrs[4 * i:4 * i + 4], sizes[i])],
                                dtype=torch.int64).pin_memory()
            ent["desc"], ent["ptrs"] = host.to(dev, non_blocking=True), ptrs
        return ent["desc"], ent["owner"], ent["start"], len(ps), ent["nchunks"]

    def _fused_step(self, gi, group, ps, grads, m, v, step_size, grad_scale=None, found_inf=None):
        from ._lib import AdamwArgs, check, lib, on_device
        for t in ps + grads + m + v:
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise RuntimeError("csa_adamw_step: parameters, grads and state must be contiguous fp32")
        desc, owner, start, nt, nc = self._chunk_tables(gi, ps, grads, m, v)
        b1, b2 = group["betas"]
        a = AdamwArgs(tensors=desc.data_ptr(), chunk_tensor=owner.data_ptr(), chunk_start=start.data_ptr(),
                      ntensors=nt, nchunks=nc, beta1=b1, beta2=b2, one_minus_beta1=1.0 - b1,
                      one_minus_beta2=1.0 - b2, eps=group["eps"], step_size=step_size,
                      decay=group["lr"] * group["weight_decay"] if group["weight_decay"] > 0.0 else 0.0,
                      grad_scale=None if grad_scale is None else grad_scale.data_ptr(),
                      found_inf=None if found_inf is None else found_inf.data_ptr())
        stream = ctypes.c_void_p(torch.cuda.current_stream(ps[0].device).cuda_stream)
        with on_device(ps[0].device):
            check(lib().csa_adamw_step(ctypes.byref(a), stream), "csa_adamw_step")

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        grad_scale = getattr(self, "grad_scale", None)  # set by GradScaler.step (device tensors)
        found_inf = getattr(self, "found_inf", None)
        if grad_scale is not None:
            grad_scale = grad_scale.to(torch.float32).contiguous()
        if found_inf is not None:
            found_inf = found_inf.to(torch.float32).contiguous()
            on_host = any(p.grad is not None and not p.is_cuda for g in self.param_groups for p in g["params"])
            if (on_host or any(g["correct_bias"] for g in self.param_groups)) and found_inf.item() != 0.0:
                return loss  # GradScaler skip, decided on the host (no state change)
        for gi, group in enumerate(self.param_groups):
            ps = [p for p in group["params"] if p.grad is not None]
            if not ps:
                continue
            grads = [p.grad for p in ps]
            m, v = [], []
            for p in ps:
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = 0
                    st["exp_avg"] = torch.zeros_like(p)
                    st["exp_avg_sq"] = torch.zeros_like(p)
                st["step"] += 1
                m.append(st["exp_avg"])
                v.append(st["exp_avg_sq"])
            b1, b2 = group["betas"]
            step_size = group["lr"]
            if group["correct_bias"]:
                t = self.state[ps[0]]["step"]
                step_size = step_size * (1.0 - b2 ** t) ** 0.5 / (1.0 - b1 ** t)
            if ps[0].is_cuda:
                self._fused_step(gi, group, ps, grads, m, v, step_size, grad_scale, found_inf)
                continue
            if grad_scale is not None:
                grads = torch._foreach_mul(grads, (1.0 / grad_scale.double()).float().item())
            torch._foreach_mul_(m, b1)
            torch._foreach_add_(m, grads, alpha=1.0 - b1)
            torch._foreach_mul_(v, b2)
            torch._foreach_addcmul_(v, grads, grads, value=1.0 - b2)
            denom = torch._foreach_sqrt(v)
            torch._foreach_add_(denom, group["eps"])
            torch._foreach_addcdiv_(ps, m, denom, value=-step_size)
            if group["weight_decay"] > 0.0:
                torch._foreach_add_(ps, ps, alpha=-group["lr"] * group["weight_decay"])
        return loss


def init_distributed():
    """torchrun env -> (rank, world, local_rank, device); RCCL process group when world > 1."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        if device.type == "cuda":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")
    return rank, world, local, device


GEMM_TABLE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "gemm_tuned_gfx950.csv")


def use_tuned_gemms(on=True, path=GEMM_TABLE, tune=False):
    """Select the stock fp32 GEMMs of the model (encoder/decoder Linears, the fused QKV projection, the
    generator) from a per-shape table instead of hipBLASLt's default heuristic: PyTorch TunableOp with
    the committed table `gemm_tuned_gfx950.csv` (tools/tune_gemms.py measured every GEMM shape of the
    config/java.py train step at 64 ASTs per GPU and of the config/python.py protocol at B=32 on an
    MI355X, picking the fastest hipBLASLt or rocBLAS solution per shape). Same fp32 arithmetic, only
    the kernel (tile shape, summation order) differs; shapes not in the table keep the default.
    The table is validated against the running PyTorch / HIP / hipBLASLt / rocBLAS versions and the
    gfx arch (its Validator rows); on a mismatch nothing is loaded. Process-global (torch.cuda.tunable),
    so every rank of a DDP job calls it for itself. Returns the number of table entries in effect.
    tune=True searches shapes missing from the table (tools/tune_gemms.py)."""
    import torch.cuda.tunable as tunable
    if not on:
        tunable.enable(False)
        return 0
    tunable.enable(True)
    tunable.tuning_enable(tune)
    tunable.set_max_tuning_duration(15)
    tunable.set_filename(path, insert_device_ordinal=False)
    if os.path.exists(path) and not tunable.read_file(path):
        tunable.enable(False)
        return 0
    if not tune:
        # results may be written back to the current filename at exit (this torch has no switch to turn that
        # off): point it at a per-process scratch file, so concurrent ranks never rewrite the shared table,
        # remove it at exit and sweep the scratch files of processes that are gone
        import atexit
        import glob
        import tempfile
        for f in glob.glob(os.path.join(tempfile.gettempdir(), "csa_tunableop_*.csv")):
            try:
                pid = int(os.path.basename(f)[len("csa_tunableop_"):-len(".csv")])
                os.kill(pid, 0)
            except ProcessLookupError:
                _remove_quiet(f)
            except (ValueError, PermissionError):
                pass
        scratch = os.path.join(tempfile.gettempdir(), f"csa_tunableop_{os.getpid()}.csv")
        tunable.set_filename(scratch, insert_device_ordinal=False)
        atexit.register(_remove_quiet, scratch)
    return len(tunable.get_results())


def _remove_quiet(path):
    try:
        os.remove(path)
    except OSError:
        pass


def set_bwd_schedule(model, schedule):
    """Set the attention backward schedule ("auto" | "in_order" | "concurrent") of every SBM / dense / CSE
    attention module inside `model` (csa_amd.module.*: bwd_schedule)."""
    n = 0
    for m in model.modules():
        if hasattr(m, "bwd_schedule"):
            m.bwd_schedule = schedule
            n += 1
    return n


def _world1_no_comm_hook(state, bucket):
    """Diagnostic DDP comm hook (tools/ddp_variants.py): a world-size-1 group's all-reduce is the identity, so the
    bucket is returned as it is (no division by 1, no RCCL call). Only ever registered at world size 1."""
    fut = torch.futures.Future()
    fut.set_result(bucket.buffer())
    return fut


class BucketedDataParallel(torch.nn.Module):
    """Data-parallel gradient averaging over the initialised process group, the semantics of
    idist.auto_model's DistributedDataParallel (script/train.py:83): identical initial parameters on
    every rank (rank 0's, broadcast once), and after each backward every parameter gradient is the mean
    of the per-rank gradients. `.module` is the wrapped model, as in DDP (state_dict keys "module.*",
    GreedyGenerator's `model.module`).

    The reducer is built for this model's gradient traffic instead of DDP's per-parameter one. DDP copies
    every parameter gradient into its bucket with its own kernel (283 tensors in config/java.py: 283
    copy launches per step, 1.7 ms at world size 1, tools/ddp_variants.py). Here each bucket of
    parameters (~`bucket_cap_mb`, in gradient arrival order) is packed by ONE torch.cat into its slice
    of a persistent flat fp32 gradient buffer the moment its last gradient has been accumulated
    (post-accumulate-grad hooks), its all-reduce is issued right away on RCCL's stream (overlapping the
    rest of the backward), and every `p.grad` becomes a view of the flat buffer, so the optimizer's
    gradient pointers stay fixed from step to step. One autograd-engine callback at the end of the
    backward packs any bucket left incomplete (parameters without a gradient contribute zeros, as in
    DDP's find_unused_parameters), waits for the all-reduces and averages.

    Averaging: RCCL's AVG reduction (a pre-multiply by 1/world, DDP's `div_(world)` then SUM), gloo:
    SUM then one division per bucket. For power-of-two world sizes both are exact scalings, so the
    result is bit-identical to DDP's. Buffers (the positional-encoding table) are broadcast once at
    construction; the model has no buffer that changes in training. `no_sync()` skips the reduction
    (local gradient accumulation); the next synchronised backward reduces the accumulated gradients.
    The first backward records the order in which gradients arrive; the buckets are then re-laid in
    that order (DDP's bucket rebuild), so later steps start all-reducing as early as possible. Every rank
    adopts RANK 0's arrival order (broadcast, as DDP's sync_bucket_indices), and bucket all-reduces are
    issued strictly in bucket-index order (a complete bucket waits until every lower-index bucket has been
    issued, DDP's next_bucket_), so the collectives of all ranks pair up bucket for bucket even when the
    ranks see different gradient arrival orders or different unused parameters.

    Multi-GPU status: the world > 1 all-reduce path is exercised by the 2-rank gloo tests
    (tests/test_train_cpu.py, including ranks with different unused parameters) and on one GPU by
    tools/ddp_one_gpu.py (gloo); it has not been run over RCCL with more than one rank, so wrap_ddp keeps
    torch DDP as the multi-GPU default and this reducer is opt-in there (impl="bucketed")."""

    def __init__(self, module, bucket_cap_mb=16, process_group=None):
        super().__init__()
        self.module = module
        self.group = process_group
        self.world = dist.get_world_size(process_group)
        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise ValueError("BucketedDataParallel: the module has no trainable parameters")
        if len({(p.dtype, p.device) for p in params}) != 1:
            raise ValueError("BucketedDataParallel: all parameters must share one dtype and device")
        self._params = params
        self._cap = max(1, int(bucket_cap_mb * 2 ** 20 // params[0].element_size()))
        with torch.no_grad():  # DDP's _sync_module_states: rank 0's parameters and buffers everywhere
            if self.world > 1:
                for t in params + list(module.buffers()):
                    dist.broadcast(t.data, 0, group=process_group)
        self._op = (dist.ReduceOp.AVG if dist.get_backend(process_group) == "nccl" else dist.ReduceOp.SUM)
        self._layout(list(reversed(range(len(params)))))  # DDP's initial guess: reverse registration order
        self._arrival, self._rebuilt = [], False
        self._sync, self._queued = True, False
        self._next = 0  # lowest bucket index whose all-reduce has not been issued in this backward
        self.timeline = None  # list -> (tag, bucket, cuda Event) per forward end / bucket pack / finish (tools/)
        self._hooks = [p.register_post_accumulate_grad_hook(self._make_hook(i)) for i, p in enumerate(params)]

    def _layout(self, order):
        """Buckets of consecutive parameters in `order` (~cap elements each) and one flat buffer."""
        p0 = self._params[0]
        self._bucket_of = [0] * len(self._params)
        self._buckets, cur, size = [], [], 0
        for i in order:
            n = self._params[i].numel()
            if cur and size + n > self._cap:
                self._buckets.append(cur)
                cur, size = [], 0
            cur.append(i)
            size += n
        self._buckets.append(cur)
        self._spans, self._views, off = [], [None] * len(self._params), 0
        total = sum(p.numel() for p in self._params)
        self.flat = torch.zeros(total, dtype=p0.dtype, device=p0.device)
        for b, idx in enumerate(self._buckets):
            lo = off
            for i in idx:
                p = self._params[i]
                self._bucket_of[i] = b
                self._views[i] = self.flat[off:off + p.numel()].view_as(p)
                off += p.numel()
            self._spans.append((lo, off))
        self._pending = [len(idx) for idx in self._buckets]
        self._works = []
        self._next = 0

    def _make_hook(self, i):
        def hook(p):
            if not self._sync:
                return
            if not self._queued:  # first gradient of this backward: finish at its end
                torch.autograd.Variable._execution_engine.queue_callback(self._finish)
                self._queued = True
            if not self._rebuilt:
                self._arrival.append(i)
            b = self._bucket_of[i]
            self._pending[b] -= 1
            if self._rebuilt:  # issue every complete bucket whose lower-index buckets are all issued
                while self._next < len(self._buckets) and self._pending[self._next] == 0:
                    self._reduce(self._next)
                    self._next += 1
        return hook

    @torch.no_grad()
    def _reduce(self, b):
        lo, hi = self._spans[b]
        dst = self.flat[lo:hi]
        grads = []
        for i in self._buckets[b]:
            g = self._params[i].grad
            grads.append(torch.zeros_like(self._params[i]) if g is None else g)
        aliased = [g.data_ptr() == self._views[i].data_ptr() for g, i in zip(grads, self._buckets[b])]
        if not any(aliased):
            torch.cat([g.reshape(-1) for g in grads], out=dst)
        else:  # gradients accumulated in place into the flat views (no_sync / set_to_none=False)
            for g, i, a in zip(grads, self._buckets[b], aliased):
                if not a:
                    self._views[i].copy_(g)
        for i in self._buckets[b]:
            self._params[i].grad = self._views[i]
        self._mark("pack", b)
        if self.world > 1:
            self._works.append((b, dist.all_reduce(dst, op=self._op, group=self.group, async_op=True)))

    @torch.no_grad()
    def _finish(self):
        self._queued = False
        if not self._rebuilt:  # first step: adopt rank 0's observed arrival order, then reduce everything
            seen = set(self._arrival)
            order = self._arrival + [i for i in reversed(range(len(self._params))) if i not in seen]
            if self.world > 1:  # every rank lays its buckets out in rank 0's order (DDP's sync_bucket_indices)
                dev = self.flat.device if dist.get_backend(self.group) == "nccl" else torch.device("cpu")
                t = torch.tensor(order, dtype=torch.int64, device=dev)
                dist.broadcast(t, 0, group=self.group)
                order = t.tolist()
            self._layout(order)
            self._rebuilt = True
            self._arrival = []
        # the buckets not issued yet, in index order (incomplete ones: parameters without a gradient add zeros)
        for b in range(self._next, len(self._buckets)):
            self._reduce(b)
        for b, w in self._works:
            w.wait()
            if self._op == dist.ReduceOp.SUM:
                lo, hi = self._spans[b]
                self.flat[lo:hi].div_(self.world)
        self._works = []
        self._pending = [len(idx) for idx in self._buckets]
        self._next = 0
        self._mark("finish", -1)

    def _mark(self, tag, b):
        if self.timeline is not None and self.flat.is_cuda:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record()
            self.timeline.append((tag, b, ev))

    def bucket_table(self):
        """[(bucket, elements, parameter names count)] of the current layout (tools/ddp_timeline.py)."""
        return [(b, hi - lo, len(self._buckets[b])) for b, (lo, hi) in enumerate(self._spans)]

    def forward(self, *args, **kwargs):
        if self._queued or self._works:  # a previous backward ended early (it raised): start this one clean
            for _, w in self._works:
                w.wait()
            self._works, self._queued, self._next = [], False, 0
            self._pending = [len(idx) for idx in self._buckets]
            if not self._rebuilt:  # the arrival record of the failed first backward is incomplete
                self._arrival = []
        out = self.module(*args, **kwargs)
        self._mark("forward", -1)
        return out

    def no_sync(self):
        """Context manager: backwards inside it accumulate local gradients without reducing them."""
        import contextlib

        @contextlib.contextmanager
        def ctx():
            old, self._sync = self._sync, False
            try:
                yield
            finally:
                self._sync = old
        return ctx()


def wrap_ddp(model, device, force=False, bucket_cap_mb=None, impl="torch", broadcast_buffers=True,
             static_graph=False, comm_hook=None):
    """Data parallelism over the initialised process group (idist.auto_model, script/train.py:83).
    Without a process group of more than one rank the model is returned unwrapped, unless `force`
    (the wrapper over a world-size-1 group: the reducer's own cost, tests).

    impl "torch" (default): torch DistributedDataParallel, 64 MB buckets (gradient_as_bucket_view; broadcast_buffers,
    static_graph and the world-size-1 diagnostic comm_hook "world1_none" apply to it only). The default for
    multi-GPU runs: its RCCL path is the one known to work with more than one rank.
    impl "bucketed": BucketedDataParallel, 16 MB buckets (bucket_cap_mb=None), one pack launch per bucket
    (+0.7% on the java step at world size 1 against torch DDP's +7-9%). 16 MB: the java step's bucket-ready
    timeline (tools/ddp_timeline.py) leaves 0.2 ms of a projected 8-rank all-reduce exposed at
    300 GB/s bus bandwidth, against 0.4 ms with 64 MB buckets. Verified at world size 2 over gloo and over a
    world-size-1 RCCL group; unverified over RCCL with more than one rank (opt-in there).

    The modules' packed parameters (Attention W_q/W_k/W_v, the CSE q/k/v linears) are packed at
    construction and after every device move, so the reducer's buckets and hooks see the final storages.
    The all-reduces overlap the backward on RCCL's stream; with 4 hardware queues per process
    (GPU_MAX_HW_QUEUES) an attention backward's side stream could share a queue with it and wait behind
    an in-flight all-reduce, so multi-rank GPU training keeps each attention backward on one stream
    (bwd_schedule "in_order", per module: no process-global switch)."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world > 1 or (force and dist.is_initialized()):
        if device.type == "cuda" and world > 1:
            set_bwd_schedule(model, "in_order")
        if impl == "bucketed":
            return BucketedDataParallel(model, bucket_cap_mb=16 if bucket_cap_mb is None else bucket_cap_mb)
        if impl != "torch":
            raise ValueError(f"wrap_ddp: unknown impl {impl!r}")
        ddp = torch.nn.parallel.DistributedDataParallel(
            model, device_ids=[device.index] if device.type == "cuda" else None,
            gradient_as_bucket_view=True, bucket_cap_mb=64 if bucket_cap_mb is None else bucket_cap_mb,
            broadcast_buffers=bool(broadcast_buffers),
            static_graph=bool(static_graph))
        if comm_hook == "world1_none":
            assert world == 1, "the no-communication hook is a world-size-1 diagnostic"
            ddp.register_comm_hook(None, _world1_no_comm_hook)
        return ddp
    return model


def make_train_step(model, optimizer, loss_fn, sw=1e-2, scaler=None, sync_loss=False, train_mode=True):
    """Returns step(x, y) implementing script/train.py:_update (lines 103-116). train_mode=False runs the
    same step in eval mode (dropouts off; the parity tests against the eval-mode reference fixtures)."""

    def step(x, y):
        model.train(train_mode)
        optimizer.zero_grad(set_to_none=True)
        y_pred, sparsity, src_pe, graphs, attns = model(x)
        loss = loss_fn(y_pred, y)
        total = loss + sw * sparsity
        if scaler is not None:
            scaler.scale(total).backward()
            scaler.step(optimizer)
            scaler.update()
        else:
            total.backward()
            optimizer.step()
        return loss.item() if sync_loss else loss.detach()

    return step
