"""Round-5 BucketedDataParallel (commit 90d2cd6), kept only for the same-box train-step A/B of tools/runs/train_reducer_ab.py."""
import torch
import torch.distributed as dist

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
    that order (DDP's bucket rebuild), so later steps start all-reducing as early as possible."""

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
            if self._pending[b] == 0 and self._rebuilt:
                self._reduce(b)
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
        if not self._rebuilt:  # first step: adopt the observed arrival order, then reduce everything
            seen = set(self._arrival)
            order = self._arrival + [i for i in reversed(range(len(self._params))) if i not in seen]
            self._layout(order)
            self._rebuilt = True
            self._arrival = []
            for b in range(len(self._buckets)):
                self._reduce(b)
        else:
            for b in range(len(self._buckets)):
                if self._pending[b] > 0:
                    self._reduce(b)
        for b, w in self._works:
            w.wait()
            if self._op == dist.ReduceOp.SUM:
                lo, hi = self._spans[b]
                self.flat[lo:hi].div_(self.world)
        self._works = []
        self._pending = [len(idx) for idx in self._buckets]
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
            self._works, self._queued = [], False
            self._pending = [len(idx) for idx in self._buckets]
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


