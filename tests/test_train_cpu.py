"""CPU tests of the training-step machinery (script/train.py:103-116): loss, optimizer, DDP (gloo, 2 ranks)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import multiprocessing as mp


def test_label_smoothing_matches_reference(golden):
    from csa_amd.model import label_smoothing_loss
    z = golden("label_smoothing")
    logits = torch.from_numpy(z["logits"]).requires_grad_(True)
    x = torch.log(torch.softmax(logits, -1))
    loss = label_smoothing_loss(x, torch.from_numpy(z["target"]))
    np.testing.assert_allclose(loss.item(), z["loss"][0], rtol=1e-6)
    loss.backward()
    np.testing.assert_allclose(logits.grad.numpy(), z["dlogits"], rtol=1e-5, atol=1e-7)


def test_adamw_matches_reference(golden):
    from csa_amd.train import AdamW
    z = golden("adamw_nobias")
    a, b = torch.nn.Parameter(torch.from_numpy(z["p0"])), torch.nn.Parameter(torch.from_numpy(z["p1"]))
    opt = AdamW([a, b], lr=1e-2, correct_bias=False)
    for i in range(3):
        a.grad, b.grad = torch.from_numpy(z["g0"][i]), torch.from_numpy(z["g1"][i])
        opt.step()
    np.testing.assert_allclose(a.detach().numpy(), z["out0"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(b.detach().numpy(), z["out1"], rtol=1e-6, atol=1e-7)


def test_synthetic_relations_follow_reference_encoding():
    from csa_amd.data import synthetic_batch
    sb = synthetic_batch(3, max_size=40, seed=3, min_nodes=10, max_nodes=40)
    for b in range(3):
        n = sb["num_node"][b]
        L = sb["L"][b].astype(int) - 75
        T = sb["T"][b].astype(int) - 75
        # antisymmetric raw distances, zero (=masked) diagonal and padding (my_ast.py:252-263)
        assert np.array_equal(L, -L.T) and np.array_equal(T, -T.T)
        assert np.all(sb["L_mask"][b] == (L == 0)) and np.all(sb["T_mask"][b] == (T == 0))
        assert np.all(np.diag(sb["L_mask"][b])) and np.all(sb["L_mask"][b][n:, :])
        assert (L[0, 1:n] > 0).all()  # the root is an ancestor of every node
        assert sb["src_mask"][b].sum() == 40 - n


class Tiny(torch.nn.Module):
    """Stand-in with the CSATrans output signature (out, sparsity, pe, graphs, attns) around a packed QKV
    triple, as csa_amd.module.sbm_attn.Attention has: glue.Linear q / k / v packed back to back at
    construction (pack_linears_), one GEMM over the packed memory (glue.linear3 -> _LinearPackedFn)."""

    def __init__(self, packed=True):
        super().__init__()
        from csa_amd.glue import Linear, pack_linears_
        self.packed = packed
        self.q, self.k, self.v = Linear(6, 6), Linear(6, 6), Linear(6, 6)
        self.lin = torch.nn.Linear(6, 5)
        self.gate = torch.nn.Linear(6, 1)
        if packed:
            pack_linears_((self.q, self.k, self.v))

    def _apply(self, fn, *args, **kwargs):
        from csa_amd.glue import pack_linears_
        out = super()._apply(fn, *args, **kwargs)
        if self.packed:
            pack_linears_((self.q, self.k, self.v))
        return out

    def forward(self, x):
        if self.packed:
            from csa_amd.glue import linear3
            q, k, v = linear3(x, (self.q, self.k, self.v)).split(6, -1)
        else:  # the plain per-layer reference
            q, k, v = (torch.nn.functional.linear(x, l.weight, l.bias) for l in (self.q, self.k, self.v))
        h = q * torch.sigmoid(k) + v
        out = torch.log(torch.softmax(self.lin(h), -1))
        return out, torch.sigmoid(self.gate(x)).mean(), None, [], []


def _packed_storage(model):
    ws = [model.q.weight, model.k.weight, model.v.weight]
    return len({w.untyped_storage().data_ptr() for w in ws}) == 1


def _batch(rank, i):
    g = torch.Generator().manual_seed(100 + 10 * i + rank)  # per-rank shard (set_seed(seed + rank))
    return torch.randn(4, 3, 6, generator=g), torch.randint(1, 5, (4, 3), generator=g)


def _worker(rank, world, port, q, cases, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from csa_amd.model import label_smoothing_loss
    from csa_amd.train import AdamW, BucketedDataParallel, init_distributed, make_train_step, wrap_ddp
    r, w, _, dev = init_distributed()
    out = {}
    for impl, cap_mb in cases:
        torch.manual_seed(0 if rank == 0 else 1 + rank)  # different replicas: the wrapper broadcasts rank 0's
        model = Tiny()
        assert _packed_storage(model)
        ddp = wrap_ddp(model, dev, impl=impl, bucket_cap_mb=cap_mb)
        assert isinstance(ddp, BucketedDataParallel if impl == "bucketed" else torch.nn.parallel.DistributedDataParallel)
        opt = AdamW(model.parameters(), lr=1e-3, correct_bias=False)
        step = make_train_step(ddp, opt, label_smoothing_loss, sw=1e-2)
        grads, weights = [], []
        for i in range(steps):
            step(*_batch(rank, i))
            assert _packed_storage(model)  # the reducer and the optimizer kept the packed storages
            grads.append([p.grad.numpy().copy() for p in model.parameters()])
            weights.append([p.detach().numpy().copy() for p in model.parameters()])
        # local accumulation under no_sync, then one synchronised backward over the accumulated gradients
        opt.zero_grad(set_to_none=True)
        with ddp.no_sync():
            o, sp, *_ = ddp(_batch(rank, 7)[0])
            (label_smoothing_loss(o, _batch(rank, 7)[1]) + 1e-2 * sp).backward()
        o, sp, *_ = ddp(_batch(rank, 8)[0])
        (label_smoothing_loss(o, _batch(rank, 8)[1]) + 1e-2 * sp).backward()
        grads.append([p.grad.numpy().copy() for p in model.parameters()])
        out[(impl, cap_mb)] = (grads, weights)
    q.put((rank, out))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_ddp_two_ranks_average_gradients():
    """2-rank gloo data-parallel steps through the packed QKV path (parameters packed before the wrapper is
    built, one GEMM forward, three gradient views of one GEMM backward): the bucketed reducer (one bucket, and
    a tiny bucket cap giving one bucket per few parameters) and torch DDP. Step 1 == the mean of the per-rank
    single-process gradients against plain unpacked per-rank GEMMs (DDP semantics) from rank 0's initial
    weights (the wrapper's broadcast); every step's gradients and weights, and a no_sync accumulation
    followed by a synchronised backward, are bit-identical between the bucketed reducer and DDP."""
    from csa_amd.model import label_smoothing_loss
    cases = [("torch", 64), ("bucketed", 64), ("bucketed", 1e-4)]
    steps = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, cases, steps)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single-process per-rank gradients of step 1 from rank 0's initial weights
    ref = []
    for rank in range(2):
        torch.manual_seed(0)
        m = Tiny(packed=False)  # same initial values, plain per-layer GEMMs
        x, y = _batch(rank, 0)
        out, sp, *_ = m(x)
        (label_smoothing_loss(out, y) + 1e-2 * sp).backward()
        ref.append([p.grad.clone() for p in m.parameters()])
    mean = [(a + b) / 2 for a, b in zip(*ref)]
    for case in cases:
        for rank in range(2):
            for gd, gm in zip(res[rank][case][0][0], mean):
                np.testing.assert_allclose(gd, gm.numpy(), rtol=1e-5, atol=1e-6)
            for s in range(steps):  # replicas stay identical after every step
                for wa, wb in zip(res[0][case][1][s], res[1][case][1][s]):
                    np.testing.assert_array_equal(wa, wb)
    for case in cases[1:]:
        for rank in range(2):
            for ga, gb in zip(res[rank][case][0], res[rank][cases[0]][0]):  # steps + the no_sync round
                for x, y in zip(ga, gb):
                    np.testing.assert_array_equal(x, y)
            for wa, wb in zip(res[rank][case][1], res[rank][cases[0]][1]):
                for x, y in zip(wa, wb):
                    np.testing.assert_array_equal(x, y)


class Branchy(torch.nn.Module):
    """Two branches a / b plus a shared trunk; forward(x, use) runs the branches named in `use` in that order, so
    ranks can leave different parameters unused and see different gradient arrival orders."""

    def __init__(self):
        super().__init__()
        self.trunk = torch.nn.Linear(6, 6)
        self.a1, self.a2 = torch.nn.Linear(6, 6), torch.nn.Linear(6, 6)
        self.b1, self.b2 = torch.nn.Linear(6, 6), torch.nn.Linear(6, 6)
        self.head = torch.nn.Linear(6, 3)

    def forward(self, x, use):
        h = torch.tanh(self.trunk(x))
        for br in use:
            h = h + torch.tanh(getattr(self, br + "2")(torch.tanh(getattr(self, br + "1")(h))))
        return self.head(h)


def _branchy_use(rank, i):
    # rank 0 leaves branch b unused on even steps, rank 1 leaves branch a unused; the order of the branches
    # (hence the gradient arrival order) also differs between the ranks
    if rank == 0:
        return ("a",) if i % 2 == 0 else ("a", "b")
    return ("b",) if i % 2 == 0 else ("b", "a")


def _worker_unused(rank, world, port, q, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    from csa_amd.train import BucketedDataParallel, init_distributed
    init_distributed()
    torch.manual_seed(0)
    model = Branchy()
    ddp = BucketedDataParallel(model, bucket_cap_mb=40 * 4 / 2 ** 20)  # ~40 floats per bucket: many buckets
    grads = []
    for i in range(steps):
        for p in model.parameters():
            p.grad = None
        g = torch.Generator().manual_seed(50 + 7 * i + rank)
        x, y = torch.randn(5, 6, generator=g), torch.randn(5, 3, generator=g)
        ((ddp(x, _branchy_use(rank, i)) - y) ** 2).sum().backward()
        grads.append([p.grad.numpy().copy() for p in model.parameters()])
    # a backward that raises part-way through (before the reducer has finished its first layout on a fresh
    # wrapper), then normal steps on the same wrapper
    torch.manual_seed(0)
    m2 = Branchy()
    d2 = BucketedDataParallel(m2, bucket_cap_mb=40 * 4 / 2 ** 20)
    g = torch.Generator().manual_seed(99)
    x, y = torch.randn(5, 6, generator=g), torch.randn(5, 3, generator=g)
    out = d2(x, ("a", "b"))

    def boom(grad):
        raise RuntimeError("injected")
    h = torch.tanh(m2.trunk(x))
    raised = False
    try:
        out.register_hook(lambda g_: g_)  # the head's gradients arrive, then the trunk path raises
        h2 = d2.module.a1.weight * 1.0
        h2.register_hook(boom)
        (((out - y) ** 2).sum() + h2.sum()).backward()
    except RuntimeError as e:
        raised = "injected" in str(e)
    after = []
    for i in range(2):
        for p in m2.parameters():
            p.grad = None
        g = torch.Generator().manual_seed(50 + 7 * i + rank)
        x, y = torch.randn(5, 6, generator=g), torch.randn(5, 3, generator=g)
        ((d2(x, _branchy_use(rank, i)) - y) ** 2).sum().backward()
        after.append([p.grad.numpy().copy() for p in m2.parameters()])
    q.put((rank, grads, raised, after))
    dist.barrier()
    dist.destroy_process_group()


def test_bucketed_reducer_ranks_with_different_unused_parameters():
    """2-rank gloo: the ranks leave DIFFERENT parameters unused and see different gradient arrival orders, over
    many small buckets. Every rank adopts rank 0's bucket layout and issues the bucket all-reduces in index order,
    so each gradient is the mean of the per-rank gradients (an unused parameter contributes zero, DDP's
    find_unused_parameters); a wrapper whose first backward raised part-way reduces correctly afterwards."""
    steps = 4
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_unused, args=(r, 2, port, q, steps)) for r in range(2)]
    for p in procs:
        p.start()
    res = {}
    for _ in range(2):
        rank, grads, raised, after = q.get(timeout=180)
        res[rank] = (grads, raised, after)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0

    def ref_grads(i):
        per_rank = []
        for rank in range(2):
            torch.manual_seed(0)
            m = Branchy()
            g = torch.Generator().manual_seed(50 + 7 * i + rank)
            x, y = torch.randn(5, 6, generator=g), torch.randn(5, 3, generator=g)
            ((m(x, _branchy_use(rank, i)) - y) ** 2).sum().backward()
            per_rank.append([torch.zeros_like(p) if p.grad is None else p.grad for p in m.parameters()])
        return [(a + b) / 2 for a, b in zip(*per_rank)]

    for i in range(steps):
        # the weights never change (no optimizer), so every step's reference starts from the same parameters
        ref = ref_grads(i)
        for rank in range(2):
            for got, want in zip(res[rank][0][i], ref):
                np.testing.assert_allclose(got, want.numpy(), rtol=1e-6, atol=1e-7)
    for rank in range(2):
        assert res[rank][1], "the injected error did not propagate"
        for i in range(2):
            for got, want in zip(res[rank][2][i], ref_grads(i)):
                np.testing.assert_allclose(got, want.numpy(), rtol=1e-6, atol=1e-7)


def _reference_label_smoothing(x, target, padding_idx, smoothing):
    """utils/label_smooth.py:24-40 restated (materialised true_dist + KLDiv(sum) / ntokens)."""
    x = x.contiguous().view(-1, x.size(-1))
    ntokens = (target != 0).sum()
    t = target.contiguous().view(-1)
    td = torch.full_like(x, smoothing / (x.size(1) - 2))
    td.scatter_(1, t.unsqueeze(1), 1.0 - smoothing)
    td[:, padding_idx] = 0
    td[t == padding_idx] = 0
    return torch.nn.functional.kl_div(x, td, reduction="sum") / ntokens


@pytest.mark.parametrize("case,smoothing", [("label_smoothing", 0.0), ("label_smoothing_s01", 0.1)])
def test_label_smoothing_module_matches_reference_golden(golden, case, smoothing):
    from csa_amd.model import LabelSmoothing
    z = golden(case)
    logits = torch.from_numpy(z["logits"]).requires_grad_(True)
    x = torch.log(torch.softmax(logits, -1))
    loss = LabelSmoothing(0, smoothing)(x, torch.from_numpy(z["target"]))
    np.testing.assert_allclose(loss.item(), z["loss"][0], rtol=1e-6)
    loss.backward()
    np.testing.assert_allclose(logits.grad.numpy(), z["dlogits"], rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("smoothing", [0.0, 0.1])
def test_label_smoothing_nan_semantics_of_underflowed_logprobs(smoothing):
    """kl_div's 0 * (-inf) = NaN where true_dist is 0, +inf where it is > 0 (reference behaviour)."""
    from csa_amd.model import LabelSmoothing
    g = torch.Generator().manual_seed(9)
    x = torch.log_softmax(torch.randn(2, 4, 11, generator=g), -1)
    target = torch.randint(2, 11, (2, 4), generator=g)
    target[1, 3] = 0
    cases = []
    a = x.clone(); a[0, 1, 0] = float("-inf"); cases.append(a)  # padding column (td = 0)
    b = x.clone(); b[1, 3, 5] = float("-inf"); cases.append(b)  # padded row
    c = x.clone(); c[0, 0, target[0, 0]] = float("-inf"); cases.append(c)  # at the target: +inf
    for xx in cases:
        mine = LabelSmoothing(0, smoothing)(xx, target).item()
        ref = _reference_label_smoothing(xx, target, 0, smoothing).item()
        assert (np.isnan(mine) and np.isnan(ref)) or mine == pytest.approx(ref, rel=1e-6), (mine, ref)


def test_native_relation_planes_match_python_restatement():
    """csa_ast_relations (csrc/csa_host.cpp) == relation_matrices + collate_relations
    (my_ast.py:198-273, dataset/base_data_set.py:33-36), bit-exact, incl. 1-node and deep trees."""
    from csa_amd.data import synthetic_batch
    for kw in (dict(batch=6, max_size=150, seed=5, min_nodes=1, max_nodes=150),
               dict(batch=3, max_size=40, seed=6, min_nodes=40, max_nodes=40)):
        a = synthetic_batch(**kw)
        b = synthetic_batch(native=False, **kw)
        for k in ("L", "T", "L_mask", "T_mask", "src_seq", "tgt_seq"):
            assert np.array_equal(a[k], b[k]), k


def test_native_relation_planes_reject_malformed_tree():
    from csa_amd._lib import CsaError
    from csa_amd.data import relation_planes
    par = np.full((1, 8), -1, np.int32)
    par[0, 1:4] = [0, 2, 1]  # node 2's parent 2 is not < 2
    with pytest.raises(CsaError, match="pre-order"):
        relation_planes(par, np.array([4]), 8)


def test_native_relation_planes_match_reference_my_ast(golden):
    """F2 pinned to the reference: csa_ast_relations (native) and the Python restatement vs
    MyAst.__get_matrices + BaseASTDataSet.collect_fn run on the same trees, including trees longer
    than max_size (MyAst.__sub_tree truncation) and 1-node trees (tests/golden/ast_relations.npz)."""
    from csa_amd.data import relation_planes
    z = golden("ast_relations")
    L, T, Lm, Tm = relation_planes(z["parents"], z["n_nodes"], 150)
    np.testing.assert_array_equal(L, z["L"])
    np.testing.assert_array_equal(T, z["T"])
    np.testing.assert_array_equal(Lm, z["L_mask"])
    np.testing.assert_array_equal(Tm, z["T_mask"])


def test_native_collect_fn_matches_reference_encoding(golden):
    """csa_amd.data.collect_fn (native csa_collate_relations) on raw L / T matrices rebuilt from the
    fixture's trees reproduces the reference collate output bit for bit."""
    from csa_amd.data import collect_fn, random_tree, relation_matrices  # noqa: F401
    z = golden("ast_relations")
    batch = []
    for b in range(len(z["n_nodes"])):
        n = int(z["n_nodes"][b])
        par = z["parents"][b, :n].astype(np.int64)
        kids = [[] for _ in range(n)]
        for v in range(1, n):
            kids[par[v]].append(v)
        rl, rt = relation_matrices(par, kids, 150)
        batch.append(({"L": torch.from_numpy(rl), "T": torch.from_numpy(rt), "src_seq": torch.zeros(150, dtype=torch.long),
                       "tgt_seq": torch.zeros(49, dtype=torch.long), "target": torch.zeros(49, dtype=torch.long),
                       "num_node": n}, None))
    data, target = collect_fn(batch)
    np.testing.assert_array_equal(data.L.numpy(), z["L"])
    np.testing.assert_array_equal(data.T.numpy(), z["T"])
    np.testing.assert_array_equal(data.L_mask.numpy(), z["L_mask"])
    np.testing.assert_array_equal(data.T_mask.numpy(), z["T_mask"])
    assert data.num_node.tolist() == z["n_nodes"].tolist() and target.shape == (len(batch), 49)
    # the clamp edges: raw distances beyond +-74 saturate to 0 / 149
    raw = torch.tensor([[-200.0, -75.0, -74.0, 0.0], [1.0, 74.0, 75.0, 300.0]])
    d2, _ = collect_fn([({"L": raw, "T": -raw, "src_seq": torch.zeros(1), "tgt_seq": torch.zeros(1),
                          "target": torch.zeros(1), "num_node": 1}, None)])
    assert d2.L.tolist() == [[[0, 0, 1, 75], [76, 149, 149, 149]]]
    assert d2.L_mask.tolist() == [[[False, False, False, True], [False] * 4]]


from hypothesis import given, settings  # noqa: E402
from hypothesis import strategies as st  # noqa: E402


@settings(max_examples=40, deadline=None, derandomize=True)
@given(sizes=st.lists(st.integers(1, 150), min_size=1, max_size=4), max_children=st.integers(1, 9),
       seed=st.integers(0, 2 ** 31 - 1))
def test_native_relation_planes_property(sizes, max_children, seed):
    """csa_ast_relations vs the Python restatement of my_ast.py:198-273 + collate on random trees (any
    branching, sizes 1..150): bit-exact; L antisymmetric around 75 away from the clamp (|raw| >= 75
    saturates to 0 / 149, dataset/base_data_set.py:35), diagonal masked."""
    from csa_amd.data import collate_relations, random_tree, relation_matrices, relation_planes
    rng = np.random.default_rng(seed)
    B, N = len(sizes), 150
    parents = np.full((B, N), -1, np.int32)
    want = []
    for b, n in enumerate(sizes):
        par, kids = random_tree(n, rng, max_children=max_children)
        parents[b, :n] = par
        rl, rt = relation_matrices(par, kids, N)
        want.append((collate_relations(rl), collate_relations(rt)))
    L, T, Lm, Tm = relation_planes(parents, np.array(sizes, np.int32), N)
    for b in range(B):
        (wl, wlm), (wt, wtm) = want[b]
        np.testing.assert_array_equal(L[b], wl)
        np.testing.assert_array_equal(T[b], wt)
        np.testing.assert_array_equal(Lm[b], wlm)
        np.testing.assert_array_equal(Tm[b], wtm)
        assert np.all(np.diag(Lm[b])) and np.all(np.diag(Tm[b]))
        li = L[b].astype(int) - 75
        inner = (np.abs(li) < 74) & (np.abs(li.T) < 74)
        np.testing.assert_array_equal(li[inner], -li.T[inner])
