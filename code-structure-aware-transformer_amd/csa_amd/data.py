"""Synthetic AST batches with the reference's relation encoding (no datasets offline).

The real pipeline parses code with tree-sitter and builds, per AST truncated to ``max_size``
nodes in pre-order (my_ast.py:129-143):

* L (ancestor/descendant relation): for every ancestor a and descendant c on a root-to-leaf
  path, L[a,c] = depth(c)-depth(a) and L[c,a] = -(depth(c)-depth(a)) (my_ast.py:223-263);
* T (sibling relation): for siblings i before j among one parent's children,
  T[i,j] = j_idx - i_idx and T[j,i] = -(j_idx - i_idx) (my_ast.py:232-270);
* zeros elsewhere (diagonal, unrelated pairs, padding);

and the collate step encodes them as ``mask = raw.eq(0)`` and ``idx = clamp(raw + 75, 0, 149)``
(dataset/base_data_set.py:33-36). This module generates random trees (uniform parent
attachment, at most 6 children per node) and produces exactly that encoding, vectorised
in numpy. The hot-path kernels consume the uint8 (B,N,N) relation/mask planes directly
(head stride 0), instead of the reference's repeated int64 (B,8,N,N) copies
(module/csa_trans.py:206-211).
"""
import numpy as np

PAD, UNK, BOS, EOS = 0, 1, 2, 3  # utils/vocab.py:10-13
REL_OFFSET, REL_MAX = 75, 149  # dataset/base_data_set.py:35-36


def random_tree(n, rng, max_children=6):
    """Random rooted tree with n nodes; returns parent[] in PRE-ORDER numbering (root = 0)."""
    parent = np.full(n, -1, dtype=np.int64)
    nchild = np.zeros(n, dtype=np.int64)
    children = [[] for _ in range(n)]
    for v in range(1, n):
        while True:
            p = int(rng.integers(0, v))
            if nchild[p] < max_children:
                break
        parent[v] = p
        nchild[p] += 1
        children[p].append(v)
    # pre-order renumbering (children in insertion order), as MyAst numbers nodes
    order = []
    stack = [0]
    while stack:
        v = stack.pop()
        order.append(v)
        stack.extend(reversed(children[v]))
    newid = np.empty(n, dtype=np.int64)
    newid[np.array(order)] = np.arange(n)
    par = np.full(n, -1, dtype=np.int64)
    for v in range(1, n):
        par[newid[v]] = newid[parent[v]]
    kids = [[] for _ in range(n)]
    for v in range(1, n):  # pre-order ids are increasing along sibling order
        kids[par[v]].append(v)
    return par, kids


def relation_matrices(par, kids, max_size):
    """Raw signed L/T matrices (max_size x max_size, float32) of one tree (my_ast.py:198-273)."""
    n = len(par)
    L = np.zeros((max_size, max_size), dtype=np.float32)
    T = np.zeros((max_size, max_size), dtype=np.float32)
    depth = np.zeros(n, dtype=np.int64)
    for v in range(1, n):
        depth[v] = depth[par[v]] + 1
    for c in range(1, n):
        a = par[c]
        while a >= 0:
            dist = depth[c] - depth[a]
            L[a, c] = dist
            L[c, a] = -dist
            a = par[a]
    for p in range(n):
        ch = kids[p]
        for i in range(len(ch)):
            for j in range(i + 1, len(ch)):
                T[ch[i], ch[j]] = j - i
                T[ch[j], ch[i]] = -(j - i)
    return L, T


def collate_relations(raw):
    """dataset/base_data_set.py:33-36 -> (idx uint8, mask bool)."""
    mask = raw == 0
    idx = np.clip(raw + REL_OFFSET, 0, REL_MAX).astype(np.uint8)
    return idx, mask


def relation_planes(parents, n_nodes, max_size, nthreads=None):
    """Native (csrc/csa_host.cpp: csa_ast_relations) relation planes of a batch of pre-order trees:
    parents (B, max_size) int32 (parent[v] < v, root -1), n_nodes (B,) -> L, T (B,N,N) uint8 relation
    indices and L_mask, T_mask (B,N,N) bool, identical to relation_matrices + collate_relations."""
    import ctypes
    import os
    from ._lib import check, lib
    parents = np.ascontiguousarray(parents, dtype=np.int32)
    n_nodes = np.ascontiguousarray(n_nodes, dtype=np.int32)
    B = parents.shape[0]
    out = [np.empty((B, max_size, max_size), np.uint8) for _ in range(4)]
    p = lambda a: ctypes.c_void_p(a.ctypes.data)
    nt = nthreads or min(16, os.cpu_count() or 1)
    check(lib().csa_ast_relations(p(parents), p(n_nodes), B, max_size, *(p(o) for o in out), nt),
          "csa_ast_relations")
    L, T, Lm, Tm = out
    return L, T, Lm.view(bool), Tm.view(bool)


def collect_fn(batch, nthreads=None):
    """BaseASTDataSet.collect_fn (dataset/base_data_set.py:20-75) for the accelerated path: `batch` is a
    list of (item, _) with item dicts holding the preprocessed per-AST tensors -- src_seq, tgt_seq,
    target (equal lengths across the batch), raw fp32 L / T (N, N) from split_matrices.npz, num_node.
    Returns (namespace, target) like the reference's (Data, target), with the relation planes encoded
    by the native csa_collate_relations as the uint8 L, T and bool L_mask, T_mask the kernels read
    (idx = clamp(raw + 75, 0, 149), mask = raw == 0). The ablation-only fields of the reference
    (adj, tree_pos, triplet) are not on this path and are not collated."""
    import ctypes
    import os
    from types import SimpleNamespace

    import torch
    from ._lib import check, lib
    items = [it for it, _ in batch]
    stack = lambda k: torch.stack([torch.as_tensor(it[k]) for it in items], 0)
    Lr = stack("L").to(torch.float32).contiguous()
    Tr = stack("T").to(torch.float32).contiguous()
    if Lr.shape != Tr.shape:
        raise ValueError("L and T must have the same shape")
    outs = [torch.empty(Lr.shape, dtype=torch.uint8) for _ in range(4)]
    nt = nthreads or min(16, os.cpu_count() or 1)
    check(lib().csa_collate_relations(ctypes.c_void_p(Lr.data_ptr()), ctypes.c_void_p(Tr.data_ptr()), Lr.numel(),
                                      *(ctypes.c_void_p(o.data_ptr()) for o in outs), nt), "csa_collate_relations")
    L, T, Lm, Tm = outs
    target = stack("target")
    data = SimpleNamespace(src_seq=stack("src_seq"), tgt_seq=stack("tgt_seq"), target=target, L=L, T=T,
                           L_mask=Lm.view(torch.bool), T_mask=Tm.view(torch.bool),
                           num_node=torch.tensor([int(it["num_node"]) for it in items]))
    return data, target


def synthetic_batch(batch, max_size=150, seed=1, min_nodes=None, max_nodes=None, src_vocab=10000,
                    tgt_vocab=20000, max_tgt_len=50, native=True):
    """A batch of synthetic ASTs. Returns a dict of numpy arrays:

    L, T (B,N,N) uint8 relation indices; L_mask, T_mask (B,N,N) bool; src_mask (B,N) bool
    (True = padded node); num_node (B,); src_seq (B,N) int64 in [2, src_vocab) with PAD beyond
    num_node; tgt_seq/target (B, max_tgt_len-1) int64 (BOS ... EOS, PAD). Relation planes come from
    the native builder (relation_planes) unless native=False."""
    rng = np.random.default_rng(seed)
    lo = max_size if min_nodes is None else min_nodes
    hi = max_size if max_nodes is None else max_nodes
    L = np.zeros((batch, max_size, max_size), np.uint8)
    T = np.zeros_like(L)
    Lm = np.zeros((batch, max_size, max_size), bool)
    Tm = np.zeros_like(Lm)
    nn = np.zeros(batch, np.int64)
    src = np.zeros((batch, max_size), np.int64)
    tgt = np.zeros((batch, max_tgt_len), np.int64)
    parents = np.full((batch, max_size), -1, np.int32)
    for b in range(batch):
        n = int(rng.integers(lo, hi + 1))
        par, _ = random_tree(n, rng)
        parents[b, :n] = par
        nn[b] = n
        src[b, :n] = rng.integers(2, src_vocab, n)
        tl = int(rng.integers(5, max_tgt_len - 1))
        tgt[b, 0] = BOS
        tgt[b, 1:tl + 1] = rng.integers(4, tgt_vocab, tl)
        tgt[b, tl + 1] = EOS
    if native:
        L, T, Lm, Tm = relation_planes(parents, nn, max_size)
    else:  # the Python restatement (tests compare the two)
        for b in range(batch):
            n = int(nn[b])
            kids = [[] for _ in range(n)]
            for v in range(1, n):
                kids[parents[b, v]].append(v)
            rl, rt = relation_matrices(parents[b, :n].astype(np.int64), kids, max_size)
            L[b], Lm[b] = collate_relations(rl)
            T[b], Tm[b] = collate_relations(rt)
    src_mask = np.arange(max_size)[None, :] >= nn[:, None]
    return dict(L=L, T=T, L_mask=Lm, T_mask=Tm, num_node=nn, src_seq=src, src_mask=src_mask,
                tgt_seq=tgt[:, :-1], target=tgt[:, 1:])
