"""ORACLE (test infrastructure only): op-for-op torch-CPU restatement of the SBM attention path.

Restates, in the same ATen op order as the reference (so fp32 results agree to the last
few ulps), the following reference code (paths relative to /root/reference):

* module/STE.py:8-19        SampleGraphSparseGraph (Bernoulli sample, hardtanh STE backward)
* module/sbm_attn.py:11-66  SBMAttention.forward
* module/sbm_attn.py:69-87  FullAttention.forward
* module/sbm_attn.py:90-140 Attention (W_q/W_k/W_v, split/combine heads, ff)

Host-supplied uniforms: the reference draws ``torch.bernoulli(tmp)``; on CPU that is
bit-identical to ``torch.rand(tmp.shape) < tmp`` under the same generator state
(verified by tools/gen_golden.py). Every function here therefore takes the uniforms ``u``
explicitly, which is also the contract of the HIP kernel's parity mode.

Backward is torch autograd, exactly as in the reference. Only ``tests/``, ``__graft_entry__``
and ``bench.py``'s cpu_baseline leg may import this module.
"""
import math

import torch
import torch.nn.functional as F

PROJ_KEYS = ("proj.0.weight", "proj.0.bias", "proj.3.weight", "proj.3.bias", "proj.6.weight", "proj.6.bias")


class STESample(torch.autograd.Function):
    """module/STE.py:8-19 with the Bernoulli draw expressed as ``u < p`` (STE.py:13)."""

    @staticmethod
    def forward(ctx, p, u):
        tmp = p.clamp(0.01, 0.99)  # STE.py:11
        A = (u < tmp).to(p.dtype)  # STE.py:13 (torch.bernoulli == rand < p)
        ctx.save_for_backward(A)  # STE.py:14
        return A

    @staticmethod
    def backward(ctx, g):
        (A,) = ctx.saved_tensors
        return F.hardtanh(A * g), None  # STE.py:17-19


def cluster_matrix(cluster_weight, num_head, num_clusters):
    """S = softmax over all k^2 entries of C_h C_h^T (module/sbm_attn.py:37-39)."""
    clusters = cluster_weight.reshape(num_head, num_clusters, -1)
    dist = torch.matmul(clusters, clusters.transpose(-1, -2))
    S = torch.softmax(dist.reshape(num_head, num_clusters ** 2), dim=-1).reshape(num_head, num_clusters, num_clusters)
    return clusters, S


def proj_mlp(x, params, keep0=None, keep1=None, p=0.0):
    """module/sbm_attn.py:22-30: Linear -> Dropout -> ReLU -> Linear -> Dropout -> ReLU -> Linear.

    ``keep0``/``keep1`` are optional pre-scaled dropout multipliers (0 or 1/(1-p)) applied
    after the first/second Linear (eval mode when None); p > 0 instead draws torch's own dropout
    (train mode, the reference's RNG use)."""
    h = F.linear(x, params["proj.0.weight"], params["proj.0.bias"])
    if keep0 is not None:
        h = h * keep0
    elif p > 0.0:
        h = F.dropout(h, p, True)
    h = F.relu(h)
    h = F.linear(h, params["proj.3.weight"], params["proj.3.bias"])
    if keep1 is not None:
        h = h * keep1
    elif p > 0.0:
        h = F.dropout(h, p, True)
    h = F.relu(h)
    return F.linear(h, params["proj.6.weight"], params["proj.6.bias"])


def sbm_attention(Q, K, V, mask, params, u, num_clusters, attn_keep=None, proj_keep=None, attn_p=0.0, proj_p=0.0):
    """module/sbm_attn.py:32-66. Returns (X, sparsity, graph, attn).

    Q,K,V: (B,H,N,d) fp32; mask: (B,M) float, 1.0 = padded key; params: dict with the
    reference state_dict keys ('layer.weight', 'proj.*'); u: (B,H,N,M) uniforms.
    attn_keep: optional (B,H,N,M) pre-scaled attention-dropout multiplier (sbm_attn.py:63);
    proj_keep: optional dict {q0,q1,k0,k1} of pre-scaled proj-dropout multipliers.
    attn_p / proj_p > 0 (without keep tensors): torch's own dropout draws (train mode)."""
    b, h, n, d = Q.shape
    m = V.shape[2]
    clusters, S = cluster_matrix(params["layer.weight"], h, num_clusters)
    S = S.unsqueeze(0).repeat((b, 1, 1, 1))  # sbm_attn.py:39
    pk = proj_keep or {}
    Qhat = torch.sigmoid(torch.matmul(proj_mlp(Q, params, pk.get("q0"), pk.get("q1"), proj_p),
                                      clusters.transpose(-1, -2)))
    Khat = torch.sigmoid(torch.matmul(proj_mlp(K, params, pk.get("k0"), pk.get("k1"), proj_p),
                                      clusters.transpose(-1, -2)))
    expA = torch.matmul(Qhat, torch.matmul(S, Khat.transpose(-1, -2)))  # sbm_attn.py:55
    graph = STESample.apply(expA, u)  # sbm_attn.py:57
    dot = torch.matmul(Q, K.transpose(-2, -1)) / math.sqrt(d)  # sbm_attn.py:59-60
    dot = dot.masked_fill(mask[:, None, None, :] == 1, float("-inf"))  # sbm_attn.py:61
    attn = F.normalize(torch.softmax(dot, dim=-1) * graph, p=1, dim=-1)  # sbm_attn.py:62
    a = attn if attn_keep is None else attn * attn_keep
    if attn_keep is None and attn_p > 0.0:
        a = F.dropout(attn, attn_p, True)
    X = torch.matmul(a, V)  # sbm_attn.py:63
    sparsity = torch.sum(graph, dim=(0, -1, -2)) / (b * n * m)  # sbm_attn.py:64
    return X, sparsity, graph, attn


def full_attention(Q, K, V, mask, attn_keep=None, attn_p=0.0):
    """module/sbm_attn.py:77-87 (dense ablation). Returns (X, None, mask, attn)."""
    d = Q.shape[-1]
    dot = torch.matmul(Q, K.transpose(-2, -1)) / math.sqrt(d)
    dot = dot.masked_fill(mask[:, None, None, :] == 1, float("-inf"))
    attn = F.normalize(torch.softmax(dot, dim=-1), p=1, dim=-1)
    a = attn if attn_keep is None else attn * attn_keep
    if attn_keep is None and attn_p > 0.0:
        a = F.dropout(attn, attn_p, True)
    X = torch.matmul(a, V)
    return X, None, mask, attn


def split_heads(X, num_head, head_dim):
    """module/sbm_attn.py:137-140 (a non-contiguous view)."""
    return X.reshape(X.size(0), X.size(1), num_head, head_dim).transpose(1, 2)


def combine_heads(X, num_head, head_dim):
    """module/sbm_attn.py:132-135."""
    X = X.transpose(1, 2)
    return X.reshape(X.size(0), X.size(1), num_head * head_dim)


def attention_layer(X, mask, params, u, num_head, head_dim, num_clusters, full_att=False, attn_p=0.0, proj_p=0.0):
    """module/sbm_attn.py:113-130 (Attention.forward with attn = SBM or Full).

    params holds the Attention state_dict keys: W_q/W_k/W_v/ff .weight/.bias and
    attn.layer.weight / attn.proj.* (the SBMAttention submodule)."""
    Q = split_heads(F.linear(X, params["W_q.weight"], params["W_q.bias"]), num_head, head_dim)
    K = split_heads(F.linear(X, params["W_k.weight"], params["W_k.bias"]), num_head, head_dim)
    V = split_heads(F.linear(X, params["W_v.weight"], params["W_v.bias"]), num_head, head_dim)
    # the reference forces fp32 here (sbm_attn.py:120-126); an fp64 X (the error-budget runs of
    # tools/gen_golden.py) stays fp64
    cd = torch.float64 if X.dtype == torch.float64 else torch.float32
    if full_att:
        out, sparsity, graph, attn = full_attention(Q.to(cd), K.to(cd), V.to(cd), mask.to(cd), attn_p=attn_p)
    else:
        sp = {k[len("attn."):]: v for k, v in params.items() if k.startswith("attn.")}
        out, sparsity, graph, attn = sbm_attention(Q.to(cd), K.to(cd), V.to(cd), mask.to(cd), sp, u, num_clusters,
                                                   attn_p=attn_p, proj_p=proj_p)
    out = combine_heads(out, num_head, head_dim)
    return F.linear(out, params["ff.weight"], params["ff.bias"]), sparsity, graph, attn
