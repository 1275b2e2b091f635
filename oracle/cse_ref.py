"""ORACLE (test infrastructure only): op-for-op restatement of the CSE disentangled attention.

Restates (paths relative to /root/reference):
* module/disentangled_attn.py:44-65  DisentangledAttn.rel_attn (c2c + gathered p2c + gathered c2p,
                                      scale sqrt(3 d_k), masked_fill -1e9, softmax, @ v)
* module/disentangled_attn.py:23-42  DisentangledAttn.forward (q/k/v/out linears, l_linear/t_linear
                                      relation projections, 4 parent + 4 sibling heads)
* module/csa_trans.py:204-211        CSE.forward rel/mask construction (repeat x4, cat, int64)
* dataset/base_data_set.py:33-36     collate encoding: mask = raw.eq(0), idx = clamp(raw+75, 0, 149)
Backward is torch autograd, as in the reference.
"""
import math

import torch
import torch.nn.functional as F


def transpose_for_scores(x, num_heads):
    """module/components.py:transpose_for_scores (view + permute, non-contiguous)."""
    x = x.view(*(x.size()[:-1] + (num_heads, -1)))
    return x.permute(0, 2, 1, 3)


def rel_attn(q, k, v, lq, lk, rel, mask):
    """module/disentangled_attn.py:44-65. q,k,v (B,H,N,dk); lq,lk (1,H,L,dk); rel (B,H,N,N) int64;
    mask (B,H,N,N) bool."""
    B, H, N, d_k = q.size()
    scale = math.sqrt(d_k * 3)
    c2c = (q @ k.permute(0, 1, 3, 2)) / scale
    p2c = lq @ k.permute(0, 1, 3, 2)  # (B,H,L,N)
    p2c = torch.gather(p2c, 2, rel.transpose(-2, -1)) / scale  # score[x,y] uses rel[y,x]
    c2p = q @ lk.permute(0, 1, 3, 2)  # (B,H,N,L)
    c2p = torch.gather(c2p, 3, rel) / scale  # score[x,y] uses rel[x,y]
    att = (c2c + p2c + c2p).masked_fill(mask == 1, -1e9)
    att = F.softmax(att, dim=-1)
    return att @ v


def build_rel_mask(L, T, L_mask, T_mask):
    """module/csa_trans.py:206-211: (B,N,N) -> rel (B,8,N,N) int64, mask (B,8,N,N) bool."""
    rel = torch.cat([L.unsqueeze(1).repeat(1, 4, 1, 1), T.unsqueeze(1).repeat(1, 4, 1, 1)], dim=1).to(torch.int64)
    mask = torch.cat([L_mask.unsqueeze(1).repeat(1, 4, 1, 1), T_mask.unsqueeze(1).repeat(1, 4, 1, 1)], dim=1)
    return rel, mask


def collate_relations(raw):
    """dataset/base_data_set.py:33-36: returns (idx, mask) from raw signed distances."""
    return torch.clamp(raw + 75, min=0, max=149), raw.eq(0)


def disentangled_attn(x, params, rel_q, rel, mask, h=8):
    """module/disentangled_attn.py:23-42 with query = key = value = x (CSE_layer, csa_trans.py:233).

    params: DisentangledAttn state_dict keys (linear_layers.{0..3}, l_linear.{0,1}, t_linear.{0,1});
    rel_q: (2, L, d_model) = stack(L_q.weight, T_q.weight) (csa_trans.py:196-202)."""
    lin = lambda i, t: F.linear(t, params[f"linear_layers.{i}.weight"], params[f"linear_layers.{i}.bias"])
    q, k, v = [transpose_for_scores(lin(i, x), h) for i in range(3)]
    l = rel_q[0].unsqueeze(0)
    t = rel_q[1].unsqueeze(0)
    ll = lambda n, i, z: F.linear(z, params[f"{n}.{i}.weight"], params[f"{n}.{i}.bias"])
    lq, lk = transpose_for_scores(ll("l_linear", 0, l), 4), transpose_for_scores(ll("l_linear", 1, l), 4)
    tq, tk = transpose_for_scores(ll("t_linear", 0, t), 4), transpose_for_scores(ll("t_linear", 1, t), 4)
    lq = torch.cat([lq, tq], dim=1)
    lk = torch.cat([lk, tk], dim=1)
    out = rel_attn(q, k, v, lq, lk, rel, mask)
    out = out.permute(0, 2, 1, 3).contiguous()
    out = out.view(*(out.size()[:-2] + (-1,)))
    return lin(3, out), None
