"""Drop-in DisentangledAttn (module/disentangled_attn.py:11-65): same constructor, forward signature,
return tuple and state_dict keys; the relation attention runs in torch.ops.csa.rel_attn_*.
``module.attn_precision = "bf16"`` runs its c2c / PV contractions and their gradients on bf16 MFMA
(d_k = 64; default "fp32", the reference's precision); ``module.bwd_schedule`` as in
csa_amd.module.sbm_attn. linear_layers[0..2] (the self-attention q / k / v) stay packed back to back
from construction on and after every device move (one QKV GEMM)."""
import copy

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import rel_ops
from ..glue import Linear, linear3, pack_linears_, split_heads3

__all__ = ["DisentangledAttn", "transpose_for_scores", "_get_clones"]


def _get_clones(module, N):
    """module/components.py:_get_clones."""
    return nn.ModuleList([copy.deepcopy(module) for _ in range(N)])


def transpose_for_scores(x, num_heads):
    """module/components.py:transpose_for_scores (a strided view; the kernels consume it in place)."""
    x = x.view(*(x.size()[:-1] + (num_heads, -1)))
    return x.permute(0, 2, 1, 3)


class DisentangledAttn(nn.Module):
    def __init__(self, h, d_model, dropout=0.1):
        super().__init__()
        assert d_model % h == 0
        self.d_k = d_model // h
        self.h = h
        self.linear_layers = _get_clones(Linear(d_model, d_model), 4)
        self.attn = None
        self.dropout = nn.Dropout(p=dropout)  # unused, as in the reference
        self.l_linear = _get_clones(Linear(d_model, self.d_k * 4), 2)
        self.t_linear = _get_clones(Linear(d_model, self.d_k * 4), 2)
        self.attn_precision = "fp32"
        self.bwd_schedule = "auto"
        pack_linears_(self.linear_layers[:3])

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        pack_linears_(self.linear_layers[:3])
        return out

    def forward(self, query, key, value, rel_emb, rel, mask):
        if query is key and key is value:  # self-attention (CSE_layer, csa_trans.py:231-233): one QKV GEMM
            query, key, value = split_heads3(linear3(query, self.linear_layers[:3]), self.h)
        else:
            query, key, value = [transpose_for_scores(l(x), self.h)
                                 for l, x in zip(self.linear_layers, (query, key, value))]
        # rel_emb[0]: the (L_q, T_q) embedding tables (the reference stacks them and selects each back out;
        # unbind takes both at once, so the backward is one stack instead of two zero-filled select
        # gradients accumulated into the stack's gradient, per layer)
        tables = rel_emb[0]
        l, t = (tables.unbind(0) if torch.is_tensor(tables) else tables)
        l, t = l.unsqueeze(0), t.unsqueeze(0)  # 1, L, d
        lq, lk = [transpose_for_scores(lin(x), 4) for lin, x in zip(self.l_linear, (l, l))]
        tq, tk = [transpose_for_scores(lin(x), 4) for lin, x in zip(self.t_linear, (t, t))]
        lq = torch.cat([lq, tq], dim=1)  # 1, 8, L, d
        lk = torch.cat([lk, tk], dim=1)
        output = rel_ops.rel_attn(query, key, value, lq, lk, rel, mask, bf16=self.attn_precision == "bf16",
                                  schedule=self.bwd_schedule)
        output = output.permute(0, 2, 1, 3).contiguous()
        output = output.view(*(output.size()[:-2] + (-1,)))
        output = self.linear_layers[-1](output)
        return output, None

    @staticmethod
    def rel_attn(q, k, v, lq, lk, rel, mask):
        return rel_ops.rel_attn(q, k, v, lq, lk, rel, mask)
