"""Drop-in DisentangledAttn (module/disentangled_attn.py:11-65) — see rel_ops for the kernels."""
import torch
import torch.nn as nn

__all__ = ["DisentangledAttn"]


def _get_clones(module, N):
    import copy
    return nn.ModuleList([copy.deepcopy(module) for _ in range(N)])


class DisentangledAttn(nn.Module):
    def __init__(self, h, d_model, dropout=0.1):
        super().__init__()
        assert d_model % h == 0
        self.d_k = d_model // h
        self.h = h
        self.linear_layers = _get_clones(nn.Linear(d_model, d_model), 4)
        self.attn = None
        self.dropout = nn.Dropout(p=dropout)  # unused, as in the reference
        self.l_linear = _get_clones(nn.Linear(d_model, self.d_k * 4), 2)
        self.t_linear = _get_clones(nn.Linear(d_model, self.d_k * 4), 2)

    def forward(self, query, key, value, rel_emb, rel, mask):
        raise NotImplementedError("rel_attn kernels not built yet")
