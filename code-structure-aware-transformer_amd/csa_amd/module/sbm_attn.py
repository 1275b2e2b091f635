"""Drop-in SBMAttention / FullAttention / Attention (module/sbm_attn.py:11-140) on fused HIP kernels.

Same constructor signatures, forward signatures, return tuples and state_dict keys as the
reference, so module/sbm_model.py and module/csa_trans.py use them unchanged and reference
checkpoints load. The forward/backward run in ``torch.ops.csa.sbm_fwd`` / ``sbm_bwd``.

Extensions (all default to the reference behaviour):
  * ``config["return_maps"]`` (default True): also return the (B,H,N,M) ``graph`` and ``attn``
    maps. The training step discards them (script/train.py:107), so the encoder can set it to
    False and skip materialising two fp32 N x M tensors per layer.
  * ``module.uniforms``: optional (B,H,N,M) uniforms for the next forward's Bernoulli draws
    (host-supplied-draw parity mode, bit-identical to torch.bernoulli given the same draws).
  * ``config["attn_precision"]`` / ``module.attn_precision`` (default "fp32", the reference's
    forced precision, sbm_attn.py:120-126): "bf16" runs QK^T, PV and their gradients, the projection MLP
    and sigmoid(. C^T) (forward and backward) on bf16 MFMA with fp32 accumulation; T = Kh S^T, expA, the
    sampling and all elementwise work stay fp32.
  * ``module.bwd_schedule`` (default "auto"): accepted for the CSE attention's schedule vocabulary; the
    SBM backward is one stream-ordered chain since ABI v6 (its query half consumes the ds / G tiles the
    key half writes), so every value gives the same launches and bitwise-identical results.
  * ``Attention`` keeps W_q / W_k / W_v packed back to back (one QKV GEMM) from construction on and after
    every ``.to()`` / ``.cuda()``: the packing exists before DDP or an optimizer sees the parameters.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ..glue import Linear, linear3, pack_linears_, split_heads3

__all__ = ["SBMAttention", "FullAttention", "Attention"]


class SBMAttention(nn.Module):
    def __init__(self, config, idx):
        super().__init__()
        self.drop_attn = nn.Dropout(p=config["attention_dropout"])
        self.head_dim = config["head_dim"]
        self.num_head = config["num_head"]
        self.num_clusters = config["num_clusters"][idx]
        self.dropout = nn.Dropout(0.2)  # unused, as in the reference (sbm_attn.py:18)
        self.layer = nn.Embedding(self.num_head * self.num_clusters, self.head_dim)
        self.orth_clusters = self.layer
        self.proj = nn.Sequential(
            nn.Linear(self.head_dim, self.head_dim),
            nn.Dropout(0.2),
            nn.ReLU(),
            nn.Linear(self.head_dim, self.head_dim),
            nn.Dropout(0.2),
            nn.ReLU(),
            nn.Linear(self.head_dim, self.head_dim),
        )
        self.return_maps = config.get("return_maps", True)
        self.attn_precision = config.get("attn_precision", "fp32")
        self.bwd_schedule = "auto"
        self.uniforms = None

    def forward(self, Q, K, V, mask):
        b, h, n, d = Q.shape
        k = self.num_clusters
        self.clusters = self.orth_clusters.weight.reshape(h, k, -1)  # side effect kept (sbm_attn.py:37)
        attn_p = self.drop_attn.p if self.training else 0.0
        proj_p = self.proj[1].p if self.training else 0.0
        u, self.uniforms = self.uniforms, None
        X, sparsity, graph, attn = ops.sbm_attention(
            Q, K, V, mask, self.layer.weight,
            [self.proj[0].weight, self.proj[0].bias, self.proj[3].weight, self.proj[3].bias,
             self.proj[6].weight, self.proj[6].bias],
            k, uniforms=u, attn_p=attn_p, proj_p=proj_p, want_maps=self.return_maps,
            bf16=self.attn_precision == "bf16", schedule=self.bwd_schedule)
        return X, sparsity, graph, attn


class FullAttention(nn.Module):
    def __init__(self, config, idx):
        super().__init__()
        self.drop_attn = nn.Dropout(p=config["attention_dropout"])
        self.head_dim = config["head_dim"]
        self.num_head = config["num_head"]
        self.dropout = nn.Dropout(0.2)
        self.return_maps = config.get("return_maps", True)
        self.attn_precision = config.get("attn_precision", "fp32")
        self.bwd_schedule = "auto"

    def forward(self, Q, K, V, mask):
        attn_p = self.drop_attn.p if self.training else 0.0
        X, _, _, attn = ops.dense_attention(Q, K, V, mask, attn_p=attn_p, want_maps=self.return_maps,
                                            bf16=self.attn_precision == "bf16", schedule=self.bwd_schedule)
        return X, None, mask, attn  # sbm_attn.py:84-87


class Attention(nn.Module):
    def __init__(self, config, idx, full_att=False):
        super().__init__()
        self.grad_checkpointing = config["attention_grad_checkpointing"]
        self.dim = config["transformer_dim"]
        self.head_dim = config["head_dim"]
        self.num_head = config["num_head"]
        self.attn_type = config["attn_type"]
        self.W_q = Linear(self.dim, self.num_head * self.head_dim)
        self.W_k = Linear(self.dim, self.num_head * self.head_dim)
        self.W_v = Linear(self.dim, self.num_head * self.head_dim)
        if full_att:
            self.attn = FullAttention(config, idx)
        else:
            self.attn = SBMAttention(config, idx)
        self.ff = Linear(self.num_head * self.head_dim, self.dim)
        pack_linears_((self.W_q, self.W_k, self.W_v))

    def _apply(self, fn, *args, **kwargs):
        out = super()._apply(fn, *args, **kwargs)
        pack_linears_((self.W_q, self.W_k, self.W_v))  # a device / dtype move gives each parameter its own storage
        return out

    def forward(self, inputs):
        X, mask, deliver = inputs
        # W_q / W_k / W_v as ONE (3 H d x dim) GEMM (parameters and state_dict keys unchanged); Q, K, V
        # are strided (B, H, N, d) views of its output, consumed in place by the kernels
        Q, K, V = split_heads3(linear3(X, (self.W_q, self.W_k, self.W_v)), self.num_head)
        with torch.autocast(device_type="cuda", enabled=False):  # sbm_attn.py:120
            attn_out, sparsity, graph, attn = self.attn(Q.float(), K.float(), V.float(), mask.float())
        attn_out = self.combine_heads(attn_out)
        out = self.ff(attn_out)
        return out, sparsity, graph, attn

    def combine_heads(self, X):
        X = X.transpose(1, 2)
        X = X.reshape(X.size(0), X.size(1), self.num_head * self.head_dim)
        return X

    def split_heads(self, X):
        X = X.reshape(X.size(0), X.size(1), self.num_head, self.head_dim)
        X = X.transpose(1, 2)
        return X
