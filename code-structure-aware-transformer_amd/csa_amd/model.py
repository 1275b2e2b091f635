"""CSATrans assembled around the MI355X attention kernels (the caller side of the hot path).

Mirrors module/csa_trans.py:67-236, module/sbm_model.py, module/base_seq2seq.py:40-114 and
module/components.py with the SAME module attribute names, so the state_dict keys match the
reference's and reference checkpoints load. What changes:

* SBM encoder attention = csa_amd.module.sbm_attn.Attention (fused HIP SBM/dense kernels); the
  per-layer (B,H,N,N) graph/attn maps are not materialised unless ``return_maps=True``
  (the train step discards them, script/train.py:107).
* CSE relation attention = csa_amd.module.disentangled_attn.DisentangledAttn fed the compact
  (B,2,N,N) uint8 relation planes (parent L, sibling T) directly, instead of the reference's
  repeat(4)+cat int64 (B,8,N,N) copies (module/csa_trans.py:206-211).
* Glue (csa_amd/glue.py): Linear (bias gradient kernel), LayerNorm kernels and the decoder's
  MultiheadAttention keep nn's parameters and state_dict keys; they run the decoder's permuted
  sequence-first views on their batch-first memory instead of copying them. Embeddings, dropout,
  GELU and SDPA are stock PyTorch-ROCm, as in the reference.
"""
import copy
import math
from types import SimpleNamespace

import torch
import torch.nn as nn
import torch.nn.functional as F

from .data import BOS, UNK
from .glue import LayerNorm, Linear, MultiheadAttention, gelu_dropout, residual_dropout
from .module.disentangled_attn import DisentangledAttn
from .module.sbm_attn import Attention

PAD = 0


def _clones(m, n):
    return nn.ModuleList([copy.deepcopy(m) for _ in range(n)])


class PositionalEncoding(nn.Module):
    """components.py:PositionalEncoding (sinusoidal, buffer `pe`)."""

    def __init__(self, emb_size, max_len=5000):
        super().__init__()
        position = torch.arange(0, max_len).unsqueeze(1)
        div = torch.exp(torch.arange(0, emb_size, 2) * -(math.log(10000.0) / emb_size))
        pe = torch.zeros(max_len, emb_size)
        pe[:, 0::2] = torch.sin(position * div)
        pe[:, 1::2] = torch.cos(position * div)
        self.register_buffer("pe", pe.unsqueeze(0))

    def forward(self, x):
        return x + self.pe[:, : x.size(1)]


class Embeddings(nn.Module):
    """components.py:Embeddings: word embedding (+ positional) -> LayerNorm -> dropout."""

    def __init__(self, hidden_size, vocab_size, dropout=0.1, with_pos=False):
        super().__init__()
        self.word_embeddings = nn.Embedding(vocab_size, hidden_size, padding_idx=0)
        self.pos_emb = PositionalEncoding(hidden_size) if with_pos else None
        self.norm = LayerNorm(hidden_size)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        e = self.word_embeddings(x)
        if self.pos_emb is not None:
            e = self.pos_emb(e)
        return self.dropout(self.norm(e))


class FeedForward(nn.Module):
    def __init__(self, d_model, dim_feed_forward, dropout=0.1):
        super().__init__()
        self.linear1 = Linear(d_model, dim_feed_forward)
        self.linear2 = Linear(dim_feed_forward, d_model)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x):
        return self.linear2(gelu_dropout(self.linear1(x), self.dropout)), None


class SublayerConnection(nn.Module):
    """Pre-LN residual: x + dropout(sublayer(norm(x)))."""

    def __init__(self, size, dropout):
        super().__init__()
        self.norm = LayerNorm(size)
        self.dropout = nn.Dropout(dropout)

    def forward(self, x, sublayer):
        out, w = sublayer(self.norm(x))
        return residual_dropout(x, out, self.dropout), w


class CSE_layer(nn.Module):  # noqa: N801 (reference name)
    def __init__(self, hidden_size, num_heads, dim_feed_forward, dropout):
        super().__init__()
        self.num_heads = num_heads
        self.hidden_size = hidden_size
        self.self_attn = DisentangledAttn(num_heads, hidden_size, dropout)
        self.feed_forward = FeedForward(hidden_size, dim_feed_forward, dropout=dropout)
        self.dropout = nn.Dropout(dropout)
        self.sublayer = _clones(SublayerConnection(hidden_size, dropout), 2)

    def forward(self, src, rel_emb, rel, mask):
        src, _ = self.sublayer[0](src, lambda x: self.self_attn(x, x, x, rel_emb, rel, mask))
        src, _ = self.sublayer[1](src, self.feed_forward)
        return src


class CSE(nn.Module):
    """module/csa_trans.py:180-217 with zero-copy relation planes."""

    def __init__(self, encoder_layer, num_layers, num_heads, hidden_size, dropout=0.2, max_src_len=150):
        super().__init__()
        self.layers = _clones(encoder_layer, num_layers)
        self.num_heads = num_heads
        self.hidden_size = hidden_size
        self.d_k = hidden_size // num_heads
        self.max_src_len = max_src_len
        self.edge_dim = self.d_k
        self.L_q = nn.Embedding(max_src_len, hidden_size)
        self.T_q = nn.Embedding(max_src_len, hidden_size)
        self.f = nn.ReLU()
        self.dropout = nn.Dropout(dropout)
        self.norm = LayerNorm(hidden_size)

    def build_rel_emb(self):
        # the reference's torch.stack([L_q.weight, T_q.weight]), kept as the pair its layers unbind
        return [(self.L_q.weight, self.T_q.weight)]

    def forward(self, data):
        out = data.src_pe_emb
        rel = torch.stack([data.L, data.T], 1)          # (B,2,N,N) uint8: heads 0-3 read L, 4-7 read T
        mask = torch.stack([data.L_mask, data.T_mask], 1)
        rel_emb = self.build_rel_emb()
        for layer in self.layers:
            out = layer(out, rel_emb, rel, mask)
        return self.norm(out)


class Transformer(nn.Module):
    """module/sbm_model.py:10-31 pre-LN block around the fused Attention."""

    def __init__(self, config, idx):
        super().__init__()
        self.norm1 = LayerNorm(config["transformer_dim"])
        self.mha = Attention(config, idx, config["full_att"])
        self.dropout1 = nn.Dropout(p=config["dropout_prob"])
        self.norm2 = LayerNorm(config["transformer_dim"])
        self.mlpblock = nn.Sequential(
            Linear(config["transformer_dim"], config["transformer_hidden_dim"]), nn.GELU(),
            nn.Dropout(p=config["dropout_prob"]),
            Linear(config["transformer_hidden_dim"], config["transformer_dim"]), nn.Dropout(p=config["dropout_prob"]))

    def forward(self, X, mask, deliver):
        out, sparsity, graph, attn = self.mha([self.norm1(X), mask, deliver])
        X = residual_dropout(X, out, self.dropout1)  # dropout1(out) + X
        lin1, gelu, drop, lin2, drop2 = self.mlpblock  # Linear, GELU, Dropout, Linear, Dropout
        if gelu.approximate == "none":
            h = lin2(gelu_dropout(lin1(self.norm2(X)), drop))
        else:
            h = lin2(drop(gelu(lin1(self.norm2(X)))))
        X = residual_dropout(X, h, drop2)  # mlpblock(norm2(X)) + X: its last module is the Dropout
        return X, sparsity, graph, attn


class SBM(nn.Module):
    """module/sbm_model.py:34-70."""

    def __init__(self, config, sbm_enc_dim, pe_dim, pegen_dim, use_pegen):
        super().__init__()
        self.num_layers = config["sbm_layers"]
        for idx in range(self.num_layers):
            setattr(self, f"transformer_{idx}", Transformer(config, idx))
        self.norm = LayerNorm(sbm_enc_dim)
        self.out = Linear(sbm_enc_dim, config["out_dim"])
        if use_pegen == "sequential":
            self.pe = PositionalEncoding(sbm_enc_dim, config["max_src_len"])
        else:
            self.pe_expand = Linear(pegen_dim, pe_dim)
        self.use_pegen = use_pegen

    def forward(self, data, src_pe, use_pe):
        mask = data.src_mask
        if use_pe != "sequential":
            pe = self.pe_expand(src_pe)
            X = torch.cat([data.src_emb, pe], dim=-1)
        else:
            pe = None
            X = self.pe(data.src_emb)
        sparsities, graphs, attns = (), [], []
        for idx in range(self.num_layers):
            X, sp, g, a = getattr(self, f"transformer_{idx}")(X, mask, [])
            sparsities += (sp,)
            graphs.append(g)
            attns.append(a)
        X = self.norm(X) * ~mask[:, :, None]
        return self.out(X), sparsities, graphs, attns, pe


class DecoderLayer(nn.Module):
    def __init__(self, d_model, nhead, dim_feedforward=2048, dropout=0.1, activation="gelu"):
        super().__init__()
        self.self_attn = MultiheadAttention(d_model, nhead, dropout=dropout)
        self.multihead_attn = MultiheadAttention(d_model, nhead, dropout=dropout)
        self.feed_forward = FeedForward(d_model, dim_feedforward, dropout=dropout)
        self.sublayer = _clones(SublayerConnection(d_model, dropout), 3)
        self.dropout3 = nn.Dropout(dropout)

    def forward(self, tgt, memory, tgt_mask=None, memory_key_padding_mask=None):
        tgt, _ = self.sublayer[0](tgt, lambda x: self.self_attn(x, x, x, attn_mask=tgt_mask, need_weights=False))
        tgt, w = self.sublayer[1](tgt, lambda x: self.multihead_attn(
            x, memory, memory, key_padding_mask=memory_key_padding_mask, need_weights=False))
        tgt, _ = self.sublayer[2](tgt, self.feed_forward)
        return tgt, w


class BaseDecoder(nn.Module):
    def __init__(self, decoder_layer, num_layers, norm=None):
        super().__init__()
        self.layers = _clones(decoder_layer, num_layers)
        self.num_layers = num_layers
        self.norm = norm

    def forward(self, tgt, memory, tgt_mask, memory_key_padding_mask=None):
        out, w = tgt, None
        for mod in self.layers:
            out, w = mod(out, memory, tgt_mask=tgt_mask, memory_key_padding_mask=memory_key_padding_mask)
        return (self.norm(out) if self.norm is not None else out), w


class Generator(nn.Module):
    """components.py:95-102 Generator: log(softmax(dropout(linear(x))))  (log of softmax, not
    log_softmax). The linear stays on hipBLASLt; dropout + softmax + log is one HIP kernel per
    direction (csa_amd/gen_ops.py, csrc/csa_gen.hip). Module/param names as the reference."""

    def __init__(self, tgt_vocab_size, hidden_size, dropout):
        super().__init__()
        self.soft_max = nn.Softmax(-1)
        self.dropout = nn.Dropout(dropout)
        self.linear = Linear(hidden_size, tgt_vocab_size)

    def forward(self, x):
        from .gen_ops import gen_log_softmax
        return gen_log_softmax(self.linear(x), self.dropout.p if self.training else 0.0)


def make_std_mask(tgt, pad=PAD):
    """dataset/base_data_set.py:125-135: pad | future mask, (B,T,T) bool."""
    T = tgt.size(-1)
    future = torch.triu(torch.ones(T, T, dtype=torch.bool, device=tgt.device), diagonal=1)
    return (tgt == pad).unsqueeze(-2) | future.unsqueeze(0)


class CSATrans(nn.Module):
    """module/csa_trans.py:67-177 (+ BaseTrans.forward/encode/decode, base_seq2seq.py:40-114)."""

    def __init__(self, src_vocab_size, tgt_vocab_size, hidden_size, num_heads, num_layers, sbm_layers, use_pegen,
                 dim_feed_forward, dropout, pe_dim, pegen_dim, sbm_enc_dim, clusters, full_att, state_dict=None,
                 max_src_len=150, return_maps=False):
        super().__init__()
        if use_pegen != "pegen":
            raise NotImplementedError("only the pegen (CSE) structure encoding is on the accelerated path")
        self.num_heads = num_heads
        self.pe_dim, self.pegen_dim = pe_dim, pegen_dim
        self.use_pegen = use_pegen
        self.src_embedding = Embeddings(sbm_enc_dim - pe_dim, src_vocab_size, dropout, with_pos=False)
        self.tgt_embedding = Embeddings(hidden_size, tgt_vocab_size, dropout, with_pos=True)
        self.src_pe_embedding = Embeddings(pegen_dim, src_vocab_size, dropout, with_pos=False)
        self.pegen = CSE(CSE_layer(pegen_dim, num_heads, pegen_dim, dropout), num_layers, num_heads, pegen_dim,
                         dropout=dropout, max_src_len=max_src_len)
        config = {"sbm_layers": sbm_layers, "transformer_dim": sbm_enc_dim, "transformer_hidden_dim": sbm_enc_dim,
                  "head_dim": sbm_enc_dim // num_heads, "num_head": num_heads, "attn_type": "sbm",
                  "attention_grad_checkpointing": False, "attention_dropout": 0.2, "num_clusters": clusters,
                  "dropout_prob": 0.2, "out_dim": hidden_size, "max_src_len": max_src_len, "full_att": full_att,
                  "return_maps": return_maps}
        self.SBM = SBM(config, sbm_enc_dim, pe_dim, pegen_dim, use_pegen)
        self.decoder = BaseDecoder(DecoderLayer(hidden_size, num_heads, dim_feed_forward, dropout, "gelu"), 4,
                                   norm=LayerNorm(hidden_size))
        self.generator = Generator(tgt_vocab_size, hidden_size, dropout)
        if state_dict is None:
            for p in self.parameters():
                if p.dim() > 1:
                    nn.init.xavier_uniform_(p)
            if not full_att:
                for i in range(sbm_layers):
                    nn.init.orthogonal_(getattr(self.SBM, f"transformer_{i}").mha.attn.layer.weight)
        else:
            self.load_state_dict(state_dict)

    def base_process(self, data):
        """base_seq2seq.py:43-54: masks and embeddings; the target side only when tgt_seq is given
        (GreedyGenerator runs with tgt_seq None and fills tgt_mask / tgt_emb per step)."""
        data.src_mask = data.src_seq.eq(PAD)
        data.src_emb = self.src_embedding(data.src_seq)
        data.src_pe_emb = self.src_pe_embedding(data.src_seq)
        if getattr(data, "tgt_seq", None) is not None:
            data.tgt_mask = make_std_mask(data.tgt_seq, PAD)
            data.tgt_emb = self.tgt_embedding(data.tgt_seq)

    def process_data(self, data):
        """base_seq2seq.py:56-57."""
        self.base_process(data)

    def encode(self, data):
        """base_seq2seq.py:67-97 (pegen branch): CSE -> SBM; sparsity = mean over the SBM layers' head
        sparsities, or 1 for the dense ablation. Returns (enc, sparsity, pe, graphs, attns)."""
        src_pe = self.pegen(data)
        enc, sparsity, graphs, attns, pe = self.SBM(data, src_pe, self.use_pegen)
        sparsity = 1 if sparsity[0] is None else torch.mean(torch.stack(sparsity))
        return enc, sparsity, pe, graphs, attns

    def decode(self, data, encoder_outputs):
        """base_seq2seq.py:99-114: returns (decoder outputs (B,T,E), last cross-attention weights)."""
        tgt_mask = data.tgt_mask.repeat(self.num_heads, 1, 1)
        dec, w = self.decoder(data.tgt_emb.permute(1, 0, 2), encoder_outputs.permute(1, 0, 2), tgt_mask=tgt_mask,
                              memory_key_padding_mask=data.src_mask)
        return dec.permute(1, 0, 2), w

    def forward(self, data):
        """base_seq2seq.py:59-65."""
        self.process_data(data)
        enc, sparsity, pe, graphs, attns = self.encode(data)
        dec, _ = self.decode(data, enc)
        out = self.generator(dec)
        return out, sparsity, pe, graphs, attns


class GreedyGenerator(nn.Module):
    """module/base_seq2seq.py:117-145: one encode, then max_tgt_len-1 steps of decode + generator +
    argmax over the last position, starting from BOS; returns the generated ids without BOS."""

    def __init__(self, model, max_tgt_len, multi_gpu=False):
        super().__init__()
        self.model = model.module if multi_gpu else model
        self.max_tgt_len = max_tgt_len
        self.start_pos = BOS
        self.unk_pos = UNK

    def forward(self, data):
        m = self.model
        m.process_data(data)
        enc, _, _, _, _ = m.encode(data)
        ys = torch.full((enc.size(0), 1), self.start_pos, dtype=torch.long, device=enc.device)
        for _ in range(self.max_tgt_len - 1):
            data.tgt_mask = make_std_mask(ys, PAD)
            data.tgt_emb = m.tgt_embedding(ys)
            dec, _ = m.decode(data, enc)
            out = m.generator(dec)[:, -1, :]
            next_word = torch.max(out, dim=1)[1]
            ys = torch.cat([ys, next_word.unsqueeze(1)], dim=1)
        return ys[:, 1:]


class _GatherTargets(torch.autograd.Function):
    """x.gather(1, t[:, None])[:, 0] whose backward scatters into a fresh zero tensor in place (torch's
    gather backward is an out-of-place scatter_add, i.e. zeros + a full clone of the (B*T, V) grad)."""

    @staticmethod
    def forward(ctx, x, t):
        ctx.save_for_backward(t)
        ctx.shape = x.shape
        return x.gather(1, t.unsqueeze(1)).squeeze(1)

    @staticmethod
    def backward(ctx, g):
        (t,) = ctx.saved_tensors
        gx = torch.zeros(ctx.shape, device=g.device, dtype=g.dtype)
        gx.scatter_add_(1, t.unsqueeze(1), g.unsqueeze(1))
        return gx, None


def _gather_targets(x, t):
    return _GatherTargets.apply(x, t)


class LabelSmoothing(nn.Module):
    """utils/label_smooth.py:15-40 without materialising true_dist (B*T x V: 251 MB per step at the java
    config). true_dist is `confidence` at the target, 0 in the padding column and in padded rows, and
    eps = smoothing / (V - 2) elsewhere, so the KLDiv(sum) / ntokens closes to, per non-pad row,
        conf (log conf - x_t) + eps ((V-2) log eps - sum_{j != t, pad} x_j)
    (the row sum is read only when smoothing > 0). torch's kl_div gives 0 * (-inf) = NaN wherever
    true_dist is 0 and x is -inf (an underflowed log-probability); that NaN is reproduced with one
    detached compare over x. ntokens = (target != 0).sum() literally, as the reference."""

    def __init__(self, padding_idx, smoothing=0.0):
        super().__init__()
        self.padding_idx = padding_idx
        self.confidence = 1.0 - smoothing
        self.smoothing = smoothing
        self.true_dist = None  # never materialised

    def forward(self, x, target):
        V = x.size(-1)
        x = x.reshape(-1, V)
        t = target.reshape(-1)
        ntokens = (target != 0).sum()
        valid = t != self.padding_idx
        xt = _gather_targets(x, t)
        conf, sm = self.confidence, self.smoothing
        row = -conf * xt + (conf * math.log(conf) if conf > 0.0 else 0.0)
        with torch.no_grad():
            if sm > 0.0:
                bad = ~(x > float("-inf"))  # -inf or NaN
                n_bad = bad.sum()
                n_at_td = (bad[valid].sum() - bad[valid, self.padding_idx].sum()) if V > 2 else 0
            else:
                # per-row fp32 counts (exact: V < 2^24) summed in fp64: a bool .sum() would first cast
                # the whole (B*T, V) mask to int64 (500 MB at the java config)
                n_bad = torch.where(x > float("-inf"), 0.0, 1.0).sum(1).double().sum()
                n_at_td = (~(xt.detach() > float("-inf")) & valid).sum()
            poison = torch.where(n_bad > n_at_td, float("nan"), 0.0).to(x.dtype)
        if sm > 0.0:
            eps = sm / (V - 2)
            col = torch.arange(V, device=x.device).unsqueeze(0)
            off = (col == t.unsqueeze(1)) | (col == self.padding_idx)  # true_dist != eps there
            rest = torch.where(off, torch.zeros_like(x), x).sum(1)
            row = row + eps * ((V - 2) * math.log(eps) - rest)
        loss = torch.where(valid, row, torch.zeros_like(row)).sum() + poison
        return loss / ntokens


def label_smoothing_loss(logp, target, padding_idx=PAD):
    """LabelSmoothing(padding_idx, smoothing=0) as a function (all configs use smoothing 0)."""
    return LabelSmoothing(padding_idx, 0.0)(logp, target)


def batch_to_device(sb, device):
    """Synthetic batch dict (csa_amd.data.synthetic_batch) -> device-resident namespace."""
    g = lambda k, dt=None: torch.as_tensor(sb[k], dtype=dt).to(device, non_blocking=True)
    return SimpleNamespace(src_seq=g("src_seq", torch.int64), tgt_seq=g("tgt_seq", torch.int64),
                           L=g("L", torch.uint8), T=g("T", torch.uint8), L_mask=g("L_mask", torch.uint8),
                           T_mask=g("T_mask", torch.uint8)), g("target", torch.int64)


CONFIGS = {  # config/python.py, config/java.py, config/python_full_att.py (vocab sizes: create_vocab caps)
    "python": dict(src_vocab_size=10000, tgt_vocab_size=20000, hidden_size=512, num_heads=8, num_layers=4,
                   sbm_layers=4, use_pegen="pegen", dim_feed_forward=2048, dropout=0.2, pe_dim=256,
                   pegen_dim=512, sbm_enc_dim=512, clusters=[10, 10, 10, 10], full_att=False),
    "java": dict(src_vocab_size=10000, tgt_vocab_size=20000, hidden_size=512, num_heads=8, num_layers=4,
                 sbm_layers=4, use_pegen="pegen", dim_feed_forward=2048, dropout=0.2, pe_dim=128, pegen_dim=512,
                 sbm_enc_dim=768, clusters=[10, 10, 10, 10], full_att=False),
    "python_full_att": dict(src_vocab_size=10000, tgt_vocab_size=20000, hidden_size=512, num_heads=8,
                            num_layers=4, sbm_layers=4, use_pegen="pegen", dim_feed_forward=2048, dropout=0.2,
                            pe_dim=256, pegen_dim=512, sbm_enc_dim=512, clusters=[10, 10, 10, 10], full_att=True),
}
