"""ORACLE (test infrastructure only): functional torch-CPU restatement of the whole CSATrans model.

Restates, op for op and with the reference's state_dict keys (paths relative to /root/reference):

* module/csa_trans.py:67-177     CSATrans.__init__ (parameter shapes, config dict)
* module/csa_trans.py:180-236    CSE / CSE_layer (rel/mask repeat x4 + cat, pre-LN sublayers)
* module/base_seq2seq.py:40-114  process_data / encode / decode / forward
* module/sbm_model.py:10-70      Transformer block and SBM stack
* module/components.py           Embeddings, PositionalEncoding, FeedForward, SublayerConnection,
                                 DecoderLayer (nn.MultiheadAttention), BaseDecoder, Generator
* module/sbm_attn.py, module/STE.py, module/disentangled_attn.py through oracle/sbm_ref.py and
  oracle/cse_ref.py.

Used (1) by tests/test_oracle_golden.py, pinned against tests/golden/csatrans_tiny.npz (the
reference's own CSATrans output), and (2) by bench.py's cpu_baseline leg, which times the
csa_trans_time_memory.py:100-150 protocol (BASELINE config 1) on the host cores. Train mode draws
dropout masks and the STE uniforms from torch's CPU generator, as the reference does; eval mode
takes the STE uniforms per SBM layer explicitly (``u_list``). Nothing in the product imports this.
"""
import math

import torch
import torch.nn.functional as F

from . import cse_ref, sbm_ref

PAD = 0


def config(src_vocab_size, tgt_vocab_size, hidden_size, num_heads, num_layers, sbm_layers, use_pegen,
           dim_feed_forward, dropout, pe_dim, pegen_dim, sbm_enc_dim, clusters, full_att, max_src_len=150):
    """The constructor arguments of module/csa_trans.py:68-85 as a dict."""
    if use_pegen != "pegen":
        raise NotImplementedError("the oracle restates the pegen (CSE) configuration only")
    return dict(src_vocab_size=src_vocab_size, tgt_vocab_size=tgt_vocab_size, hidden_size=hidden_size,
                num_heads=num_heads, num_layers=num_layers, sbm_layers=sbm_layers, dim_feed_forward=dim_feed_forward,
                dropout=dropout, pe_dim=pe_dim, pegen_dim=pegen_dim, sbm_enc_dim=sbm_enc_dim, clusters=list(clusters),
                full_att=full_att, max_src_len=max_src_len)


def param_shapes(cfg):
    """state_dict parameter names -> shapes (module/csa_trans.py:67-177; the orth_clusters alias and the
    positional-encoding buffer are left out)."""
    S, E, P, H = cfg["sbm_enc_dim"], cfg["hidden_size"], cfg["pegen_dim"], cfg["num_heads"]
    dk, ff, hd = P // H, cfg["dim_feed_forward"], S // H
    sh = {}

    def lin(name, i, o):
        sh[name + ".weight"], sh[name + ".bias"] = (o, i), (o,)

    def ln(name, n):
        sh[name + ".weight"], sh[name + ".bias"] = (n,), (n,)

    def emb(name, V, n):
        sh[name + ".word_embeddings.weight"] = (V, n)
        ln(name + ".norm", n)

    emb("src_embedding", cfg["src_vocab_size"], S - cfg["pe_dim"])
    emb("tgt_embedding", cfg["tgt_vocab_size"], E)
    emb("src_pe_embedding", cfg["src_vocab_size"], P)
    for i in range(cfg["num_layers"]):
        pre = f"pegen.layers.{i}."
        for j in range(4):
            lin(pre + f"self_attn.linear_layers.{j}", P, P)
        for j in range(2):
            lin(pre + f"self_attn.l_linear.{j}", P, 4 * dk)
            lin(pre + f"self_attn.t_linear.{j}", P, 4 * dk)
        lin(pre + "feed_forward.linear1", P, P)
        lin(pre + "feed_forward.linear2", P, P)
        for j in range(2):
            ln(pre + f"sublayer.{j}.norm", P)
    sh["pegen.L_q.weight"] = (cfg["max_src_len"], P)
    sh["pegen.T_q.weight"] = (cfg["max_src_len"], P)
    ln("pegen.norm", P)
    for i in range(cfg["sbm_layers"]):
        pre = f"SBM.transformer_{i}."
        ln(pre + "norm1", S)
        ln(pre + "norm2", S)
        for w in ("W_q", "W_k", "W_v"):
            lin(pre + "mha." + w, S, S)
        lin(pre + "mha.ff", S, S)
        if not cfg["full_att"]:
            sh[pre + "mha.attn.layer.weight"] = (H * cfg["clusters"][i], hd)
            for j in (0, 3, 6):
                lin(pre + f"mha.attn.proj.{j}", hd, hd)
        lin(pre + "mlpblock.0", S, S)
        lin(pre + "mlpblock.3", S, S)
    ln("SBM.norm", S)
    lin("SBM.out", S, E)
    lin("SBM.pe_expand", P, cfg["pe_dim"])
    for i in range(4):
        pre = f"decoder.layers.{i}."
        for a in ("self_attn", "multihead_attn"):
            sh[pre + a + ".in_proj_weight"], sh[pre + a + ".in_proj_bias"] = (3 * E, E), (3 * E,)
            lin(pre + a + ".out_proj", E, E)
        lin(pre + "feed_forward.linear1", E, ff)
        lin(pre + "feed_forward.linear2", ff, E)
        for j in range(3):
            ln(pre + f"sublayer.{j}.norm", E)
    ln("decoder.norm", E)
    lin("generator.linear", E, cfg["tgt_vocab_size"])
    return sh


def init_params(cfg, seed=0):
    """Reference initialisation (module/csa_trans.py:165-175): nn defaults, then xavier_uniform_ on every
    matrix and orthogonal_ on each SBM layer's cluster embeddings."""
    g = torch.Generator().manual_seed(seed)
    p = {}
    for k, s in param_shapes(cfg).items():
        if len(s) > 1:
            t = torch.empty(s)
            bound = math.sqrt(6.0 / (s[0] + s[1]))
            p[k] = t.uniform_(-bound, bound, generator=g)
        elif k.endswith("norm.weight"):
            p[k] = torch.ones(s)
        else:
            p[k] = torch.zeros(s)
    for i in range(cfg["sbm_layers"]):
        k = f"SBM.transformer_{i}.mha.attn.layer.weight"
        if k in p:
            p[k] = torch.nn.init.orthogonal_(torch.empty(p[k].shape), generator=g)
    return p


def positional_encoding(n, emb_size, max_len=5000):
    """components.py:PositionalEncoding buffer rows [0, n)."""
    pe = torch.zeros(max_len, emb_size)
    position = torch.arange(0, max_len).unsqueeze(1)
    div_term = torch.exp(torch.arange(0, emb_size, 2) * -(math.log(10000.0) / emb_size))
    pe[:, 0::2] = torch.sin(position * div_term)
    pe[:, 1::2] = torch.cos(position * div_term)
    return pe[:n].unsqueeze(0)


def make_std_mask(tgt, pad=PAD):
    """dataset/base_data_set.py make_std_mask: pad | future (B,T,T) bool."""
    T = tgt.size(-1)
    future = torch.triu(torch.ones(T, T, dtype=torch.bool), diagonal=1)
    return (tgt == pad).unsqueeze(-2) | future.unsqueeze(0)


class Model:
    """CSATrans as functions of a parameter dict (reference state_dict keys)."""

    def __init__(self, cfg, params, training=False):
        self.cfg, self.p, self.training = cfg, params, training
        self.drop = cfg["dropout"]

    def _lin(self, name, x):
        return F.linear(x, self.p[name + ".weight"], self.p[name + ".bias"])

    def _ln(self, name, x):
        return F.layer_norm(x, (x.size(-1),), self.p[name + ".weight"], self.p[name + ".bias"])

    def _drop(self, x, p=None):
        return F.dropout(x, self.drop if p is None else p, self.training)

    def _emb(self, name, ids, with_pos=False):
        """components.py:Embeddings."""
        e = F.embedding(ids, self.p[name + ".word_embeddings.weight"], padding_idx=0)
        if with_pos:
            e = e + positional_encoding(ids.size(1), e.size(-1))
        return self._drop(self._ln(name + ".norm", e))

    def _ffn(self, name, x):
        """components.py:FeedForward: linear2(dropout(gelu(linear1(x))))."""
        return self._lin(name + ".linear2", self._drop(F.gelu(self._lin(name + ".linear1", x))))

    def cse(self, src_pe_emb, L, T, L_mask, T_mask):
        """csa_trans.py:204-236."""
        H = self.cfg["num_heads"]
        rel, mask = cse_ref.build_rel_mask(L, T, L_mask, T_mask)
        rel_q = torch.stack([self.p["pegen.L_q.weight"], self.p["pegen.T_q.weight"]])
        out = src_pe_emb
        for i in range(self.cfg["num_layers"]):
            pre = f"pegen.layers.{i}."
            ap = {k[len(pre + "self_attn."):]: v for k, v in self.p.items() if k.startswith(pre + "self_attn.")}
            a, _ = cse_ref.disentangled_attn(self._ln(pre + "sublayer.0.norm", out), ap, rel_q, rel, mask, H)
            out = out + self._drop(a)
            out = out + self._drop(self._ffn(pre + "feed_forward", self._ln(pre + "sublayer.1.norm", out)))
        return self._ln("pegen.norm", out)

    def sbm(self, src_emb, src_pe, src_mask, u_list=None):
        """sbm_model.py:10-70 (Attention = sbm_ref.attention_layer). Returns (X, sparsities, pe)."""
        cfg, H = self.cfg, self.cfg["num_heads"]
        hd = cfg["sbm_enc_dim"] // H
        pe = self._lin("SBM.pe_expand", src_pe)
        X = torch.cat([src_emb, pe], dim=-1)
        sps = []
        for i in range(cfg["sbm_layers"]):
            pre = f"SBM.transformer_{i}."
            ap = {k[len(pre + "mha."):]: v for k, v in self.p.items() if k.startswith(pre + "mha.")}
            Xn = self._ln(pre + "norm1", X)
            B, N = Xn.shape[:2]
            u = None if cfg["full_att"] else (u_list[i] if u_list is not None else torch.rand(B, H, N, N))
            out, sp, _, _ = sbm_ref.attention_layer(Xn, src_mask, ap, u, H, hd, cfg["clusters"][i], cfg["full_att"],
                                                    attn_p=self.drop_attn(), proj_p=self.drop_attn())
            sps.append(sp)
            X = self._drop(out) + X
            h = self._drop(F.gelu(self._lin(pre + "mlpblock.0", self._ln(pre + "norm2", X))))
            X = self._drop(self._lin(pre + "mlpblock.3", h)) + X
        X = self._ln("SBM.norm", X) * ~src_mask[:, :, None]
        return self._lin("SBM.out", X), sps, pe

    def drop_attn(self):
        """attention_dropout and the proj dropouts are fixed at 0.2 (csa_trans.py:152, sbm_attn.py:24,27)."""
        return 0.2 if self.training else 0.0

    def _mha(self, name, q, k, v, attn_mask=None, key_padding_mask=None):
        """nn.MultiheadAttention.forward (need_weights=True, as components.py:DecoderLayer calls it)."""
        E = q.size(-1)
        out, _ = F.multi_head_attention_forward(
            q, k, v, E, self.cfg["num_heads"], self.p[name + ".in_proj_weight"], self.p[name + ".in_proj_bias"],
            None, None, False, self.drop, self.p[name + ".out_proj.weight"], self.p[name + ".out_proj.bias"],
            training=self.training, key_padding_mask=key_padding_mask, need_weights=True, attn_mask=attn_mask)
        return out

    def decode(self, tgt_emb, enc, tgt_mask, src_mask):
        """base_seq2seq.py:99-114 + components.py:BaseDecoder/DecoderLayer."""
        x, mem = tgt_emb.permute(1, 0, 2), enc.permute(1, 0, 2)
        m = tgt_mask.repeat(self.cfg["num_heads"], 1, 1)
        for i in range(4):
            pre = f"decoder.layers.{i}."
            y = self._ln(pre + "sublayer.0.norm", x)
            x = x + self._drop(self._mha(pre + "self_attn", y, y, y, attn_mask=m))
            y = self._ln(pre + "sublayer.1.norm", x)
            x = x + self._drop(self._mha(pre + "multihead_attn", y, mem, mem, key_padding_mask=src_mask))
            x = x + self._drop(self._ffn(pre + "feed_forward", self._ln(pre + "sublayer.2.norm", x)))
        return self._ln("decoder.norm", x).permute(1, 0, 2)

    def forward(self, src_seq, tgt_seq, L, T, L_mask, T_mask, u_list=None):
        """base_seq2seq.py:59-65: returns (log-probabilities (B,T,V), mean sparsity)."""
        src_mask = src_seq.eq(PAD)
        src_emb = self._emb("src_embedding", src_seq)
        src_pe_emb = self._emb("src_pe_embedding", src_seq)
        tgt_mask = make_std_mask(tgt_seq, PAD)
        tgt_emb = self._emb("tgt_embedding", tgt_seq, with_pos=True)
        src_pe = self.cse(src_pe_emb, L, T, L_mask, T_mask)
        enc, sps, _ = self.sbm(src_emb, src_pe, src_mask, u_list)
        sparsity = torch.ones(()) if sps[0] is None else torch.mean(torch.stack(sps))
        dec = self.decode(tgt_emb, enc, tgt_mask, src_mask)
        logits = self._lin("generator.linear", dec)
        return torch.log(torch.softmax(self._drop(logits), -1)), sparsity


def label_smoothing(x, target, padding_idx=PAD):
    """utils/label_smooth.py:15-40 at smoothing 0 (every config): KLDiv(sum)(x, true_dist) / ntokens."""
    V = x.size(-1)
    x = x.reshape(-1, V)
    t = target.reshape(-1)
    true_dist = torch.zeros_like(x)
    true_dist.scatter_(1, t.unsqueeze(1), 1.0)
    true_dist[:, padding_idx] = 0
    true_dist[t == padding_idx] = 0
    return F.kl_div(x, true_dist, reduction="sum") / (target != 0).sum()
