"""Encoder/decoder glue of the train step: nn.Linear whose bias gradient is
csa_bias_grad (csrc/csa_glue.hip) instead of torch's generic strided reduction. Forward and the
two GEMMs of the backward stay on hipBLASLt. Same parameters and state_dict keys as nn.Linear."""
import ctypes

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._lib import check, lib, on_device


def bias_grad(gy2: torch.Tensor) -> torch.Tensor:
    """(rows, cols) contiguous fp32 on the GPU -> (cols,) column sums (deterministic order)."""
    rows, cols = gy2.shape
    db = torch.empty(cols, device=gy2.device, dtype=torch.float32)
    L = lib()
    ws = torch.empty(max(1, L.csa_bias_grad_workspace_bytes(rows, cols)), dtype=torch.uint8, device=gy2.device)
    stream = ctypes.c_void_p(torch.cuda.current_stream(gy2.device).cuda_stream)
    with on_device(gy2.device):
        check(L.csa_bias_grad(ctypes.c_void_p(gy2.data_ptr()), ctypes.c_void_p(db.data_ptr()), rows, cols, 0,
                              ctypes.c_void_p(ws.data_ptr()), stream), "csa_bias_grad")
    return db


class _LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        ctx.save_for_backward(x, w)
        return F.linear(x, w, b)

    @staticmethod
    def backward(ctx, gy):
        x, w = ctx.saved_tensors
        gy2 = gy.reshape(-1, gy.shape[-1])
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = gy @ w
        if ctx.needs_input_grad[1]:
            dw = gy2.t() @ x.reshape(-1, x.shape[-1])
        if ctx.needs_input_grad[2]:
            g = gy2 if gy2.is_contiguous() and gy2.dtype == torch.float32 else gy2.float().contiguous()
            db = bias_grad(g).to(gy.dtype)
        return dx, dw, db


def linear(x, w, b=None):
    if b is None or not x.is_cuda or x.dtype != torch.float32:
        return F.linear(x, w, b)
    if _batch_major(x):  # rows are independent: run on the batch-first memory, return the same view
        return _LinearFn.apply(x.transpose(0, 1), w, b).transpose(0, 1)
    return _LinearFn.apply(x, w, b)


def _packed(ts):
    """The tensor spanning three same-shape contiguous tensors stored back to back in one storage
    (pack_adjacent_), or None."""
    a = ts[0]
    n = a.numel()
    for i, t in enumerate(ts):
        if (not t.is_contiguous() or t.shape != a.shape or t.dtype != a.dtype or t.device != a.device
                or t.untyped_storage().data_ptr() != a.untyped_storage().data_ptr()
                or t.storage_offset() != a.storage_offset() + i * n):
            return None
    return a.detach().as_strided((len(ts) * a.shape[0],) + tuple(a.shape[1:]), a.stride())


def pack_adjacent_(params):
    """Move the data of same-shape parameters into one buffer, back to back (each keeps its own
    Parameter object, shape and state_dict key). Returns True when they are (now) packed."""
    if _packed(params) is not None:
        return True
    a = params[0]
    if any(p.shape != a.shape or p.dtype != a.dtype or p.device != a.device for p in params):
        return False
    with torch.no_grad():
        buf = torch.cat([p.detach() for p in params], 0)
        n = a.shape[0]
        for i, p in enumerate(params):
            p.data = buf[i * n:(i + 1) * n]
    return True


class _LinearPackedFn(torch.autograd.Function):
    """y = x [W_0; W_1; W_2]^T + [b_0; b_1; b_2] for weights / biases packed back to back: one GEMM
    over the packed memory, no per-forward concatenation; the backward's single dW / db GEMM is
    handed back as three views."""

    @staticmethod
    def forward(ctx, x, w0, w1, w2, b0, b1, b2):
        W, B = _packed((w0, w1, w2)), _packed((b0, b1, b2))
        ctx.save_for_backward(x, W)
        ctx.n = w0.shape[0]
        return F.linear(x, W, B)

    @staticmethod
    def backward(ctx, gy):
        x, W = ctx.saved_tensors
        n = ctx.n
        gy2 = gy.reshape(-1, gy.shape[-1])
        dx = gy @ W if ctx.needs_input_grad[0] else None
        dw = gy2.t() @ x.reshape(-1, x.shape[-1])
        if gy2.is_cuda:
            g = gy2 if gy2.is_contiguous() and gy2.dtype == torch.float32 else gy2.float().contiguous()
            db = bias_grad(g).to(gy.dtype)
        else:  # host tensors (the gloo DDP tests): the same column sums on the CPU
            db = gy2.sum(0)
        return (dx,) + tuple(dw[i * n:(i + 1) * n] for i in range(3)) + tuple(db[i * n:(i + 1) * n] for i in range(3))


def pack_linears_(linears):
    """Pack the weights and the biases of same-shape nn.Linear layers back to back (pack_adjacent_).
    Modules that own such a triple call this at construction and after every device / dtype move
    (_apply), so the packing exists before DDP builds its buckets or an optimizer sees the parameters."""
    ws, bs = [l.weight for l in linears], [l.bias for l in linears]
    if any(b is None for b in bs):
        return False
    return pack_adjacent_(ws) and pack_adjacent_(bs)


def linear3(x, linears):
    """The three nn.Linear layers `linears` applied to the same x as one GEMM, outputs concatenated on
    the last dim: (..., 3 out). Their parameters are packed back to back (pack_linears_: eagerly by the
    owning module, or here on first use), so no per-forward weight concatenation happens."""
    ws, bs = [l.weight for l in linears], [l.bias for l in linears]
    if (x.dtype == torch.float32 and x.device == ws[0].device and all(b is not None for b in bs)
            and pack_adjacent_(ws) and pack_adjacent_(bs)):
        if _batch_major(x):
            return _LinearPackedFn.apply(x.transpose(0, 1), *ws, *bs).transpose(0, 1)
        return _LinearPackedFn.apply(x, *ws, *bs)
    w = torch.cat(ws, 0)
    b = torch.cat(bs, 0) if all(b is not None for b in bs) else None
    return linear(x, w, b)


class Linear(nn.Linear):
    def forward(self, x):
        return linear(x, self.weight, self.bias)


class _LayerNormFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, eps):
        L = lib()
        cols = x.shape[-1]
        x2 = x.reshape(-1, cols)
        y = torch.empty_like(x2)
        stats = torch.empty(x2.shape[0], 2, device=x.device, dtype=torch.float32)
        stream = ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        with on_device(x.device):
            check(L.csa_layernorm_fwd(p(x2), p(w), p(b), p(y), p(stats), x2.shape[0], cols, eps, stream),
                  "csa_layernorm_fwd")
        ctx.save_for_backward(x2, w, stats)
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, gy):
        x2, w, stats = ctx.saved_tensors
        L = lib()
        rows, cols = x2.shape
        gy2 = gy.reshape(rows, cols).contiguous()
        dx = torch.empty_like(x2)
        dw = torch.empty(cols, device=x2.device, dtype=torch.float32)
        db = torch.empty_like(dw)
        ws = torch.empty(max(1, L.csa_layernorm_bwd_workspace_bytes(rows, cols)), dtype=torch.uint8,
                         device=x2.device)
        stream = ctypes.c_void_p(torch.cuda.current_stream(x2.device).cuda_stream)
        p = lambda t: ctypes.c_void_p(t.data_ptr())
        with on_device(x2.device):
            check(L.csa_layernorm_bwd(p(gy2), p(x2), p(stats), p(w), p(dx), p(dw), p(db), rows, cols, p(ws), stream),
                  "csa_layernorm_bwd")
        return dx.view(gy.shape), dw, db, None


class LayerNorm(nn.LayerNorm):
    """nn.LayerNorm (same parameters / state_dict keys) on csa_layernorm_fwd/_bwd (csrc/csa_glue.hip)
    for fp32 CUDA inputs over one normalised dim with affine weights; anything else takes torch's."""

    def forward(self, x):
        if (x.is_cuda and x.dtype == torch.float32 and len(self.normalized_shape) == 1 and self.weight is not None
                and self.bias is not None and lib().csa_layernorm_supported(x.shape[-1])):
            if x.is_contiguous():
                return _LayerNormFn.apply(x, self.weight, self.bias, float(self.eps))
            if _batch_major(x):  # per-row op: normalise the batch-first memory, return the same view
                return _LayerNormFn.apply(x.transpose(0, 1), self.weight, self.bias, float(self.eps)).transpose(0, 1)
        return super().forward(x)


def _batch_major(x):
    """A (T, B, E) tensor whose memory is (B, T, E)-contiguous (a permuted batch-first tensor)."""
    return x.dim() == 3 and not x.is_contiguous() and x.transpose(0, 1).is_contiguous()


def _float_mask(m, dtype):
    """F._canonical_mask for a bool mask: True -> -inf, False -> 0."""
    if m.dtype == torch.bool:
        return torch.zeros(m.shape, dtype=dtype, device=m.device).masked_fill_(m, float("-inf"))
    return m.to(dtype)


class MultiheadAttention(nn.MultiheadAttention):
    """nn.MultiheadAttention (same parameters / state_dict keys; the decoder's self- and
    cross-attention, reference module/base_seq2seq.py DecoderLayer) without its layout copies.

    The decoder's sequence-first inputs are permuted views of batch-first tensors
    (csa_trans.py passes `tgt_emb.permute(1, 0, 2)` and `enc.permute(1, 0, 2)`). torch's
    multi_head_attention_forward makes those contiguous, packs q/k/v as (3, T, B, E) copies and,
    in the backward, zero-fills and accumulates a full (3, T, B, E) gradient per select. Here the
    projections run on the batch-first memory, q/k/v are strided (B, H, T, hd) views of the packed
    projection (their backward is one stack), and the output is returned as a (T, B, E) view of a
    batch-first tensor. Same math as the need_weights=False path of F.multi_head_attention_forward:
    bool masks -> -inf additive masks, key padding merged per head, the (B*H, T, S) attn_mask read
    as view(B, H, T, S), SDPA with dropout_p = dropout when training, out_proj. Any other use
    (need_weights, bias_k, kdim != embed_dim, batch_first, ...) takes nn.MultiheadAttention's path."""

    def forward(self, query, key, value, key_padding_mask=None, need_weights=True, attn_mask=None,
                average_attn_weights=True, is_causal=False):
        if (need_weights or is_causal or self.batch_first or not self._qkv_same_embed_dim or self.bias_k is not None
                or self.add_zero_attn or self.in_proj_bias is None or query.dim() != 3 or not query.is_cuda
                or key is not value):
            return super().forward(query, key, value, key_padding_mask=key_padding_mask, need_weights=need_weights,
                                   attn_mask=attn_mask, average_attn_weights=average_attn_weights,
                                   is_causal=is_causal)
        T, B, E = query.shape
        S = key.shape[0]
        H = self.num_heads
        hd = E // H
        qb = query.transpose(0, 1)  # (B, T, E), contiguous when query is a permuted batch-first tensor
        if query is key:
            qkv = linear(qb, self.in_proj_weight, self.in_proj_bias).view(B, T, 3, H, hd)
            q, k, v = (t.transpose(1, 2) for t in qkv.unbind(2))
        else:
            w_q, w_kv = self.in_proj_weight.split([E, 2 * E])
            b_q, b_kv = self.in_proj_bias.split([E, 2 * E])
            q = linear(qb, w_q, b_q).view(B, T, H, hd).transpose(1, 2)
            kv = linear(key.transpose(0, 1), w_kv, b_kv).view(B, S, 2, H, hd)
            k, v = (t.transpose(1, 2) for t in kv.unbind(2))
        m = None
        if attn_mask is not None:
            m = _float_mask(attn_mask, q.dtype)
            m = m.unsqueeze(0) if m.dim() == 2 else m
        if key_padding_mask is not None:
            kpm = _float_mask(key_padding_mask, q.dtype).view(B, 1, 1, S).expand(-1, H, -1, -1).reshape(B * H, 1, S)
            m = kpm if m is None else m + kpm
        if m is not None:
            m = m.unsqueeze(0) if m.size(0) == 1 else m.view(B, H, -1, S)
        o = F.scaled_dot_product_attention(q, k, v, m, self.dropout if self.training else 0.0)
        o = o.transpose(1, 2).reshape(B, T, E)
        return linear(o, self.out_proj.weight, self.out_proj.bias).transpose(0, 1), None


class _SplitHeads3(torch.autograd.Function):
    @staticmethod
    def forward(ctx, y, num_heads):
        B, N, C = y.shape
        ctx.shape = (B, N, C)
        v = y.view(B, N, 3, num_heads, C // (3 * num_heads))
        return tuple(v[:, :, i].transpose(1, 2) for i in range(3))

    @staticmethod
    def backward(ctx, dq, dk, dv):
        B, N, C = ctx.shape
        if dq is not None and dk is not None and dv is not None:
            from .ops import packed_qkv
            if packed_qkv(dq, dk, dv):  # the kernels wrote the packed layout already (ops.packed_grads)
                return dq.as_strided((B, N, C), (N * C, C, 1), dq.storage_offset()), None
        ref = next(g for g in (dq, dk, dv) if g is not None)
        out = torch.empty(B, N, C, device=ref.device, dtype=ref.dtype)
        ov = out.view(B, N, 3, ref.shape[1], C // (3 * ref.shape[1]))
        for i, g in enumerate((dq, dk, dv)):  # three strided copies (a strided-input stack is 3x slower)
            if g is None:
                ov[:, :, i].zero_()
            else:
                ov[:, :, i].transpose(1, 2).copy_(g)
        return out, None


def split_heads3(y, num_heads):
    """Packed QKV projection (B, N, 3*H*d) -> Q, K, V as strided (B, H, N, d) views, the same values as
    split(H*d, -1) followed by view(B, N, H, d).transpose(1, 2) (sbm_attn.py:137-140,
    components.py:transpose_for_scores). The backward copies the three head-major gradients straight
    into one packed (B, N, 3*H*d) tensor; torch's reshape/view + split backward copies each gradient
    twice."""
    if y.dim() != 3 or not y.is_contiguous() or y.shape[-1] % (3 * num_heads):
        B, N, C = y.shape
        return tuple(t.reshape(B, N, num_heads, -1).transpose(1, 2) for t in y.split(C // 3, dim=-1))
    return _SplitHeads3.apply(y, num_heads)


class _ResidualDropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, o, p):
        from .ops import _draw_seed
        bm = not x.is_contiguous()  # batch-major (T, B, E) view: run on the (B, T, E) memory
        xm, om = (x.transpose(0, 1), o.transpose(0, 1)) if bm else (x, o)
        y = torch.empty_like(xm)
        seed = _draw_seed()
        p_ = lambda t: ctypes.c_void_p(t.data_ptr())
        with on_device(x.device):
            check(lib().csa_residual_dropout_fwd(p_(xm), p_(om), p_(y), y.numel(), p, seed, 0,
                                                 ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)),
                  "csa_residual_dropout_fwd")
        ctx.cfg = (bm, p, seed)
        return y.transpose(0, 1) if bm else y

    @staticmethod
    def backward(ctx, gy):
        bm, p, seed = ctx.cfg
        g = (gy.transpose(0, 1) if bm else gy).contiguous()  # same memory order as the forward
        d_o = torch.empty_like(g)
        p_ = lambda t: ctypes.c_void_p(t.data_ptr())
        with on_device(g.device):
            check(lib().csa_residual_dropout_bwd(p_(g), p_(d_o), g.numel(), p, seed, 0,
                                                 ctypes.c_void_p(torch.cuda.current_stream(g.device).cuda_stream)),
                  "csa_residual_dropout_bwd")
        return gy, (d_o.transpose(0, 1) if bm else d_o), None


def _aligned(t):
    return t.data_ptr() % 16 == 0


def residual_dropout(x, o, dropout: nn.Dropout):
    """x + dropout(o) (module/components.py SublayerConnection, module/sbm_model.py:29-31) as one
    csa_residual_dropout kernel per direction in training (Philox stream 5, oracle/philox.py:res_keep;
    no mask stored). Eval mode, p outside (0, 1), CPU tensors or mismatched layouts take torch's ops."""
    p = float(dropout.p)
    if (dropout.training and 0.0 < p < 1.0 and x.is_cuda and x.dtype == torch.float32 and o.dtype == torch.float32
            and x.shape == o.shape and x.stride() == o.stride() and _aligned(x) and _aligned(o)
            and (x.is_contiguous() or _batch_major(x))):
        return _ResidualDropoutFn.apply(x, o, p)
    return x + dropout(o)


class _GeluDropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, p):
        from .ops import _draw_seed
        bm = not h.is_contiguous()  # batch-major (T, B, F) view: run on the (B, T, F) memory
        hm = h.transpose(0, 1) if bm else h
        y = torch.empty_like(hm)
        seed = _draw_seed() if p > 0.0 else 0
        p_ = lambda t: ctypes.c_void_p(t.data_ptr())
        with on_device(h.device):
            check(lib().csa_gelu_dropout_fwd(p_(hm), p_(y), y.numel(), p, seed, 0,
                                             ctypes.c_void_p(torch.cuda.current_stream(h.device).cuda_stream)),
                  "csa_gelu_dropout_fwd")
        ctx.save_for_backward(hm)
        ctx.cfg = (bm, p, seed)
        return y.transpose(0, 1) if bm else y

    @staticmethod
    def backward(ctx, gy):
        (hm,) = ctx.saved_tensors
        bm, p, seed = ctx.cfg
        g = (gy.transpose(0, 1) if bm else gy).contiguous()
        dh = torch.empty_like(hm)
        p_ = lambda t: ctypes.c_void_p(t.data_ptr())
        with on_device(g.device):
            check(lib().csa_gelu_dropout_bwd(p_(g), p_(hm), p_(dh), g.numel(), p, seed, 0,
                                             ctypes.c_void_p(torch.cuda.current_stream(g.device).cuda_stream)),
                  "csa_gelu_dropout_bwd")
        return (dh.transpose(0, 1) if bm else dh), None


def gelu_dropout(h, dropout: nn.Dropout):
    """dropout(gelu(h)) (exact erf GELU; module/components.py FeedForward, module/sbm_model.py:22-26) as
    one csa_gelu_dropout kernel per direction (Philox stream 6, oracle/philox.py:ffn_keep; only h is
    saved). CPU tensors, non-fp32 or other layouts take torch's ops."""
    p = float(dropout.p) if dropout.training else 0.0
    if (h.is_cuda and h.dtype == torch.float32 and 0.0 <= p < 1.0 and _aligned(h)
            and (h.is_contiguous() or _batch_major(h))):
        return _GeluDropoutFn.apply(h, p)
    return dropout(F.gelu(h))
