"""ORACLE (test infrastructure only): closed-form fp64 forward/backward of SBM attention.

This is the math the HIP kernels implement (flash-style: no N x N intermediate is needed
beyond one tile), written out explicitly so it can be checked against the reference's
autograd (oracle/sbm_ref.py, itself pinned to tests/golden). Reference: module/sbm_attn.py:32-66,
module/STE.py:8-19.

Forward, per (b,h), query row i, key j (M keys, pad keys have mask=1):
    C   = layer.weight.reshape(H,k,d)[h];  S = softmax_{k^2}(C C^T)               (sbm_attn.py:37-39)
    Qh  = sigmoid(MLP(Q) C^T),  Kh = sigmoid(MLP(K) C^T),  T = Kh S^T (T_j = S Kh_j)  (:41-53)
    expA_ij = Qh_i . T_j ;  A_ij = [u_ij < clamp(expA_ij, .01, .99)]                 (:55, STE.py:10-15)
    e_ij = exp(s_ij - m_i), s = QK^T/sqrt(d) (pad keys -> e=0);  Z_i = sum_j e_ij
    Zg_i = sum_j e_ij A_ij ;  n_i = Zg_i / Z_i ;  D_i = max(n_i, 1e-12)                (:59-62)
    attn_ij = e_ij A_ij / (Z_i D_i);  X_i = sum_j attn_ij r_ij V_j  (r = dropout mult)  (:63)
    sparsity_h = sum_{b,i,j} A_ij / (B N M)                                           (:64)
Backward (F.normalize's L1 norm has grad sign(M), sign(0)=0; clamp_min passes iff n>=eps):
    gamma_i = dX_i . X_i   (= sum_j dattn_ij attn_ij)
    dattn_ij = r_ij (dX_i . V_j) (+ grad of the returned attn map)
    dM_ij = (dattn_ij - [n_i>=eps][M_ij>0] gamma_i) / D_i
    dP_ij = dM_ij A_ij ;  rho_i = sum_j P_ij dP_ij = (n_i>=eps ? 0 : gamma_i)
    ds_ij = P_ij (dP_ij - rho_i) / sqrt(d)  -> dQ += ds K, dK += ds^T Q
    dA_ij = dM_ij P_ij + dsparsity_h/(B N M) (+ grad of the returned graph)
    G_ij  = hardtanh(A_ij dA_ij)                                                      (STE.py:19)
    dQh = G T ;  dT = G^T Qh ;  dKh = dT S ;  dS += dT^T Kh (summed over b)
    then sigmoid', C^T, MLP backward; dS -> softmax_{k^2} backward -> dC += (dD + dD^T) C.
"""
import math

import torch

EPS = 1e-12


def _ident(t):
    return t


def _bf16_round(t):
    """Round to bf16 (RNE) and back: the operand rounding of a bf16-MFMA contraction (v_cvt_pk_bf16_f32)."""
    return t.to(torch.bfloat16).to(t.dtype)


def _mlp_fwd(x, W, keep, R=_ident):
    """Returns (out, [inputs of each Linear], [relu masks]). R rounds the operands of each x W^T product
    (bf16 emulation); the bias is added exactly, as the kernels do."""
    W0, b0, W1, b1, W2, b2 = W
    z0 = R(x) @ R(W0).T + b0
    if keep is not None and keep[0] is not None:
        z0 = z0 * keep[0]
    h1 = torch.relu(z0)
    z1 = R(h1) @ R(W1).T + b1
    if keep is not None and keep[1] is not None:
        z1 = z1 * keep[1]
    h2 = torch.relu(z1)
    out = R(h2) @ R(W2).T + b2
    return out, (x, h1, h2), (z0 > 0, z1 > 0)


def _mlp_bwd(dout, W, acts, masks, keep, R=_ident):
    W0, b0, W1, b1, W2, b2 = W
    x, h1, h2 = acts
    m0, m1 = masks
    g = {}
    g["proj.6.weight"] = torch.einsum("...o,...i->oi", R(dout), R(h2))
    g["proj.6.bias"] = dout.reshape(-1, dout.shape[-1]).sum(0)
    dh2 = R(dout) @ R(W2)
    dz1 = dh2 * m1
    if keep is not None and keep[1] is not None:
        dz1 = dz1 * keep[1]
    g["proj.3.weight"] = torch.einsum("...o,...i->oi", R(dz1), R(h1))
    g["proj.3.bias"] = dz1.reshape(-1, dz1.shape[-1]).sum(0)
    dh1 = R(dz1) @ R(W1)
    dz0 = dh1 * m0
    if keep is not None and keep[0] is not None:
        dz0 = dz0 * keep[0]
    g["proj.0.weight"] = torch.einsum("...o,...i->oi", R(dz0), R(x))
    g["proj.0.bias"] = dz0.reshape(-1, dz0.shape[-1]).sum(0)
    dx = R(dz0) @ R(W0)
    return dx, g


def sbm_fwd_bwd(Q, K, V, mask, params, u, num_clusters, dX, dsparsity, attn_keep=None, proj_keep=None,
                graph_override=None, bf16=False):
    """fp64 closed-form forward + backward. Returns (outputs dict, grads dict).

    bf16=True: an ideal CSA_DTYPE_BF16 implementation -- the operands of every contraction the bf16 mode
    runs on bf16 MFMA are rounded to bf16 (QK^T, dX V^T, PV with the unnormalised weights e A r, dV, dQ,
    dK, the three MLP layers and .C^T forward, C^T dZ, the W^T chains and the dW outer products backward;
    dC reads the projection output p as the bf16 mode saves it, rounded to bf16), everything else
    (accumulation, biases, softmax, sampling, expA, T, dQh, dT, dS, dZ) exact. The error of this emulation
    against the fp32 reference is what a bf16-operand implementation cannot avoid."""
    R = _bf16_round if bf16 else _ident
    f = lambda t: None if t is None else t.detach().double()
    Q, K, V, mask, u, dX, dsparsity = map(f, (Q, K, V, mask, u, dX, dsparsity))
    attn_keep = f(attn_keep)
    pk = {k: f(v) for k, v in (proj_keep or {}).items()}
    W = tuple(f(params[k]) for k in ("proj.0.weight", "proj.0.bias", "proj.3.weight", "proj.3.bias",
                                      "proj.6.weight", "proj.6.bias"))
    B, H, N, d = Q.shape
    M = V.shape[2]
    k = num_clusters
    C = f(params["layer.weight"]).reshape(H, k, d)
    D2 = C @ C.transpose(-1, -2)
    S = torch.softmax(D2.reshape(H, k * k), -1).reshape(H, k, k)
    Qp, qacts, qmasks = _mlp_fwd(Q, W, (pk.get("q0"), pk.get("q1")), R)
    Kp, kacts, kmasks = _mlp_fwd(K, W, (pk.get("k0"), pk.get("k1")), R)
    Qh = torch.sigmoid(R(Qp) @ R(C).transpose(-1, -2).unsqueeze(0))
    Kh = torch.sigmoid(R(Kp) @ R(C).transpose(-1, -2).unsqueeze(0))
    T = Kh @ S.transpose(-1, -2).unsqueeze(0)  # T_j = S Kh_j
    expA = Qh @ T.transpose(-1, -2)
    if graph_override is not None:
        A = f(graph_override)
    else:
        A = (u < expA.clamp(0.01, 0.99)).double()
    s = (R(Q) @ R(K).transpose(-1, -2)) / math.sqrt(d)
    s = s.masked_fill(mask[:, None, None, :] == 1, float("-inf"))
    mrow = s.max(-1, keepdim=True).values
    e = torch.exp(s - mrow)
    Z = e.sum(-1, keepdim=True)
    P = e / Z
    Mm = P * A
    n = Mm.sum(-1, keepdim=True)
    Dn = n.clamp_min(EPS)
    attn = Mm / Dn
    r = attn_keep if attn_keep is not None else torch.ones_like(attn)
    if bf16:  # the kernel rounds the unnormalised weights e A r (r: the dropout multiplier) and scales after
        X = (R(e * A * r) @ R(V)) / (Z * Dn)
    else:
        X = (attn * r) @ V
    sparsity = A.sum((0, 2, 3)) / (B * N * M)
    out = dict(X=X, sparsity=sparsity, graph=A, attn=attn, expA=expA, Qhat=Qh, Khat=Kh, T=T, S=S,
               rowmax=mrow[..., 0], Z=Z[..., 0], n=n[..., 0])

    g = {}
    g["V"] = R(attn * r).transpose(-1, -2) @ R(dX)
    dattn = (R(dX) @ R(V).transpose(-1, -2)) * r
    gamma = (dX * X).sum(-1, keepdim=True)
    big = (n >= EPS).double()
    dM = (dattn - big * (Mm > 0).double() * gamma) / Dn
    dP = dM * A
    rho = (1 - big) * gamma
    ds = P * (dP - rho) / math.sqrt(d)
    ds = torch.nan_to_num(ds)  # pad keys: P == 0
    dQ = R(ds) @ R(K)
    dK = R(ds).transpose(-1, -2) @ R(Q)
    dA = dM * P + (dsparsity / (B * N * M)).view(1, H, 1, 1)
    G = (A * dA).clamp(-1, 1)
    dQh = G @ T
    dT = G.transpose(-1, -2) @ Qh
    dKh = dT @ S  # T_j = S Kh_j  ->  dKh_j = S^T dT_j
    dS = torch.einsum("bhja,bhjc->hac", dT, Kh)
    dZq = dQh * Qh * (1 - Qh)
    dZk = dKh * Kh * (1 - Kh)
    dQp = R(dZq) @ R(C).unsqueeze(0)
    dKp = R(dZk) @ R(C).unsqueeze(0)
    dC = torch.einsum("bhnk,bhnd->hkd", dZq, R(Qp)) + torch.einsum("bhnk,bhnd->hkd", dZk, R(Kp))
    dD = S * (dS - (S * dS).sum((-1, -2), keepdim=True))
    dC = dC + (dD + dD.transpose(-1, -2)) @ C
    dQm, gq = _mlp_bwd(dQp, W, qacts, qmasks, (pk.get("q0"), pk.get("q1")), R)
    dKm, gk = _mlp_bwd(dKp, W, kacts, kmasks, (pk.get("k0"), pk.get("k1")), R)
    g["Q"] = dQ + dQm
    g["K"] = dK + dKm
    g["layer.weight"] = dC.reshape(H * k, d)
    for key in gq:
        g[key] = gq[key] + gk[key]
    g["_G"] = G
    g["_dQhat"] = dQh
    g["_dT"] = dT
    g["_dS"] = dS
    return out, g
