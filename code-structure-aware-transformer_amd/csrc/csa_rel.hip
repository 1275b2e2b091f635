// CSE disentangled AST-relation attention (module/disentangled_attn.py:44-65) on gfx950.
//
//   s[x,y] = (q_x.k_y + lq[rel[y,x]].k_y + q_x.lk[rel[x,y]]) / sqrt(3 d);  s[mask] = -1e9;
//   out = softmax(s) v
//
// Fused path (d_k = 64, every config; below): k_rel_logits (C2P = Q LK^T, P2CT = K LQ^T), k_rel_prep
// (permuted uint16 relation/mask code planes), k_rel_fwd_f (c2c MFMA + the two logit gathers, online
// softmax, PV; saves the gathered bias tile-major), k_rel_bwd_qf / k_rel_bwd_kf (query / key side
// backward, the gather backward as LDS bin histograms, no g/P materialised), k_rel_lgrad (dlk, dlq).
// Generic path (d_k = 16 / 32 / 96, tests only):
//   Forward:  k_bgemm   C2P  = Q LK^T   (B,H,N,Lp)   p2c/c2p relation logits, as the reference's
//             k_bgemm   P2CT = K LQ^T   (B,H,M,Lp)   lq @ k^T / q @ lk^T (disentangled_attn.py:53-58)
//             k_rel_fwd one wave per (b,h,32 queries): c2c by MFMA + per-element gathers of the two
//                       relation logits, -1e9 masking, online softmax, PV; saves (row max, 1/row sum).
//   Backward: k_rel_bwd_q    recompute P, dP = dO V^T (MFMA), g = P (dP - dO.O)/sqrt(3d) (0 where masked);
//                            dq += g K (MFMA); materialises g and P (B,H,N,N) once.
//             k_bgemm        dv = P^T dO, dk = g^T Q
//             k_rel_scatter  G_c2p[x][r] = sum_{y: rel[x,y]=r} g[x,y];  G_p2cT[y][r] = sum_{x: rel[y,x]=r} g[x,y]
//                            (the gather backward; one thread per row/column, fixed order => deterministic)
//             k_bgemm        dq += G_c2p LK ; dk += G_p2cT LQ ; dlk = sum_b G_c2p^T Q ; dlq = sum_b G_p2cT^T K
// Relation planes are uint8 (B,P,N,N) with a head->plane map (heads 0-3 parent plane L, 4-7 sibling
// plane T; module/csa_trans.py:206-211), replacing the reference's repeated int64 (B,8,N,N) copies.
#include "csa_common.hpp"
#include <algorithm>
#include "../../include/csa_hip.h"

#include <math.h>
#include <stdio.h>
#include <string.h>

using namespace csa;

namespace {

constexpr float NEG_INF = -__builtin_inff();

// ------------------------------------------------------------------------------------
// Generic batched fp32 MFMA GEMM:  C[bat](m,n) (+)= alpha * sum_{r<R} sum_{k<K} A(r,bat,m,k) * B(r,bat,n,k)
// element addresses: X[(bat / H2) * x_b1 + (bat % H2) * x_b2 + r * x_r + m * x_m + k * x_k]
// One wave per 32x32 C tile; K consumed in chunks of 32 (16 MFMA K-steps, lin perm).
// ------------------------------------------------------------------------------------
// R-split (rsplit > 1): blockIdx.z = split * nbat + bat; split s sums r in [s R / rsplit, (s+1) R / rsplit)
// into its own partial C at C + s * c_split (summed in split order by k_sum_splits: deterministic).
struct GemmArgs {
  const float* A; int64_t a_m, a_k, a_b1, a_b2, a_r;
  const float* B; int64_t b_n, b_k, b_b1, b_b2, b_r;
  float* C; int64_t c_m, c_n, c_b1, c_b2;
  int M, N, K, H2, R;
  float alpha; int accumulate;
  int rsplit, nbat; int64_t c_split;
};

// One 32-wide K chunk of lane operands: 16 consecutive k (lin permutation: half h takes
// [16h, 16h+16)). VEC: k is the contiguous dimension (x_k == 1, 16-B aligned rows whose
// allocation covers K rounded up to 4), loaded as dwordx4; otherwise strided scalar loads (the
// 32 lanes of a half are then the contiguous dimension). Addresses are always in bounds
// (clamped); validity only selects the value, so no branch surrounds a load.
template <bool VEC>
__device__ __forceinline__ void chunk_load(float* v, const float* __restrict__ row, int64_t xk, int kb, int K,
                                           bool rv) {
  if constexpr (VEC) {
#pragma unroll
    for (int s = 0; s < 16; s += 4) {
      const int kk = kb + s;
      const f32x4 x = *reinterpret_cast<const f32x4*>(row + (kk < K ? kk : 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) v[s + e] = (rv && kk + e < K) ? x[e] : 0.f;
    }
  } else {
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      const int kk = kb + s;
      const float x = row[(int64_t)(kk < K ? kk : 0) * xk];
      v[s] = (rv && kk < K) ? x : 0.f;
    }
  }
}

// AV && BV: register double buffering, chunk k0 + 32 in flight while chunk k0's 16 MFMAs run.
// Otherwise single-buffered (the strided scalar operand's address math already holds ~100 VGPRs;
// double buffering it halved occupancy and ran slower).
template <bool AV, bool BV>
__global__ __launch_bounds__(64) void k_bgemm(const GemmArgs g) {
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * 32, m0 = blockIdx.y * 32;
  const int bat = g.rsplit > 1 ? (int)blockIdx.z % g.nbat : (int)blockIdx.z;
  const int split = g.rsplit > 1 ? (int)blockIdx.z / g.nbat : 0;
  const int r_lo = (int)((int64_t)split * g.R / (g.rsplit > 1 ? g.rsplit : 1));
  const int r_hi = (int)((int64_t)(split + 1) * g.R / (g.rsplit > 1 ? g.rsplit : 1));
  const int b1 = bat / g.H2, b2 = bat % g.H2;
  const float* A = g.A + b1 * g.a_b1 + b2 * g.a_b2;
  const float* Bp = g.B + b1 * g.b_b1 + b2 * g.b_b2;
  const int m = m0 + c, n = n0 + c;
  const bool mv = m < g.M, nv = n < g.N;
  f32x16 acc = zero16();
  if constexpr (AV && BV) {
    const int mc = imin(m, g.M - 1), nc = imin(n, g.N - 1);
    for (int r = r_lo; r < r_hi; ++r) {
      const float* Ar = A + r * g.a_r + (int64_t)mc * g.a_m;
      const float* Br = Bp + r * g.b_r + (int64_t)nc * g.b_n;
      float av[16], bv[16];
      chunk_load<true>(av, Ar, 1, 16 * h, g.K, mv);
      chunk_load<true>(bv, Br, 1, 16 * h, g.K, nv);
      for (int k0 = 0; k0 < g.K; k0 += 32) {
        float an[16], bn[16];
        chunk_load<true>(an, Ar, 1, k0 + 32 + 16 * h, g.K, mv);
        chunk_load<true>(bn, Br, 1, k0 + 32 + 16 * h, g.K, nv);
#pragma unroll
        for (int s = 0; s < 16; ++s) acc = mfma(av[s], bv[s], acc);
#pragma unroll
        for (int s = 0; s < 16; ++s) { av[s] = an[s]; bv[s] = bn[s]; }
      }
    }
  } else {
    for (int r = r_lo; r < r_hi; ++r) {
      const float* Ar = A + r * g.a_r + (int64_t)(AV ? imin(m, g.M - 1) : m) * g.a_m;
      const float* Br = Bp + r * g.b_r + (int64_t)(BV ? imin(n, g.N - 1) : n) * g.b_n;
      for (int k0 = 0; k0 < g.K; k0 += 32) {
        float av[16], bv[16];
        if constexpr (AV) {
          chunk_load<true>(av, Ar, 1, k0 + 16 * h, g.K, mv);
        } else {
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            const int kk = k0 + 16 * h + s;
            av[s] = (mv && kk < g.K) ? Ar[(int64_t)kk * g.a_k] : 0.f;
          }
        }
        if constexpr (BV) {
          chunk_load<true>(bv, Br, 1, k0 + 16 * h, g.K, nv);
        } else {
#pragma unroll
          for (int s = 0; s < 16; ++s) {
            const int kk = k0 + 16 * h + s;
            bv[s] = (nv && kk < g.K) ? Br[(int64_t)kk * g.b_k] : 0.f;
          }
        }
#pragma unroll
        for (int s = 0; s < 16; ++s) acc = mfma(av[s], bv[s], acc);
      }
    }
  }
  float* C = g.C + b1 * g.c_b1 + b2 * g.c_b2 + split * g.c_split;
  if (nv) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = m0 + crow(r, h);
      if (mm < g.M) {
        float* p = C + (int64_t)mm * g.c_m + (int64_t)n * g.c_n;
        *p = g.accumulate ? *p + g.alpha * acc[r] : g.alpha * acc[r];
      }
    }
  }
}

// out[e] = sum_{s < RS} part[s * stride + e], in split order
__global__ __launch_bounds__(256) void k_sum_splits(const float* __restrict__ part, float* __restrict__ out, int64_t n,
                                                    int RS, int64_t stride) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    float v = 0.f;
    for (int s = 0; s < RS; ++s) v += part[s * stride + e];
    out[e] = v;
  }
}

// The two partial sets of k_rel_lgrad (dlk: blockIdx.y = 0, dlq: 1) in one launch: out[e] = sum_{s < RS}
// part[s * n + e] in split order (bit-identical to k_sum_splits), eight independent loads in flight per step
__global__ __launch_bounds__(256) void k_sum_splits2(const float* __restrict__ part0, const float* __restrict__ part1,
                                                     float* __restrict__ out0, float* __restrict__ out1, int64_t n,
                                                     int RS) {
  const float* part = blockIdx.y ? part1 : part0;
  float* out = blockIdx.y ? out1 : out0;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  float v = 0.f;
  int s = 0;
  for (; s + 8 <= RS; s += 8) {
    float t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) t[u] = part[(int64_t)(s + u) * n + e];
#pragma unroll
    for (int u = 0; u < 8; ++u) v += t[u];
  }
  for (; s < RS; ++s) v += part[(int64_t)s * n + e];
  out[e] = v;
}

struct RelArgs {
  int B, H, N, L, Lp, NQB, NKB, group;
  int ldg;  // row stride of the G^T / P^T images (N rounded up to 4: 16-B aligned rows)
  const float *q, *k, *v; int64_t q_sb, q_sh, q_sn, k_sb, k_sh, k_sn, v_sb, v_sh, v_sn;
  const uint8_t *rel, *mask; int64_t rel_sb, rel_sh, mask_sb, mask_sh;
  const float *c2p, *p2ct;  // (B,H,N,Lp), (B,H,N,Lp)
  float *out, *stats;
  int64_t o_sb, o_sh, o_sn;  // element strides of out (fused path; contiguous otherwise)
  float inv_scale;
  // backward
  const float* dout;
  int64_t do_sb, do_sh, do_sn, dq_sb, dq_sh, dq_sn, dk_sb, dk_sh, dk_sn, dv_sb, dv_sh, dv_sn;
  float *dq, *G, *P;
  // fused path (d_k = 64): prepared planes, plane count, padded size, bins layout, gather-backward output
  const uint16_t *RM, *RT; int P_, NP, KB2, LB; int64_t ldx;
  const float* RB;  // tile-major relation bias (written by k_rel_fwd_f)
  int bf16;         // CSA_DTYPE_BF16: bf16 MFMA for c2c, PV and their gradients
  float *dk, *dv, *gc2p, *gp2ct, *qstat;
  float* gt;  // fp32 16-row path: softmax-input gradient tiles k_rel_bwd_kh -> k_rel_bwd_qg ([key][query] 32 x 32)
  const float *lq, *lk;
  int qstat_pre;  // qstat written by k_rel_qstat (concurrent backward): k_rel_bwd_qf leaves it alone
  int LB16, Q4;   // 16-row bins (k_rel_bwd_kh / qg): row stride and the per-lane-group K range
};

__device__ __forceinline__ int64_t plane_off(const RelArgs& p, int b, int hd, int64_t sb, int64_t sh) {
  if (p.group > 0) return b * sb + (hd >= p.group ? 1 : 0) * sh;
  return b * sb + hd * sh;
}

// A lane's accumulator tiles (rows 32 t + crow(r, h) of one output row) -> out[0 .. 32 DT)
template <int DT>
__device__ __forceinline__ void store_rows_f(float* __restrict__ out, const f32x16 (&a)[DT]) {
  const int h = lane_id() >> 5;
#pragma unroll
  for (int t = 0; t < DT; ++t)
#pragma unroll
    for (int g4 = 0; g4 < 4; ++g4) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = a[t][4 * g4 + e];
      *reinterpret_cast<f32x4*>(out + 32 * t + 8 * g4 + 4 * h) = v;
    }
}

// Score of one (x, y) element; returns NEG_INF outside the matrix.
// All loads are unconditional on clamped indices (a branch around a load serialises the tile's
// loads behind vmcnt(0), see csa_common.hpp load_run); validity is applied to the value.
__device__ __forceinline__ float rel_score(const RelArgs& p, float c2c, int x, int y, const uint8_t* rp,
                                           const uint8_t* mp, const float* c2p, const float* p2ct) {
  const bool inside = x < p.N && y < p.N;
  const int xc = imin(x, p.N - 1), yc = imin(y, p.N - 1);
  int rxy = rp[(int64_t)xc * p.N + yc], ryx = rp[(int64_t)yc * p.N + xc];
  rxy = rxy < p.L ? rxy : p.L - 1;  // memory safety; the reference requires rel < L
  ryx = ryx < p.L ? ryx : p.L - 1;
  const bool masked = mp[(int64_t)xc * p.N + yc] != 0;
  const float v = (c2c + c2p[(int64_t)xc * p.Lp + rxy] + p2ct[(int64_t)yc * p.Lp + ryx]) * p.inv_scale;
  return !inside ? NEG_INF : masked ? -1e9f : v;  // masked_fill(mask == 1, -1e9) (disentangled_attn.py:62)
}

// ------------------------------------------------------------------------------------
// Forward: one wave per (b,h, 32-query block); S^T orientation (keys = acc rows, queries = lanes)
// ------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(64) void k_rel_fwd(const RelArgs p) {
  constexpr int DT = (D + 31) / 32, NS = D / 2;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const BhBlock xb = xcd_block(p.NQB, p.B * p.H);
  if (!xb.valid) return;
  const int qb = xb.blk, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const int i = qb * 32 + c;
  const bool iv = i < p.N;
  const int ic = imin(i, p.N - 1);
  float q[NS];
  load_run<NS>(q, p.q + b * p.q_sb + hd * p.q_sh + (int64_t)ic * p.q_sn + h * NS, iv);
  const float* kb = p.k + b * p.k_sb + hd * p.k_sh;
  const float* vb = p.v + b * p.v_sb + hd * p.v_sh;
  const uint8_t* rp = p.rel + plane_off(p, b, hd, p.rel_sb, p.rel_sh);
  const uint8_t* mp = p.mask + plane_off(p, b, hd, p.mask_sb, p.mask_sh);
  const float* c2p = p.c2p + (int64_t)bh * p.N * p.Lp;
  const float* p2ct = p.p2ct + (int64_t)bh * p.N * p.Lp;
  float m_run = NEG_INF, zp = 0.f;
  f32x16 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = zero16();
  for (int kt = 0; kt < p.NKB; ++kt) {
    const int j0 = kt * 32, jl = j0 + c;
    float kr[NS];
    load_run<NS>(kr, kb + (int64_t)imin(jl, p.N - 1) * p.k_sn + h * NS, jl < p.N);
    f32x16 sacc = zero16();
#pragma unroll
    for (int s = 0; s < NS; ++s) sacc = mfma(kr[s], q[s], sacc);
    float sv[16];
    float tmax = NEG_INF;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      sv[r] = rel_score(p, sacc[r], i, j0 + crow(r, h), rp, mp, c2p, p2ct);
      tmax = fmaxf(tmax, sv[r]);
    }
    tmax = xhalf_max(tmax);
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = (m_new == NEG_INF) ? 1.f : __expf(m_run - m_new);
    zp *= alpha;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
    float w[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      w[r] = (sv[r] == NEG_INF) ? 0.f : __expf(sv[r] - m_new);
      zp += w[r];
    }
    m_run = m_new;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = j0 + crow(r, h);
        const float vt = ldz(vb, (int64_t)imin(j, p.N - 1) * p.v_sn + imin(32 * t + c, D - 1), INT64_MAX,
                             j < p.N && 32 * t + c < D);
        o[t] = mfma(vt, w[r], o[t]);
      }
  }
  const float Z = xhalf_sum(zp);
  if (iv) {
    const float inv = 1.f / Z;
    float* xo = p.out + ((int64_t)bh * p.N + i) * D;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = o[t][4 * g4 + e] * inv;
        if (32 * t + 8 * g4 + 4 * h < D) *reinterpret_cast<f32x4*>(xo + 32 * t + 8 * g4 + 4 * h) = v;
      }
    if (h == 0) {
      p.stats[((int64_t)bh * p.N + i) * 2] = m_run;
      p.stats[((int64_t)bh * p.N + i) * 2 + 1] = inv;
    }
  }
}

// ------------------------------------------------------------------------------------
// Backward (query side): g, P materialised; dq (c2c part) by MFMA
// ------------------------------------------------------------------------------------
template <int D>
__global__ __launch_bounds__(64) void k_rel_bwd_q(const RelArgs p) {
  constexpr int DT = (D + 31) / 32, NS = D / 2;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const BhBlock xb = xcd_block(p.NQB, p.B * p.H);
  if (!xb.valid) return;
  const int qb = xb.blk, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const int i = qb * 32 + c;
  const bool iv = i < p.N;
  const int ic = imin(i, p.N - 1);
  float q[NS], dO[NS];
  load_run<NS>(q, p.q + b * p.q_sb + hd * p.q_sh + (int64_t)ic * p.q_sn + h * NS, iv);
  load_run<NS>(dO, p.dout + ((int64_t)bh * p.N + ic) * D + h * NS, iv);
  float dp = 0.f;
  {
    float o[NS];
    load_run<NS>(o, p.out + ((int64_t)bh * p.N + ic) * D + h * NS, iv);
#pragma unroll
    for (int s = 0; s < NS; ++s) dp = fmaf(dO[s], o[s], dp);
  }
  const float delta = xhalf_sum(dp);
  const float rmax = p.stats[((int64_t)bh * p.N + ic) * 2];
  const float rinv = p.stats[((int64_t)bh * p.N + ic) * 2 + 1];
  const float* kb = p.k + b * p.k_sb + hd * p.k_sh;
  const float* vb = p.v + b * p.v_sb + hd * p.v_sh;
  const uint8_t* rp = p.rel + plane_off(p, b, hd, p.rel_sb, p.rel_sh);
  const uint8_t* mp = p.mask + plane_off(p, b, hd, p.mask_sb, p.mask_sh);
  const float* c2p = p.c2p + (int64_t)bh * p.N * p.Lp;
  const float* p2ct = p.p2ct + (int64_t)bh * p.N * p.Lp;
  float* __restrict__ Gb = p.G + (int64_t)bh * p.N * p.ldg;
  float* __restrict__ Pb = p.P + (int64_t)bh * p.N * p.ldg;
  f32x16 dq[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) dq[t] = zero16();
  for (int kt = 0; kt < p.NKB; ++kt) {
    const int j0 = kt * 32, jl = j0 + c;
    const bool jv = jl < p.N;
    const int jc = imin(jl, p.N - 1);
    f32x16 sacc = zero16(), dpacc = zero16();
    {
      float kr[NS];
      load_run<NS>(kr, kb + (int64_t)jc * p.k_sn + h * NS, jv);
#pragma unroll
      for (int s = 0; s < NS; ++s) sacc = mfma(kr[s], q[s], sacc);
    }
    {
      float vr[NS];
      load_run<NS>(vr, vb + (int64_t)jc * p.v_sn + h * NS, jv);
#pragma unroll
      for (int s = 0; s < NS; ++s) dpacc = mfma(vr[s], dO[s], dpacc);
    }
    // all of the tile's score gathers first, so they are issued back to back instead of each
    // waiting behind the previous element's G/P stores (G/P are __restrict__)
    float sc[16];
    bool msk[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int y = j0 + crow(r, h);
      sc[r] = rel_score(p, sacc[r], i, y, rp, mp, c2p, p2ct);
      msk[r] = mp[(int64_t)ic * p.N + imin(y, p.N - 1)] != 0;
    }
    float gv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int y = j0 + crow(r, h);
      const bool inside = sc[r] != NEG_INF;
      const float P = inside ? __expf(sc[r] - rmax) * rinv : 0.f;
      const float g = (inside && !msk[r]) ? P * (dpacc[r] - delta) * p.inv_scale : 0.f;
      // transposed images G^T / P^T [y][x] (row stride ldg): the 32 query lanes store one
      // contiguous 128-B run per key
      if (inside) {
        Gb[(int64_t)y * p.ldg + i] = g;
        Pb[(int64_t)y * p.ldg + i] = P;
      }
      gv[r] = g;
    }
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int j = j0 + crow(r, h);
        const float kv = ldz(kb, (int64_t)imin(j, p.N - 1) * p.k_sn + imin(32 * t + c, D - 1), INT64_MAX,
                             j < p.N && 32 * t + c < D);
        dq[t] = mfma(kv, gv[r], dq[t]);
      }
  }
  if (iv) {
    float* dst = p.dq + ((int64_t)bh * p.N + i) * D;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        f32x4 v;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = dq[t][4 * g4 + e];
        if (32 * t + 8 * g4 + 4 * h < D) *reinterpret_cast<f32x4*>(dst + 32 * t + 8 * g4 + 4 * h) = v;
      }
  }
}

// Gather backward as a deterministic scatter: one thread owns one row (mode 0: G_c2p[x][.], bins
// over rel[x,y] along y) or one column (mode 1: G_p2cT[y][.], bins over rel[y,x] along x).
__global__ __launch_bounds__(64) void k_rel_scatter(const RelArgs p, float* __restrict__ out, int mode) {
  extern __shared__ __attribute__((aligned(16))) float bins[];
  const int t = threadIdx.x;
  const int64_t rowid = (int64_t)blockIdx.x * 64 + t;  // over B*H*N
  float* my = bins + t * p.Lp;
  for (int r = 0; r < p.Lp; ++r) my[r] = 0.f;
  if (rowid < (int64_t)p.B * p.H * p.N) {
    const int bh = (int)(rowid / p.N), x = (int)(rowid % p.N);
    const int b = bh / p.H, hd = bh % p.H;
    const uint8_t* rp = p.rel + plane_off(p, b, hd, p.rel_sb, p.rel_sh);
    const float* Gb = p.G + (int64_t)bh * p.N * p.ldg;  // G^T [y][x]
    if (mode == 0) {
      for (int y = 0; y < p.N; ++y) {
        int r = rp[(int64_t)x * p.N + y];
        r = r < p.L ? r : p.L - 1;
        my[r] += Gb[(int64_t)y * p.ldg + x];
      }
    } else {
      for (int xx = 0; xx < p.N; ++xx) {
        int r = rp[(int64_t)x * p.N + xx];  // rel[y = x][xx]
        r = r < p.L ? r : p.L - 1;
        my[r] += Gb[(int64_t)x * p.ldg + xx];
      }
    }
    float* o = out + rowid * p.Lp;
    for (int r = 0; r < p.Lp; ++r) o[r] = my[r];
  }
}


// ------------------------------------------------------------------------------------
// Fused path (d_k = 64): prepared relation planes, LDS-DMA tile images, in-kernel gather backward
// ------------------------------------------------------------------------------------
// Prepared planes per (batch element, relation plane), NP = 32 ceil(N/32) rows and columns, uint16:
//   RM[a][tile_pos(b)] = rel[a][b] | mask[a][b] << 8      RT[a][tile_pos(b)] = rel[b][a] | mask[b][a] << 8
// Columns are permuted inside each 32-wide tile so that the 16 elements a lane holds in MFMA
// accumulator registers r = 0..15 of half h (column crow(r, h)) sit at positions 16 h + r: a lane's
// codes for one tile are 32 contiguous bytes (two dwordx4 loads) of ITS OWN row. The forward (lane =
// query x) reads rel[x][y] + mask[x][y] from RM and rel[y][x] from RT for its two logit gathers; the
// query-side backward reads rel[x][y] (its c2p bin) from RM, the key-side backward (lane = key y)
// rel[y][x] (its p2c bin) from RM -- no byte-wise or transposed access anywhere, and a general
// (asymmetric) mask stays exact. Entries outside [0,N)^2 hold 0x0100.
__host__ __device__ constexpr int tile_pos(int j) { return 16 * ((j >> 2) & 1) + (j & 3) + 4 * (j >> 3); }

// One 32-row block of one plane per workgroup (round 5; was one 32 x 32 tile per workgroup, 5x the workgroups
// for the same bytes: 11.6 us at B = 64, latency-bound). The block's rel / mask rows are one contiguous byte
// range of the (.., N, N) plane, staged into LDS (dword loads when it is 4-byte aligned, as at N = 150); a
// thread then codes 4 consecutive columns of one row in every column tile, which tile_pos keeps contiguous
// (positions 16 (k & 1) + 4 (k >> 1) + 0..3 for column group k): RM takes one 8-B store per thread and tile, and
// so does RT, whose row y of this block reads the staged column y.
// Dynamic LDS: rel_prep_lds_bytes(N) = two staged 32 x N byte blocks (64 KB at N = 1024).
inline size_t rel_prep_lds_bytes(int64_t N) { return 2 * (size_t)((32 * N + 15) / 16 * 16); }
// One (32-row block at, plane bp) item on NTH threads (tid < NTH): k_rel_prep runs it on 256, k_rel_logits' extra
// one-wave workgroups on 64 (the same stores, so the planes are identical either way).
template <int NTH>
__device__ __forceinline__ void rel_prep_item(const RelArgs& p, uint16_t* __restrict__ RM, uint16_t* __restrict__ RT,
                                              uint8_t* srel, int at, int bp, int tid) {
  uint8_t* const smask = srel + (32 * p.N + 15) / 16 * 16;
  const int NT = p.NP / 32;
  const int b = bp / p.P_, pl = bp % p.P_;
  const int hd = p.group > 0 ? (pl == 0 ? 0 : p.group) : pl;  // a head that reads plane pl
  const int a0 = at * 32, nrow = imin(32, p.N - a0);
  const uint8_t* rp = p.rel + plane_off(p, b, hd, p.rel_sb, p.rel_sh) + (int64_t)a0 * p.N;
  const uint8_t* mp = p.mask + plane_off(p, b, hd, p.mask_sb, p.mask_sh) + (int64_t)a0 * p.N;
  const int nbytes = nrow * p.N;
  if ((((uintptr_t)rp | (uintptr_t)mp | (uintptr_t)nbytes) & 3) == 0) {
    for (int e = tid; e < nbytes / 4; e += NTH) {
      reinterpret_cast<uint32_t*>(srel)[e] = reinterpret_cast<const uint32_t*>(rp)[e];
      reinterpret_cast<uint32_t*>(smask)[e] = reinterpret_cast<const uint32_t*>(mp)[e];
    }
  } else {
    for (int e = tid; e < nbytes; e += NTH) { srel[e] = rp[e]; smask[e] = mp[e]; }
  }
  __syncthreads();
  uint16_t* rm = RM + (size_t)bp * p.NP * p.NP;
  uint16_t* rt = RT + (size_t)bp * p.NP * p.NP;
  auto code = [&](int row, int col) -> uint32_t {  // staged (row, col) of this block; 0x0100 outside [0,N)^2
    if (row >= nrow || col >= p.N) return 0x0100u;
    int r = srel[row * p.N + col];
    r = r < p.L ? r : p.L - 1;  // memory safety; the reference requires rel < L
    return (uint32_t)r | (smask[row * p.N + col] ? 0x100u : 0u);
  };
  for (int t = tid; t < 256; t += NTH) {  // 32 rows x 8 column groups
    const int rl = t >> 3, k = t & 7, pos = 16 * (k & 1) + 4 * (k >> 1);
    const int a = a0 + rl;
    for (int bt = 0; bt < NT; ++bt) {
      const int c0 = bt * 32 + 4 * k;
      // RM row a, columns c0 .. c0 + 3: rel[a][c] | mask[a][c] << 8
      *reinterpret_cast<uint2*>(rm + (size_t)a * p.NP + bt * 32 + pos) =
          uint2{code(rl, c0) | (code(rl, c0 + 1) << 16), code(rl, c0 + 2) | (code(rl, c0 + 3) << 16)};
      // RT row y = bt * 32 + rl, columns a0 + 4 k .. + 3: rel[x][y] of the staged rows x
      const int y = bt * 32 + rl, x0 = 4 * k;
      *reinterpret_cast<uint2*>(rt + (size_t)y * p.NP + a0 + pos) =
          uint2{code(x0, y) | (code(x0 + 1, y) << 16), code(x0 + 2, y) | (code(x0 + 3, y) << 16)};
    }
  }
}

__global__ __launch_bounds__(256) void k_rel_prep(const RelArgs p, uint16_t* __restrict__ RM, uint16_t* __restrict__ RT) {
  extern __shared__ __attribute__((aligned(16))) uint8_t srel[];
  rel_prep_item<256>(p, RM, RT, srel, (int)blockIdx.x, (int)blockIdx.y, (int)threadIdx.x);
}

// k_rel_prep for N > 1024 (its staged rows would exceed 64 KB of LDS): one 32 x 32 tile of one plane per workgroup; a thread codes 4 consecutive columns of one row, which
// tile_pos keeps contiguous (positions 16 (k & 1) + 4 (k >> 1) + 0..3 for column group k), so RM and RT
// take one 8-B store per thread (RT through the LDS transpose).
__global__ __launch_bounds__(256) void k_rel_prep_t(const RelArgs p, uint16_t* __restrict__ RM, uint16_t* __restrict__ RT) {
  __shared__ uint16_t tile[32][36];  // [row a][column b] of the tile's codes (36: 8-B aligned rows)
  const int NT = p.NP / 32, at = (int)blockIdx.x / NT, bt = (int)blockIdx.x % NT;
  const int bp = blockIdx.y, b = bp / p.P_, pl = bp % p.P_;
  const int hd = p.group > 0 ? (pl == 0 ? 0 : p.group) : pl;  // a head that reads plane pl
  const uint8_t* rp = p.rel + plane_off(p, b, hd, p.rel_sb, p.rel_sh);
  const uint8_t* mp = p.mask + plane_off(p, b, hd, p.mask_sb, p.mask_sh);
  uint16_t* rm = RM + (size_t)bp * p.NP * p.NP;
  uint16_t* rt = RT + (size_t)bp * p.NP * p.NP;
  const int t = (int)threadIdx.x, rl = t >> 3, k = t & 7, pos = 16 * (k & 1) + 4 * (k >> 1);
  const int a = at * 32 + rl;
  uint16_t code[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int bb = bt * 32 + 4 * k + i;
    code[i] = 0x0100;
    if (a < p.N && bb < p.N) {
      int r = rp[(int64_t)a * p.N + bb];
      r = r < p.L ? r : p.L - 1;  // memory safety; the reference requires rel < L
      code[i] = (uint16_t)(r | (mp[(int64_t)a * p.N + bb] ? 0x100 : 0));
    }
    tile[rl][4 * k + i] = code[i];
  }
  *reinterpret_cast<uint2*>(rm + (size_t)a * p.NP + bt * 32 + pos) =
      uint2{(uint32_t)code[0] | ((uint32_t)code[1] << 16), (uint32_t)code[2] | ((uint32_t)code[3] << 16)};
  __syncthreads();
  // RT row bt * 32 + rl, columns a = at * 32 + 4 k + i: tile[4 k + i][rl]
  *reinterpret_cast<uint2*>(rt + (size_t)(bt * 32 + rl) * p.NP + at * 32 + pos) =
      uint2{(uint32_t)tile[4 * k][rl] | ((uint32_t)tile[4 * k + 1][rl] << 16),
            (uint32_t)tile[4 * k + 2][rl] | ((uint32_t)tile[4 * k + 3][rl] << 16)};
}

struct Codes { uint32_t w[8]; };
// a lane's 16 codes of one tile (32 B of its own prepared row)
__device__ __forceinline__ Codes load_codes(const uint16_t* __restrict__ row, int tile) {
  Codes k;
  const uint32_t* q = reinterpret_cast<const uint32_t*>(row + 32 * tile + 16 * (lane_id() >> 5));
  const u32x4 a = *reinterpret_cast<const u32x4*>(q), bq = *reinterpret_cast<const u32x4*>(q + 4);
  k.w[0] = a.x; k.w[1] = a.y; k.w[2] = a.z; k.w[3] = a.w; k.w[4] = bq.x; k.w[5] = bq.y; k.w[6] = bq.z; k.w[7] = bq.w;
  return k;
}
__device__ __forceinline__ uint32_t code_of(const Codes& k, int r) { return (k.w[r >> 1] >> (16 * (r & 1))) & 0xffffu; }

__device__ __forceinline__ const uint16_t* prep_row(const RelArgs& p, const uint16_t* plane, int b, int hd, int row) {
  const int pl = p.group > 0 ? (hd >= p.group ? 1 : 0) : (p.P_ == 1 ? 0 : hd);
  return plane + ((size_t)(b * p.P_ + pl) * p.NP + row) * p.NP;
}

// bins (32 rows x LB floats, LB / 4 odd: the 16 rows of a ds_read_b128 lane group hit 16 distinct
// 16-B bank slots) += g at column rel, the two lane halves one after the other (they share rows),
// lanes of a half own distinct rows: no two lanes ever add to one address in the same instruction and
// a row's additions happen in a fixed order -> deterministic.
__device__ __forceinline__ void bins_scatter(float* bins, int LB, const float (&g)[16], const uint32_t (&col)[16]) {
  const int c = lane_id() & 31, h = lane_id() >> 5;
  float* row = bins + c * LB;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    if (h == pass) {
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (g[r] != 0.f) atomicAdd(row + col[r], g[r]);
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): pass 0's adds land before pass 1's
  }
}

// acc[t] (rows d = 32 t + crow(r,h), lanes = the bins' rows) += sum_r Lmat[r][d] * bins[lane row][r]
// (dq_rel = G_c2p LK or dk_rel = G_p2cT LQ), K = 2 KB2 (lin perm: k = s + KB2 h), Lmat rows >= L read 0.
// The Lmat operand comes from L2 (the head's L x d matrix): a ring of RING groups of 4 K-steps is kept in
// flight (RING - 1 groups ahead, ~1500 MFMA cycles), which covers the L2 latency at one wave per SIMD;
// a lookahead of one group left this phase latency-bound. The chunks of RING groups run unguarded
// (a prefetch past the end loads a clamped, never-used row); the < RING leftover groups follow.
template <int DT>
__device__ __forceinline__ void bins_times(f32x16 (&acc)[DT], const float* bins, int LB, int KB2,
                                           const float* __restrict__ Lmat, int L, int D) {
  constexpr int RING = 4;
  const int c = lane_id() & 31, h = lane_id() >> 5;
  const float* brow = bins + c * LB + KB2 * h;
  auto lmat = [&](int s4, float (&v)[4][DT]) {  // Lmat rows s4 + e + KB2 h (0 beyond L), columns 32 t + c
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = s4 + e + KB2 * h;
      const float* lr = Lmat + (int64_t)(r < L ? r : 0) * D;
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        const float lv = lr[32 * t + c];
        v[e][t] = r < L ? lv : 0.f;
      }
    }
  };
  auto group = [&](int g, const float (&v)[4][DT]) {
    const f32x4 bv = *reinterpret_cast<const f32x4*>(brow + 4 * g);
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int t = 0; t < DT; ++t) acc[t] = mfma(v[e][t], bv[e], acc[t]);
  };
  const int ng = KB2 / 4, ngf = ng / RING * RING;  // groups of 4 K-steps per half; in whole chunks
  float lv[RING][4][DT];
#pragma unroll
  for (int u = 0; u < RING - 1; ++u) lmat(4 * u, lv[u]);
  for (int g0 = 0; g0 < ngf; g0 += RING) {
#pragma unroll
    for (int u = 0; u < RING; ++u) {
      lmat(4 * (g0 + u + RING - 1), lv[(u + RING - 1) % RING]);
      group(g0 + u, lv[u]);
    }
  }
#pragma unroll
  for (int u = 0; u < RING - 1; ++u)  // leftover groups ngf + u < ng: already in ring slot u
    if (ngf + u < ng) group(ngf + u, lv[u]);
}

// bins row of this lane (row = lane & 31, the half's columns [KB2 h, KB2 h + KB2) clipped to Lp) -> column
// `row` of a transposed (Lp, ldx) table: for each bin r the 32 lanes of a half store 32 consecutive
// floats (coalesced), and the dlq / dlk GEMMs then read it with x contiguous (dwordx4 operand loads).
__device__ __forceinline__ void bins_store_t(float* __restrict__ outT, int64_t ldx, int row, const float* bins, int LB,
                                             int KB2, int Lp, bool valid) {
  if (!valid) return;
  const int c = lane_id() & 31, h = lane_id() >> 5;
  const float* brow = bins + c * LB;
  const int r1 = imin(KB2 * h + KB2, Lp);
  for (int r = KB2 * h; r < r1; ++r) outT[(int64_t)r * ldx + row] = brow[r];
}

// One l-tile of k_rel_logits: both chains from the slab image (TWO: the pair's second block exists; a
// wave-uniform choice of body, so the single-block tail wave issues half the MFMAs), the refill, the stores.
template <int D, bool TWO>
__device__ __forceinline__ void logits_tile(const RelArgs& p, const float* lds, uint32_t L0, __amdgpu_buffer_rsrc_t lr,
                                            const DmaPat& pat, int rbase, const float (&xr0)[D / 2],
                                            const float (&xr1)[D / 2], float* out, int rp, int lt, int NLT, int lane) {
  constexpr int NS = D / 2;
  const int c = lane & 31, h = lane >> 5;
  const int l = lt * 32 + c;
  // slab lt has landed: vector memory operations retire in issue order, so waiting until only the previous
  // tile's stores (issued after slab lt's DMA) are outstanding suffices
  if (lt == 0) wait_vm_all();
  else if constexpr (TWO) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  f32x16 acc0 = zero16(), acc1 = zero16();
#pragma unroll
  for (int j = 0; j < NS / 4; ++j) {
    const f32x4 lv = lds_f4(lds, rbase ^ (16 * j));
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc0 = mfma(xr0[4 * j + e], lv[e], acc0);  // D[x][l]
      if constexpr (TWO) acc1 = mfma(xr1[4 * j + e], lv[e], acc1);
    }
  }
  if (lt + 1 < NLT) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slab lt read out before it is refilled
    dma64(L0, lr, pat, D * 4, (lt + 1) * 32);
  }
  // buffer stores: rows past N fall outside the descriptor and columns past L get an out-of-range offset, so
  // the range check drops both (no per-element branches); the row part of the offset is wave-uniform (soffset)
  const __amdgpu_buffer_rsrc_t orr = make_rsrc(out, p.N * p.Lp * 4);
  const int voff = l < p.L ? ((64 * rp + 4 * h) * p.Lp + l) * 4 : 0x40000000;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int soff = crow(r, 0) * p.Lp * 4;
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc0[r]), orr, voff, soff, 0);
    if constexpr (TWO) __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(acc1[r]), orr, voff, soff + 32 * p.Lp * 4, 0);
  }
}

// Relation logits C2P = Q LK_h^T and P2CT = K LQ_h^T, (B,H,N,Lp) each: one wave per (b,h, table, pair of
// 32-row blocks). The wave's 2 x 32 rows stay in registers as the A operands of two independent accumulator
// chains; each 32-row slab of LK / LQ (L2-resident, shared by the whole batch) comes in by LDS-DMA into one
// SW_ROW image and feeds both chains (64 MFMAs per slab; per-lane row loads from global would touch 64 cache
// lines per instruction). One 8 KiB image per wave (not two): the refill waits for the slab's reads, and the
// other waves of the SIMD (<= 20 per CU by LDS, ~100 VGPRs) cover it, so the grid (2 x ceil(NQB / 2) x B x H
// waves) runs in one round. Stores are coalesced along the relation index.
template <int D>
__global__ __launch_bounds__(64, 4) void k_rel_logits(const RelArgs p, float* __restrict__ c2p, float* __restrict__ p2ct,
                                                     uint16_t* __restrict__ RM, uint16_t* __restrict__ RT, int nlog) {
  constexpr int NS = D / 2;
  static_assert(D == 64, "fused CSE path is d_k = 64");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  if ((int)blockIdx.x >= nlog) {  // the relation-plane prep (k_rel_prep's items), one wave each, beside the logits
    const int it = (int)blockIdx.x - nlog, NT = p.NP / 32;
    rel_prep_item<64>(p, RM, RT, reinterpret_cast<uint8_t*>(lds), it % NT, it / NT, lane_id());
    return;
  }
  const uint32_t L0 = lds_offset(lds);
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const int NRP = (p.NQB + 1) / 2;  // pairs of row blocks
  const BhBlock xb = xcd_block(2 * NRP, p.B * p.H);
  if (!xb.valid) return;
  const int which = xb.blk & 1, rp = xb.blk >> 1, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const bool two = 2 * rp + 1 < p.NQB;  // (wave-uniform) the pair's second block exists
  const float* X0 = which ? p.k + b * p.k_sb + hd * p.k_sh : p.q + b * p.q_sb + hd * p.q_sh;
  const int64_t xs = which ? p.k_sn : p.q_sn;
  const int x0 = 64 * rp + c, x1 = x0 + 32;
  const float* Lm = (which ? p.lq : p.lk) + (int64_t)hd * p.L * D;
  const __amdgpu_buffer_rsrc_t lr = make_rsrc(Lm, p.L * D * 4);
  lds_zero<32 * D>(lds);
  const DmaPat pat = dma_pat(SW_ROW, D * 4);
  dma64(L0, lr, pat, D * 4, 0);
  float xr0[NS], xr1[NS];
  load_run<NS>(xr0, X0 + (int64_t)imin(x0, p.N - 1) * xs + h * NS, x0 < p.N);
  load_run<NS>(xr1, X0 + (int64_t)imin(x1, p.N - 1) * xs + h * NS, two && x1 < p.N);
  float* out = (which ? p2ct : c2p) + (int64_t)bh * p.N * p.Lp;
  const int NLT = (p.L + 31) / 32;
  const int rbase = row_base64(c, h);
  if (two) {
    for (int lt = 0; lt < NLT; ++lt) logits_tile<D, true>(p, lds, L0, lr, pat, rbase, xr0, xr1, out, rp, lt, NLT, lane);
  } else {
    for (int lt = 0; lt < NLT; ++lt) logits_tile<D, false>(p, lds, L0, lr, pat, rbase, xr0, xr1, out, rp, lt, NLT, lane);
  }
}

// Tile-major relation bias, written by the forward for the two backward kernels: RB[b,h][qb][kt] is the
// 32 x 32 tile (query rows x, key columns y) of
//   c2p[x][rel[x][y]] + p2ct[y][rel[y][x]]      (the reference's two gathers, disentangled_attn.py:55-58)
// or -inf where mask[x][y] (the -1e9 masked_fill), 0 outside [0,N)^2. Inside a tile, column y sits at
// tile_pos(y) and the 16-B chunks of row x are XOR-swizzled by (x >> 1) & 7, so a 4 KB tile DMA'd to
// LDS serves both orientations conflict-free: a query lane's 16 columns (4 ds_read_b128) and a key
// lane's 16 rows (ds_read_b32).
__host__ __device__ constexpr int rb_off(int x, int pos) { return x * 32 + 4 * ((pos >> 2) ^ ((x >> 1) & 7)) + (pos & 3); }

// Forward, one wave per (b,h, 32 queries), S^T orientation (keys = accumulator rows, queries = lanes):
// K (SW_ROW) and V (SW_COL) tile images by LDS-DMA one tile ahead; the relation codes of the next tile
// prefetched with it; the two logit gathers per element from the L2-resident C2P / P2CT tables.
template <int D, bool BF>
__global__ __launch_bounds__(64, 2) void k_rel_fwd_f(const RelArgs p) {
  constexpr int DT = D / 32, NS = D / 2, IMG = 32 * D * 4;
  static_assert(D == 64, "fused CSE path is d_k = 64");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const uint32_t Kl = lds_offset(lds), Vl = Kl + IMG;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const BhBlock xb = xcd_block(p.NQB, p.B * p.H);
  if (!xb.valid) return;
  const int qb = xb.blk, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const int i = qb * 32 + c;
  const bool iv = i < p.N;
  const int ic = imin(i, p.N - 1);
  const int kld = (int)p.k_sn * 4, vld = (int)p.v_sn * 4;
  const __amdgpu_buffer_rsrc_t kr = make_rsrc(p.k + b * p.k_sb + hd * p.k_sh, (p.N - 1) * kld + D * 4);
  const __amdgpu_buffer_rsrc_t vr = make_rsrc(p.v + b * p.v_sb + hd * p.v_sh, (p.N - 1) * vld + D * 4);
  lds_zero<2 * IMG / 4>(lds);
  const DmaPat kpat = dma_pat(SW_ROW, kld), vpat = dma_pat(SW_COL, vld);
  const uint16_t* rmrow = prep_row(p, p.RM, b, hd, ic);
  const uint16_t* rtrow = prep_row(p, p.RT, b, hd, ic);
  Codes cm = load_codes(rmrow, 0), ct = load_codes(rtrow, 0);
  float q[NS];
  load_run<NS>(q, p.q + b * p.q_sb + hd * p.q_sh + (int64_t)ic * p.q_sn + h * NS, iv);
  dma64(Kl, kr, kpat, kld, 0);
  dma64(Vl, vr, vpat, vld, 0);
  const float* c2prow = p.c2p + ((int64_t)bh * p.N + ic) * p.Lp;
  const float* p2ct = p.p2ct + (int64_t)bh * p.N * p.Lp;
  // this lane's 16 bias columns of tile kt: row c of the tile, chunk j at byte rboff ^ 16 j
  char* rbase_g = reinterpret_cast<char*>(const_cast<float*>(p.RB) + ((int64_t)bh * p.NQB + qb) * p.NKB * 1024);
  const int rboff = 4 * rb_off(c, 16 * h);
  const int kbase = row_base64(c, h);
  int vb[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) vb[t] = IMG + col_base64(t, c, h);
  float m_run = NEG_INF, zp = 0.f;
  f32x16 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = zero16();
  for (int kt = 0; kt < p.NKB; ++kt) {
    const int j0 = kt * 32;
    wait_vm_all();  // tile kt's K / V images and its codes have landed
    // the 32 logit gathers (disentangled_attn.py:55-58) first: their latency runs under the QK^T MFMAs
    float gl[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t a = code_of(cm, r), t2 = code_of(ct, r);
      const int y = imin(j0 + crow(r, h), p.N - 1);
      const float v = c2prow[a & 0xffu] + p2ct[(int64_t)y * p.Lp + (t2 & 0xffu)];
      gl[r] = (a & 0x100u) ? NEG_INF : v;  // the bias table marks masked entries -inf
    }
    f32x16 sacc = zero16();
    if constexpr (BF) {
#pragma unroll
      for (int j2 = 0; j2 < NS / 8; ++j2)
        sacc = mfma_bf(pack8(lds_f4(lds, kbase ^ (32 * j2)), lds_f4(lds, kbase ^ (32 * j2 + 16))), pack8(&q[8 * j2]),
                       sacc);
    } else {
#pragma unroll
      for (int j = 0; j < NS / 4; ++j) {
        const f32x4 kv = lds_f4(lds, kbase ^ (16 * j));
#pragma unroll
        for (int e = 0; e < 4; ++e) sacc = mfma(kv[e], q[4 * j + e], sacc);
      }
    }
    float vt[DT][16];
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) vt[t][r] = lds_f1(lds, vb[t] + 256 * crow(r, 0));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (kt + 1 < p.NKB) {
      dma64(Kl, kr, kpat, kld, j0 + 32);
      dma64(Vl, vr, vpat, vld, j0 + 32);
      cm = load_codes(rmrow, kt + 1);
      ct = load_codes(rtrow, kt + 1);
    }
    // save the gathered bias for the backward kernels (tile-major, 4 x 16 B per lane)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = (iv && j0 + crow(4 * j + e, h) < p.N) ? gl[4 * j + e] : 0.f;
      *reinterpret_cast<f32x4*>(rbase_g + kt * 4096 + (rboff ^ (16 * j))) = v;
    }
    float sv[16];
    float tmax = NEG_INF;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const bool inside = j0 + crow(r, h) < p.N;
      const float v = (sacc[r] + gl[r]) * p.inv_scale;
      // masked_fill(mask == 1, -1e9) (disentangled_attn.py:62)
      sv[r] = !inside ? NEG_INF : (gl[r] == NEG_INF) ? -1e9f : v;
      tmax = fmaxf(tmax, sv[r]);
    }
    tmax = xhalf_max(tmax);
    const float m_new = fmaxf(m_run, tmax);
    const float alpha = (m_new == NEG_INF) ? 1.f : __expf(m_run - m_new);
    zp *= alpha;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
    float w[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      w[r] = (sv[r] == NEG_INF) ? 0.f : __expf(sv[r] - m_new);
      zp += w[r];
    }
    m_run = m_new;
    if constexpr (BF) {
      const bf16x8 w0 = pack8(&w[0]), w1 = pack8(&w[8]);
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        o[t] = mfma_bf(pack8(&vt[t][0]), w0, o[t]);
        o[t] = mfma_bf(pack8(&vt[t][8]), w1, o[t]);
      }
    } else {
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t] = mfma(vt[t][r], w[r], o[t]);
    }
  }
  const float Z = xhalf_sum(zp);
  if (iv) {
    const float inv = 1.f / Z;
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) o[t][r] *= inv;
    store_rows_f<DT>(p.out + b * p.o_sb + hd * p.o_sh + (int64_t)i * p.o_sn, o);
    if (h == 0) {
      p.stats[((int64_t)bh * p.N + i) * 2] = m_run;
      p.stats[((int64_t)bh * p.N + i) * 2 + 1] = inv;
    }
  }
}

// Backward, query side: one wave per (b,h, 32 queries), S^T orientation. Recomputes P and dP = dO V^T,
// g = P (dP - delta) / sqrt(3 d) (0 where masked); dq = g K + G_c2p LK with G_c2p[x][r] = sum over y
// with rel[x][y] = r of g[x][y] accumulated in LDS bins (the gather backward of disentangled_attn.py:58);
// writes dq, the G_c2p rows (for dlk) and (row max, 1/row sum, delta) per query for the key side.
template <int D, bool BF>
__global__ __launch_bounds__(64, 1) void k_rel_bwd_qf(const RelArgs p) {
  constexpr int DT = D / 32, NS = D / 2, IMG = 32 * D * 4;
  static_assert(D == 64, "fused CSE path is d_k = 64");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const uint32_t Kl = lds_offset(lds), Vl = Kl + IMG, Rl = Kl + 2 * IMG;
  float* bins = lds + (2 * IMG + 4096) / 4;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const BhBlock xb = xcd_block(p.NQB, p.B * p.H);
  if (!xb.valid) return;
  const int qb = xb.blk, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const int i = qb * 32 + c;
  const bool iv = i < p.N;
  const int ic = imin(i, p.N - 1);
  const int kld = (int)p.k_sn * 4, vld = (int)p.v_sn * 4;
  const __amdgpu_buffer_rsrc_t kr = make_rsrc(p.k + b * p.k_sb + hd * p.k_sh, (p.N - 1) * kld + D * 4);
  const __amdgpu_buffer_rsrc_t vr = make_rsrc(p.v + b * p.v_sb + hd * p.v_sh, (p.N - 1) * vld + D * 4);
  const __amdgpu_buffer_rsrc_t rbr = make_rsrc(p.RB + ((int64_t)bh * p.NQB + qb) * p.NKB * 1024, p.NKB * 4096);
  lds_zero<2 * IMG / 4>(lds);
  for (int e = lane; e < 32 * p.LB; e += 64) bins[e] = 0.f;
  const DmaPat kpat = dma_pat(SW_BOTH, kld), vpat = dma_pat(SW_ROW, vld);
  const uint16_t* rmrow = prep_row(p, p.RM, b, hd, ic);
  Codes cm = load_codes(rmrow, 0);
  float q[NS], dO[NS];
  load_run<NS>(q, p.q + b * p.q_sb + hd * p.q_sh + (int64_t)ic * p.q_sn + h * NS, iv);
  load_run<NS>(dO, p.dout + b * p.do_sb + hd * p.do_sh + (int64_t)ic * p.do_sn + h * NS, iv);
  dma64(Kl, kr, kpat, kld, 0);
  dma64(Vl, vr, vpat, vld, 0);
  dma_block16<4096>(Rl, rbr, 0);
  const int rbase = 2 * IMG + rb_off(c, 16 * h) * 4;
  float dp = 0.f;
  {
    float o[NS];
    load_run<NS>(o, p.out + b * p.o_sb + hd * p.o_sh + (int64_t)ic * p.o_sn + h * NS, iv);
#pragma unroll
    for (int s = 0; s < NS; ++s) dp = fmaf(dO[s], o[s], dp);
  }
  const float delta = xhalf_sum(dp);
  const float rmax = p.stats[((int64_t)bh * p.N + ic) * 2];
  const float rinv = p.stats[((int64_t)bh * p.N + ic) * 2 + 1];
  f32x16 dq[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) dq[t] = zero16();
  for (int kt = 0; kt < p.NKB; ++kt) {
    int ln = threadIdx.x;  // opaque per iteration: keeps the per-row LDS addresses out of the prologue
    asm volatile("" : "+v"(ln));
    const int c = ln & 31, h = (ln >> 5) & 1;
    const int j0 = kt * 32;
    wait_vm_all();
    float gl[16];
    uint32_t col[16];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 v = lds_f4(lds, rbase ^ (16 * j));
#pragma unroll
      for (int e = 0; e < 4; ++e) gl[4 * j + e] = v[e];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) col[r] = code_of(cm, r) & 0xffu;  // rel[x][y]: the c2p gather's column
    f32x16 sacc = zero16(), dpacc = zero16();
    const int kb = row_base64(c, h, SW_BOTH);
    const int vbb = IMG + row_base64(c, h, SW_ROW);
    if constexpr (BF) {
#pragma unroll
      for (int j2 = 0; j2 < NS / 8; ++j2) {
        sacc = mfma_bf(pack8(lds_f4(lds, kb ^ (32 * j2)), lds_f4(lds, kb ^ (32 * j2 + 16))), pack8(&q[8 * j2]), sacc);
        dpacc = mfma_bf(pack8(lds_f4(lds, vbb ^ (32 * j2)), lds_f4(lds, vbb ^ (32 * j2 + 16))), pack8(&dO[8 * j2]),
                        dpacc);
      }
    } else {
#pragma unroll
      for (int j = 0; j < NS / 4; ++j) {
        const f32x4 kv = lds_f4(lds, kb ^ (16 * j));
#pragma unroll
        for (int e = 0; e < 4; ++e) sacc = mfma(kv[e], q[4 * j + e], sacc);
      }
#pragma unroll
      for (int j = 0; j < NS / 4; ++j) {
        const f32x4 vv = lds_f4(lds, vbb ^ (16 * j));
#pragma unroll
        for (int e = 0; e < 4; ++e) dpacc = mfma(vv[e], dO[4 * j + e], dpacc);
      }
    }
    float kT[DT][16];
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const int tb = both_base64(t, c, h);
#pragma unroll
      for (int r = 0; r < 16; ++r) kT[t][r] = both_read(lds, tb, r, 0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (kt + 1 < p.NKB) {
      dma64(Kl, kr, kpat, kld, j0 + 32);
      dma64(Vl, vr, vpat, vld, j0 + 32);
      dma_block16<4096>(Rl, rbr, (kt + 1) * 4096);
      cm = load_codes(rmrow, kt + 1);
    }
    float gv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const bool inside = iv && (j0 + crow(r, h) < p.N);
      const bool msk = gl[r] == NEG_INF;
      const float s = msk ? -1e9f : (sacc[r] + gl[r]) * p.inv_scale;
      const float P = inside ? __expf(s - rmax) * rinv : 0.f;
      gv[r] = (inside && !msk) ? P * (dpacc[r] - delta) * p.inv_scale : 0.f;
    }
    if constexpr (BF) {
      const bf16x8 g0 = pack8(&gv[0]), g1 = pack8(&gv[8]);
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        dq[t] = mfma_bf(pack8(&kT[t][0]), g0, dq[t]);
        dq[t] = mfma_bf(pack8(&kT[t][8]), g1, dq[t]);
      }
    } else {
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) dq[t] = mfma(kT[t][r], gv[r], dq[t]);
    }
    bins_scatter(bins, p.LB, gv, col);
  }
  __syncthreads();
  bins_times<DT>(dq, bins, p.LB, p.KB2, p.lk + (int64_t)hd * p.L * D, p.L, D);
  if (iv) {
    store_rows_f<DT>(p.dq + b * p.dq_sb + hd * p.dq_sh + (int64_t)i * p.dq_sn, dq);
    if (h == 0 && !p.qstat_pre) {
      f32x4 st;
      st[0] = rmax; st[1] = rinv; st[2] = delta; st[3] = 0.f;
      *reinterpret_cast<f32x4*>(p.qstat + ((int64_t)bh * p.N + i) * 4) = st;
    }
  }
  bins_store_t(p.gc2p + ((int64_t)hd * p.B + b) * p.Lp * p.ldx, p.ldx, i, bins, p.LB, p.KB2, p.Lp, iv);
}

// Per-query (row max, 1/row sum, delta = rowsum(dO * O), 0) into qstat for the key-side kernel when it runs
// beside the query-side one on a second stream (csa_rel_attn_bwd). PARTS lanes per row, each a run of
// 64 / PARTS elements in the query-side kernel's order (sequential fma, then the parts added pairwise:
// PARTS = 2 for k_rel_bwd_qf; 4 for the 16-row kernels: (q0 + q1) + (q2 + q3) over 16-element runs). HBM-bound (2 x 256 B per row).
template <int PARTS>
__global__ __launch_bounds__(256) void k_rel_qstat(const RelArgs p) {
  constexpr int NS = 64 / PARTS;
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x, row = t / PARTS;
  const int h = (int)(t % PARTS);
  const bool rv = row < (int64_t)p.B * p.H * p.N;
  const int64_t rc = rv ? row : 0;
  const int i = (int)(rc % p.N), bh = (int)(rc / p.N), b = bh / p.H, hd = bh % p.H;
  float dO[NS], o[NS];
  load_run<NS>(dO, p.dout + b * p.do_sb + hd * p.do_sh + (int64_t)i * p.do_sn + h * NS, rv);
  load_run<NS>(o, p.out + b * p.o_sb + hd * p.o_sh + (int64_t)i * p.o_sn + h * NS, rv);
  float dp = 0.f;
#pragma unroll
  for (int s = 0; s < NS; ++s) dp = fmaf(dO[s], o[s], dp);
  float delta = dp + __shfl_xor(dp, 1, 64);
  if constexpr (PARTS == 4) delta = delta + __shfl_xor(delta, 2, 64);
  if (rv && h == 0) {
    f32x4 st;
    st[0] = p.stats[rc * 2]; st[1] = p.stats[rc * 2 + 1]; st[2] = delta; st[3] = 0.f;
    *reinterpret_cast<f32x4*>(p.qstat + rc * 4) = st;
  }
}

// Backward, key side: one wave per (b,h, 32 keys), S orientation (queries = accumulator rows, keys =
// lanes); Q and dO tile images (SW_BOTH) and the per-query (max, 1/sum, delta) by LDS-DMA. dv = P^T dO,
// dk = g^T q + G_p2cT LQ with G_p2cT[y][r] = sum over x with rel[y][x] = r of g[x][y] in LDS bins
// (the gather backward of disentangled_attn.py:55); writes dk, dv and the G_p2cT rows (for dlq).
template <int D, bool BF>
__global__ __launch_bounds__(64, 1) void k_rel_bwd_kf(const RelArgs p) {
  constexpr int DT = D / 32, NS = D / 2, IMG = 32 * D * 4;
  static_assert(D == 64, "fused CSE path is d_k = 64");
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const uint32_t L0 = lds_offset(lds), Ql = L0, Xl = L0 + IMG, Sl = L0 + 2 * IMG, Rl = L0 + 2 * IMG + 512;
  float* bins = lds + (2 * IMG + 512 + 4096) / 4;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const BhBlock xb = xcd_block(p.NKB, p.B * p.H);
  if (!xb.valid) return;
  const int kbi = xb.blk, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const int j = kbi * 32 + c;
  const bool jv = j < p.N;
  const int jc = imin(j, p.N - 1);
  const int qld = (int)p.q_sn * 4;
  const __amdgpu_buffer_rsrc_t qr_ = make_rsrc(p.q + b * p.q_sb + hd * p.q_sh, (p.N - 1) * qld + D * 4);
  const int xld = (int)p.do_sn * 4;
  const __amdgpu_buffer_rsrc_t xr_ = make_rsrc(p.dout + b * p.do_sb + hd * p.do_sh, (p.N - 1) * xld + D * 4);
  const __amdgpu_buffer_rsrc_t sr_ = make_rsrc(p.qstat + (int64_t)bh * p.N * 4, p.N * 16);
  // bias tiles (qb, kbi) for qb = 0.. are NKB tiles apart: descriptor over the whole (b,h) table
  const __amdgpu_buffer_rsrc_t rbr = make_rsrc(p.RB + (int64_t)bh * p.NQB * p.NKB * 1024, p.NQB * p.NKB * 4096);
  lds_zero<(2 * IMG + 512) / 4>(lds);
  for (int e = lane; e < 32 * p.LB; e += 64) bins[e] = 0.f;
  const DmaPat qpat = dma_pat(SW_BOTH, qld), xpat = dma_pat(SW_BOTH, xld);
  const uint16_t* rmrow = prep_row(p, p.RM, b, hd, jc);
  Codes cm = load_codes(rmrow, 0);
  float kr[NS], vr[NS];
  load_run<NS>(kr, p.k + b * p.k_sb + hd * p.k_sh + (int64_t)jc * p.k_sn + h * NS, jv);
  load_run<NS>(vr, p.v + b * p.v_sb + hd * p.v_sh + (int64_t)jc * p.v_sn + h * NS, jv);
  dma64(Ql, qr_, qpat, qld, 0);
  dma64(Xl, xr_, xpat, xld, 0);
  dma_tile_contig<4>(Sl, sr_, 0);
  dma_block16<4096>(Rl, rbr, kbi * 4096);
  const int rcol = 2 * IMG + 512 + 4 * rb_off(0, tile_pos(c));  // + 128 row: this key's bias in row `row`
  f32x16 dv[DT], dk[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) { dv[t] = zero16(); dk[t] = zero16(); }
  for (int qb = 0; qb < p.NQB; ++qb) {
    int ln = threadIdx.x;
    asm volatile("" : "+v"(ln));
    const int c = ln & 31, h = (ln >> 5) & 1;
    const int i0 = qb * 32;
    wait_vm_all();
    float gl[16];
    uint32_t col[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int x = crow(r, h);  // the row's chunk swizzle depends on x: fold it into the column offset
      gl[r] = lds_f1(lds, 2 * IMG + 512 + 4 * rb_off(x, tile_pos(c)));
      col[r] = code_of(cm, r) & 0xffu;  // rel[y][x]: the p2c gather's column
    }
    (void)rcol;
    f32x16 sacc = zero16(), dpacc = zero16();
    const int qrb = row_base64(c, h, SW_BOTH);
    if constexpr (BF) {
#pragma unroll
      for (int j2 = 0; j2 < NS / 8; ++j2) {
        sacc = mfma_bf(pack8(lds_f4(lds, qrb ^ (32 * j2)), lds_f4(lds, qrb ^ (32 * j2 + 16))), pack8(&kr[8 * j2]),
                       sacc);
        dpacc = mfma_bf(pack8(lds_f4(lds, IMG + (qrb ^ (32 * j2))), lds_f4(lds, IMG + (qrb ^ (32 * j2 + 16)))),
                        pack8(&vr[8 * j2]), dpacc);
      }
    } else {
#pragma unroll
      for (int s4 = 0; s4 < NS / 4; ++s4) {
        const f32x4 qv = lds_f4(lds, qrb ^ (16 * s4));
#pragma unroll
        for (int e = 0; e < 4; ++e) sacc = mfma(qv[e], kr[4 * s4 + e], sacc);
      }
#pragma unroll
      for (int s4 = 0; s4 < NS / 4; ++s4) {
        const f32x4 xv = lds_f4(lds, IMG + (qrb ^ (16 * s4)));
#pragma unroll
        for (int e = 0; e < 4; ++e) dpacc = mfma(xv[e], vr[4 * s4 + e], dpacc);
      }
    }
    float Pv[16], gv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int x = i0 + crow(r, h);
      const bool inside = (x < p.N) && jv;
      const f32x4 st = lds_f4(lds, 2 * IMG + 16 * crow(r, h));
      const bool msk = gl[r] == NEG_INF;
      const float s = msk ? -1e9f : (sacc[r] + gl[r]) * p.inv_scale;
      const float P = inside ? __expf(s - st[0]) * st[1] : 0.f;
      Pv[r] = P;
      gv[r] = (inside && !msk) ? P * (dpacc[r] - st[2]) * p.inv_scale : 0.f;
    }
    int cb[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) cb[t] = both_base64(t, c, h);
    if constexpr (BF) {
      const bf16x8 p0 = pack8(&Pv[0]), p1 = pack8(&Pv[8]), g0 = pack8(&gv[0]), g1 = pack8(&gv[8]);
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        float xc[16], qc[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) { xc[r] = both_read(lds, cb[t], r, IMG); qc[r] = both_read(lds, cb[t], r, 0); }
        dv[t] = mfma_bf(pack8(&xc[0]), p0, dv[t]);
        dv[t] = mfma_bf(pack8(&xc[8]), p1, dv[t]);
        dk[t] = mfma_bf(pack8(&qc[0]), g0, dk[t]);
        dk[t] = mfma_bf(pack8(&qc[8]), g1, dk[t]);
      }
    } else {
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) dv[t] = mfma(both_read(lds, cb[t], r, IMG), Pv[r], dv[t]);
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) dk[t] = mfma(both_read(lds, cb[t], r, 0), gv[r], dk[t]);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (qb + 1 < p.NQB) {
      dma64(Ql, qr_, qpat, qld, i0 + 32);
      dma64(Xl, xr_, xpat, xld, i0 + 32);
      dma_tile_contig<4>(Sl, sr_, i0 + 32);
      dma_block16<4096>(Rl, rbr, ((qb + 1) * p.NKB + kbi) * 4096);
      cm = load_codes(rmrow, qb + 1);
    }
    bins_scatter(bins, p.LB, gv, col);
  }
  __syncthreads();
  bins_times<DT>(dk, bins, p.LB, p.KB2, p.lq + (int64_t)hd * p.L * D, p.L, D);
  if (jv) {
    store_rows_f<DT>(p.dk + b * p.dk_sb + hd * p.dk_sh + (int64_t)j * p.dk_sn, dk);
    store_rows_f<DT>(p.dv + b * p.dv_sb + hd * p.dv_sh + (int64_t)j * p.dv_sn, dv);
  }
  bins_store_t(p.gp2ct + ((int64_t)hd * p.B + b) * p.Lp * p.ldx, p.ldx, j, bins, p.LB, p.KB2, p.Lp, jv);
}

// ------------------------------------------------------------------------------------
// fp32 backward with 16-row waves (k_rel_bwd_kh, then k_rel_bwd_qg from its g tiles). The 32-row kernels above hold 40 KB of
// LDS per wave (K/V images 16 KB, bias tile 4 KB, bins 20 KB): one wave per SIMD, latency-bound. Here a
// workgroup of two waves covers the same 32-row block: the two waves share the tile images and the bias
// tile (each DMAs half of them), and each owns 16 rows and a 16-row bins table (~10 KB), so the workgroup
// needs ~40 KB for two waves and a CU holds four: two waves per SIMD. The contractions run on the exact
// fp32 v_mfma_f32_16x16x4_f32 (same FLOP rate as 32x32x2). Lane l = (x16 = l & 15, g = l >> 4):
//   query side: S^T / dP^T tiles D[key 16 st + 4 g + i][query x16] (st = 0, 1: the two 16-key halves of
//               a 32-key tile), dq^T[d][query] += K^T[d][key] g^T[key][query] (acc K-permutation);
//   key side:   S / dP tiles D[query 16 st + 4 g + i][key x16], dv^T / dk^T[d][key] += X^T[d][query] (.).
// A lane's 8 elements (st, i) of one tile sit at prepared-plane / bias-tile positions
// pbase(g) + 8 st + i with pbase(g) = 16 (g & 1) + 4 (g >> 1) (= tile_pos(16 st + 4 g + i)): two 8-B code
// loads and two 16-B bias reads per tile.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int pbase16(int g) { return 16 * (g & 1) + 4 * (g >> 1); }

struct Codes8 { uint32_t w[4]; };
// the lane's 8 codes (e = 4 st + i) of one tile from ITS OWN prepared row
__device__ __forceinline__ Codes8 load_codes8(const uint16_t* __restrict__ row, int tile) {
  const uint16_t* q = row + 32 * tile + pbase16(lane_id() >> 4);
  const uint2 a = *reinterpret_cast<const uint2*>(q), b = *reinterpret_cast<const uint2*>(q + 8);
  return Codes8{{a.x, a.y, b.x, b.y}};
}
__device__ __forceinline__ uint32_t code8(const Codes8& k, int e) { return (k.w[e >> 1] >> (16 * (e & 1))) & 0xffffu; }

// byte offset of element (row, col) of a SW_BOTH / SW_ROW 32 x 64 image
__device__ __forceinline__ int img_elem(int row, int col, const int sw) { return 256 * row + 16 * ((col >> 2) ^ swz(sw, row)) + 4 * (col & 3); }

// 16-row bins (16 rows x LB floats, LB / 2 odd: the 16 rows of a b64 read hit distinct bank pairs) += g at
// column rel; the four lane groups share the rows, so they add in four exec-masked passes, lanes of a pass
// own distinct rows and a row's additions happen in a fixed order -> deterministic. An element whose g is
// zero in every lane of the pass (masked relations: most of the matrix) skips its add. The passes need no
// wait between them: one wave's LDS instructions execute in issue order, and the empty asm keeps the compiler
// from merging or reordering them (round 5: 8 of 9 same-box rounds faster, java layer -1.3 us,
// profiles/r05_ab_cse_passwait.txt).
__device__ __forceinline__ void bins_scatter16(float* bins, int LB, const float (&gv)[8], const uint32_t (&col)[8]) {
  const int x16 = lane_id() & 15, g = lane_id() >> 4;
  float* row = bins + x16 * LB;
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    if (g == pass) {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (gv[e] != 0.f) atomicAdd(row + col[e], gv[e]);
    }
    asm volatile("" ::: "memory");  // keeps the passes apart (the compiler would merge them into one)
  }
}

// acc[t] (register i of lane group g: d = 16 g + 4 i + t, lanes = the bins' rows) += sum_r Lmat[r][d] bins[row][r]
// (dq_rel = G_c2p LK or dk_rel = G_p2cT LQ): tile t's MFMA row m is d = 4 m + t, so lane x16's four A operands
// of a K-step are one dwordx4, Lmat[r][4 x16 .. 4 x16 + 3]. K-step s of lane group g is r = g Q4 + s (Q4 even,
// 4 Q4 >= L; rows >= L read 0); the Lmat operand comes from L2 with a ring of RING groups of two K-steps in flight.
__device__ __forceinline__ void bins_times16(f32x4 (&acc)[4], const float* bins, int LB, int Q4,
                                             const float* __restrict__ Lmat, int L) {
  constexpr int D = 64, RING = 8;
  const int x16 = lane_id() & 15, g = lane_id() >> 4;
  const float* brow = bins + x16 * LB + g * Q4;
  auto lmat = [&](int s2, float (&v)[2][4]) {
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int r = g * Q4 + 2 * s2 + e;
      const float* lr = Lmat + (int64_t)(r < L ? r : 0) * D;
      const f32x4 lv = *reinterpret_cast<const f32x4*>(lr + 4 * x16);
#pragma unroll
      for (int t = 0; t < 4; ++t) v[e][t] = r < L ? lv[t] : 0.f;
    }
  };
  auto group = [&](int s2, const float (&v)[2][4]) {
    const float2 bv = *reinterpret_cast<const float2*>(brow + 2 * s2);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      acc[t] = mfma16(v[0][t], bv.x, acc[t]);
      acc[t] = mfma16(v[1][t], bv.y, acc[t]);
    }
  };
  const int ng = Q4 / 2, ngf = ng / RING * RING;
  float lv[RING][2][4];
#pragma unroll
  for (int u = 0; u < RING - 1; ++u) lmat(u, lv[u]);
  for (int g0 = 0; g0 < ngf; g0 += RING) {
#pragma unroll
    for (int u = 0; u < RING; ++u) {
      lmat(g0 + u + RING - 1, lv[(u + RING - 1) % RING]);  // past the end: a clamped, never-used row
      group(g0 + u, lv[u]);
    }
  }
#pragma unroll
  for (int u = 0; u < RING - 1; ++u)
    if (ngf + u < ng) group(ngf + u, lv[u]);
}

// bins row of this lane (row x16, the group's columns [g Q4, g Q4 + Q4) clipped to Lp) -> column `row` of the
// transposed (Lp, ldx) table (16 lanes of a group store 16 consecutive floats per bin)
__device__ __forceinline__ void bins_store16(float* __restrict__ outT, int64_t ldx, int row, const float* bins, int LB,
                                             int Q4, int Lp, bool valid) {
  if (!valid) return;
  const int x16 = lane_id() & 15, g = lane_id() >> 4;
  const float* brow = bins + x16 * LB;
  const int r1 = imin(g * Q4 + Q4, Lp);
  for (int r = g * Q4; r < r1; ++r) outT[(int64_t)r * ldx + row] = brow[r];
}

// LDS of the 16-row kernels: images | (key side: 512 B of query stats) | 4 KB bias tile | 2 x 16-row bins
__host__ __device__ constexpr int rel16_bins_off(bool key_side) { return 2 * 32 * 64 * 4 + (key_side ? 512 : 0) + 4096; }

typedef uint32_t u32x4v_t __attribute__((ext_vector_type(4)));

// Key side, 16-row waves: workgroup = (b,h, 32-key block), wave w = keys 16 w .. 16 w + 15. Same algebra and
// outputs as k_rel_bwd_kf.
__global__ __launch_bounds__(128, 2) void k_rel_bwd_kh(const RelArgs p) {
  constexpr int D = 64, IMG = 32 * D * 4;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const uint32_t L0 = lds_offset(lds), Ql = L0, Xl = L0 + IMG, Sl = L0 + 2 * IMG, Rl = L0 + 2 * IMG + 512;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = lane_id(), x16 = lane & 15, g = lane >> 4;
  float* bins = lds + rel16_bins_off(true) / 4 + w * 16 * p.LB16;
  const BhBlock xb = xcd_block(p.NKB, p.B * p.H);
  if (!xb.valid) return;
  const int kbi = xb.blk, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const int yr = 16 * w + x16, j = kbi * 32 + yr;
  const bool jv = j < p.N;
  const int jc = imin(j, p.N - 1);
  const int qld = (int)p.q_sn * 4, xld = (int)p.do_sn * 4;
  const __amdgpu_buffer_rsrc_t qr_ = make_rsrc(p.q + b * p.q_sb + hd * p.q_sh, (p.N - 1) * qld + D * 4);
  const __amdgpu_buffer_rsrc_t xr_ = make_rsrc(p.dout + b * p.do_sb + hd * p.do_sh, (p.N - 1) * xld + D * 4);
  const __amdgpu_buffer_rsrc_t sr_ = make_rsrc(p.qstat + (int64_t)bh * p.N * 4, p.N * 16);
  const __amdgpu_buffer_rsrc_t rbr = make_rsrc(p.RB + (int64_t)bh * p.NQB * p.NKB * 1024, p.NQB * p.NKB * 4096);
  for (int e = (int)threadIdx.x; e < (2 * IMG + 512) / 16; e += 128)
    reinterpret_cast<f32x4*>(lds)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int e = lane; e < 16 * p.LB16; e += 64) bins[e] = 0.f;
  __syncthreads();
  const DmaPat qpat = dma_pat(SW_BOTH, qld), xpat = dma_pat(SW_BOTH, xld);
  const uint16_t* rmrow = prep_row(p, p.RM, b, hd, jc);
  Codes8 cm = load_codes8(rmrow, 0);
  float kr[16], vr[16];
  load_run<16>(kr, p.k + b * p.k_sb + hd * p.k_sh + (int64_t)jc * p.k_sn + 16 * g, jv);
  load_run<16>(vr, p.v + b * p.v_sb + hd * p.v_sh + (int64_t)jc * p.v_sn + 16 * g, jv);
  dma64(Ql, qr_, qpat, qld, 0, 4 * w, 4 * w + 4);
  dma64(Xl, xr_, xpat, xld, 0, 4 * w, 4 * w + 4);
  dma_tile_contig<4>(Sl, sr_, 0, w, w + 1);
  dma_block16<2048>(Rl + 2048 * w, rbr, kbi * 4096 + 2048 * w);
  const int ypos = tile_pos(yr);
  f32x4 dv[4], dk[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) { dv[t] = f32x4{0.f, 0.f, 0.f, 0.f}; dk[t] = dv[t]; }
  float gsv[8];  // deferred bins scatter
  uint32_t csv[8];
  for (int qb = 0; qb < p.NQB; ++qb) {
    const int i0 = qb * 32;
    wait_vm_all();
    __syncthreads();
    float gl[8], rm[8], ri[8], dl[8];
    uint32_t col[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int x = 16 * (e >> 2) + 4 * g + (e & 3);  // query of element e in the tile
      gl[e] = lds_f1(lds, 2 * IMG + 512 + 4 * rb_off(x, ypos));
      const f32x4 st = lds_f4(lds, 2 * IMG + 16 * x);
      rm[e] = st[0]; ri[e] = st[1]; dl[e] = st[2];
      col[e] = code8(cm, e) & 0xffu;  // rel[y][x]: the p2c gather's column
    }
    // four interleaved chains (S, dP of both query halves): a 16x16x4 result feeds its own chain after 40 cycles,
    // its issue slot is 32, so one chain alone would run at 80% of the pipe rate
    f32x4 sacc[2], dpacc[2];
#pragma unroll
    for (int st = 0; st < 2; ++st) { sacc[st] = f32x4{0.f, 0.f, 0.f, 0.f}; dpacc[st] = sacc[st]; }
    f32x4 qv[2][2], xv[2][2];
    auto rd = [&](int s4, f32x4 (&qd)[2], f32x4 (&xd)[2]) {
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        qd[st] = lds_f4(lds, img_elem(16 * st + x16, 16 * g + 4 * s4, SW_BOTH));
        xd[st] = lds_f4(lds, IMG + img_elem(16 * st + x16, 16 * g + 4 * s4, SW_BOTH));
      }
    };
    rd(0, qv[0], xv[0]);
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      if (s4 + 1 < 4) rd(s4 + 1, qv[(s4 + 1) & 1], xv[(s4 + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int st = 0; st < 2; ++st) {
          sacc[st] = mfma16(qv[s4 & 1][st][e], kr[4 * s4 + e], sacc[st]);
          dpacc[st] = mfma16(xv[s4 & 1][st][e], vr[4 * s4 + e], dpacc[st]);
        }
    }
    // elementwise first: the bias / statistics registers die before the column operands are read
    float Pv[8], gv[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sa = sacc[e >> 2][e & 3], dpa = dpacc[e >> 2][e & 3];
      const bool inside = (i0 + 16 * (e >> 2) + 4 * g + (e & 3) < p.N) && jv;
      const bool msk = gl[e] == NEG_INF;
      const float s = msk ? -1e9f : (sa + gl[e]) * p.inv_scale;
      const float P = inside ? __expf(s - rm[e]) * ri[e] : 0.f;
      Pv[e] = P;
      gv[e] = (inside && !msk) ? P * (dpa - dl[e]) * p.inv_scale : 0.f;
    }
    if (p.gt) {  // this key's row of tile (qb, kbi) for k_rel_bwd_qg: queries 16 st + 4 g .. + 3 (read once: non-temporal)
      const __amdgpu_buffer_rsrc_t gr = make_rsrc(p.gt + (int64_t)bh * p.NQB * p.NKB * 1024, p.NQB * p.NKB * 4096);
#pragma unroll
      for (int st = 0; st < 2; ++st)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4v_t, f32x4{gv[4 * st], gv[4 * st + 1], gv[4 * st + 2], gv[4 * st + 3]}), gr,
            4 * (yr * 32 + 4 * g + 16 * st), (qb * p.NKB + kbi) * 4096, 2);
    }
    float xc[4][8], qc[4][8];  // A operands of dv / dk: X[query 16 st + 4 g + i][d = 4 x16 + t], b128 per query
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int off = img_elem(16 * (e >> 2) + 4 * g + (e & 3), 4 * x16, SW_BOTH);
      const f32x4 xv = lds_f4(lds, IMG + off), qv4 = lds_f4(lds, off);
#pragma unroll
      for (int t = 0; t < 4; ++t) { xc[t][e] = xv[t]; qc[t][e] = qv4[t]; }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    if (qb + 1 < p.NQB) {
      dma64(Ql, qr_, qpat, qld, i0 + 32, 4 * w, 4 * w + 4);
      dma64(Xl, xr_, xpat, xld, i0 + 32, 4 * w, 4 * w + 4);
      dma_tile_contig<4>(Sl, sr_, i0 + 32, w, w + 1);
      dma_block16<2048>(Rl + 2048 * w, rbr, ((qb + 1) * p.NKB + kbi) * 4096 + 2048 * w);
      cm = load_codes8(rmrow, qb + 1);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        dv[t] = mfma16(xc[t][e], Pv[e], dv[t]);
        dk[t] = mfma16(qc[t][e], gv[e], dk[t]);
      }
    bins_scatter16(bins, p.LB16, gv, col);
  }
  bins_times16(dk, bins, p.LB16, p.Q4, p.lq + (int64_t)hd * p.L * D, p.L);
  if (jv) {
    float* dkp = p.dk + b * p.dk_sb + hd * p.dk_sh + (int64_t)j * p.dk_sn + 16 * g;  // d = 16 g + 4 r + t
    float* dvp = p.dv + b * p.dv_sb + hd * p.dv_sh + (int64_t)j * p.dv_sn + 16 * g;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      *reinterpret_cast<f32x4*>(dkp + 4 * r) = f32x4{dk[0][r], dk[1][r], dk[2][r], dk[3][r]};
      *reinterpret_cast<f32x4*>(dvp + 4 * r) = f32x4{dv[0][r], dv[1][r], dv[2][r], dv[3][r]};
    }
  }
  bins_store16(p.gp2ct + ((int64_t)hd * p.B + b) * p.Lp * p.ldx, p.ldx, j, bins, p.LB16, p.Q4, p.Lp, jv);
}

// Query side, 16-row waves, from the key side's g tiles (fp32): workgroup = (b,h, 32-query block), wave w =
// queries 16 w .. 16 w + 15. k_rel_bwd_kh stored the softmax-input gradient g = P (dP - delta) / sqrt(3 d)
// of every element as [key][query] tiles, so this kernel neither recomputes the scores (no V image, no bias
// tile, no exp) nor dP: dq = g K (16x16x4 MFMA, K image by LDS-DMA) and the c2p gather backward
// (G_c2p bins, then dq += G_c2p LK) in the 16-row operand layouts above.
__global__ __launch_bounds__(128, 2) void k_rel_bwd_qg(const RelArgs p) {
  constexpr int D = 64, IMG = 32 * D * 4;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const uint32_t Kl = lds_offset(lds);
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int lane = lane_id(), x16 = lane & 15, g = lane >> 4;
  float* bins = lds + rel16_bins_off(false) / 4 + w * 16 * p.LB16;
  const BhBlock xb = xcd_block(p.NQB, p.B * p.H);
  if (!xb.valid) return;  // whole workgroup
  const int qb = xb.blk, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const int xr = 16 * w + x16, i = qb * 32 + xr;
  const bool iv = i < p.N;
  const int ic = imin(i, p.N - 1);
  const int kld = (int)p.k_sn * 4;
  const __amdgpu_buffer_rsrc_t kr = make_rsrc(p.k + b * p.k_sb + hd * p.k_sh, (p.N - 1) * kld + D * 4);
  // rows past N are never fetched: the image holds zeros there (zeroed before any DMA can land)
  for (int e = (int)threadIdx.x; e < IMG / 16; e += 128) reinterpret_cast<f32x4*>(lds)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int e = lane; e < 16 * p.LB16; e += 64) bins[e] = 0.f;
  __syncthreads();
  const DmaPat kpat = dma_pat(SW_BOTH, kld);
  const uint16_t* rmrow = prep_row(p, p.RM, b, hd, ic);
  Codes8 cm = load_codes8(rmrow, 0);
  // element e = 4 st + i of tile kt (key 16 st + 4 g + i, query xr): tg + kt * 1024 + 32 (16 st + 4 g + i)
  const float* tg = p.gt + ((int64_t)bh * p.NQB + qb) * p.NKB * 1024 + 128 * g + xr;
  float gn[8];
  auto load_g = [&](int kt) {
#pragma unroll
    for (int e = 0; e < 8; ++e) gn[e] = tg[kt * 1024 + 32 * (16 * (e >> 2) + (e & 3))];
  };
  dma64(Kl, kr, kpat, kld, 0, 4 * w, 4 * w + 4);  // wave w fetches rows 16 w .. 16 w + 15
  load_g(0);
  f32x4 dq[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) dq[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kt = 0; kt < p.NKB; ++kt) {
    const int j0 = kt * 32;
    wait_vm_all();
    __syncthreads();  // both waves' pieces of tile kt landed
    float gv[8];
    uint32_t col[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { gv[e] = gn[e]; col[e] = code8(cm, e) & 0xffu; }  // rel[x][y]: the c2p column
    float kT[4][8];  // A operands of dq: K[key 16 st + 4 g + i][d = 4 x16 + t], one b128 read per key
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const f32x4 kv = lds_f4(lds, img_elem(16 * (e >> 2) + 4 * g + (e & 3), 4 * x16, SW_BOTH));
#pragma unroll
      for (int t = 0; t < 4; ++t) kT[t][e] = kv[t];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();  // both waves read tile kt out: refill
    if (kt + 1 < p.NKB) {
      dma64(Kl, kr, kpat, kld, j0 + 32, 4 * w, 4 * w + 4);
      cm = load_codes8(rmrow, kt + 1);
      load_g(kt + 1);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e)
#pragma unroll
      for (int t = 0; t < 4; ++t) dq[t] = mfma16(kT[t][e], gv[e], dq[t]);
    bins_scatter16(bins, p.LB16, gv, col);
  }
  bins_times16(dq, bins, p.LB16, p.Q4, p.lk + (int64_t)hd * p.L * D, p.L);
  if (iv) {
    float* dst = p.dq + b * p.dq_sb + hd * p.dq_sh + (int64_t)i * p.dq_sn + 16 * g;  // d = 16 g + 4 r + t
#pragma unroll
    for (int r = 0; r < 4; ++r) *reinterpret_cast<f32x4*>(dst + 4 * r) = f32x4{dq[0][r], dq[1][r], dq[2][r], dq[3][r]};
  }
  bins_store16(p.gc2p + ((int64_t)hd * p.B + b) * p.Lp * p.ldx, p.ldx, i, bins, p.LB16, p.Q4, p.Lp, iv);
}

// Relation-embedding gradients of the fused path, split over the batch (deterministic):
//   part[s][h](l, dd) = sum over the chunks of split s of G_h[l][x] X_h[x][dd]
// (dlk: G = G_c2p, X = Q; dlq: G = G_p2cT, X = K; disentangled_attn.py:51-52 backward). The G tables are
// (H, B, Lp, NP), x = n (written by bins_store_t; columns n >= N are never written and masked here).
// One wave per (32-row l tile, head, split) computes both 32-column halves of dd: A = G rows (dwordx4 runs
// of x in the acc K-permutation), B = the chunk's 32 X rows by LDS-DMA into a double-buffered SW_COL image
// (column reads conflict-free); chunk c + 1 lands while chunk c's 32 MFMAs run. k_sum_splits2 adds the
// splits in order.
struct LgradArgs {
  const float* G[2];   // G_c2p, G_p2cT tables (H, Lp, ldx)
  const float* X[2];   // Q, K
  int64_t x_sb[2], x_sh[2], x_sn[2];
  float* part[2];      // (nsplit, H, L, 64) partials of dlk, dlq
  int64_t ldx; int Lp, L, NP, B, N, H, nsplit;
};
// Workgroup = one wave per 32-row l tile (all of L), grid (H, 2 splits-sets): the chunk's X image is shared
// by the waves (each DMAs some of its eight 1 KiB pieces; a barrier per chunk publishes it). One wave per
// (l tile, head, split) workgroup, each DMAing whole images with no barrier, measured 47 -> 77 us
// (profiles/r04_ab_lgrad.txt).
__global__ __launch_bounds__(512) void k_rel_lgrad(const LgradArgs g) {
  constexpr int D = 64, IMG = 32 * D * 4;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const uint32_t L0 = lds_offset(lds);
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const int lt = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6)), NW = (int)(blockDim.x >> 6);
  const int hd = blockIdx.x, which = (int)blockIdx.y / g.nsplit, sp = (int)blockIdx.y % g.nsplit;
  const int cpb = g.NP / 32, nch = g.B * cpb;  // 32-row chunks per batch element / in all
  const int c0 = (int)((int64_t)sp * nch / g.nsplit), c1 = (int)((int64_t)(sp + 1) * nch / g.nsplit);
  const int l = lt * 32 + c;
  const float* arow = g.G[which] + ((int64_t)hd * g.B * g.Lp + imin(l, g.L - 1)) * g.ldx;  // + b Lp ldx per chunk
  const float* X = g.X[which] + hd * g.x_sh[which];
  const int64_t x_sb = g.x_sb[which];
  const int ld = (int)g.x_sn[which] * 4, N = g.N;
  const DmaPat pat = dma_pat(SW_COL, ld);
  for (int e = threadIdx.x; e < 2 * IMG / 16; e += blockDim.x)  // rows >= N are never fetched: finite zeros
    reinterpret_cast<f32x4*>(lds)[e] = f32x4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  // chunk ch: this wave's pieces of rows n0 .. n0 + 31 of batch element b into image buf, and its G runs
  // G[l][x0 + 8 q + 4 h + e] = the A operand of K-step r = 4 q + e (acc perm: x = x0 + crow(r, h))
  // piece q (rows 4q .. 4q + 3) of a chunk: the lane's pattern entry q & 3 picked by selects (q is a runtime
  // value here; dma64's array index would put the pattern in scratch and a scratch load before every piece)
  auto piece = [&](uint32_t img, __amdgpu_buffer_rsrc_t xr, int n0, int q) {
    const int m = q & 3;
    const int pv = m == 0 ? pat.v[0] : m == 1 ? pat.v[1] : m == 2 ? pat.v[2] : pat.v[3];
    __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, lds_at(img + 1024 * q), 16, pv + (n0 + 4 * q) * ld, 0, 0, 0);
  };
  auto issue_x = [&](int ch, int buf) {
    const int b = ch / cpb, n0 = (ch % cpb) * 32;
    const __amdgpu_buffer_rsrc_t xr = make_rsrc(X + b * x_sb, (N - 1) * ld + D * 4);
    for (int q = lt; q < 8; q += NW) piece(L0 + IMG * buf, xr, n0, q);
  };
  auto issue_g = [&](int ch, f32x4 (&a4)[4]) {
    const int b = ch / cpb, n0 = (ch % cpb) * 32;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      a4[q] = *reinterpret_cast<const f32x4*>(arow + (int64_t)b * g.Lp * g.ldx + n0 + 8 * q + 4 * h);
  };
  int vb[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) vb[t] = col_base64(t, c, h);
  f32x16 acc[2] = {zero16(), zero16()};
  // The G runs (the kernel's HBM stream: 100 MB at B = 64) are loaded two chunks ahead into a ring of three
  // register buffers (the loop unrolled by three, so no buffer is copied while its loads are in flight), the
  // X images one chunk ahead. Issue order per chunk: X pieces of chunk ch + 1, then the G runs of ch + 2
  // (compiler fences keep the order; past the split's last chunk the last chunk's runs are loaded again, so
  // every chunk issues exactly four G loads), and the vmcnt(4) at the top of the next chunk retires
  // everything but those last four (vmcnt counts in issue order).
  f32x4 B0[4], B1[4], B2[4];
  auto step = [&](int ch, const f32x4 (&use)[4], f32x4 (&nxt)[4]) {
    const int cur = (ch - c0) & 1, n0 = (ch % cpb) * 32;
    // vmcnt(4) as the builtin (0x0f74: lgkmcnt / expcnt left open), which the compiler's wait insertion sees:
    // behind an inline-asm wait it would still count the older loads as pending and wait for them again
    __builtin_amdgcn_s_waitcnt(0x0f74);
    __syncthreads();   // every wave's pieces landed; every wave read out image cur ^ 1 (chunk ch - 1)
    if (ch + 1 < c1) issue_x(ch + 1, cur ^ 1);
    asm volatile("" ::: "memory");
    issue_g(imin(ch + 2, c1 - 1), nxt);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float a = (n0 + crow(r, h) < N) ? use[r >> 2][r & 3] : 0.f;
        acc[t] = mfma(a, lds_f1(lds, IMG * cur + vb[t] + 256 * crow(r, 0)), acc[t]);
      }
  };
  if (c0 < c1) {
    issue_x(c0, 0);
    asm volatile("" ::: "memory");
    issue_g(c0, B0);
    issue_g(imin(c0 + 1, c1 - 1), B1);
    asm volatile("" ::: "memory");
  }
  for (int ch = c0; ch < c1; ch += 3) {
    step(ch, B0, B2);
    if (ch + 1 >= c1) break;
    step(ch + 1, B1, B0);
    if (ch + 2 >= c1) break;
    step(ch + 2, B2, B1);
  }
  float* out = g.part[which] + ((int64_t)sp * g.H + hd) * g.L * D;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ll = lt * 32 + crow(r, h);
      if (ll < g.L) out[(int64_t)ll * D + 32 * t + c] = acc[t][r];
    }
}

csa_status rfail(csa_status s, const char* m) {
  csa::set_error("%s", m);
  return s;
}

csa_status rfail_hip(const char* what) {
  const hipError_t e = hipGetLastError();
  csa::set_error("%s: %s", what, hipGetErrorString(e));
  return CSA_LAUNCH_FAILED;
}

csa_status rcheck(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    csa::set_error("%s: %s", what, hipGetErrorString(e));
    return CSA_LAUNCH_FAILED;
  }
  return CSA_OK;
}

void gemm(hipStream_t st, const GemmArgs& g, int nbat) {
  dim3 grid((unsigned)((g.N + 31) / 32), (unsigned)((g.M + 31) / 32), (unsigned)(nbat * (g.rsplit > 1 ? g.rsplit : 1)));
  // dwordx4 operand loads where k is contiguous and every row start is 16-B aligned
  auto vec = [](const float* base, int64_t xk, int64_t xm, int64_t xb1, int64_t xb2, int64_t xr) {
    return xk == 1 && ((uintptr_t)base) % 16 == 0 && xm % 4 == 0 && xb1 % 4 == 0 && xb2 % 4 == 0 && xr % 4 == 0;
  };
  const bool av = vec(g.A, g.a_k, g.a_m, g.a_b1, g.a_b2, g.a_r), bv = vec(g.B, g.b_k, g.b_n, g.b_b1, g.b_b2, g.b_r);
  if (av && bv) hipLaunchKernelGGL((k_bgemm<true, true>), grid, dim3(64), 0, st, g);
  else if (av) hipLaunchKernelGGL((k_bgemm<true, false>), grid, dim3(64), 0, st, g);
  else if (bv) hipLaunchKernelGGL((k_bgemm<false, true>), grid, dim3(64), 0, st, g);
  else hipLaunchKernelGGL((k_bgemm<false, false>), grid, dim3(64), 0, st, g);
}

struct RelLayout {
  int64_t Lp, ldg, NP, ldx;
  int RS;                                    // batch splits of the dlq / dlk reductions
  bool fused;                                // d_k = 64: prepared planes + in-kernel gather backward
  size_t c2p, p2ct, RM, RT, RB, state_total;  // forward state
  size_t G, P, gc2p, gp2ct, part, qstat, gt, ws_total;  // backward workspace
};

inline size_t ral(size_t x) { return (x + 255) & ~size_t(255); }

RelLayout rel_layout(int64_t B, int64_t H, int64_t N, int64_t L, int64_t d) {
  RelLayout R;
  R.Lp = ((L + 3) / 4) * 4;
  // dlq / dlk sum over the whole batch: RS partial sums of B / RS elements each fill the GPU
  // (a single reduction chain per output tile left only H * 10 waves)
  R.fused = (d == 64);
  R.NP = ((N + 31) / 32) * 32;
  // fused: k_rel_lgrad splits the B * NP / 32 chunks of x over RS waves per (l tile, head); otherwise the
  // k_bgemm R-split sums RS partials of B / RS elements each (one chain per tile left only H * 10 waves)
  R.RS = R.fused ? (int)std::min<int64_t>(32, B * R.NP / 32) : (int)(B < 16 ? B : 16);
  size_t o = 0;
  auto take = [&](size_t bytes) { size_t r = o; o += ral(bytes); return r; };
  R.c2p = take(sizeof(float) * B * H * N * R.Lp);
  R.p2ct = take(sizeof(float) * B * H * N * R.Lp);
  // prepared planes: at most one per head (fewer when heads share planes, e.g. the CSE's 2)
  R.RM = take(R.fused ? sizeof(uint16_t) * B * H * R.NP * R.NP : 0);
  R.RT = take(R.fused ? sizeof(uint16_t) * B * H * R.NP * R.NP : 0);
  R.RB = take(R.fused ? sizeof(float) * B * H * R.NP * R.NP : 0);  // tile-major relation bias
  R.state_total = o;
  o = 0;
  R.ldg = ((N + 3) / 4) * 4;
  R.G = take(R.fused ? 0 : sizeof(float) * B * H * N * R.ldg);
  R.P = take(R.fused ? 0 : sizeof(float) * B * H * N * R.ldg);
  R.ldx = R.NP;  // fused: G tables stored transposed (H, B, Lp, ldx), x = n
  R.gc2p = take(R.fused ? sizeof(float) * H * B * R.Lp * R.ldx : sizeof(float) * B * H * N * R.Lp);
  R.gp2ct = take(R.fused ? sizeof(float) * H * B * R.Lp * R.ldx : sizeof(float) * B * H * N * R.Lp);
  R.part = take(sizeof(float) * (R.fused ? 2 : 1) * R.RS * H * L * d);  // fused: dlk and dlq partials
  R.qstat = take(R.fused ? sizeof(float) * B * H * N * 4 : 0);
  R.gt = take(R.fused ? sizeof(float) * B * H * R.NP * R.NP : 0);
  R.ws_total = o;
  return R;
}

// a zero stride triple, or the (B,H,N,d)-contiguous one
inline bool contig3(int64_t sb, int64_t sh, int64_t sn, int64_t H, int64_t N, int64_t d) {
  return (sb == 0 && sh == 0 && sn == 0) || (sb == H * N * d && sh == N * d && sn == d);
}

csa_status validate_rel(const csa_rel_attn_args* a) {
  if (!a) return rfail(CSA_INVALID_ARG, "null args");
  if (a->B < 1 || a->H < 1 || a->N < 1 || a->L < 1) return rfail(CSA_INVALID_ARG, "B, H, N, L must be >= 1");
  if (a->d != 16 && a->d != 32 && a->d != 64 && a->d != 96)
    return rfail(CSA_UNSUPPORTED_SHAPE, "d_k must be 16, 32, 64 or 96");
  if (a->L > 256) return rfail(CSA_UNSUPPORTED_SHAPE, "relation vocabulary L must be <= 256 (uint8 indices)");
  if (!a->q || !a->k || !a->v || !a->lq || !a->lk || !a->rel || !a->mask || !a->out || !a->row_stats || !a->state)
    return rfail(CSA_INVALID_ARG, "null pointer");
  if (a->rel_head_group < 0 || a->rel_head_group > a->H) return rfail(CSA_INVALID_ARG, "bad rel_head_group");
  if (a->dtype != CSA_DTYPE_F32 && a->dtype != CSA_DTYPE_BF16) return rfail(CSA_INVALID_ARG, "bad dtype");
  if (a->dtype == CSA_DTYPE_BF16 && a->d != 64) return rfail(CSA_UNSUPPORTED_SHAPE, "bf16 CSE needs d_k = 64");
  auto al16 = [](const void* ptr, int64_t sb, int64_t sh, int64_t sn) {
    return (((uintptr_t)ptr) % 16 == 0) && sb % 4 == 0 && sh % 4 == 0 && sn % 4 == 0;
  };
  if (!al16(a->q, a->q_sb, a->q_sh, a->q_sn) || !al16(a->k, a->k_sb, a->k_sh, a->k_sn) ||
      !al16(a->v, a->v_sb, a->v_sh, a->v_sn) || !al16(a->out, a->o_sb, a->o_sh, a->o_sn))
    return rfail(CSA_INVALID_ARG, "q/k/v/out must be 16-byte aligned with strides multiple of 4 elements");
  if (a->d != 64 && !contig3(a->o_sb, a->o_sh, a->o_sn, a->H, a->N, a->d))
    return rfail(CSA_UNSUPPORTED_SHAPE, "a strided out needs d_k = 64");
  return CSA_OK;
}

RelArgs make_rel(const csa_rel_attn_args* a, const RelLayout& R) {
  void* ws = a->state;
  RelArgs p;
  memset(&p, 0, sizeof(p));
  p.B = (int)a->B; p.H = (int)a->H; p.N = (int)a->N; p.L = (int)a->L; p.Lp = (int)R.Lp;
  p.NQB = (int)((a->N + 31) / 32); p.NKB = p.NQB; p.group = (int)a->rel_head_group; p.ldg = (int)R.ldg;
  p.q = a->q; p.k = a->k; p.v = a->v;
  p.q_sb = a->q_sb; p.q_sh = a->q_sh; p.q_sn = a->q_sn;
  p.k_sb = a->k_sb; p.k_sh = a->k_sh; p.k_sn = a->k_sn;
  p.v_sb = a->v_sb; p.v_sh = a->v_sh; p.v_sn = a->v_sn;
  p.rel = a->rel; p.mask = a->mask;
  p.rel_sb = a->rel_sb; p.rel_sh = a->rel_sh; p.mask_sb = a->mask_sb; p.mask_sh = a->mask_sh;
  p.c2p = (const float*)((char*)ws + R.c2p);
  p.p2ct = (const float*)((char*)ws + R.p2ct);
  p.out = a->out; p.stats = a->row_stats;
  {
    const bool oc = a->o_sb == 0 && a->o_sh == 0 && a->o_sn == 0;  // zero triple: contiguous
    p.o_sb = oc ? a->H * a->N * a->d : a->o_sb;
    p.o_sh = oc ? a->N * a->d : a->o_sh;
    p.o_sn = oc ? a->d : a->o_sn;
  }
  p.inv_scale = 1.f / sqrtf(3.f * (float)a->d);
  p.lq = a->lq; p.lk = a->lk;
  p.bf16 = a->dtype == CSA_DTYPE_BF16;
  if (R.fused) {
    p.NP = (int)R.NP;
    p.P_ = a->rel_head_group > 0 ? 2 : (a->rel_sh == 0 && a->mask_sh == 0 ? 1 : (int)a->H);
    p.RM = (const uint16_t*)((char*)ws + R.RM);
    p.RT = (const uint16_t*)((char*)ws + R.RT);
    p.RB = (const float*)((char*)ws + R.RB);
    p.ldx = R.ldx;
    p.KB2 = (int)(((a->L + 7) / 8) * 4);  // bins K loop: 2 KB2 >= L, KB2 a multiple of 4
    p.LB = 2 * p.KB2 + (((2 * p.KB2 / 4) % 2 == 0) ? 4 : 0);  // LB / 4 odd (conflict-free b128 rows)
    p.Q4 = (int)(((a->L + 7) / 8) * 2);  // 16-row bins: 4 Q4 >= L, Q4 even (b64 reads)
    p.LB16 = 4 * p.Q4 + 2;               // LB16 / 2 odd (conflict-free b64 rows)
  }
  return p;
}

size_t bins_lds_bytes(const RelArgs& p) { return sizeof(float) * 32 * (size_t)p.LB; }
size_t bins16_lds_bytes(const RelArgs& p) { return sizeof(float) * 2 * 16 * (size_t)p.LB16; }

// fp32 backward on the 16-row kernels (two waves per SIMD); bf16 mode keeps the 32-row kernels.
inline bool rel_use16(const RelArgs& p) {
  return !p.bf16;
}


// relation logits: C2P[b,h] = Q LK_h^T (N x L), P2CT[b,h] = K LQ_h^T (N x L)
void rel_logits(const csa_rel_attn_args* a, const RelLayout& R, hipStream_t st) {
  void* ws = a->state;
  for (int which = 0; which < 2; ++which) {
    GemmArgs g;
    memset(&g, 0, sizeof(g));
    const float* X = which == 0 ? a->q : a->k;
    g.A = X; g.a_m = which == 0 ? a->q_sn : a->k_sn; g.a_k = 1;
    g.a_b1 = which == 0 ? a->q_sb : a->k_sb; g.a_b2 = which == 0 ? a->q_sh : a->k_sh;
    g.B = which == 0 ? a->lk : a->lq; g.b_n = a->d; g.b_k = 1; g.b_b1 = 0; g.b_b2 = a->L * a->d;
    g.C = (float*)((char*)ws + (which == 0 ? R.c2p : R.p2ct));
    g.c_m = R.Lp; g.c_n = 1; g.c_b1 = a->H * a->N * R.Lp; g.c_b2 = a->N * R.Lp;
    g.M = (int)a->N; g.N = (int)a->L; g.K = (int)a->d; g.H2 = (int)a->H; g.R = 1; g.alpha = 1.f; g.accumulate = 0;
    gemm(st, g, (int)(a->B * a->H));
  }
}

// ABI v9 stage timing: records the caller's events around one CSE stage (no-op when prof is NULL)
struct RelStage {
  const csa_prof* pf; int s; hipStream_t st;
  RelStage(const csa_prof* pf_, int s_, hipStream_t st_) : pf(pf_), s(s_), st(st_) {
    if (pf && pf->start[s]) (void)hipEventRecord((hipEvent_t)pf->start[s], st);
  }
  ~RelStage() {
    if (pf && pf->stop[s]) (void)hipEventRecord((hipEvent_t)pf->stop[s], st);
  }
};

void rel_param_grads(const csa_rel_attn_args* a, const csa_rel_attn_bwd_args* b, const RelLayout& R, float* gc2p,
                     float* gp2ct, hipStream_t st) {
  void* ws = b->workspace;
  const int B = (int)a->B, H = (int)a->H, N = (int)a->N, L = (int)a->L, D = (int)a->d;
  const int64_t Lp = R.Lp;
  // dlk_h = sum_b G_c2p^T Q ; dlq_h = sum_b G_p2cT^T K    (C(m=r, n=dd) = sum_b sum_x G(x,r) X(x,dd))
  if (R.fused) {
    const RelStage sg(b->prof, CSA_REL_STAGE_LGRAD, st);
    float* part = (float*)((char*)ws + R.part);
    const int64_t n = (int64_t)H * L * D;
    LgradArgs g;
    g.G[0] = gc2p; g.G[1] = gp2ct; g.X[0] = a->q; g.X[1] = a->k;
    g.x_sb[0] = a->q_sb; g.x_sh[0] = a->q_sh; g.x_sn[0] = a->q_sn;
    g.x_sb[1] = a->k_sb; g.x_sh[1] = a->k_sh; g.x_sn[1] = a->k_sn;
    g.part[0] = part; g.part[1] = part + (int64_t)R.RS * n;
    g.ldx = R.ldx; g.Lp = (int)Lp; g.L = L; g.NP = (int)R.NP; g.B = B; g.N = N; g.H = H; g.nsplit = R.RS;
    hipLaunchKernelGGL(k_rel_lgrad, dim3((unsigned)H, (unsigned)(2 * R.RS)), dim3(64 * (unsigned)((L + 31) / 32)),
                       2 * 32 * 64 * 4, st, g);
    hipLaunchKernelGGL(k_sum_splits2, dim3((unsigned)((n + 255) / 256), 2), dim3(256), 0, st, g.part[0], g.part[1],
                       b->dlk, b->dlq, n, R.RS);
    return;
  }
  for (int which = 0; which < 2; ++which) {
    GemmArgs g;
    memset(&g, 0, sizeof(g));
    g.A = which == 0 ? gc2p : gp2ct;
    g.a_m = 1; g.a_k = Lp; g.a_b1 = 0; g.a_b2 = (int64_t)N * Lp; g.a_r = (int64_t)H * N * Lp;
    const float* X = which == 0 ? a->q : a->k;
    g.B = X; g.b_n = 1; g.b_k = which == 0 ? a->q_sn : a->k_sn; g.b_b1 = 0;
    g.b_b2 = which == 0 ? a->q_sh : a->k_sh; g.b_r = which == 0 ? a->q_sb : a->k_sb;
    float* part = (float*)((char*)ws + R.part);
    g.C = R.RS > 1 ? part : (which == 0 ? b->dlk : b->dlq);
    g.c_m = D; g.c_n = 1; g.c_b1 = 0; g.c_b2 = (int64_t)L * D;
    g.M = L; g.N = D; g.K = N; g.H2 = H; g.R = B; g.alpha = 1.f; g.accumulate = 0;
    g.rsplit = R.RS; g.nbat = H; g.c_split = (int64_t)H * L * D;
    gemm(st, g, H);
    if (R.RS > 1) {
      const int64_t n = (int64_t)H * L * D;
      hipLaunchKernelGGL(k_sum_splits, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, part,
                         which == 0 ? b->dlk : b->dlq, n, R.RS, g.c_split);
    }
  }
}

}  // namespace

extern "C" {

size_t csa_rel_attn_state_bytes(int64_t B, int64_t H, int64_t N, int64_t L, int64_t d) {
  return rel_layout(B, H, N, L, d).state_total;
}

size_t csa_rel_attn_bwd_workspace_bytes(int64_t B, int64_t H, int64_t N, int64_t L, int64_t d) {
  return rel_layout(B, H, N, L, d).ws_total;
}

csa_status csa_rel_attn_fwd(const csa_rel_attn_args* a, void* stream) {
  csa_status s = validate_rel(a);
  if (s != CSA_OK) return s;
  const RelLayout R = rel_layout(a->B, a->H, a->N, a->L, a->d);
  hipStream_t st = (hipStream_t)stream;
  const DeviceGuard guard(st);
  RelArgs p = make_rel(a, R);
  const dim3 grid(xcd_grid(p.NQB, (int)(a->B * a->H)));
  if (R.fused) {
    {
    const RelStage sg(a->prof, CSA_REL_STAGE_LOGITS, st);
    const int NT = (int)(R.NP / 32);
    const unsigned nlog = xcd_grid(2 * (int)((p.NQB + 1) / 2), (int)(a->B * a->H));
    const size_t prep_lds = rel_prep_lds_bytes(a->N);
    // N <= 256: the prep items ride in the logits launch as extra one-wave workgroups (its LDS then grows to the
    // staged rows, <= 16 KB, and the logits grid still fits one round); larger N keeps the separate launch
    const bool merged = prep_lds <= 16384;
    const size_t logits_lds = merged ? std::max<size_t>(32 * 64 * 4, prep_lds) : 32 * 64 * 4;
    const unsigned nprep = merged ? (unsigned)(NT * a->B * p.P_) : 0u;
    hipLaunchKernelGGL(k_rel_logits<64>, dim3(nlog + nprep), dim3(64), logits_lds, st, p, (float*)p.c2p, (float*)p.p2ct,
                       (uint16_t*)p.RM, (uint16_t*)p.RT, (int)nlog);
    if (merged) {
    } else if (prep_lds <= 65536) {
      set_dyn_lds((const void*)k_rel_prep, (int)rel_prep_lds_bytes(a->N));
      hipLaunchKernelGGL(k_rel_prep, dim3((unsigned)NT, (unsigned)(a->B * p.P_)), dim3(256), rel_prep_lds_bytes(a->N),
                         st, p, (uint16_t*)p.RM, (uint16_t*)p.RT);
    } else {
      hipLaunchKernelGGL(k_rel_prep_t, dim3((unsigned)(NT * NT), (unsigned)(a->B * p.P_)), dim3(256), 0, st, p,
                         (uint16_t*)p.RM, (uint16_t*)p.RT);
    }
    }
    const RelStage sg(a->prof, CSA_REL_STAGE_FWD, st);
    if (p.bf16) hipLaunchKernelGGL((k_rel_fwd_f<64, true>), grid, dim3(64), 2 * 32 * 64 * 4, st, p);
    else hipLaunchKernelGGL((k_rel_fwd_f<64, false>), grid, dim3(64), 2 * 32 * 64 * 4, st, p);
    return rcheck("csa_rel_attn_fwd");
  }
  rel_logits(a, R, st);
  if (a->d == 64) hipLaunchKernelGGL(k_rel_fwd<64>, grid, dim3(64), 0, st, p);
  else if (a->d == 32) hipLaunchKernelGGL(k_rel_fwd<32>, grid, dim3(64), 0, st, p);
  else if (a->d == 16) hipLaunchKernelGGL(k_rel_fwd<16>, grid, dim3(64), 0, st, p);
  else hipLaunchKernelGGL(k_rel_fwd<96>, grid, dim3(64), 0, st, p);
  return rcheck("csa_rel_attn_fwd");
}

csa_status csa_rel_attn_bwd(const csa_rel_attn_bwd_args* b, void* stream) {
  if (!b || !b->fwd) return rfail(CSA_INVALID_ARG, "null args");
  const csa_rel_attn_args* a = b->fwd;
  csa_status s = validate_rel(a);
  if (s != CSA_OK) return s;
  if (!b->dout || !b->dq || !b->dk || !b->dv || !b->dlq || !b->dlk || !b->workspace)
    return rfail(CSA_INVALID_ARG, "null gradient pointer / workspace");
  if (b->schedule > CSA_SCHED_CONCURRENT) return rfail(CSA_INVALID_ARG, "schedule must be a CSA_SCHED_* value");
  const RelLayout R = rel_layout(a->B, a->H, a->N, a->L, a->d);
  hipStream_t st = (hipStream_t)stream;
  const DeviceGuard guard(st);
  void* ws = b->workspace;
  RelArgs p = make_rel(a, R);
  p.dout = b->dout; p.dq = b->dq;
  {
    auto al16 = [](const void* ptr, int64_t sb, int64_t sh, int64_t sn) {
      return (((uintptr_t)ptr) % 16 == 0) && sb % 4 == 0 && sh % 4 == 0 && sn % 4 == 0;
    };
    const int64_t t[4][3] = {{b->do_sb, b->do_sh, b->do_sn}, {b->dq_sb, b->dq_sh, b->dq_sn},
                             {b->dk_sb, b->dk_sh, b->dk_sn}, {b->dv_sb, b->dv_sh, b->dv_sn}};
    const void* ptrs[4] = {b->dout, b->dq, b->dk, b->dv};
    int64_t* dst[4][3] = {{&p.do_sb, &p.do_sh, &p.do_sn}, {&p.dq_sb, &p.dq_sh, &p.dq_sn},
                          {&p.dk_sb, &p.dk_sh, &p.dk_sn}, {&p.dv_sb, &p.dv_sh, &p.dv_sn}};
    for (int u = 0; u < 4; ++u) {
      const bool c = t[u][0] == 0 && t[u][1] == 0 && t[u][2] == 0;
      if (!R.fused && !contig3(t[u][0], t[u][1], t[u][2], a->H, a->N, a->d))
        return rfail(CSA_UNSUPPORTED_SHAPE, "strided dout/dq/dk/dv need d_k = 64");
      if (!al16(ptrs[u], t[u][0], t[u][1], t[u][2]))
        return rfail(CSA_INVALID_ARG, "dout/dq/dk/dv must be 16-byte aligned with strides multiple of 4 elements");
      *dst[u][0] = c ? a->H * a->N * a->d : t[u][0];
      *dst[u][1] = c ? a->N * a->d : t[u][1];
      *dst[u][2] = c ? a->d : t[u][2];
    }
  }
  p.G = (float*)((char*)ws + R.G);
  p.P = (float*)((char*)ws + R.P);
  const int B = (int)a->B, H = (int)a->H, N = (int)a->N, L = (int)a->L, D = (int)a->d;
  const int64_t Lp = R.Lp;
  float* gc2p = (float*)((char*)ws + R.gc2p);
  float* gp2ct = (float*)((char*)ws + R.gp2ct);
  if (R.fused) {
    p.dk = b->dk; p.dv = b->dv; p.gc2p = gc2p; p.gp2ct = gp2ct;
    p.qstat = (float*)((char*)ws + R.qstat);
    const bool w16 = rel_use16(p);
    const size_t lq_bytes = w16 ? rel16_bins_off(false) + bins16_lds_bytes(p) : 2 * 32 * 64 * 4 + 4096 + bins_lds_bytes(p);
    const size_t lk_bytes = w16 ? rel16_bins_off(true) + bins16_lds_bytes(p) : 2 * 32 * 64 * 4 + 512 + 4096 + bins_lds_bytes(p);
    const dim3 gq(xcd_grid(p.NQB, B * H)), gk(xcd_grid(p.NKB, B * H)), blk(w16 ? 128 : 64);
    const bool concur = b->side_stream && b->side_fork && b->side_join &&
                        bwd_concurrent(b->schedule, b->side_stream, stream_device(st), (int64_t)p.NQB * B * H, 1);
    const SideLane lane{(hipStream_t)b->side_stream, (hipEvent_t)b->side_fork, (hipEvent_t)b->side_join};
    const SideLane* side = concur ? &lane : nullptr;
    auto launch_q = [&](hipStream_t s_) {  // (bf16 mode: the fp32 path runs k_rel_bwd_qg below)
      if (p.bf16) {
        hipLaunchKernelGGL((k_rel_bwd_qf<64, true>), gq, blk, lq_bytes, s_, p);
      } else {
        hipLaunchKernelGGL((k_rel_bwd_qf<64, false>), gq, blk, lq_bytes, s_, p);
      }
    };
    auto launch_k = [&](hipStream_t s_) {
      if (w16) {
        set_dyn_lds((const void*)k_rel_bwd_kh, (int)lk_bytes);
        hipLaunchKernelGGL(k_rel_bwd_kh, gk, blk, lk_bytes, s_, p);
      } else if (p.bf16) {
        hipLaunchKernelGGL((k_rel_bwd_kf<64, true>), gk, blk, lk_bytes, s_, p);
      } else {
        hipLaunchKernelGGL((k_rel_bwd_kf<64, false>), gk, blk, lk_bytes, s_, p);
      }
    };
    // fp32: row statistics, key side (g tiles out), then the query side from the key side's g tiles (no score / dP
    // recompute on the query side; the round-3 recomputing query kernel measured slower, DESIGN.md §3 CSE A/B)
    if (w16) {
      p.qstat_pre = 1;
      p.gt = (float*)((char*)ws + R.gt);
      const int64_t threads = 4LL * B * H * N;
      {
        const RelStage sg(b->prof, CSA_REL_STAGE_QSTAT, st);
        hipLaunchKernelGGL(k_rel_qstat<4>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, st, p);
      }
      {
        const RelStage sg(b->prof, CSA_REL_STAGE_BWD_K, st);
        launch_k(st);
      }
      const size_t lg_bytes = rel16_bins_off(false) + bins16_lds_bytes(p);
      set_dyn_lds((const void*)k_rel_bwd_qg, (int)lg_bytes);
      const RelStage sg(b->prof, CSA_REL_STAGE_BWD_Q, st);
      hipLaunchKernelGGL(k_rel_bwd_qg, gq, blk, lg_bytes, st, p);
    } else if (side) {  // fork: row statistics + key side on the side stream, query side here, join before the lgrad
      if (!side->fork(st)) return rfail_hip("csa_rel_attn_bwd: side-stream fork");
      p.qstat_pre = 1;
      const int parts = w16 ? 4 : 2;
      const int64_t threads = (int64_t)parts * B * H * N;
      if (w16) hipLaunchKernelGGL(k_rel_qstat<4>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, side->s, p);
      else hipLaunchKernelGGL(k_rel_qstat<2>, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, side->s, p);
      launch_k(side->s);
      launch_q(st);
      if (!side->join(st)) return rfail_hip("csa_rel_attn_bwd: side-stream join");
    } else {
      launch_q(st);
      launch_k(st);
    }
    rel_param_grads(a, b, R, gc2p, gp2ct, st);
    return rcheck("csa_rel_attn_bwd");
  }
  // G^T / P^T: columns x >= N of each row are never written; the GEMMs select zeros there
  const dim3 grid(xcd_grid(p.NQB, B * H));
  if (D == 64) hipLaunchKernelGGL(k_rel_bwd_q<64>, grid, dim3(64), 0, st, p);
  else if (D == 32) hipLaunchKernelGGL(k_rel_bwd_q<32>, grid, dim3(64), 0, st, p);
  else if (D == 16) hipLaunchKernelGGL(k_rel_bwd_q<16>, grid, dim3(64), 0, st, p);
  else hipLaunchKernelGGL(k_rel_bwd_q<96>, grid, dim3(64), 0, st, p);
  // dv = P^T dO ; dk = G^T Q    (per (b,h): C(m=y, n=dd) = sum_x X(x,y) Y(x,dd))
  for (int which = 0; which < 2; ++which) {
    GemmArgs g;
    memset(&g, 0, sizeof(g));
    g.A = which == 0 ? p.P : p.G; g.a_m = R.ldg; g.a_k = 1; g.a_b1 = (int64_t)H * N * R.ldg;
    g.a_b2 = (int64_t)N * R.ldg;
    if (which == 0) { g.B = b->dout; g.b_n = 1; g.b_k = D; g.b_b1 = (int64_t)H * N * D; g.b_b2 = (int64_t)N * D; }
    else { g.B = a->q; g.b_n = 1; g.b_k = a->q_sn; g.b_b1 = a->q_sb; g.b_b2 = a->q_sh; }
    g.C = which == 0 ? b->dv : b->dk; g.c_m = D; g.c_n = 1; g.c_b1 = (int64_t)H * N * D; g.c_b2 = (int64_t)N * D;
    g.M = N; g.N = D; g.K = N; g.H2 = H; g.R = 1; g.alpha = 1.f; g.accumulate = 0;
    gemm(st, g, B * H);
  }
  // gather backward
  const unsigned nrow = (unsigned)(((int64_t)B * H * N + 63) / 64);
  const size_t lds = sizeof(float) * 64 * Lp;
  set_dyn_lds((const void*)k_rel_scatter, (int)lds);
  hipLaunchKernelGGL(k_rel_scatter, dim3(nrow), dim3(64), lds, st, p, gc2p, 0);
  hipLaunchKernelGGL(k_rel_scatter, dim3(nrow), dim3(64), lds, st, p, gp2ct, 1);
  // dq += G_c2p LK_h ; dk += G_p2cT LQ_h    (C(m=x, n=dd) = sum_r G(x,r) LK(r,dd))
  for (int which = 0; which < 2; ++which) {
    GemmArgs g;
    memset(&g, 0, sizeof(g));
    g.A = which == 0 ? gc2p : gp2ct; g.a_m = Lp; g.a_k = 1; g.a_b1 = (int64_t)H * N * Lp; g.a_b2 = (int64_t)N * Lp;
    g.B = which == 0 ? a->lk : a->lq; g.b_n = 1; g.b_k = D; g.b_b1 = 0; g.b_b2 = (int64_t)L * D;
    g.C = which == 0 ? b->dq : b->dk; g.c_m = D; g.c_n = 1; g.c_b1 = (int64_t)H * N * D; g.c_b2 = (int64_t)N * D;
    g.M = N; g.N = D; g.K = L; g.H2 = H; g.R = 1; g.alpha = 1.f; g.accumulate = 1;
    gemm(st, g, B * H);
  }
  rel_param_grads(a, b, R, gc2p, gp2ct, st);
  return rcheck("csa_rel_attn_bwd");
}

}  // extern "C"
