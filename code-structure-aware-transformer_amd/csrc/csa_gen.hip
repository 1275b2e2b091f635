// Generator head of module/components.py:95-102 on gfx950:
//
//   out = linear(x)                (hipBLASLt, unchanged)
//   logp = log(softmax(dropout(out), -1))   <- this file, one kernel per direction
//
// The reference runs dropout (2 passes + a bool mask), softmax and log as separate kernels over the
// (B*T, V) logits, i.e. 3 reads + 3 writes of a 251 MB tensor per step at the java config
// (B=64, T=49, V=20000), and 3 more kernels in the backward. Here:
//   fwd: read out once (a second read of the row hits L2), write logp once;
//   bwd: read dlogp and logp (second pass from L2), write dout once.
// Semantics kept: log OF softmax (an underflowed probability gives -inf, as torch.log(softmax));
// backward is the autograd chain log -> softmax -> dropout literally, t = g / s,
// dz = keep/(1-p) * s * (t - sum_k t_k s_k), so a 0/0 propagates exactly as in the reference.
//
// Dropout draws come from the stateless Philox4x32-7 stream RNG_GEN_DROP keyed by (seed, offset):
// element (row, col) uses 16-bit uniform (col & 7) of philox(ctr = {col >> 3, row, 0,
// (RNG_GEN_DROP << 28) ^ offset}); keep <=> u16 >= ceil(p * 65536) (oracle/philox.py:gen_keep).
//
// One workgroup per row; each thread owns groups of 8 consecutive columns (one Philox call per
// group, two dwordx4 loads when the row is 16-B aligned). Rows up to V = 24576 stay in registers
// (k_gen_*_r, 512 threads: one HBM read per element); longer rows take the two-pass loop kernels
// (second pass from L2).
#include "csa_common.hpp"
#include "../../include/csa_hip.h"

#include <math.h>

using namespace csa;

namespace {

constexpr uint32_t RNG_GEN_DROP = 4u;
constexpr int GT = 256;

struct GenArgs {
  int64_t rows, V;
  uint32_t seed_lo, seed_hi, off, thr;  // thr = ceil(p * 65536); 0 = no dropout
  float scale;                          // 1 / (1 - p)
};

__device__ __forceinline__ uint32_t gen_u16(const u32x4& r, int e) {
  const uint32_t w = (e >> 1) == 0 ? r.x : (e >> 1) == 1 ? r.y : (e >> 1) == 2 ? r.z : r.w;
  return (e & 1) ? (w >> 16) : (w & 0xffffu);
}

// 8 values of group gi of a row (zero beyond V), and their keep bits (all 1 without dropout).
__device__ __forceinline__ void load8(const float* __restrict__ row, int64_t V, int64_t gi, bool vec, float* v) {
  const int64_t c0 = 8 * gi;
  if (vec && c0 + 8 <= V) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(row + c0);
    const f32x4 b = *reinterpret_cast<const f32x4*>(row + c0 + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) { v[e] = a[e]; v[4 + e] = b[e]; }
  } else {
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (c0 + e < V) ? row[c0 + e] : 0.f;
  }
}

__device__ __forceinline__ uint32_t keep8(const GenArgs& a, int64_t row, int64_t gi) {
  if (a.thr == 0) return 0xffu;
  const u32x4 r = philox4x32(u32x4{(uint32_t)gi, (uint32_t)row, 0u, (RNG_GEN_DROP << 28) ^ a.off}, a.seed_lo,
                             a.seed_hi);
  uint32_t k = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) k |= (gen_u16(r, e) >= a.thr ? 1u : 0u) << e;
  return k;
}

__device__ __forceinline__ float dropv(float z, uint32_t keep, int e, const GenArgs& a) {
  return a.thr == 0 ? z : (((keep >> e) & 1u) ? z * a.scale : 0.f * z);  // nn.Dropout: z * mask * scale
}

// block-wide (max, sum) merge of per-thread online-softmax states, fixed order
__device__ __forceinline__ void block_maxsum(float& m, float& s, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    const float mo = __shfl_xor(m, o, 64), so = __shfl_xor(s, o, 64);
    const float mn = fmaxf(m, mo);
    s = (mn == -INFINITY ? 0.f : s * expf(m - mn) + so * expf(mo - mn));
    m = mn;
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[2 * w] = m; red[2 * w + 1] = s; }
  __syncthreads();
  m = red[0]; s = red[1];
#pragma unroll
  for (int i = 1; i < GT / 64; ++i) {
    const float mo = red[2 * i], so = red[2 * i + 1];
    const float mn = fmaxf(m, mo);
    s = (mn == -INFINITY ? 0.f : s * expf(m - mn) + so * expf(mo - mn));
    m = mn;
  }
}

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  float t = red[0];
#pragma unroll
  for (int i = 1; i < GT / 64; ++i) t += red[i];
  return t;
}

__global__ __launch_bounds__(GT) void k_gen_fwd(const float* __restrict__ z, float* __restrict__ logp, const GenArgs a) {
  __shared__ float red[2 * GT / 64];
  const int64_t row = blockIdx.x;
  const float* zr = z + row * a.V;
  float* out = logp + row * a.V;
  const bool vec = (a.V % 4 == 0) && ((((uintptr_t)z) | ((uintptr_t)logp)) & 15) == 0;
  const int64_t ng = (a.V + 7) / 8;
  float m = -INFINITY, s = 0.f;
  for (int64_t gi = threadIdx.x; gi < ng; gi += GT) {
    float v[8];
    load8(zr, a.V, gi, vec, v);
    const uint32_t keep = keep8(a, row, gi);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (8 * gi + e >= a.V) continue;
      const float x = dropv(v[e], keep, e, a);
      if (x > m) { s = s * expf(m - x) + 1.f; m = x; }
      else s += expf(x - m);
    }
  }
  block_maxsum(m, s, red);
  for (int64_t gi = threadIdx.x; gi < ng; gi += GT) {
    float v[8];
    load8(zr, a.V, gi, vec, v);
    const uint32_t keep = keep8(a, row, gi);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = logf(expf(dropv(v[e], keep, e, a) - m) / s);  // log(softmax)
    const int64_t c0 = 8 * gi;
    if (vec && c0 + 8 <= a.V) {
      *reinterpret_cast<f32x4*>(out + c0) = f32x4{o[0], o[1], o[2], o[3]};
      *reinterpret_cast<f32x4*>(out + c0 + 4) = f32x4{o[4], o[5], o[6], o[7]};
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c0 + e < a.V) out[c0 + e] = o[e];
    }
  }
}

__global__ __launch_bounds__(GT) void k_gen_bwd(const float* __restrict__ g, const float* __restrict__ logp,
                                                float* __restrict__ dz, const GenArgs a) {
  __shared__ float red[GT / 64];
  const int64_t row = blockIdx.x;
  const float* gr = g + row * a.V;
  const float* lr = logp + row * a.V;
  float* out = dz + row * a.V;
  const bool vec = (a.V % 4 == 0) && ((((uintptr_t)g) | ((uintptr_t)logp) | ((uintptr_t)dz)) & 15) == 0;
  const int64_t ng = (a.V + 7) / 8;
  float acc = 0.f;
  for (int64_t gi = threadIdx.x; gi < ng; gi += GT) {
    float gv[8], lv[8];
    load8(gr, a.V, gi, vec, gv);
    load8(lr, a.V, gi, vec, lv);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (8 * gi + e >= a.V) continue;
      const float sv = expf(lv[e]);
      acc += (gv[e] / sv) * sv;  // sum_k t_k s_k of softmax_backward, t = g / s (log backward)
    }
  }
  const float tot = block_sum(acc, red);
  for (int64_t gi = threadIdx.x; gi < ng; gi += GT) {
    float gv[8], lv[8];
    load8(gr, a.V, gi, vec, gv);
    load8(lr, a.V, gi, vec, lv);
    const uint32_t keep = keep8(a, row, gi);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float sv = expf(lv[e]);
      o[e] = dropv(sv * (gv[e] / sv - tot), keep, e, a);
    }
    const int64_t c0 = 8 * gi;
    if (vec && c0 + 8 <= a.V) {
      *reinterpret_cast<f32x4*>(out + c0) = f32x4{o[0], o[1], o[2], o[3]};
      *reinterpret_cast<f32x4*>(out + c0 + 4) = f32x4{o[4], o[5], o[6], o[7]};
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c0 + e < a.V) out[c0 + e] = o[e];
    }
  }
}

// Register-resident variants (V <= RT * 8 * NG): each thread keeps its NG groups of 8 columns in
// registers across both passes, so every element is read from HBM exactly once and the row max is
// taken before any exp (sum_j exp(x_j - max) as the reference softmax computes it).
constexpr int RT = 512;

template <int NG>
__global__ __launch_bounds__(RT) void k_gen_fwd_r(const float* __restrict__ z, float* __restrict__ logp, const GenArgs a) {
  __shared__ float red[RT / 64];
  const int64_t row = blockIdx.x;
  const float* zr = z + row * a.V;
  float* out = logp + row * a.V;
  const bool vec = (a.V % 4 == 0) && ((((uintptr_t)z) | ((uintptr_t)logp)) & 15) == 0;
  const int64_t ng = (a.V + 7) / 8;
  float x[NG][8];
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int64_t gi = threadIdx.x + (int64_t)q * RT;
    load8(zr, a.V, gi < ng ? gi : 0, vec, x[q]);
  }
  float m = -INFINITY;
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int64_t gi = threadIdx.x + (int64_t)q * RT;
    const uint32_t keep = keep8(a, row, gi);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool in = gi < ng && 8 * gi + e < a.V;
      x[q][e] = in ? dropv(x[q][e], keep, e, a) : -INFINITY;
      m = fmaxf(m, x[q][e]);
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  m = red[0];
#pragma unroll
  for (int i = 1; i < RT / 64; ++i) m = fmaxf(m, red[i]);
  __syncthreads();
  float sum = 0.f;
#pragma unroll
  for (int q = 0; q < NG; ++q)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      x[q][e] = expf(x[q][e] - m);  // 0 beyond V (exp(-inf))
      sum += x[q][e];
    }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) sum += __shfl_xor(sum, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = sum;
  __syncthreads();
  float S = red[0];
#pragma unroll
  for (int i = 1; i < RT / 64; ++i) S += red[i];
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int64_t gi = threadIdx.x + (int64_t)q * RT;
    if (gi >= ng) continue;
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = logf(x[q][e] / S);  // log(softmax)
    const int64_t c0 = 8 * gi;
    if (vec && c0 + 8 <= a.V) {
      __builtin_nontemporal_store(f32x4{o[0], o[1], o[2], o[3]}, reinterpret_cast<f32x4*>(out + c0));
      __builtin_nontemporal_store(f32x4{o[4], o[5], o[6], o[7]}, reinterpret_cast<f32x4*>(out + c0 + 4));
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c0 + e < a.V) out[c0 + e] = o[e];
    }
  }
}

template <int NG>
__global__ __launch_bounds__(RT) void k_gen_bwd_r(const float* __restrict__ g, const float* __restrict__ logp,
                                                  float* __restrict__ dz, const GenArgs a) {
  __shared__ float red[RT / 64];
  const int64_t row = blockIdx.x;
  const float* gr = g + row * a.V;
  const float* lr = logp + row * a.V;
  float* out = dz + row * a.V;
  const bool vec = (a.V % 4 == 0) && ((((uintptr_t)g) | ((uintptr_t)logp) | ((uintptr_t)dz)) & 15) == 0;
  const int64_t ng = (a.V + 7) / 8;
  float sv[NG][8], tv[NG][8];
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int64_t gi = threadIdx.x + (int64_t)q * RT;
    load8(gr, a.V, gi < ng ? gi : 0, vec, tv[q]);
    load8(lr, a.V, gi < ng ? gi : 0, vec, sv[q]);
  }
  float acc = 0.f;
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int64_t gi = threadIdx.x + (int64_t)q * RT;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const bool in = gi < ng && 8 * gi + e < a.V;
      sv[q][e] = expf(sv[q][e]);
      tv[q][e] = tv[q][e] / sv[q][e];  // log backward: t = g / s
      acc += in ? tv[q][e] * sv[q][e] : 0.f;
    }
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  float tot = red[0];
#pragma unroll
  for (int i = 1; i < RT / 64; ++i) tot += red[i];
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int64_t gi = threadIdx.x + (int64_t)q * RT;
    if (gi >= ng) continue;
    const uint32_t keep = keep8(a, row, gi);
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = dropv(sv[q][e] * (tv[q][e] - tot), keep, e, a);
    const int64_t c0 = 8 * gi;
    if (vec && c0 + 8 <= a.V) {
      *reinterpret_cast<f32x4*>(out + c0) = f32x4{o[0], o[1], o[2], o[3]};
      *reinterpret_cast<f32x4*>(out + c0 + 4) = f32x4{o[4], o[5], o[6], o[7]};
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (c0 + e < a.V) out[c0 + e] = o[e];
    }
  }
}

// groups per thread covering the row (1..6), 0 = loop kernels
inline int reg_groups(int64_t V) {
  const int64_t per = ((V + 7) / 8 + RT - 1) / RT;
  return per <= 6 ? (int)per : 0;
}

csa_status gfail(csa_status s, const char* m) {
  csa::set_error("%s", m);
  return s;
}

bool make_gen(int64_t rows, int64_t V, float p, uint64_t seed, uint64_t offset, GenArgs* a) {
  if (rows < 0 || V < 1 || rows > 0x7fffffff || !(p >= 0.f && p < 1.f)) return false;
  a->rows = rows; a->V = V;
  a->seed_lo = (uint32_t)seed; a->seed_hi = (uint32_t)(seed >> 32); a->off = (uint32_t)offset;
  a->thr = p > 0.f ? (uint32_t)ceil((double)p * 65536.0) : 0u;
  a->scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  return true;
}

}  // namespace

extern "C" {

csa_status csa_gen_logsoftmax_fwd(const float* logits, float* logp, int64_t rows, int64_t V, float dropout,
                                  uint64_t seed, uint64_t offset, void* stream) {
  GenArgs a;
  if (!make_gen(rows, V, dropout, seed, offset, &a)) return gfail(CSA_INVALID_ARG, "csa_gen_logsoftmax_fwd: bad rows/V/p");
  if (rows == 0) return CSA_OK;
  if (!logits || !logp) return gfail(CSA_INVALID_ARG, "csa_gen_logsoftmax_fwd: null pointer");
  const hipStream_t st = (hipStream_t)stream;
  const DeviceGuard guard(st);
  const dim3 grid((unsigned)rows);
  switch (reg_groups(V)) {
    case 1: hipLaunchKernelGGL(k_gen_fwd_r<1>, grid, dim3(RT), 0, st, logits, logp, a); break;
    case 2: hipLaunchKernelGGL(k_gen_fwd_r<2>, grid, dim3(RT), 0, st, logits, logp, a); break;
    case 3: hipLaunchKernelGGL(k_gen_fwd_r<3>, grid, dim3(RT), 0, st, logits, logp, a); break;
    case 4: hipLaunchKernelGGL(k_gen_fwd_r<4>, grid, dim3(RT), 0, st, logits, logp, a); break;
    case 5: hipLaunchKernelGGL(k_gen_fwd_r<5>, grid, dim3(RT), 0, st, logits, logp, a); break;
    case 6: hipLaunchKernelGGL(k_gen_fwd_r<6>, grid, dim3(RT), 0, st, logits, logp, a); break;
    default: hipLaunchKernelGGL(k_gen_fwd, grid, dim3(GT), 0, st, logits, logp, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    csa::set_error("csa_gen_logsoftmax_fwd: %s", hipGetErrorString(e));
    return CSA_LAUNCH_FAILED;
  }
  return CSA_OK;
}

csa_status csa_gen_logsoftmax_bwd(const float* dlogp, const float* logp, float* dlogits, int64_t rows, int64_t V,
                                  float dropout, uint64_t seed, uint64_t offset, void* stream) {
  GenArgs a;
  if (!make_gen(rows, V, dropout, seed, offset, &a)) return gfail(CSA_INVALID_ARG, "csa_gen_logsoftmax_bwd: bad rows/V/p");
  if (rows == 0) return CSA_OK;
  if (!dlogp || !logp || !dlogits) return gfail(CSA_INVALID_ARG, "csa_gen_logsoftmax_bwd: null pointer");
  const hipStream_t st = (hipStream_t)stream;
  const DeviceGuard guard(st);
  const dim3 grid((unsigned)rows);
  switch (reg_groups(V)) {
    case 1: hipLaunchKernelGGL(k_gen_bwd_r<1>, grid, dim3(RT), 0, st, dlogp, logp, dlogits, a); break;
    case 2: hipLaunchKernelGGL(k_gen_bwd_r<2>, grid, dim3(RT), 0, st, dlogp, logp, dlogits, a); break;
    case 3: hipLaunchKernelGGL(k_gen_bwd_r<3>, grid, dim3(RT), 0, st, dlogp, logp, dlogits, a); break;
    case 4: hipLaunchKernelGGL(k_gen_bwd_r<4>, grid, dim3(RT), 0, st, dlogp, logp, dlogits, a); break;
    case 5: hipLaunchKernelGGL(k_gen_bwd_r<5>, grid, dim3(RT), 0, st, dlogp, logp, dlogits, a); break;
    case 6: hipLaunchKernelGGL(k_gen_bwd_r<6>, grid, dim3(RT), 0, st, dlogp, logp, dlogits, a); break;
    default: hipLaunchKernelGGL(k_gen_bwd, grid, dim3(GT), 0, st, dlogp, logp, dlogits, a);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    csa::set_error("csa_gen_logsoftmax_bwd: %s", hipGetErrorString(e));
    return CSA_LAUNCH_FAILED;
  }
  return CSA_OK;
}

}  // extern "C"
