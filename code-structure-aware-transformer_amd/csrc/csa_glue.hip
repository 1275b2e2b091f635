// Linear-layer bias gradient (db = sum over rows of dY) for the encoder glue of the train step
// (module/sbm_model.py:27-31, module/csa_trans.py FeedForward / CSE_layer, components.py Generator).
//
// torch's Linear backward reduces dY (rows x cols, rows = B*N = 9600 at the java step) with its
// generic strided reduce_kernel: ~18 us per call for a 29 MB read (1.6 TB/s), 95 calls per step.
// Here: pass 1, grid (cols / 64, RS row slices), each 256-thread workgroup sums a 64-column x
// (rows / RS) slab with dwordx4 loads (16 threads per row x 16 rows in flight), reduces its 16 row
// lanes through LDS in a fixed order and writes one partial row; pass 2 sums the RS partials in
// slice order. The summation order depends only on (rows, cols): deterministic.
#include <algorithm>
#include <cmath>

#include "csa_common.hpp"
#include "../../include/csa_hip.h"

using csa::f32x4;
using csa::philox4x32;
using csa::u32x4;

namespace {

constexpr int BG_COLS = 64, BG_RL = 16;

__global__ __launch_bounds__(256) void k_bias_grad_part(const float* __restrict__ dy, float* __restrict__ part,
                                                        int64_t rows, int64_t cols, int64_t rows_per_slice) {
  __shared__ float red[BG_RL][BG_COLS + 4];
  const int cq = threadIdx.x & 15, rl = threadIdx.x >> 4;
  const int64_t c0 = (int64_t)blockIdx.x * BG_COLS + 4 * cq;
  const int64_t r_lo = (int64_t)blockIdx.y * rows_per_slice;
  const int64_t r_hi = r_lo + rows_per_slice < rows ? r_lo + rows_per_slice : rows;
  const bool vec = (cols % 4 == 0) && (((uintptr_t)dy) & 15) == 0;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (vec && c0 + 4 <= cols) {
#pragma unroll 4
    for (int64_t r = r_lo + rl; r < r_hi; r += BG_RL) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(dy + r * cols + c0);
      acc[0] += v[0]; acc[1] += v[1]; acc[2] += v[2]; acc[3] += v[3];
    }
  } else {
    for (int64_t r = r_lo + rl; r < r_hi; r += BG_RL)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c0 + e < cols) acc[e] += dy[r * cols + c0 + e];
  }
#pragma unroll
  for (int e = 0; e < 4; ++e) red[rl][4 * cq + e] = acc[e];
  __syncthreads();
  if (threadIdx.x < BG_COLS) {
    const int64_t c = (int64_t)blockIdx.x * BG_COLS + threadIdx.x;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < BG_RL; ++i) s += red[i][threadIdx.x];
    if (c < cols) part[(int64_t)blockIdx.y * cols + c] = s;
  }
}

// Partials -> column sums. One workgroup per 16 columns; its 16 row groups each sum the partials
// i = rg, rg + 16, ... (8 loads in flight, added in index order), then one thread per column adds
// the 16 row-group sums in order. The order depends only on (rs, cols): deterministic. (One thread
// per column summing all rs partials left only cols / 256 workgroups: 8.7 us per LayerNorm call.)
constexpr int BS_COLS = 16, BS_RG = 16;

// Columns c >= split go to db2[c - split] (LayerNorm: dgamma | dbeta partials side by side, one launch).
__global__ __launch_bounds__(256) void k_bias_grad_sum(const float* __restrict__ part, float* __restrict__ db,
                                                       int64_t cols, int rs, int accumulate, int64_t stride,
                                                       float* __restrict__ db2, int64_t split) {
  __shared__ float red[BS_RG][BS_COLS + 1];
  const int cl = threadIdx.x % BS_COLS, rg = threadIdx.x / BS_COLS;
  const int64_t c = (int64_t)blockIdx.x * BS_COLS + cl;
  float s = 0.f;
  if (c < cols) {
    for (int i0 = rg; i0 < rs; i0 += 8 * BS_RG) {
      float v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * BS_RG;
        v[u] = i < rs ? part[(int64_t)i * stride + c] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
  }
  red[rg][cl] = s;
  __syncthreads();
  if (rg == 0 && c < cols) {
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < BS_RG; ++i) t += red[i][cl];
    float* out = c < split ? db + c : db2 + (c - split);
    *out = accumulate ? *out + t : t;
  }
}

inline int bg_slices(int64_t rows) {
  const int64_t rs = (rows + 255) / 256;  // >= 256 rows per slice
  return (int)(rs < 1 ? 1 : rs > 64 ? 64 : rs);
}

// ------------------------------------------------------------------------------------
// LayerNorm over the last dim (nn.LayerNorm(size), eps 1e-5, the encoder's pre-norm sublayers):
// one wave per row, the row in registers (CPL dwordx4 chunks per lane, cols <= 256 CPL), two-pass
// mean / variance in registers (no E[x^2] - mean^2 cancellation). Backward: dx per row from the
// saved (mean, rstd); dgamma / dbeta as per-workgroup column partials (fixed order) summed by
// k_bias_grad_sum, so the whole backward is deterministic.
// ------------------------------------------------------------------------------------
constexpr int LN_ROWS_PER_WG = 32;  // 4 waves x 8 rows (300 workgroups at 9600 rows)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int CPL>
__global__ __launch_bounds__(256) void k_ln_fwd(const float* __restrict__ x, const float* __restrict__ gamma,
                                                const float* __restrict__ beta, float* __restrict__ y,
                                                float* __restrict__ stats, int64_t rows, int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const float* xr = x + row * cols;
  f32x4 v[CPL];
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int c = 4 * (lane + 64 * q);
    v[q] = c < cols ? *reinterpret_cast<const f32x4*>(xr + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    s += (v[q][0] + v[q][1]) + (v[q][2] + v[q][3]);
  }
  const float mean = wave_sum(s) / (float)cols;
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int c = 4 * (lane + 64 * q);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float d = c < cols ? v[q][e] - mean : 0.f;
      ss = fmaf(d, d, ss);
    }
  }
  const float rstd = 1.f / sqrtf(wave_sum(ss) / (float)cols + eps);
  float* yr = y + row * cols;
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int c = 4 * (lane + 64 * q);
    if (c < cols) {
      const f32x4 g = *reinterpret_cast<const f32x4*>(gamma + c);
      const f32x4 b = *reinterpret_cast<const f32x4*>(beta + c);
      f32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = fmaf((v[q][e] - mean) * rstd, g[e], b[e]);
      *reinterpret_cast<f32x4*>(yr + c) = o;
    }
  }
  if (lane == 0) { stats[2 * row] = mean; stats[2 * row + 1] = rstd; }
}

template <int CPL>
__global__ __launch_bounds__(256) void k_ln_bwd(const float* __restrict__ dy, const float* __restrict__ x,
                                                const float* __restrict__ stats, const float* __restrict__ gamma,
                                                float* __restrict__ dx, float* __restrict__ part, int64_t rows,
                                                int cols) {
  __shared__ float red[4][2][256 * CPL > 1024 ? 1024 : 256 * CPL];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  f32x4 g[CPL], pg[CPL], pb[CPL];
#pragma unroll
  for (int q = 0; q < CPL; ++q) {
    const int c = 4 * (lane + 64 * q);
    g[q] = c < cols ? *reinterpret_cast<const f32x4*>(gamma + c) : f32x4{0.f, 0.f, 0.f, 0.f};
    pg[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    pb[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const int64_t r0 = (int64_t)blockIdx.x * LN_ROWS_PER_WG + w;
  for (int i = 0; i < LN_ROWS_PER_WG / 4; ++i) {
    const int64_t row = r0 + 4 * i;
    if (row >= rows) break;
    const float mean = stats[2 * row], rstd = stats[2 * row + 1];
    f32x4 xh[CPL], gy[CPL];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int c = 4 * (lane + 64 * q);
      const f32x4 xv = c < cols ? *reinterpret_cast<const f32x4*>(x + row * cols + c) : f32x4{0.f, 0.f, 0.f, 0.f};
      const f32x4 dv = c < cols ? *reinterpret_cast<const f32x4*>(dy + row * cols + c) : f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xh[q][e] = c < cols ? (xv[e] - mean) * rstd : 0.f;
        gy[q][e] = dv[e] * g[q][e];
        s1 += gy[q][e];
        s2 = fmaf(gy[q][e], xh[q][e], s2);
        pg[q][e] = fmaf(dv[e], xh[q][e], pg[q][e]);
        pb[q][e] += dv[e];
      }
    }
    const float m1 = wave_sum(s1) / (float)cols, m2 = wave_sum(s2) / (float)cols;
#pragma unroll
    for (int q = 0; q < CPL; ++q) {
      const int c = 4 * (lane + 64 * q);
      if (c < cols) {
        f32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rstd * (gy[q][e] - m1 - xh[q][e] * m2);
        *reinterpret_cast<f32x4*>(dx + row * cols + c) = o;
      }
    }
  }
#pragma unroll
  for (int q = 0; q < CPL; ++q)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int c = 4 * (lane + 64 * q) + e;
      red[w][0][c] = pg[q][e];
      red[w][1][c] = pb[q][e];
    }
  __syncthreads();
  // part layout: [slice][0: dgamma | 1: dbeta][cols]
  for (int c = threadIdx.x; c < cols; c += 256) {
    const float a = (red[0][0][c] + red[1][0][c]) + (red[2][0][c] + red[3][0][c]);
    const float b = (red[0][1][c] + red[1][1][c]) + (red[2][1][c] + red[3][1][c]);
    part[(int64_t)blockIdx.x * 2 * cols + c] = a;
    part[(int64_t)blockIdx.x * 2 * cols + cols + c] = b;
  }
}

inline int ln_cpl(int64_t cols) {
  if (cols < 4 || cols % 4) return 0;
  const int64_t cpl = (cols + 255) / 256;
  return cpl <= 4 ? (int)cpl : 0;
}

}  // namespace

extern "C" {

size_t csa_bias_grad_workspace_bytes(int64_t rows, int64_t cols) {
  return sizeof(float) * (size_t)bg_slices(rows) * (size_t)(cols > 0 ? cols : 0);
}

csa_status csa_bias_grad(const float* dy, float* db, int64_t rows, int64_t cols, int accumulate, void* workspace,
                         void* stream) {
  if (rows < 0 || cols < 0) {
    csa::set_error("csa_bias_grad: negative size");
    return CSA_INVALID_ARG;
  }
  if (cols == 0) return CSA_OK;
  if (!db || (rows > 0 && (!dy || !workspace))) {
    csa::set_error("csa_bias_grad: null pointer");
    return CSA_INVALID_ARG;
  }
  const hipStream_t st = (hipStream_t)stream;
  const csa::DeviceGuard guard(st);
  if (rows == 0) {
    if (!accumulate && hipMemsetAsync(db, 0, sizeof(float) * cols, st) != hipSuccess) {
      csa::set_error("csa_bias_grad: memset failed");
      return CSA_LAUNCH_FAILED;
    }
    return CSA_OK;
  }
  const int rs = bg_slices(rows);
  const int64_t per = (rows + rs - 1) / rs;
  float* part = (float*)workspace;
  hipLaunchKernelGGL(k_bias_grad_part, dim3((unsigned)((cols + BG_COLS - 1) / BG_COLS), (unsigned)rs), dim3(256), 0,
                     st, dy, part, rows, cols, per);
  hipLaunchKernelGGL(k_bias_grad_sum, dim3((unsigned)((cols + BS_COLS - 1) / BS_COLS)), dim3(256), 0, st, part, db, cols, rs,
                     accumulate, cols, nullptr, cols);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    csa::set_error("csa_bias_grad: %s", hipGetErrorString(e));
    return CSA_LAUNCH_FAILED;
  }
  return CSA_OK;
}

int csa_layernorm_supported(int64_t cols) { return ln_cpl(cols) > 0 ? 1 : 0; }

size_t csa_layernorm_bwd_workspace_bytes(int64_t rows, int64_t cols) {
  return sizeof(float) * 2 * (size_t)((rows + LN_ROWS_PER_WG - 1) / LN_ROWS_PER_WG) * (size_t)(cols > 0 ? cols : 0);
}

csa_status csa_layernorm_fwd(const float* x, const float* gamma, const float* beta, float* y, float* stats,
                             int64_t rows, int64_t cols, float eps, void* stream) {
  const int cpl = ln_cpl(cols);
  if (rows < 0 || cpl == 0) {
    csa::set_error("csa_layernorm_fwd: cols must be a multiple of 4 in [4, 1024]");
    return CSA_UNSUPPORTED_SHAPE;
  }
  if (rows == 0) return CSA_OK;
  if (!x || !gamma || !beta || !y || !stats || ((((uintptr_t)x) | ((uintptr_t)y) | ((uintptr_t)gamma) |
                                                 ((uintptr_t)beta)) & 15)) {
    csa::set_error("csa_layernorm_fwd: null or misaligned pointer");
    return CSA_INVALID_ARG;
  }
  const hipStream_t st = (hipStream_t)stream;
  const csa::DeviceGuard guard(st);
  const dim3 grid((unsigned)((rows + 3) / 4));
  switch (cpl) {
    case 1: hipLaunchKernelGGL(k_ln_fwd<1>, grid, dim3(256), 0, st, x, gamma, beta, y, stats, rows, (int)cols, eps); break;
    case 2: hipLaunchKernelGGL(k_ln_fwd<2>, grid, dim3(256), 0, st, x, gamma, beta, y, stats, rows, (int)cols, eps); break;
    case 3: hipLaunchKernelGGL(k_ln_fwd<3>, grid, dim3(256), 0, st, x, gamma, beta, y, stats, rows, (int)cols, eps); break;
    default: hipLaunchKernelGGL(k_ln_fwd<4>, grid, dim3(256), 0, st, x, gamma, beta, y, stats, rows, (int)cols, eps);
  }
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    csa::set_error("csa_layernorm_fwd: %s", hipGetErrorString(e));
    return CSA_LAUNCH_FAILED;
  }
  return CSA_OK;
}

csa_status csa_layernorm_bwd(const float* dy, const float* x, const float* stats, const float* gamma, float* dx,
                             float* dgamma, float* dbeta, int64_t rows, int64_t cols, void* workspace, void* stream) {
  const int cpl = ln_cpl(cols);
  if (rows < 0 || cpl == 0) {
    csa::set_error("csa_layernorm_bwd: cols must be a multiple of 4 in [4, 1024]");
    return CSA_UNSUPPORTED_SHAPE;
  }
  if (!dgamma || !dbeta || (rows > 0 && (!dy || !x || !stats || !gamma || !dx || !workspace)) ||
      ((((uintptr_t)dy) | ((uintptr_t)x) | ((uintptr_t)dx) | ((uintptr_t)gamma)) & 15)) {
    csa::set_error("csa_layernorm_bwd: null or misaligned pointer");
    return CSA_INVALID_ARG;
  }
  const hipStream_t st = (hipStream_t)stream;
  const csa::DeviceGuard guard(st);
  if (rows == 0) {
    if (hipMemsetAsync(dgamma, 0, sizeof(float) * cols, st) != hipSuccess ||
        hipMemsetAsync(dbeta, 0, sizeof(float) * cols, st) != hipSuccess) {
      csa::set_error("csa_layernorm_bwd: memset failed");
      return CSA_LAUNCH_FAILED;
    }
    return CSA_OK;
  }
  const int nwg = (int)((rows + LN_ROWS_PER_WG - 1) / LN_ROWS_PER_WG);
  float* part = (float*)workspace;
  const dim3 grid((unsigned)nwg);
  switch (cpl) {
    case 1: hipLaunchKernelGGL(k_ln_bwd<1>, grid, dim3(256), 0, st, dy, x, stats, gamma, dx, part, rows, (int)cols); break;
    case 2: hipLaunchKernelGGL(k_ln_bwd<2>, grid, dim3(256), 0, st, dy, x, stats, gamma, dx, part, rows, (int)cols); break;
    case 3: hipLaunchKernelGGL(k_ln_bwd<3>, grid, dim3(256), 0, st, dy, x, stats, gamma, dx, part, rows, (int)cols); break;
    default: hipLaunchKernelGGL(k_ln_bwd<4>, grid, dim3(256), 0, st, dy, x, stats, gamma, dx, part, rows, (int)cols);
  }
  // dgamma = rows 0, 2, 4, ... of part; dbeta = rows 1, 3, 5, ... (stride 2 cols between slices)
  const dim3 g2((unsigned)((2 * cols + BS_COLS - 1) / BS_COLS));  // dgamma and dbeta in one launch
  hipLaunchKernelGGL(k_bias_grad_sum, g2, dim3(256), 0, st, part, dgamma, 2 * cols, nwg, 0, (int64_t)2 * cols, dbeta,
                     cols);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    csa::set_error("csa_layernorm_bwd: %s", hipGetErrorString(e));
    return CSA_LAUNCH_FAILED;
  }
  return CSA_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// Residual + dropout of the pre-LN blocks (module/components.py SublayerConnection
// `x + dropout(sublayer(norm(x)))`, module/sbm_model.py:29-31 `dropout1(out) + X`):
//   y = x + keep(i) * o * scale,  do = keep(i) * dy * scale   (dx = dy needs no kernel).
// keep(i) for memory element i is 16-bit uniform (i & 7) of Philox4x32-7
// {lo32(i >> 3), hi32(i >> 3), 0, (RNG_RES_DROP << 28) ^ offset} keyed by the 64-bit seed, keep <=>
// u16 >= ceil(p * 65536) (oracle/philox.py:res_keep). The backward regenerates the bits, so no
// mask is stored. One thread per 8 consecutive elements (two dwordx4 loads per operand).
constexpr uint32_t RNG_RES_DROP = 5u;

struct ResArgs {
  uint32_t seed_lo, seed_hi, off, thr;
  float scale;
  int64_t n;
};

template <uint32_t STREAM = RNG_RES_DROP>
__device__ __forceinline__ uint32_t res_keep8(const ResArgs& a, int64_t g) {
  const u32x4 r = philox4x32(u32x4{(uint32_t)g, (uint32_t)((uint64_t)g >> 32), 0u, (STREAM << 28) ^ a.off},
                             a.seed_lo, a.seed_hi);
  const uint32_t w[4] = {r.x, r.y, r.z, r.w};
  uint32_t k = 0;
#pragma unroll
  for (int e = 0; e < 8; ++e) k |= ((((e & 1) ? (w[e >> 1] >> 16) : (w[e >> 1] & 0xffffu)) >= a.thr) ? 1u : 0u) << e;
  return k;
}

// BWD: x == nullptr, o = dy, y = do.
template <bool BWD>
__global__ __launch_bounds__(256) void k_res_drop(const float* __restrict__ x, const float* __restrict__ o,
                                                  float* __restrict__ y, ResArgs a) {
#pragma clang fp contract(off)  // dropout then add, two roundings as torch (no fma of o * scale + x)
  const int64_t groups = (a.n + 7) >> 3;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < groups; g += (int64_t)gridDim.x * 256) {
    const uint32_t keep = res_keep8(a, g);
    const int64_t i0 = g << 3;
    if (i0 + 8 <= a.n) {
      const f32x4 o0 = *reinterpret_cast<const f32x4*>(o + i0), o1 = *reinterpret_cast<const f32x4*>(o + i0 + 4);
      f32x4 r0, r1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        r0[e] = ((keep >> e) & 1u) ? o0[e] * a.scale : 0.f * o0[e];
        r1[e] = ((keep >> (e + 4)) & 1u) ? o1[e] * a.scale : 0.f * o1[e];
      }
      if (!BWD) {
        const f32x4 x0 = *reinterpret_cast<const f32x4*>(x + i0), x1 = *reinterpret_cast<const f32x4*>(x + i0 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { r0[e] = x0[e] + r0[e]; r1[e] = x1[e] + r1[e]; }
      }
      *reinterpret_cast<f32x4*>(y + i0) = r0;
      *reinterpret_cast<f32x4*>(y + i0 + 4) = r1;
    } else {
      for (int e = 0; i0 + e < a.n; ++e) {
        const float v = ((keep >> e) & 1u) ? o[i0 + e] * a.scale : 0.f * o[i0 + e];
        y[i0 + e] = BWD ? v : x[i0 + e] + v;
      }
    }
  }
}

static csa_status res_launch(bool bwd, const float* x, const float* o, float* y, int64_t n, float p, uint64_t seed,
                             uint64_t offset, void* stream, const char* name) {
  if (n < 0 || !(p > 0.f && p < 1.f)) {
    csa::set_error("%s: need n >= 0 and 0 < p < 1", name);
    return CSA_INVALID_ARG;
  }
  if (n == 0) return CSA_OK;
  if (!o || !y || (!bwd && !x)) {
    csa::set_error("%s: null pointer", name);
    return CSA_INVALID_ARG;
  }
  if ((((uintptr_t)o | (uintptr_t)y | (uintptr_t)x) & 15u) != 0) {
    csa::set_error("%s: pointers must be 16-byte aligned", name);
    return CSA_INVALID_ARG;
  }
  ResArgs a;
  a.seed_lo = (uint32_t)seed; a.seed_hi = (uint32_t)(seed >> 32); a.off = (uint32_t)offset;
  a.thr = (uint32_t)ceil((double)p * 65536.0);
  a.scale = 1.f / (1.f - p);
  a.n = n;
  const int64_t groups = (n + 7) >> 3;
  const unsigned blocks = (unsigned)std::min<int64_t>((groups + 255) / 256, 256 * 16);
  const hipStream_t st = (hipStream_t)stream;
  const csa::DeviceGuard guard(st);
  if (bwd) hipLaunchKernelGGL(k_res_drop<true>, dim3(blocks), dim3(256), 0, st, nullptr, o, y, a);
  else hipLaunchKernelGGL(k_res_drop<false>, dim3(blocks), dim3(256), 0, st, x, o, y, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    csa::set_error("%s: %s", name, hipGetErrorString(e));
    return CSA_LAUNCH_FAILED;
  }
  return CSA_OK;
}

extern "C" {

csa_status csa_residual_dropout_fwd(const float* x, const float* o, float* y, int64_t n, float p, uint64_t seed,
                                    uint64_t offset, void* stream) {
  return res_launch(false, x, o, y, n, p, seed, offset, stream, "csa_residual_dropout_fwd");
}

csa_status csa_residual_dropout_bwd(const float* dy, float* d_o, int64_t n, float p, uint64_t seed, uint64_t offset,
                                    void* stream) {
  return res_launch(true, nullptr, dy, d_o, n, p, seed, offset, stream, "csa_residual_dropout_bwd");
}

}  // extern "C"

// ---------------------------------------------------------------------------------------
// GELU + dropout of the feed-forward blocks (module/components.py FeedForward
// `linear2(dropout(gelu(linear1(x))))`, module/sbm_model.py:22-26 mlpblock GELU -> Dropout):
//   y = keep(i) * gelu(h) * scale,  dh = keep(i) * scale * dy * gelu'(h)   (exact erf GELU, torch's
// formulas: gelu = h * 0.5 * (1 + erf(h / sqrt 2)), gelu' = cdf + h * exp(-h^2 / 2) / sqrt(2 pi)).
// keep(i): Philox stream 6 over memory order, same layout as the residual stream
// (oracle/philox.py:ffn_keep); p = 0 keeps everything (plain GELU).
constexpr uint32_t RNG_FFN_DROP = 6u;

__device__ __forceinline__ float gelu_f(float h) { return h * 0.5f * (1.f + erff(h * 0.70710678118654752440f)); }
__device__ __forceinline__ float gelu_d(float h) {
  const float cdf = 0.5f * (1.f + erff(h * 0.70710678118654752440f));
  const float pdf = expf(-0.5f * h * h) * 0.39894228040143267794f;
  return cdf + h * pdf;
}

template <bool BWD>
__global__ __launch_bounds__(256) void k_gelu_drop(const float* __restrict__ h, const float* __restrict__ dy,
                                                   float* __restrict__ out, ResArgs a) {
#pragma clang fp contract(off)
  const int64_t groups = (a.n + 7) >> 3;
  for (int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x; g < groups; g += (int64_t)gridDim.x * 256) {
    const uint32_t keep = a.thr ? res_keep8<RNG_FFN_DROP>(a, g) : 0xffu;
    const int64_t i0 = g << 3;
    float hv[8], gv[8], r[8];
    const bool full = i0 + 8 <= a.n;
    if (full) {
      const f32x4 h0 = *reinterpret_cast<const f32x4*>(h + i0), h1 = *reinterpret_cast<const f32x4*>(h + i0 + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { hv[e] = h0[e]; hv[e + 4] = h1[e]; }
      if (BWD) {
        const f32x4 g0 = *reinterpret_cast<const f32x4*>(dy + i0), g1 = *reinterpret_cast<const f32x4*>(dy + i0 + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) { gv[e] = g0[e]; gv[e + 4] = g1[e]; }
      }
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        hv[e] = i0 + e < a.n ? h[i0 + e] : 0.f;
        gv[e] = (BWD && i0 + e < a.n) ? dy[i0 + e] : 0.f;
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      if (BWD) {
        const float gd = a.thr ? (((keep >> e) & 1u) ? gv[e] * a.scale : 0.f * gv[e]) : gv[e];  // dropout bwd
        r[e] = gd * gelu_d(hv[e]);
      } else {
        const float z = gelu_f(hv[e]);
        r[e] = a.thr ? (((keep >> e) & 1u) ? z * a.scale : 0.f * z) : z;
      }
    }
    if (full) {
      *reinterpret_cast<f32x4*>(out + i0) = f32x4{r[0], r[1], r[2], r[3]};
      *reinterpret_cast<f32x4*>(out + i0 + 4) = f32x4{r[4], r[5], r[6], r[7]};
    } else {
      for (int e = 0; i0 + e < a.n; ++e) out[i0 + e] = r[e];
    }
  }
}

static csa_status ffn_launch(bool bwd, const float* h, const float* dy, float* out, int64_t n, float p, uint64_t seed,
                             uint64_t offset, void* stream, const char* name) {
  if (n < 0 || !(p >= 0.f && p < 1.f)) {
    csa::set_error("%s: need n >= 0 and 0 <= p < 1", name);
    return CSA_INVALID_ARG;
  }
  if (n == 0) return CSA_OK;
  if (!h || !out || (bwd && !dy)) {
    csa::set_error("%s: null pointer", name);
    return CSA_INVALID_ARG;
  }
  if ((((uintptr_t)h | (uintptr_t)out | (uintptr_t)dy) & 15u) != 0) {
    csa::set_error("%s: pointers must be 16-byte aligned", name);
    return CSA_INVALID_ARG;
  }
  ResArgs a;
  a.seed_lo = (uint32_t)seed; a.seed_hi = (uint32_t)(seed >> 32); a.off = (uint32_t)offset;
  a.thr = p > 0.f ? (uint32_t)ceil((double)p * 65536.0) : 0u;
  a.scale = p > 0.f ? 1.f / (1.f - p) : 1.f;
  a.n = n;
  const int64_t groups = (n + 7) >> 3;
  const unsigned blocks = (unsigned)std::min<int64_t>((groups + 255) / 256, 256 * 16);
  const hipStream_t st = (hipStream_t)stream;
  const csa::DeviceGuard guard(st);
  if (bwd) hipLaunchKernelGGL(k_gelu_drop<true>, dim3(blocks), dim3(256), 0, st, h, dy, out, a);
  else hipLaunchKernelGGL(k_gelu_drop<false>, dim3(blocks), dim3(256), 0, st, h, nullptr, out, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    csa::set_error("%s: %s", name, hipGetErrorString(e));
    return CSA_LAUNCH_FAILED;
  }
  return CSA_OK;
}

extern "C" {

csa_status csa_gelu_dropout_fwd(const float* h, float* y, int64_t n, float p, uint64_t seed, uint64_t offset,
                                void* stream) {
  return ffn_launch(false, h, nullptr, y, n, p, seed, offset, stream, "csa_gelu_dropout_fwd");
}

csa_status csa_gelu_dropout_bwd(const float* dy, const float* h, float* dh, int64_t n, float p, uint64_t seed,
                                uint64_t offset, void* stream) {
  return ffn_launch(true, h, dy, dh, n, p, seed, offset, stream, "csa_gelu_dropout_bwd");
}

}  // extern "C"
