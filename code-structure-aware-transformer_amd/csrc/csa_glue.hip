// Linear-layer bias gradient (db = sum over rows of dY) for the encoder glue of the train step
// (module/sbm_model.py:27-31, module/csa_trans.py FeedForward / CSE_layer, components.py Generator).
//
// torch's Linear backward reduces dY (rows x cols, rows = B*N = 9600 at the java step) with its
// generic strided reduce_kernel: ~18 us per call for a 29 MB read (1.6 TB/s), 95 calls per step.
// Here: pass 1, grid (cols / 64, RS row slices), each 256-thread workgroup sums a 64-column x
// (rows / RS) slab with dwordx4 loads (16 threads per row x 16 rows in flight), reduces its 16 row
// lanes through LDS in a fixed order and writes one partial row; pass 2 sums the RS partials in
// slice order. The summation order depends only on (rows, cols): deterministic.
#include "csa_common.hpp"
#include "../../include/csa_hip.h"

using csa::f32x4;

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

__global__ __launch_bounds__(256) void k_bias_grad_sum(const float* __restrict__ part, float* __restrict__ db,
                                                       int64_t cols, int rs, int accumulate) {
  const int64_t c = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (c >= cols) return;
  // loads issued 8 at a time (independent), then added in slice order: the sum is the same fixed
  // left-to-right chain, without one L2 round trip per partial
  float s = 0.f;
  for (int i0 = 0; i0 < rs; i0 += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = i0 + u < rs ? part[(int64_t)(i0 + u) * cols + c] : 0.f;
#pragma unroll
    for (int u = 0; u < 8; ++u) s += v[u];
  }
  db[c] = accumulate ? db[c] + s : s;
}

inline int bg_slices(int64_t rows) {
  const int64_t rs = (rows + 255) / 256;  // >= 256 rows per slice
  return (int)(rs < 1 ? 1 : rs > 64 ? 64 : rs);
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
  hipLaunchKernelGGL(k_bias_grad_sum, dim3((unsigned)((cols + 255) / 256)), dim3(256), 0, st, part, db, cols, rs,
                     accumulate);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    csa::set_error("csa_bias_grad: %s", hipGetErrorString(e));
    return CSA_LAUNCH_FAILED;
  }
  return CSA_OK;
}

}  // extern "C"
