// Dev probe (not part of the library): how much vector-ALU issue overlaps an exact-fp32 MFMA stream on gfx950.
//
// One 512-thread workgroup per CU; waves w and w + 4 share a SIMD. Each wave runs one of three programs and stamps
// its own cycle count (s_memtime) into out[]:
//   M  : NM x v_mfma_f32_32x32x2_f32 on 4 independent accumulators (the matrix pipe paced, no VALU)
//   V  : NV x v_fma_f32 in 8 independent chains (VALU only)
//   MV : both streams in one wave, F VALU per MFMA interleaved by sched_group_barrier
// Configurations (argv): mode 0 = waves 0-3 MV alone (4-7 exit), 1 = waves 0-3 M beside 4-7 V, 2 = 0-3 M alone,
// 3 = 0-3 V alone, 4 = 0-7 all MV (two interleaving waves per SIMD).
// build: hipcc --offload-arch=gfx950 -O3 tools/mfma_valu_probe.hip -o tools/mfma_valu_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int F>
__global__ __launch_bounds__(512) void probe(int mode, int iters, float* out, unsigned long long* cyc) {
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const bool lo = w < 4;
  int prog;  // 0 = M, 1 = V, 2 = MV, -1 = exit
  if (mode == 0) prog = lo ? 2 : -1;
  else if (mode == 1) prog = lo ? 0 : 1;
  else if (mode == 2) prog = lo ? 0 : -1;
  else if (mode == 3) prog = lo ? 1 : -1;
  else prog = 2;
  if (prog < 0) return;
  float a = 1.0f + lane * 1e-3f, b = 0.5f;
  f32x16 acc[4];
  for (int i = 0; i < 4; ++i)
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  float v[8];
  for (int i = 0; i < 8; ++i) v[i] = lane * 0.01f + i;
  __syncthreads();
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    if (prog == 0) {
#pragma unroll
      for (int m = 0; m < 16; ++m) acc[m & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m & 3], 0, 0, 0);
    } else if (prog == 1) {
#pragma unroll
      for (int m = 0; m < 16 * F; ++m) v[m & 7] = fmaf(v[m & 7], 0.999f, 0.001f);
    } else {
#pragma unroll
      for (int m = 0; m < 16; ++m) {
        acc[m & 3] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[m & 3], 0, 0, 0);
#pragma unroll
        for (int f = 0; f < F; ++f) v[(m * F + f) & 7] = fmaf(v[(m * F + f) & 7], 0.999f, 0.001f);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // one MFMA
        if (F > 0) __builtin_amdgcn_sched_group_barrier(0x002, F, 0);  // then F VALU
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int i = 0; i < 4; ++i)
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  for (int i = 0; i < 8; ++i) s += v[i];
  out[blockIdx.x * 512 + threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * 8 + w] = t1 - t0;
  if (lane == 0 && blockIdx.x == 0 && w == 0 && mode == 2)
    printf("  calib: memtime ticks %llu, realtime ticks %llu (100 MHz) -> %.3f GHz memtime rate\n", t1 - t0, r1 - r0,
           (double)(t1 - t0) / (double)(r1 - r0) * 0.1);
}

template <int F>
void run(int mode, int iters, float* out, unsigned long long* cyc, unsigned long long* h) {
  hipLaunchKernelGGL(probe<F>, dim3(256), dim3(512), 0, 0, mode, iters, out, cyc);
  (void)hipMemset(cyc, 0, 256 * 8 * 8);
  hipLaunchKernelGGL(probe<F>, dim3(256), dim3(512), 0, 0, mode, iters, out, cyc);
  (void)hipMemcpy(h, cyc, 256 * 8 * 8, hipMemcpyDeviceToHost);
  double lo = 0, hi = 0;
  int nlo = 0, nhi = 0;
  for (int bl = 0; bl < 256; ++bl)
    for (int w = 0; w < 8; ++w) {
      const unsigned long long c = h[bl * 8 + w];
      if (!c) continue;
      if (w < 4) { lo += c; ++nlo; } else { hi += c; ++nhi; }
    }
  const double nm = 16.0 * iters;
  printf("F=%d mode=%d  waves0-3: %.1f cyc/MFMA-slot  waves4-7: %.1f cyc/MFMA-slot\n", F, mode,
         nlo ? lo / nlo / nm : 0.0, nhi ? hi / nhi / nm : 0.0);
}

int main() {
  float* out;
  unsigned long long *cyc, h[256 * 8];
  (void)hipMalloc(&out, 256 * 512 * 4);
  (void)hipMalloc(&cyc, 256 * 8 * 8);
  const int iters = 2000;
  for (int mode = 0; mode < 5; mode += (mode == 0 ? 2 : 2)) {
    run<0>(mode, iters, out, cyc, h);
    run<4>(mode, iters, out, cyc, h);
    run<8>(mode, iters, out, cyc, h);
    run<12>(mode, iters, out, cyc, h);
    run<16>(mode, iters, out, cyc, h);
    run<24>(mode, iters, out, cyc, h);
  }
  return 0;
}
