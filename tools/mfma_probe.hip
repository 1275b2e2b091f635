// Dev probe (not part of the library): C/D lane layout and issue cost of the fp32 multi-block MFMA forms on
// gfx950 (v_mfma_f32_16x16x1_4b_f32, v_mfma_f32_32x32x1_2b_f32, v_mfma_f32_4x4x1_16b_f32) next to the
// single-block v_mfma_f32_32x32x2_f32 / v_mfma_f32_16x16x4_f32 the kernels use.
// build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_probe tools/mfma_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x32 __attribute__((ext_vector_type(32)));

// mode 0: A = lane + 1, B = 1 (D names the A lane); mode 1: A = 1, B = lane + 1 (D names the B lane)
__global__ void k_layout(float* out, int mode, int which) {
  const int l = threadIdx.x;
  const float a = mode == 0 ? (float)(l + 1) : 1.f, b = mode == 0 ? 1.f : (float)(l + 1);
  if (which == 0) {
    f32x16 d = {};
    d = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, d, 0, 0, 0);
    for (int r = 0; r < 16; ++r) out[r * 64 + l] = d[r];
  } else {
    f32x4 d = {};
    d = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, d, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[r * 64 + l] = d[r];
  }
}

__global__ void k_layout32(float* out, int mode) {
  const int l = threadIdx.x;
  const float a = mode == 0 ? (float)(l + 1) : 1.f, b = mode == 0 ? 1.f : (float)(l + 1);
  f32x32 d = {};
  d = __builtin_amdgcn_mfma_f32_32x32x1f32(a, b, d, 0, 0, 0);
  for (int r = 0; r < 32; ++r) out[r * 64 + l] = d[r];
}

// cycles per instruction, 4 independent accumulators, one wave per SIMD (4 waves per block)
template <int W>
__global__ void k_rate(float* out, long long* cyc, int n) {
  const int l = threadIdx.x & 63;
  float a = 1.f + l * 1e-3f, b = 2.f - l * 1e-3f;
  long long t0 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  if constexpr (W == 0) {
    f32x16 d0 = {}, d1 = {}, d2 = {}, d3 = {};
    for (int i = 0; i < n; ++i) {
      d0 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, d3, 0, 0, 0);
    }
    s = d0[0] + d1[1] + d2[2] + d3[3];
  } else if constexpr (W == 1) {
    f32x16 d0 = {}, d1 = {}, d2 = {}, d3 = {};
    for (int i = 0; i < n; ++i) {
      d0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, d3, 0, 0, 0);
    }
    s = d0[0] + d1[1] + d2[2] + d3[3];
  } else if constexpr (W == 2) {
    f32x4 d0 = {}, d1 = {}, d2 = {}, d3 = {};
    for (int i = 0; i < n; ++i) {
      d0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, d3, 0, 0, 0);
    }
    s = d0[0] + d1[1] + d2[2] + d3[3];
  } else if constexpr (W == 3) {
    f32x4 d0 = {}, d1 = {}, d2 = {}, d3 = {};
    for (int i = 0; i < n; ++i) {
      d0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, d1, 0, 0, 0);
      d2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, d2, 0, 0, 0);
      d3 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, d3, 0, 0, 0);
    }
    s = d0[0] + d1[1] + d2[2] + d3[3];
  } else if constexpr (W == 5) {
    f32x16 d0 = {};  // one dependent chain of 32x32x2 (W == 6: the same at two waves per SIMD)
    for (int i = 0; i < 4 * n; ++i) d0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, d0, 0, 0, 0);
    s = d0[0];
  } else if constexpr (W == 7) {
    f32x16 d0 = {}, d1 = {};  // two interleaved chains of 32x32x2
    for (int i = 0; i < 2 * n; ++i) {
      d0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, d1, 0, 0, 0);
    }
    s = d0[0] + d1[1];
  } else {
    f32x16 d0 = {};  // one dependent chain of 16x16x1_4b
    for (int i = 0; i < 4 * n; ++i) d0 = __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, d0, 0, 0, 0);
    s = d0[0];
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float *d, h[64 * 64];
  long long* c;
  hipMalloc(&d, 64 * 64 * 4 * 256);
  hipMalloc(&c, 8 * 1024);
  const char* names[] = {"16x16x1_4b", "32x32x1_2b(unused)", "4x4x1_16b"};
  for (int which = 0; which < 3; which += 2) {
    const int nreg = which == 0 ? 16 : 4;
    float A[16][64], Bv[16][64];
    for (int mode = 0; mode < 2; ++mode) {
      k_layout<<<1, 64>>>(d, mode, which);
      hipMemcpy(h, d, nreg * 64 * 4, hipMemcpyDeviceToHost);
      for (int r = 0; r < nreg; ++r)
        for (int l = 0; l < 64; ++l) (mode == 0 ? A : Bv)[r][l] = h[r * 64 + l];
    }
    printf("%s: (reg, lane) -> (A lane, B lane)\n", names[which]);
    for (int r = 0; r < nreg; ++r) {
      printf(" r%2d:", r);
      for (int l = 0; l < 64; ++l) printf(" %d/%d", (int)A[r][l] - 1, (int)Bv[r][l] - 1);
      printf("\n");
    }
  }
  {
    float A[32][64], Bv[32][64];
    for (int mode = 0; mode < 2; ++mode) {
      k_layout32<<<1, 64>>>(d, mode);
      hipMemcpy(h, d, 32 * 64 * 4, hipMemcpyDeviceToHost);
      for (int r = 0; r < 32; ++r)
        for (int l = 0; l < 64; ++l) (mode == 0 ? A : Bv)[r][l] = h[r * 64 + l];
    }
    printf("32x32x1_2b: (reg, lane) -> (A lane, B lane)\n");
    for (int r = 0; r < 32; ++r) {
      printf(" r%2d:", r);
      for (int l = 0; l < 64; ++l) printf(" %d/%d", (int)A[r][l] - 1, (int)Bv[r][l] - 1);
      printf("\n");
    }
  }
  const char* rn[] = {"16x16x1_4b x4 indep", "32x32x2 x4 indep", "16x16x4 x4 indep", "4x4x1_16b x4 indep",
                      "16x16x1_4b dependent chain", "32x32x2 dependent chain", "32x32x2 dep, 2 waves/SIMD",
                      "32x32x2 two chains"};
  for (int w = 0; w < 8; ++w) {
    const int n = 4096;
    for (int rep = 0; rep < 2; ++rep) {
      if (w == 0) k_rate<0><<<256, 256>>>(d, c, n);
      if (w == 1) k_rate<1><<<256, 256>>>(d, c, n);
      if (w == 2) k_rate<2><<<256, 256>>>(d, c, n);
      if (w == 3) k_rate<3><<<256, 256>>>(d, c, n);
      if (w == 4) k_rate<4><<<256, 256>>>(d, c, n);
      if (w == 5) k_rate<5><<<256, 256>>>(d, c, n);
      if (w == 6) k_rate<5><<<256, 512>>>(d, c, n);
      if (w == 7) k_rate<7><<<256, 256>>>(d, c, n);
    }
    long long hc[256];
    hipMemcpy(hc, c, sizeof(hc), hipMemcpyDeviceToHost);
    double s = 0;
    for (int i = 0; i < 256; ++i) s += hc[i];
    printf("%-28s %.2f cycles per MFMA (s_memtime)\n", rn[w], s / 256 / (4.0 * n));
  }
  return 0;
}
