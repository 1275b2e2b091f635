// Device-side building blocks shared by the CSA-Trans attention kernels (gfx950 / CDNA4 only).
//
// Everything here is built around ONE matrix instruction, the exact-fp32 MFMA
// v_mfma_f32_32x32x2_f32 (64 cycles/SIMD, result == k-ordered fmaf chain): the reference
// computes the whole hot path in fp32 (module/sbm_attn.py:120-126 disables autocast and
// casts to .float()), and parity is judged at rtol 1e-4 / atol 1e-5, so the contractions
// run on fp32 MFMA.
//
// Lane conventions for one wave64 (c = lane & 31, h = lane >> 5):
//   D[i][j] += sum_{k in step} A[i][k] B[k][j]
//   A operand: lane holds A[i = c][k = kperm(s, h)]       (one float per K-step s)
//   B operand: lane holds B[k = kperm(s, h)][j = c]
//   C/D      : lane holds D[crow(r, h)][c] in register r (r = 0..15)
// Any bijection kperm(s, h) is valid as long as both operands use the same one; we use
//   "lin"  : k = s + (K/2) h          (operand loaded from a row-major row: each lane reads a
//                                       contiguous run of K/2 floats -> dwordx4 loads)
//   "acc"  : k = 32 t + crow(r, h)    (operand that IS a previous accumulator tile: the
//                                       16 registers of tile t feed K-steps 16t .. 16t+15)
// so an accumulator tile can feed the next product with no data movement whenever that
// product sums over the tile's ROW index.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>
#include <math.h>
#include <stdlib.h>

namespace csa {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
__host__ __device__ __forceinline__ constexpr int crow(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 acc) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
}

// v_mfma_f32_16x16x4_f32 (exact fp32, 32 cycles/SIMD, the same rate per FLOP): lane l = (x16 = l & 15,
// g = l >> 4) holds A[x16][k = g] / B[k = g][x16]; C/D register i holds D[4 g + i][x16].
__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
}

// v_mfma_f32_16x16x1_4b_f32 (exact fp32, four independent 16x16 blocks, K = 1 each, 32 cycles/SIMD: the same
// rate per FLOP). Block b takes its operands from lanes 16b .. 16b+15 (A[i = l & 15], B[j = l & 15]); C/D
// register 4b + e of lane l holds block b's D[4 (l >> 4) + e][l & 15] (tools/mfma_probe.hip). Used where one
// product dimension is a 16-wide cluster index: a 32x32 tile would be half padding.
__device__ __forceinline__ f32x16 mfma4b(float a, float b, f32x16 acc) {
  return __builtin_amdgcn_mfma_f32_16x16x1f32(a, b, acc, 0, 0, 0);
}

// bf16 mode (CSA_DTYPE_BF16): the N^2 contractions run on v_mfma_f32_32x32x16_bf16 (16x the f32 MFMA
// rate, fp32 accumulation). One instruction takes 8 consecutive K-steps of the f32 chains above from
// each lane (lane half h, element j <-> K-step 8 s + j), so a chain keeps its K permutation and both
// operands stay consistent: f32 operands are rounded to bf16 (RNE, v_cvt_pk_bf16_f32) when packed.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x16 mfma_bf(bf16x8 a, bf16x8 b, f32x16 acc) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
}
__device__ __forceinline__ bf16x8 pack8(const float* v) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)v[j];
  return r;
}
__device__ __forceinline__ bf16x8 pack8(f32x4 a, f32x4 b) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) { r[j] = (__bf16)a[j]; r[4 + j] = (__bf16)b[j]; }
  return r;
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int r = 0; r < 16; ++r) z[r] = 0.f;
  return z;
}

// Sum of a value over the two 32-lane halves (lane l <-> l ^ 32).
__device__ __forceinline__ float xhalf_sum(float v) { return v + __shfl_xor(v, 32, 64); }
__device__ __forceinline__ float xhalf_max(float v) { return fmaxf(v, __shfl_xor(v, 32, 64)); }

// Reduce over the 32 lanes of each half (result replicated in every lane of the half).
__device__ __forceinline__ float half_sum32(float v) {
#pragma unroll
  for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Load `NV` consecutive floats from p (16-B aligned) into dst, zeroed when !valid.
// p must ALWAYS be a dereferenceable address (callers clamp the row index): the load is issued
// unconditionally and only the value is selected. A branch around a load makes hipcc wait
// vmcnt(0) inside it, serialising every load of a tile (guide §5, trap (c)).
template <int NV>
__device__ __forceinline__ void load_run(float* dst, const float* __restrict__ p, bool valid) {
#pragma unroll
  for (int i = 0; i < NV; i += 4) {
    f32x4 v = *reinterpret_cast<const f32x4*>(p + i);
    dst[i] = valid ? v[0] : 0.f; dst[i + 1] = valid ? v[1] : 0.f;
    dst[i + 2] = valid ? v[2] : 0.f; dst[i + 3] = valid ? v[3] : 0.f;
  }
}

// Unconditional scalar load of p[min(idx, hi)], zeroed when !valid (see load_run).
__device__ __forceinline__ float ldz(const float* __restrict__ p, int64_t idx, int64_t hi, bool valid) {
  const float v = p[idx < hi ? idx : hi];
  return valid ? v : 0.f;
}
__device__ __forceinline__ int imin(int a, int b) { return a < b ? a : b; }

// Scalar-load variant (no alignment requirement).
template <int NV>
__device__ __forceinline__ void load_run_s(float* dst, const float* __restrict__ p, int n_avail, bool valid) {
#pragma unroll
  for (int i = 0; i < NV; ++i) dst[i] = (valid && i < n_avail) ? p[i] : 0.f;
}

// ---------------------------------------------------------------------------------------
// Philox4x32 counter-based RNG (Salmon et al., SC'11): stateless, so forward sampling is
// reproducible from (seed, offset, element coordinates) on any launch geometry. 7 rounds: the
// Random123 paper reports Philox4x32-7 passing TestU01 BigCrush (10 is the conservative default).
// ---------------------------------------------------------------------------------------
struct u32x4 { uint32_t x, y, z, w; };

constexpr int PHILOX_ROUNDS = 7;

__device__ __forceinline__ u32x4 philox4x32(u32x4 ctr, uint32_t k0, uint32_t k1) {
  const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int i = 0; i < PHILOX_ROUNDS; ++i) {
    // one v_mad_u64_u32 per 32x32->64 product (measured 20% cheaper than mul_hi + mul_lo)
    const uint64_t p0 = (uint64_t)M0 * ctr.x, p1 = (uint64_t)M1 * ctr.z;
    ctr = u32x4{(uint32_t)(p1 >> 32) ^ ctr.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ ctr.w ^ k1, (uint32_t)p0};
    k0 += W0; k1 += W1;
  }
  return ctr;
}

// 24-bit uniform in [0,1) (same resolution as torch's fp32 uniform).
__device__ __forceinline__ float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// Stream ids (Philox counter word 3 high bits) so independent draws never share counters.
enum : uint32_t { RNG_STE = 1u, RNG_ATTN_DROP = 2u, RNG_PROJ_DROP = 3u };

// ---------------------------------------------------------------------------------------
// Wave-private LDS tile images filled by LDS-DMA (buffer_load_dword ... lds: 64 lanes x 4 B per
// instruction straight into LDS, no VGPR round trip, completion tracked by vmcnt).
// K/V tiles are stored with a padded row stride of D+4 floats. Both operand read patterns are
// then conflict-free and reduce to one lane base plus a compile-time offset, so no per-read
// address registers are needed:
//   row segments (MFMA A operand, ds_read_b128: 16 lanes = 16 rows) -> 4-bank row skew;
//   transposed reads (ds_read_b32: 32 lanes = 32 consecutive columns of one row).

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Byte offset of a dynamic-LDS pointer (taken once, outside hot loops: the generic->LDS cast
// carries a null check).
__device__ __forceinline__ uint32_t lds_offset(const float* p) {
  return (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const float*)p;
}
__device__ __forceinline__ lds_ptr_t lds_at(uint32_t off) { return (lds_ptr_t)(uintptr_t)off; }

// Raw buffer resource over [base, base + nbytes).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const float* base, int nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base), (short)0, nbytes, 0x00020000);
}

// Rows r0..r0+31 of a row-major fp32 matrix (row stride ld_bytes; rows >= M repeat row M-1,
// so the image only ever holds real, finite data) into an LDS image at byte offset img with
// row stride (D+4) floats. One 64-lane dword DMA per 64 columns of a row; the clamped row
// offset goes in soffset (SGPR), the lane's column in voffset (one VGPR for the whole tile).
template <int D>
__device__ __forceinline__ void dma_rows(uint32_t img, __amdgpu_buffer_rsrc_t src, int ld_bytes, int r0, int M) {
  // opaque per call: otherwise hipcc hoists all 32 (img + const) M0 values out of the caller's
  // loop and spills them to VGPR lanes
  asm volatile("" : "+s"(img));
  const int voff = lane_id() * 4;
  const int smax = (M - 1) * ld_bytes;
  int soff = imin(r0, M - 1) * ld_bytes;
#pragma unroll
  for (int r = 0; r < 32; ++r) {
    // running row offset, opaque per row: computed right before its DMA instead of all 32 up front
    asm volatile("" : "+s"(soff));
#pragma unroll
    for (int piece = 0; piece < (D + 63) / 64; ++piece) {
      const uint32_t dst = img + 4 * (r * (D + 4) + 64 * piece);
      if (D - 64 * piece >= 64) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(src, lds_at(dst), 4, voff + 256 * piece, soff, 0, 0);
      } else if (lane_id() < D - 64 * piece) {  // exec-masked tail piece (D = 96)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(src, lds_at(dst), 4, voff + 256 * piece, soff, 0, 0);
      }
    }
    soff = imin(soff + ld_bytes, smax);
  }
}

// Rows r0..r0+31 of a contiguous (M, W) row-major matrix into an unpadded image (32*W floats).
// src must span exactly M rows: rows >= M fall outside the buffer and are not real data.
template <int W>
__device__ __forceinline__ void dma_tile_contig(uint32_t img, __amdgpu_buffer_rsrc_t src, int r0, const int f0 = 0,
                                                const int f1 = 2) {
  asm volatile("" : "+s"(img));
  const int voff = lane_id() * 4 + r0 * W * 4;
#pragma unroll
  for (int i = f0 * W / 4; i < f1 * W / 4; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(src, lds_at(img + 256 * i), 4, voff + 256 * i, 0, 0, 0);
}

// Contiguous NBYTES (multiple of 1 KiB) from src at src_byte_off into LDS at lds_off: one 16-B-per-lane
// DMA instruction per KiB (buffer_load_dwordx4 ... lds). lds_off and src must be wave-uniform.
template <int NBYTES>
__device__ __forceinline__ void dma_block16(uint32_t lds_off, __amdgpu_buffer_rsrc_t src, int src_byte_off) {
  static_assert(NBYTES % 1024 == 0, "whole 1 KiB pieces");
  asm volatile("" : "+s"(lds_off));
  const int voff = lane_id() * 16;
#pragma unroll
  for (int i = 0; i < NBYTES / 1024; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(src, lds_at(lds_off + 1024 * i), 16, voff, src_byte_off + 1024 * i, 0, 0);
}

// ---------------------------------------------------------------------------------------
// Unpadded 32 x 64 fp32 tile images (8 KiB) filled by 8 x buffer_load_dwordx4 ... lds (1 KiB each).
// An x4 DMA writes 1 KiB contiguously, so bank conflicts are avoided by a per-row XOR swizzle of the
// 16-B chunks instead of row padding: LDS chunk p of row r holds logical chunk p ^ swz(r).
//   SW_ROW: swz = r & 15         row-segment reads (16 lanes = 16 rows, same logical chunk) are
//                                conflict-free; a lane's 8 chunks of one half sit at base ^ (16 j).
//   SW_COL: swz = 8 * bit2(r)    column reads (lanes = 32 consecutive columns of rows R and R + 4)
//                                are conflict-free and reduce to two lane bases + immediate offsets.
//   SW_BOTH: swz = (r & 7) | 8 * (bit2(r) ^ bit3(r))   both patterns conflict-free; a row read sits at
//                                row_base ^ (16 j), a column read at (col_base_t ^ K_r) + 256 crow(r, 0).
// Instruction q covers rows 4q..4q+3: lane i -> row 4q + i/16, LDS chunk i%16. The source offset
// carries the whole row offset in voffset, so rows >= M fall outside the buffer range given by the
// descriptor (never outside the allocation) and do not load real data; callers zero the image once.
// ---------------------------------------------------------------------------------------
enum { SW_ROW = 1, SW_COL = 2, SW_BOTH = 3 };
__host__ __device__ constexpr int swz(int sw, int row) {
  return sw == SW_ROW ? (row & 15) : sw == SW_COL ? 8 * ((row >> 2) & 1) : (row & 7) | ((((row >> 2) ^ (row >> 3)) & 1) << 3);
}

// Per-lane DMA source patterns (q mod 4 for SW_ROW, q mod 2 for SW_COL). The swizzle kind is a plain
// argument (callers pass a constant and the helpers are inlined): templated versions of these
// helpers lost their host-side kernel stubs under hipcc 7.2.
struct DmaPat { int v[4]; };
__device__ __forceinline__ DmaPat dma_pat(const int sw, int ld_bytes) {
  DmaPat P;
  const int i = lane_id(), s = i >> 4;
#pragma unroll
  for (int q = 0; q < 4; ++q) P.v[q] = s * ld_bytes + 16 * ((i & 15) ^ swz(sw, 4 * q + s));
  return P;
}
// Rows row0..row0+31 of a row-major (ld_bytes) fp32 matrix with 64 columns -> swizzled image at img.
// (Instructions q0 <= q < q1 only: rows 4 q0 .. 4 q1 - 1.)
__device__ __forceinline__ void dma64(uint32_t img, __amdgpu_buffer_rsrc_t src, const DmaPat& P, int ld_bytes, int row0,
                                      const int q0 = 0, const int q1 = 8) {
  asm volatile("" : "+s"(img));
  int rowoff = (row0 + 4 * q0) * ld_bytes;
#pragma unroll
  for (int q = q0; q < q1; ++q) {
    asm volatile("" : "+s"(rowoff));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(src, lds_at(img + 1024 * q), 16, P.v[q & 3] + rowoff, 0, 0, 0);
    rowoff += 4 * ld_bytes;
  }
}
// SW_ROW / SW_BOTH image: byte address of logical chunk (8h + j) of row c is row_base ^ (16 j), j < 8.
__device__ __forceinline__ int row_base64(int c, int h, const int sw = SW_ROW) { return 256 * c + 16 * ((8 * h) ^ swz(sw, c)); }
// SW_BOTH image: element (crow(r,h), 32t + c) is at (both_base64(t) ^ both_k(r)) + 256 * crow(r, 0).
__device__ __forceinline__ int both_base64(int t, int c, int h) {
  return 1024 * h + 128 * (t ^ h) + 16 * ((c >> 2) ^ (4 * h)) + 4 * (c & 3);
}
__host__ __device__ constexpr int both_k(int r) { return 128 * ((r >> 2) & 1) + 16 * (r & 3); }
// SW_BOTH column read (rows crow(r,h) and crow(r+8,h) share the XOR term; the rest is the offset field)
__device__ __forceinline__ float both_read(const float* lds, int base_t, int r, int off) {
  return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(lds) + off + 256 * crow(r, 0) + (base_t ^ both_k(r)));
}

// SW_COL image: element (crow(r,h), 32t + c) is at col_base64(t) + 256 * crow(r, 0).
__device__ __forceinline__ int col_base64(int t, int c, int h) { return 1024 * h + 128 * (t ^ h) + 4 * c; }

// Narrow row images (32 rows x KP floats, KP in {16,32,64,128}) of a contiguous (rows, KP) matrix:
// chunk p of row r holds logical chunk p ^ nsw(r), which makes 16-lane row reads conflict-free.
template <int KP>
__device__ __forceinline__ int nsw(int row) {
  return KP == 16 ? ((row >> 2) & 3) : KP == 32 ? ((row >> 1) & 7) : (row & 15);
}
// (KP is a plain argument: every caller passes a compile-time constant and the call is inlined.)
// (Rows [32 f0, 32 f1) / 2 of the tile only when a half range (f0, f1) in {0, 1, 2} is given.)
__device__ __forceinline__ void dma_narrow(uint32_t img, __amdgpu_buffer_rsrc_t src, int row0, const int KP,
                                          const int f0 = 0, const int f1 = 2) {
  const int CPR = KP / 4, RB = KP * 4;
  asm volatile("" : "+s"(img));
  const int i = lane_id();
#pragma unroll
  for (int q = f0 * KP / 16; q < f1 * KP / 16; ++q) {
    const int byte = 1024 * q + 16 * i, row = byte / RB, p = (byte / 16) % CPR;
    const int sw = KP == 16 ? ((row >> 2) & 3) : KP == 32 ? ((row >> 1) & 7) : (row & 15);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(src, lds_at(img + 1024 * q), 16, (row0 + row) * RB + 16 * (p ^ sw), 0, 0,
                                             0);
  }
}
// element (row, col) of a narrow image with KP floats per row
__device__ __forceinline__ int narrow_elem(int row, int col, const int KP) {
  const int sw = KP == 16 ? ((row >> 2) & 3) : KP == 32 ? ((row >> 1) & 7) : (row & 15);
  return row * KP * 4 + 16 * ((col >> 2) ^ sw) + 4 * (col & 3);
}
// byte address of logical chunk (L0 + j) of row c is narrow_base ^ (16 j) (L0 a multiple of the j range)
template <int KP>
__device__ __forceinline__ int narrow_base(int c, int L0) { return c * KP * 4 + 16 * (L0 ^ nsw<KP>(c)); }

__device__ __forceinline__ f32x4 lds_f4(const float* lds, int byte) {
  return *reinterpret_cast<const f32x4*>(reinterpret_cast<const char*>(lds) + byte);
}
__device__ __forceinline__ float lds_f1(const float* lds, int byte) {
  return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(lds) + byte);
}

// Zero an LDS image of NF floats before its first DMA, so rows a DMA leaves
// untouched (out-of-range rows of dma_tile_contig) hold zeros or earlier finite data, never garbage.
template <int NF>
__device__ __forceinline__ void lds_zero(float* img) {
  static_assert(NF % 4 == 0, "whole f32x4 stores");
  const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < (NF / 4 + 63) / 64; ++i)
    if (64 * i + lane_id() < NF / 4) reinterpret_cast<f32x4*>(img)[64 * i + lane_id()] = z;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// Wait for every outstanding vector-memory op of this wave (incl. LDS-DMA) before reading LDS.
__device__ __forceinline__ void wait_vm_all() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// XCD-aware block mapping. MI355X dispatches consecutive workgroups round-robin over its 8 XCDs,
// each with a private L2; the NB blocks of one (b,h) re-read the same K/V (or Q/dX) tiles, so they
// should share an XCD. Grid = 8 * ceil(BH/8) * NB one-dimensional blocks; block id -> (bh, blk) with
// bh = 8*(slot / NB) + id % 8, blk = slot % NB, slot = id / 8 (bh >= BH: idle block). Placement only
// affects speed (guide §1), never results.
struct BhBlock { int bh, blk; bool valid; };
__device__ __forceinline__ BhBlock xcd_block(int nb, int BH) {
  const int id = blockIdx.x, x = id & 7, slot = id >> 3;
  BhBlock r;
  r.bh = 8 * (slot / nb) + x;
  r.blk = slot % nb;
  r.valid = r.bh < BH;
  return r;
}
inline unsigned xcd_grid(int nb, int BH) { return (unsigned)(8 * ((BH + 7) / 8) * nb); }
// The same blocks on the same XCDs, walked in the reverse order inside each XCD: a consumer of the previous kernel's
// per-(b,h) output starts with the (b,h)s that kernel wrote last, still in the XCD's L2 (k_attn_bwd_kv after the
// forward, which k_attn_bwd_qg then walks against: profiles/r06_ab_xcd_order.txt).
__device__ __forceinline__ BhBlock xcd_block_rev(int nb, int BH) {
  const int id = blockIdx.x, x = id & 7, slot = (int)(gridDim.x >> 3) - 1 - (id >> 3);
  BhBlock r;
  r.bh = 8 * (slot / nb) + x;
  r.blk = slot % nb;
  r.valid = r.bh < BH;
  return r;
}

// ---------------------------------------------------------------------------------------
// Host-side launch plumbing. Every entry point runs on the device of the stream it is given, not
// on the calling thread's current device (DeviceGuard), and keeps no library-owned streams or events.
// ---------------------------------------------------------------------------------------
inline int stream_device(hipStream_t st) {
  int dev = -1;
  if (hipStreamGetDevice(st, &dev) != hipSuccess || dev < 0) {
    (void)hipGetLastError();
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  }
  return dev;
}
// Makes the stream's device current for the scope (restores the caller's on exit).
struct DeviceGuard {
  int dev = 0, prev = -1;
  explicit DeviceGuard(hipStream_t st) : dev(stream_device(st)) {
    int cur = -1;
    if (hipGetDevice(&cur) == hipSuccess && cur != dev && hipSetDevice(dev) == hipSuccess) prev = cur;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel instantiation, current device): the
// attribute is idempotent, and this table of (kernel, device bits) is the library's only cached state.
void set_dyn_lds(const void* kernel, int bytes);

// The two halves of an attention backward side by side (SBM: bwd_q | gamma pass + bwd_kv; CSE: bwd_qf |
// row-statistics pass + bwd_kf): the key half on the CALLER's side stream (csa_*_bwd_args.side_stream),
// forked from and joined back into the caller's stream with the caller's two events (capture-safe).
// CSA_SCHED_AUTO picks it when the query half's grid leaves a partial last round of workgroups on the
// chip (SBM java dims, B=64: 2.5 rounds, -4% per layer step) and not when the grid is whole rounds (SBM
// python dims, B=256: exactly 5 rounds, +3%: the statistics pass is not hidden).
inline bool bwd_concurrent(uint32_t sched, const void* side, int dev, int64_t wgs, int waves_per_simd) {
  if (!side || sched == 1u /* CSA_SCHED_IN_ORDER */) return false;
  if (sched == 2u /* CSA_SCHED_CONCURRENT */) return true;
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) {
    (void)hipGetLastError();
    return false;
  }
  const double r = (double)wgs / (4.0 * cus * waves_per_simd), full = ceil(r);
  return (full - r) / full >= 0.1;
}
// Caller-owned fork/join lane. fork(): record on the caller's stream, make the side stream wait;
// join(): the reverse. Each returns false on a HIP error (the caller then reports CSA_LAUNCH_FAILED;
// a failed fork launches nothing on the side stream).
struct SideLane {
  hipStream_t s; hipEvent_t fork_ev, join_ev;
  bool fork(hipStream_t st) const {
    return hipEventRecord(fork_ev, st) == hipSuccess && hipStreamWaitEvent(s, fork_ev, 0) == hipSuccess;
  }
  bool join(hipStream_t st) const {
    return hipEventRecord(join_ev, s) == hipSuccess && hipStreamWaitEvent(st, join_ev, 0) == hipSuccess;
  }
};

// Per-thread last-error text shared by every translation unit (csa_last_error_str).
void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
const char* get_error();

}  // namespace csa
