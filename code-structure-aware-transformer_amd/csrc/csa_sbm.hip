// SBM attention (module/sbm_attn.py:11-87 + module/STE.py) as gfx950 HIP kernels.
//
// The throw-away experiment variants of earlier rounds live in git history (round-5
// tree, commit 0b877e5), not in these sources.
// Pipeline (one forward + one backward = 10 launches, all stream-ordered, no host sync):
//   fwd: k_prep              S_h = softmax_{k^2}(C_h C_h^T) (sbm_attn.py:37-39) and the weights ->
//                            MFMA-operand-major fragments (L2-resident), one launch
//        k_proj_fwd_l        Qh = sigmoid(MLP(Q) C^T), Kh likewise, T = Kh S^T    sbm_attn.py:41-53
//        k_attn_fwd          expA tile, u < clamp(expA) sampling, online softmax
//                            with graph-masked L1 renormalisation, dropout, PV    sbm_attn.py:55-64, STE.py:10-15
//        k_sparsity_finish   integer edge counts -> head-wise sparsity            sbm_attn.py:64
//   bwd: k_attn_rowprep      gamma = rowsum(dX*X) and the per-row constants of the elementwise backward
//        k_attn_bwd_kv       S, dP, the elementwise backward once per element; dK (attention path),
//                            dV, dT; one float per element (w, or W_NO_EDGE) to the workspace
//        k_attn_bwd_qg       dQ (attention path) = ds K, dQh = G T, ds and G rebuilt from those tiles
//        k_proj_bwd_s        STE/sigmoid/cluster/MLP backward (+dQ, +dK second path),
//                            per-workgroup fixed-order partial slabs for dW, db, dC, dS
//        k_reduce_slabs      fixed-order slab reduction
//        k_cluster_grad      softmax_{k^2} backward -> dC
// The N x N intermediates of the reference (expA, graph, dot, softmax, attn: ~11 fp32
// (B,H,N,M) tensors) are never materialised in the forward: the sampled graph and the dropout
// keep-mask are kept as 1 bit per edge for the backward, and the optional attn/graph maps are
// produced by k_maps only when the caller asks for them. The fp32 backward hands one (with
// clusters at most two) fp32 value per element from k_attn_bwd_kv to k_attn_bwd_qg through the
// workspace (Layout::w_dsg, O(B*H*N*M)); bf16 mode recomputes instead and sizes it away
// (CSA_FLAG_BF16_WS).
#include "csa_common.hpp"
#include "../../include/csa_hip.h"

#include <algorithm>
#include <type_traits>
#include <mutex>
#include <stdint.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

using namespace csa;

namespace csa {
static thread_local char g_err[512] = "";
void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
const char* get_error() { return g_err; }

void set_dyn_lds(const void* kernel, int bytes) {
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) dev = -1;
  struct Ent { const void* k; int bytes; uint64_t devs; };
  static std::mutex mu;
  static Ent tab[256];
  static int n = 0;
  const uint64_t bit = (dev >= 0 && dev < 64) ? (1ull << dev) : 0ull;
  // held across the HIP call: concurrent first calls for one kernel must not record a smaller size
  std::lock_guard<std::mutex> lock(mu);
  Ent* e = nullptr;
  for (int i = 0; i < n; ++i)
    if (tab[i].k == kernel) e = &tab[i];
  if (e && bit && (e->devs & bit) && e->bytes >= bytes) return;
  const int target = e && e->bytes > bytes ? e->bytes : bytes;  // never lower an attribute already set
  if (hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, target) != hipSuccess) {
    (void)hipGetLastError();  // the launch reports it
    return;
  }
  if (!e && n < 256) e = &(tab[n++] = Ent{kernel, target, 0});
  if (!e) return;
  if (target > e->bytes) e->devs = 0;  // a larger size re-arms every device
  e->bytes = target;
  e->devs |= bit;
}
}  // namespace csa

namespace {

constexpr float NEG_INF = -__builtin_inff();
constexpr float NORM_EPS = 1e-12f;  // F.normalize default eps (sbm_attn.py:62)
constexpr float LOG2E = 1.4426950408889634f;
typedef float f2 __attribute__((ext_vector_type(2)));  // register pairs for packed fp32 (v_pk_*)

// ------------------------------------------------------------------------------------
// Layout of the saved forward state (caller-allocated, csa_sbm_state_bytes)
// ------------------------------------------------------------------------------------
struct Layout {
  int64_t B, H, N, M, D, k, kp, KT, NQB, NKB, Mpad;
  size_t S, Qh, Kh, T, stats, Abits, Rbits, cnt, tdead, Wf[3], WfT[3], Cf, CfT, Sf, SfT, Act, total;
  // bwd workspace
  size_t w_dQh, w_dT, w_slab, w_dS, w_dC, w_gx, w_dsg, w_brow, w_total;
  int64_t G, slab_floats, w_dsg_plane;
  int64_t G_K, G_Q;  // k_proj_bwd_s split by item kind (concurrent schedule): workgroups per head of each launch
};

inline size_t al(size_t x) { return (x + 255) & ~size_t(255); }

// Projection-backward workgroups per head. The head's I = B * items_per_b items (32-row Q / K blocks)
// are split evenly over G workgroups of 4 waves (one item per wave per group of 4). G minimises
// (dispatch rounds over the 256 CUs) x (groups of 4 items per workgroup); the smallest G wins ties
// (fewer slabs to reduce). java B = 64, H = 8, 10 items per AST, 1 workgroup per CU: G = 32, one round
// of 5 full groups (a whole-batch split, G = 64, ran two rounds of 3 groups, the last half empty).
int64_t proj_bwd_groups(int64_t B, int64_t H, int64_t items_per_b, int wg_per_cu, int share = 1) {
  const int64_t I = B * items_per_b, slots = std::max<int64_t>(1, 256LL * wg_per_cu / share);
  const int64_t gmax = std::min<int64_t>(I, std::max<int64_t>(1, 4 * slots / H));
  int64_t best = 1, best_cost = INT64_MAX;
  for (int64_t G = 1; G <= gmax; ++G) {
    const int64_t cost = ((H * G + slots - 1) / slots) * (((I + G - 1) / G + 3) / 4);
    if (cost < best_cost) { best_cost = cost; best = G; }
  }
  return best;
}

Layout make_layout(int64_t B, int64_t H, int64_t N, int64_t M, int64_t D, int64_t k, uint32_t flags) {
  const bool dense = flags & CSA_FLAG_DENSE;
  Layout L;
  L.B = B; L.H = H; L.N = N; L.M = M; L.D = D; L.k = dense ? 0 : k;
  // kp (stored cluster width) is exactly 2*KPH of the instantiation used: 16, 32, 64 or 128
  L.kp = dense ? 0 : (k <= 16 ? 16 : k <= 32 ? 32 : k <= 64 ? 64 : 128);
  L.KT = dense ? 0 : (L.kp <= 32 ? 1 : L.kp / 32);
  L.NQB = (N + 31) / 32; L.NKB = (M + 31) / 32; L.Mpad = L.NKB * 32;
  size_t o = 0;
  auto take = [&](size_t bytes) { size_t r = o; o += al(bytes); return r; };
  const int64_t KP32 = 32 * L.KT;
  L.S = take(sizeof(float) * H * KP32 * KP32);
  L.Qh = take(sizeof(float) * B * H * N * L.kp);
  L.Kh = take(sizeof(float) * B * H * M * L.kp);
  L.T = take(sizeof(float) * B * H * M * L.kp);
  L.stats = take(sizeof(float) * B * H * N * 4);
  L.Abits = take(sizeof(uint32_t) * B * H * L.NQB * L.Mpad);
  L.Rbits = take(sizeof(uint32_t) * B * H * L.NQB * L.Mpad);
  L.cnt = take(sizeof(uint32_t) * B * H * L.NQB);  // per (b,h, query block): sampled edges (k_attn_fwd)
  L.tdead = take(sizeof(unsigned long long) * B);  // per AST: key tiles whose every key is masked (bit kt)
  for (int l = 0; l < 3; ++l) L.Wf[l] = take(sizeof(float) * (dense ? 0 : D * D));
  for (int l = 0; l < 3; ++l) L.WfT[l] = take(sizeof(float) * (dense ? 0 : D * D));
  L.Cf = take(sizeof(float) * H * KP32 * D);
  L.CfT = take(sizeof(float) * H * KP32 * D);
  L.Sf = take(sizeof(float) * H * KP32 * KP32);
  L.SfT = take(sizeof(float) * H * KP32 * KP32);
  // MLP activations of every 32-row item (h1 | h2 | po | hat), saved by k_proj_fwd for k_proj_bwd
  // (absent for CSA_FLAG_FWD_ONLY: only the backward reads them)
  L.Act = take(sizeof(float) * ((dense || (flags & CSA_FLAG_FWD_ONLY)) ? 0 : B * H * (L.NQB + L.NKB) * (3 * D + KP32) * 32));
  L.total = o;
  // backward workspace
  // two workgroups per CU for d = 64 with KT = 1 (k_proj_bwd_s / k_proj_bwd<64, 1>: 80 / 64 KiB LDS)
  L.G = dense ? 0 : proj_bwd_groups(B, H, L.NQB + L.NKB, (D == 64 && L.KT == 1) ? 2 : 1);
  // the key / query split (k_proj_bwd_s kinds 1 and 2, or both in one launch) sizes each kind for half the
  // workgroup slots, so the two together take the machine once (each sized for all of it: 2 rounds, and at
  // java dims 3 groups of 4 items per workgroup where the unsplit grid had 5 in one round: 210 -> 256 us)
  L.G_K = dense ? 0 : proj_bwd_groups(B, H, L.NKB, (D == 64 && L.KT == 1) ? 2 : 1, 2);
  L.G_Q = dense ? 0 : proj_bwd_groups(B, H, L.NQB, (D == 64 && L.KT == 1) ? 2 : 1, 2);
  L.slab_floats = dense ? 0 : (3 * D * D + 3 * D + KP32 * D + KP32 * KP32);
  o = 0;
  L.w_dQh = take(sizeof(float) * B * H * N * L.kp);
  L.w_dT = take(sizeof(float) * B * H * M * L.kp);
  L.w_slab = take(sizeof(float) * H * std::max(L.G, L.G_K + L.G_Q) * L.slab_floats);
  L.w_dS = take(sizeof(float) * H * KP32 * KP32);
  L.w_dC = take(sizeof(float) * H * KP32 * D);
  L.w_gx = take(sizeof(float) * B * H * N);  // used only when an attn-map gradient is passed
  // ds and G (STE gradient) tiles handed from k_attn_bwd_kv to k_attn_bwd_qg: (b,h, query block, key block)
  // 32 x 32 fp32 tiles [key][query]; G only with clusters
  L.w_dsg_plane = B * H * L.NQB * L.NKB * 1024;
  L.w_dsg = take(sizeof(float) * ((flags & CSA_FLAG_BF16_WS) ? 0 : L.w_dsg_plane * (dense ? 1 : 2)));
  // per query row (NQB * 32 rows per (b,h), padded rows included) the constants of k_attn_bwd_kv's elementwise
  // backward, written by k_attn_rowprep
  L.w_brow = take(sizeof(float) * B * H * L.NQB * 32 * 4);
  L.w_total = o;
  return L;
}

template <typename T> __device__ __forceinline__ T* at(void* base, size_t off) {
  return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + off);
}

// Scheduling fence: bounds how far the scheduler hoists the (L2-resident) fragment loads ahead of
// their MFMAs, which otherwise inflates register pressure past two waves per SIMD.
__device__ __forceinline__ void fence_sched() { __builtin_amdgcn_sched_barrier(0); }

// Fragment of an MFMA A operand, stored operand-major: ((it * nsteps/4 + s/4) * 64 + lane) * 4 + s%4.
// Loaded with a buffer load: one wave-uniform descriptor (SGPRs), the lane's byte offset as the only
// VGPR and the fragment's offset as a scalar. A plain pointer load makes the compiler materialise a
// 64-bit per-lane address for every one of the ~100 fragment loads of a layer chain and hoist them
// all to kernel entry, which spilled k_proj_bwd to scratch (guide T8/T20).
__device__ __forceinline__ f32x4 frag4(const float* __restrict__ f, int it, int nsteps, int s4) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(f), (short)0, 0x7fffffff, 0x00020000);
  const int soff = (it * (nsteps >> 2) + s4) * 1024;
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, lane_id() * 16, soff, 0));
}

// out[t] += sum_{s < 4 S4N} frag(t)[s] * bval(s) for t < NTO, fragments fetched LA K-groups (4 steps
// each) ahead: LA = 1 covers the L2 latency when the 4 NTO MFMAs of a group (>= 256 cycles) and other
// waves fill the gap; the sched fence keeps the lookahead (and its registers) at LA groups.
// The same fragment layout copied into LDS (FL): one ds_read_b128 per lane per K-group and tile.
__device__ __forceinline__ f32x4 frag4_lds(const float* __restrict__ f, int it, int nsteps, int s4) {
  return *reinterpret_cast<const f32x4*>(f + ((it * (nsteps >> 2) + s4) * 64 + lane_id()) * 4);
}

// BF16: the same chain on v_mfma_f32_32x32x16_bf16 (CSA_DTYPE_BF16's projection contractions): one
// instruction takes two consecutive K-groups (8 K-steps, csa_common.hpp pack8), both operands rounded to
// bf16 (RNE) as they are packed; accumulation stays fp32. S4N must be even.
// side(g) runs inside K-group g's scheduling region (g = 0 .. groups - 1; a compile-time constant once the loop is
// unrolled): independent work (activation stores, ActStager) that the scheduler interleaves with the group's MFMAs.
struct NoSide { __device__ __forceinline__ void operator()(int) const {} };
template <int NTO, int S4N, int LA = 1, bool FL = false, bool BF16 = false, typename BV, typename SIDE = NoSide>
__device__ __forceinline__ void frag_chain(const float* __restrict__ frag, int nsteps, f32x16 (&out)[NTO], BV bval,
                                           SIDE side = SIDE()) {
  static_assert(LA == 1 || LA == 2, "lookahead of one or two K-groups");
  auto ld = [&](int t, int s4) { return FL ? frag4_lds(frag, t, nsteps, s4) : frag4(frag, t, nsteps, s4); };
  if constexpr (BF16) {
    static_assert(S4N % 2 == 0, "bf16 chains take K-groups in pairs");
    constexpr int S8N = S4N / 2;
    f32x4 wq[2][NTO][2];
#pragma unroll
    for (int t = 0; t < NTO; ++t) { wq[0][t][0] = ld(t, 0); wq[0][t][1] = ld(t, 1); }
#pragma unroll
    for (int s8 = 0; s8 < S8N; ++s8) {
      if (s8 + 1 < S8N) {
#pragma unroll
        for (int t = 0; t < NTO; ++t) {
          wq[(s8 + 1) & 1][t][0] = ld(t, 2 * s8 + 2);
          wq[(s8 + 1) & 1][t][1] = ld(t, 2 * s8 + 3);
        }
      }
      float bv[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) bv[e] = bval(8 * s8 + e);
      const bf16x8 b8 = pack8(bv);
#pragma unroll
      for (int t = 0; t < NTO; ++t) out[t] = mfma_bf(pack8(wq[s8 & 1][t][0], wq[s8 & 1][t][1]), b8, out[t]);
      side(s8);
      fence_sched();
    }
    return;
  }
  f32x4 wq[LA + 1][NTO];
#pragma unroll
  for (int a = 0; a < LA; ++a)
    if (a < S4N)
#pragma unroll
      for (int t = 0; t < NTO; ++t) wq[a][t] = ld(t, a);
#pragma unroll
  for (int s4 = 0; s4 < S4N; ++s4) {
    if (s4 + LA < S4N) {
#pragma unroll
      for (int t = 0; t < NTO; ++t) wq[(s4 + LA) % (LA + 1)][t] = ld(t, s4 + LA);
    }
#pragma unroll
    for (int t = 0; t < NTO; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) out[t] = mfma(wq[s4 % (LA + 1)][t][e], bval(4 * s4 + e), out[t]);
    if constexpr (FL) {
      // LDS fragments: the scheduler otherwise sinks the lookahead reads to the group's last MFMA (register
      // pressure heuristics), so the next group starts on lgkmcnt(0); pin them ahead of the group's MFMAs
      if (s4 + LA < S4N) __builtin_amdgcn_sched_group_barrier(0x100, NTO, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4 * NTO, 0);
    }
    side(s4);
    fence_sched();
  }
}

// ------------------------------------------------------------------------------------
// Fragment prep: dst(it, s, lane) = Mat[32 it + c][kperm(s, h)] (or Mat^T), 0 outside.
// ------------------------------------------------------------------------------------
struct FragJob {
  const float* src; float* dst;
  int rows, cols, ld;         // source matrix (rows x cols, row stride ld)
  int transpose;              // value = src[kk][r] instead of src[r][kk]
  int acc_perm;               // kperm: 0 = lin (k = s + nsteps*h), 1 = acc (k = 32(s/16)+crow(s%16,h))
  int nit, nsteps;            // output tiles x K-steps
  int batch; int64_t src_bstride, dst_bstride;  // repeated per head
};
struct FragJobs { FragJob j[12]; int n; };

// element e of job J (e = batch index * per-batch elements + position in the fragment array)
__device__ __forceinline__ void frag_elem(const FragJob& J, int64_t e) {
  const int64_t per = (int64_t)J.nit * J.nsteps * 64;
  const int64_t bidx = e / per, rem = e % per;
  const int s4 = (int)(rem / 256) % (J.nsteps / 4);
  const int it = (int)(rem / 256) / (J.nsteps / 4);
  const int lane = (int)(rem / 4) % 64, s = s4 * 4 + (int)(rem % 4);
  const int c = lane & 31, h = lane >> 5;
  const int r = 32 * it + c;
  const int kk = J.acc_perm ? 32 * (s / 16) + crow(s % 16, h) : s + J.nsteps * h;
  const float* src = J.src + bidx * J.src_bstride;
  float v = 0.f;
  if (r < J.rows && kk < J.cols) v = J.transpose ? src[(int64_t)kk * J.ld + r] : src[(int64_t)r * J.ld + kk];
  J.dst[bidx * J.dst_bstride + rem] = v;
}

// ------------------------------------------------------------------------------------
// F1: S_h = softmax over all k^2 entries of C_h C_h^T, zero-padded to (32KT x 32KT)
// ------------------------------------------------------------------------------------
// MAXE = ceil(k^2 / 256) rounded up to 1, 4, 16 or 64 (host-selected instantiation)
// The forward's prep stage in one launch: blocks 0 .. H-1 compute S_h (one head each) and then lay out S_h's
// fragments (jobs [0, nS), batch index = the head); blocks H .. run the weight / cluster fragment jobs
// [nS, n), which do not depend on S, grid-stride.
template <int MAXE>
__global__ __launch_bounds__(256) void k_prep(const float* __restrict__ C, float* __restrict__ S, int k, int D, int KP32,
                                              int H, const FragJobs jobs, int nS) {
  if ((int)blockIdx.x >= H) {
    const int64_t t0 = (int64_t)(blockIdx.x - H) * 256 + threadIdx.x, stride = (int64_t)(gridDim.x - H) * 256;
    for (int j = nS; j < jobs.n; ++j) {
      const FragJob& J = jobs.j[j];
      const int64_t total = (int64_t)J.nit * J.nsteps * 64 * J.batch;
      for (int64_t e = t0; e < total; e += stride) frag_elem(J, e);
    }
    return;
  }
  // C_h (k x D <= 128 x 96) staged in LDS; each thread keeps its (up to MAXE) logits in registers
  // across the max / sum / normalise passes (one dot product per entry instead of three).
  const int hd = blockIdx.x, tid = threadIdx.x;
  // rows padded to D + 1 floats: consecutive threads read consecutive rows b, which then sit in
  // different banks (an unpadded stride of D = 64 put every thread of a wave on one bank)
  __shared__ float Cs[128 * 97];
  __shared__ float red[256];
  const float* Ch = C + (size_t)hd * k * D;
  const int LD = D + 1;
  for (int e = tid; e < k * D; e += 256) Cs[(e / D) * LD + e % D] = Ch[e];
  __syncthreads();
  const int kk = k * k;
  float v[MAXE];
  float mx = NEG_INF;
#pragma unroll
  for (int q = 0; q < MAXE; ++q) {
    const int e = tid + 256 * q;
    v[q] = NEG_INF;
    if (e < kk) {
      const int a = e / k, b = e % k;
      float acc = 0.f;
      for (int t = 0; t < D; ++t) acc = fmaf(Cs[a * LD + t], Cs[b * LD + t], acc);
      v[q] = acc;
      mx = fmaxf(mx, acc);
    }
  }
  red[tid] = mx;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] = fmaxf(red[tid], red[tid + s]);
    __syncthreads();
  }
  mx = red[0];
  __syncthreads();
  float sm = 0.f;
#pragma unroll
  for (int q = 0; q < MAXE; ++q) {
    const int e = tid + 256 * q;
    v[q] = e < kk ? expf(v[q] - mx) : 0.f;
    sm += v[q];
  }
  red[tid] = sm;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  sm = red[0];
  float* Sh = S + (size_t)hd * KP32 * KP32;
  for (int e = tid; e < KP32 * KP32; e += 256) Sh[e] = 0.f;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < MAXE; ++q) {
    const int e = tid + 256 * q;
    if (e < kk) Sh[(e / k) * KP32 + e % k] = v[q] / sm;
  }
  __syncthreads();  // S_h complete (the workgroup's global writes are visible to it after the barrier)
  for (int j = 0; j < nS; ++j) {
    const FragJob& J = jobs.j[j];
    const int64_t per = (int64_t)J.nit * J.nsteps * 64;
    for (int64_t e = tid; e < per; e += 256) frag_elem(J, hd * per + e);
  }
}

// ------------------------------------------------------------------------------------
// Shared kernel arguments
// ------------------------------------------------------------------------------------
struct KArgs {
  int B, H, N, M, k, kp, NQB, NKB, Mpad;
  const float *Q, *K, *V; int64_t q_sb, q_sh, q_sn, k_sb, k_sh, k_sn, v_sb, v_sh, v_sn;
  const float* mask; int64_t mask_sb;
  const float* pb[3];  // proj biases
  const float *Wf[3], *WfT[3], *Cf, *CfT, *Sf, *SfT, *S;
  float *Qh, *Kh, *T, *stats, *Act;  // Act NULL for CSA_FLAG_FWD_ONLY (no activation blocks saved)
  uint32_t *Abits, *Rbits;
  uint32_t* cnt;  // per (b,h, query block) sampled-edge counts, summed per head by k_sparsity_finish
  unsigned long long* tdead;  // per AST: fully masked key tiles (k_attn_fwd; bit 0 never set), NKB <= 64
  const float* U;
  uint32_t seed_lo, seed_hi, off;
  float attn_p, proj_p, scale;
  uint32_t drop_thr, pdrop_thr;  // 16-bit keep thresholds: keep <=> u16 >= thr (thr = ceil(p * 65536))
  int bf16;                      // CSA_DTYPE_BF16: bf16 MFMA for the N^2 contractions (wave-uniform branch)
  // outputs
  float* X; int64_t x_sb, x_sh, x_sn;
  // backward
  const float *dX, *dsp, *dgraph, *dattn;  // dgraph / dattn: upstream grads of the returned maps (or null)
  float* gx;                               // dattn: per query row sum_j dattn_ij attn_ij (k_attn_gx)
  float *dQ, *dK, *dV, *dQh, *dT, *slab;
  float* dsg; int64_t gplane;  // ds | G tiles (Layout::w_dsg), G at dsg + gplane
  float* brow;                 // per query row (c0, u, v, rho) of the elementwise backward (k_attn_rowprep)
  int64_t dx_sb, dx_sh, dx_sn, dq_sb, dq_sh, dq_sn, dk_sb, dk_sh, dk_sn, dv_sb, dv_sh, dv_sn;
  int G; int64_t slab_floats;
  // k_proj_bwd_s items: 0 all, 1 key blocks, 2 query blocks, 3 both in one launch (workgroups [0, pb_gk) key
  // blocks, the rest query blocks); pb_goff: the launch's first slab of the head's G
  int pb_kind, pb_goff, pb_gk;
};

// One 16-bit uniform per element: Philox word e/2, low half for even e.
__device__ __forceinline__ uint32_t u16_of(const u32x4& r, int e) {
  const uint32_t w = (e >> 1) == 0 ? r.x : (e >> 1) == 1 ? r.y : (e >> 1) == 2 ? r.z : r.w;
  return (e & 1) ? (w >> 16) : (w & 0xffffu);
}

// MLP forward pieces for one 32-row block held as lin-perm rows x[D/2] (see csa_common.hpp).
// Hidden activations are accumulator tiles (feature rows in registers, data rows on lanes).
// Proj dropout p>0 applies Linear -> Dropout -> ReLU (sbm_attn.py:22-30) with a stateless Philox
// mask keyed by (row, feature, layer, Q/K), so the backward regenerates it bit-identically.
// The layer's Philox words (one call -> 8 x 16-bit uniforms for registers 8gp..8gp+7 of tile ot; keep <=>
// u16 >= pdrop_thr) are generated one call per K-group as side work of the layer's own MFMA chain (gen(g) inside
// the chain's scheduling regions), then applied (apply) to the finished accumulators. PD (a dropout launch): with
// p = 0 the keep test passes everywhere and the scale is 1, so PD only decides whether the words are drawn.
template <int D, bool PD>
struct DropWords {
  static constexpr int DT = D / 32, NC = 2 * DT;  // Philox calls per layer
  u32x4 u[NC];
  uint32_t k0, k1, c3, c1;  // Philox key, counter word 3 (stream, offset), counter word 1's layer / Q-K bits
  int row, bh;
  __device__ __forceinline__ DropWords(const KArgs& p, int layer, int row_, int bh_, int isK)
      : k0(p.seed_lo), k1(p.seed_hi), c3((RNG_PROJ_DROP << 28) ^ p.off),
        c1(((uint32_t)layer << 16) | ((uint32_t)isK << 20)), row(row_), bh(bh_) {}
  __device__ __forceinline__ void gen(int g) {
    if constexpr (PD) {
      if (g < NC) {
        const int ot = g >> 1, gp = g & 1, h = lane_id() >> 5;
        u[g] = philox4x32(u32x4{(uint32_t)row, (uint32_t)(4 * ot + 2 * gp + h) | c1, (uint32_t)bh, c3}, k0, k1);
      }
    }
  }
  __device__ __forceinline__ void apply(const KArgs& p, f32x16 (&a)[DT]) const {
    const float ks = PD ? 1.f / (1.f - p.proj_p) : 1.f;
#pragma unroll
    for (int ot = 0; ot < DT; ++ot)
#pragma unroll
      for (int gp = 0; gp < 2; ++gp)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float v = a[ot][8 * gp + e];
          if constexpr (PD) v = (u16_of(u[2 * ot + gp], e) >= p.pdrop_thr) ? v * ks : 0.f;
          a[ot][8 * gp + e] = fmaxf(v, 0.f);
        }
  }
};

// fp32, k <= 16, d = 64 / 96 (k_proj_bwd_s): the cluster-weight gradient is formed from h2 instead of po,
//   dC_h = sum dZ^T po = (sum dZ^T h2) W2^T + (sum dZ^T 1) b2^T     (po = h2 W2^T + b2, proj.6)
// so the forward does not save po (a third of the activation bytes: 168 MB written and read per B = 256 step) and
// k_cluster_grad applies W2 / b2 once per head. A reassociation of the same sums (fp32 rounding only).
constexpr bool H2C_ON = true;
__host__ __device__ constexpr bool h2c_path(int D, int KT, bool BF) { return H2C_ON && !BF && (D == 64 || D == 96) && KT == 1; }

constexpr int MLP_LA = 2;  // forward MLP chains: fragments two K-groups ahead
constexpr int FL_LA = 1;   // LDS fragment chains: one K-group ahead covers the LDS latency

// Linear bias as one more MFMA K-step after the weight chain (x W^T + b, summed last like addmm):
// A = b[32 ot + c] on every lane (raw load issued before the chain, no select on it), B = 1 on the
// h = 0 lanes and 0 on the h = 1 lanes, so D[f][row] += b[f].
template <int D>
__device__ __forceinline__ void bias_operand(const float* __restrict__ b, float (&ba)[D / 32]) {
  const int c = lane_id() & 31;
#pragma unroll
  for (int ot = 0; ot < D / 32; ++ot) ba[ot] = b[32 * ot + c];
}
template <int D>
__device__ __forceinline__ void add_bias(const float (&ba)[D / 32], f32x16 (&a)[D / 32]) {
  const float one = (lane_id() >> 5) == 0 ? 1.f : 0.f;
#pragma unroll
  for (int ot = 0; ot < D / 32; ++ot) a[ot] = mfma(ba[ot], one, a[ot]);
}

// Fragment sources of the projection forward: global (L2-resident) or the workgroup's LDS copy (FL).
struct FwdFrags { const float* W[3]; const float* C; const float* S; const float* b[3]; };

// h1 = relu(drop(W0 x + b0)) from lin-perm input rows
template <int D, bool FL, bool BF = false, bool PD = true>
__device__ __forceinline__ void mlp_layer0(const KArgs& p, const float* W0, const float* b0, const float (&x)[D / 2],
                                           f32x16 (&h1)[D / 32], int row, int bh, int isK) {
  constexpr int DT = D / 32, NS = D / 2;
  float ba[DT];
  bias_operand<D>(b0, ba);
#pragma unroll
  for (int ot = 0; ot < DT; ++ot) h1[ot] = zero16();
  DropWords<D, PD> dw(p, 0, row, bh, isK);
  frag_chain<DT, NS / 4, FL ? FL_LA : MLP_LA, FL, BF>(W0, NS, h1, [&](int s) { return x[s]; },
                                                       [&](int g) { dw.gen(g); });
  add_bias<D>(ba, h1);
  dw.apply(p, h1);
}

// out = W_l in + b_l  (acc-perm input), l = 1, 2
template <int D, bool FL, bool BF = false, typename SIDE = NoSide>
__device__ __forceinline__ void mlp_layer(const float* Wl, const float* bl, const f32x16 (&in)[D / 32],
                                          f32x16 (&out)[D / 32], SIDE side = SIDE()) {
  constexpr int DT = D / 32, NS = D / 2;
  float ba[DT];
  bias_operand<D>(bl, ba);
#pragma unroll
  for (int ot = 0; ot < DT; ++ot) out[ot] = zero16();
  frag_chain<DT, NS / 4, FL ? FL_LA : MLP_LA, FL, BF>(Wl, NS, out, [&](int s) { return in[s / 16][s % 16]; }, side);
  add_bias<D>(ba, out);
}

// hat^T = sigmoid(C_h p^T), rows (clusters) >= k zeroed. Cf: the head's cluster fragments.
template <int D, int KT, bool FL, bool BF = false, typename SIDE = NoSide>
__device__ __forceinline__ void cluster_hat(const KArgs& p, const float* Cf, const f32x16 (&po)[D / 32], f32x16 (&hat)[KT],
                                            SIDE side = SIDE()) {
  constexpr int NS = D / 2;
  const int h = lane_id() >> 5;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) hat[kt] = zero16();
  frag_chain<KT, NS / 4, 1, FL, BF>(Cf, NS, hat, [&](int s) { return po[s / 16][s % 16]; }, side);
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int a = 32 * kt + crow(r, h);
      // sigmoid via hardware exp / divide (a few ulp; branch-free): sbm_attn.py:47,53
      hat[kt][r] = (a < p.k) ? __fdividef(1.f, 1.f + __expf(-hat[kt][r])) : 0.f;
      (void)a;
    }
  }
}

// out^T = Sfrag * in^T (K = 32 KT clusters, acc-perm input)
template <int KT, bool FL = false>
__device__ __forceinline__ void small_mm(const float* __restrict__ frag, const f32x16 (&in)[KT], f32x16 (&out)[KT]) {
#pragma unroll
  for (int at = 0; at < KT; ++at) out[at] = zero16();
  frag_chain<KT, 4 * KT, 1, FL>(frag, 16 * KT, out, [&](int s) { return in[s / 16][s % 16]; });
}

// Store an accumulator tile set (feature rows, data row = lane) to out[row][0..ncols) (row-major, ld)
template <int NT>
__device__ __forceinline__ void store_rows(float* __restrict__ out, int64_t ld, int ncols, const f32x16 (&a)[NT], bool valid) {
  if (!valid) return;
  const int h = lane_id() >> 5;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c0 = 32 * t + 8 * g + 4 * h;
      if (c0 < ncols) {
        f32x4 v; v[0] = a[t][4 * g]; v[1] = a[t][4 * g + 1]; v[2] = a[t][4 * g + 2]; v[3] = a[t][4 * g + 3];
        *reinterpret_cast<f32x4*>(out + c0) = v;
      }
    }
  (void)ld;
}

template <int NT>
__device__ __forceinline__ void load_rows(f32x16 (&a)[NT], const float* __restrict__ in, int ncols, bool valid) {
  const int h = lane_id() >> 5;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c0 = 32 * t + 8 * g + 4 * h;
      const bool ok = valid && c0 < ncols;
      const f32x4 v = *reinterpret_cast<const f32x4*>(in + (c0 < ncols ? c0 : ncols - 4));
      a[t][4 * g] = ok ? v[0] : 0.f; a[t][4 * g + 1] = ok ? v[1] : 0.f;
      a[t][4 * g + 2] = ok ? v[2] : 0.f; a[t][4 * g + 3] = ok ? v[3] : 0.f;
    }
}

// ------------------------------------------------------------------------------------
// Activation blocks. Per 32-row item, k_proj_fwd saves h1 | h2 | po | hat feature-major:
// feature f is a 128-B row of the 32 data rows, its 16-B chunks XOR-swizzled by (f>>1)&7.
// k_proj_bwd DMAs these slices unchanged into its LDS staging regions. There the outer-product
// reads (ds_read_b128 of 4 rows of feature 32t+c, one 16-lane group = 16 consecutive c) are
// bank-conflict free: lane c lands in 16-B slot (c&1)*8 + (chunk ^ ((c>>1)&7)) of 256 B.
// ------------------------------------------------------------------------------------
__device__ __forceinline__ int act_off(int f, int row) { return f * 32 + 4 * ((row >> 2) ^ ((f >> 1) & 7)) + (row & 3); }


// Accumulator tiles (feature rows 32t + crow(r,h), data row = lane c) -> block slice (features from 0),
// through a wave-private 4 KiB LDS scratch: each 32-feature tile is written to the scratch in the
// block layout (16 ds_write_b32 per lane, conflict-free: a lane half writes one feature row) and leaves
// as 4 x 1 KiB contiguous dwordx4 stores (4x fewer store instructions, half the VGPR traffic per byte).
// NF = features of the tile set (<= 32 NT; a partial last tile stores only its first NF - 32 (NT - 1)).
template <int NT, int NF = 32 * NT>
__device__ __forceinline__ void store_act_lds(float* __restrict__ blk, const f32x16 (&a)[NT], float* __restrict__ scr) {
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int nf = NF - 32 * t < 32 ? NF - 32 * t : 32;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (crow(r, 0) < nf) scr[act_off(crow(r, h), c)] = a[t][r];
#pragma unroll
    for (int k = 0; k < nf / 8; ++k) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(scr + 4 * (lane + 64 * k));
      __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(blk + 1024 * t + 4 * (lane + 64 * k)));
    }
  }
}

// CSA_DTYPE_BF16 (d = 64 / 96, k <= 16): h1 | h2 | po are saved as bf16 in the first half of their slices,
// rounded as pack8 rounds them for the bf16 MFMAs (RNE), so the backward's bf16 outer products see the same
// operands; the relu masks keep their signs. Halves the activation traffic of the bf16 mode.
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2v __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4v __attribute__((ext_vector_type(4)));
template <int NT>
__device__ __forceinline__ void store_act_lds_bf(float* __restrict__ blk, const f32x16 (&a)[NT], float* __restrict__ scr) {
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  u32x2v* out = reinterpret_cast<u32x2v*>(blk);  // element e at 16-bit slot e
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int r = 0; r < 16; ++r) scr[act_off(crow(r, h), c)] = a[t][r];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(scr + 4 * (lane + 64 * k));
      bf16x4 b;
#pragma unroll
      for (int e = 0; e < 4; ++e) b[e] = (__bf16)v[e];
      __builtin_nontemporal_store(__builtin_bit_cast(u32x2v, b), out + 256 * t + lane + 64 * k);
    }
  }
}

constexpr int CSA_AUX_NT = 2;  // buffer instruction cache policy: non-temporal (as __builtin_nontemporal_store)
// store_act_lds / store_act_lds_bf split into three stages per tile, so that the stores ride along an MFMA chain
// as its side work (frag_chain's side(g)) instead of running as a phase of their own after the item's products
// (round 5: the store phase was 25% of a k_proj_fwd_l wave's time, s_memtime stamps). Stage W: the tile's 16
// scattered ds_write_b32 into the scratch; R: its nf / 8 ds_read_b128 back; S: the non-temporal global stores.
// Chain group 2t runs S(t - 1) then W(t), group 2t + 1 runs R(t), group 2 NT runs S(NT - 1), so a chain of
// >= 2 NT + 1 K-groups carries NT tiles. A wave's LDS operations complete in order, so W(t) may follow R(t - 1)
// into the same scratch without a wait. Same bytes in the same places as store_act_lds(_bf).
// The global stores go through a buffer resource over the item's activation block (num_records 0 when the call
// saves no activations: the hardware drops them), so no branch splits the chain's scheduling regions; `off` is
// the slice's byte offset in the block.
template <int NT, int NF = 32 * NT, bool BFS = false>
struct ActStager {
  __amdgpu_buffer_rsrc_t rs;
  int off;
  float* scr;
  const f32x16* a;
  f32x4 v[4];
  __device__ __forceinline__ static constexpr int nf(int t) { return NF - 32 * t < 32 ? NF - 32 * t : 32; }
  __device__ __forceinline__ void W(int t) {
    const int c = lane_id() & 31, h = lane_id() >> 5;
#pragma unroll
    for (int r = 0; r < 16; ++r)
      if (crow(r, 0) < nf(t)) scr[act_off(crow(r, h), c)] = a[t][r];
  }
  __device__ __forceinline__ void R(int t) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (k < nf(t) / 8) v[k] = *reinterpret_cast<const f32x4*>(scr + 4 * (lane + 64 * k));
  }
  __device__ __forceinline__ void S(int t) {
    const int lane = lane_id();
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      if (k >= nf(t) / 8) continue;
      if constexpr (BFS) {
        bf16x4 b;
#pragma unroll
        for (int e = 0; e < 4; ++e) b[e] = (__bf16)v[k][e];
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2v, b), rs, 8 * lane,
                                              off + 8 * (256 * t + 64 * k), CSA_AUX_NT);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4v, v[k]), rs, 16 * lane,
                                               off + 4 * (1024 * t + 256 * k), CSA_AUX_NT);
      }
    }
  }
  // the side work of chain group g
  __device__ __forceinline__ void operator()(int g) {
    if ((g & 1) == 0) {
      if (g >= 2 && g / 2 - 1 < NT) S(g / 2 - 1);
      if (g / 2 < NT) W(g / 2);
    } else if (g / 2 < NT) {
      R(g / 2);
    }
  }
  // stages a chain of `groups` K-groups did not reach (none when groups >= 2 NT + 1)
  __device__ __forceinline__ void finish(int groups) {
#pragma unroll
    for (int g = 0; g <= 2 * NT; ++g)
      if (g >= groups) (*this)(g);
  }
};

// The bf16 slice of store_act_lds_bf, DMA'd into the upper half of a wave's R-float LDS region, widened in
// place to the fp32 slice over the whole region (element order, hence the act_off layout, unchanged).
// Elements [0, R/2) first: their fp32 lands below the bf16 data. Then [R/2, R): every read of the phase
// completes before its writes, which overlap only that phase's own (consumed) sources.
template <int R>
__device__ __forceinline__ void widen_act_bf(float* __restrict__ reg, int lane) {
  const uint32_t* src = reinterpret_cast<const uint32_t*>(reg + R / 2);
  constexpr int NJ = R / 1024;  // 8-element reads per lane per phase
#pragma unroll
  for (int ph = 0; ph < 2; ++ph) {
    u32x4v w[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) w[j] = *reinterpret_cast<const u32x4v*>(src + ph * (R / 4) + 4 * (lane + 64 * j));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      f32x4 lo, hi;
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        lo[2 * e] = __builtin_bit_cast(float, w[j][e] << 16);
        lo[2 * e + 1] = __builtin_bit_cast(float, w[j][e] & 0xffff0000u);
        hi[2 * e] = __builtin_bit_cast(float, w[j][2 + e] << 16);
        hi[2 * e + 1] = __builtin_bit_cast(float, w[j][2 + e] & 0xffff0000u);
      }
      float* dst = reg + ph * (R / 2) + 8 * (lane + 64 * j);
      *reinterpret_cast<f32x4*>(dst) = lo;
      *reinterpret_cast<f32x4*>(dst + 4) = hi;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------------------------
// F2 body: one 32-row item (block rb of Q, or of K when isK) of batch element b, head hd.
// ------------------------------------------------------------------------------------
// x rows (lin-perm half rows) of item r of (b, hd)
template <int D>
__device__ __forceinline__ void load_item_x(const KArgs& p, int b, int hd, int r, float (&x)[D / 2]) {
  const int c = lane_id() & 31, h = lane_id() >> 5;
  const int isK = r >= p.NQB;
  const int nrows = isK ? p.M : p.N;
  const int row = (isK ? r - p.NQB : r) * 32 + c;
  const int rowc = imin(row, nrows - 1);
  const float* X = isK ? p.K + b * p.k_sb + hd * p.k_sh + (int64_t)rowc * p.k_sn
                       : p.Q + b * p.q_sb + hd * p.q_sh + (int64_t)rowc * p.q_sn;
  // raw loads (rows past the end re-read the last row): nothing consumes them here, so no wait is
  // placed before the caller's stores; proj_fwd_item zeroes the padding rows when it uses them
#pragma unroll
  for (int i = 0; i < D / 2; i += 4) {
    const f32x4 v = *reinterpret_cast<const f32x4*>(X + h * (D / 2) + i);
    x[i] = v[0]; x[i + 1] = v[1]; x[i + 2] = v[2]; x[i + 3] = v[3];
  }
}

// F2 body: item r of (b, hd) from its x rows. `next` runs once every product is done and x is dead,
// before the stores (the persistent kernel issues the next item's x loads there: a later vmcnt wait
// for them then does not also wait for this item's stores, which drain under the next item).
template <int D, int KT, bool FL, typename NEXT, bool BF = false, bool PD = true>
__device__ __forceinline__ void proj_fwd_item(const KArgs& p, const FwdFrags& F, int b, int hd, int r, float (&x)[D / 2],
                                              float* scr, NEXT next) {
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const int bh = b * p.H + hd;
  const int isK = r >= p.NQB;
  const int rb = isK ? r - p.NQB : r;
  const int nrows = isK ? p.M : p.N;
  const int row = rb * 32 + c;
  const bool rv = row < nrows;
  f32x16 h1[D / 32], h2[D / 32], po[D / 32], hat[KT], t[KT];
#pragma unroll
  for (int i = 0; i < D / 2; ++i) x[i] = rv ? x[i] : 0.f;
#define PHF(i)
  constexpr bool ABF = BF && (D == 64 || D == 96) && KT == 1;  // read back by k_proj_bwd_s<D, true>
  constexpr int ABLK = (3 * D + 32 * KT) * 32;
  // fp32 activations: h1 | h2 | po leave as the side work of the chain that consumes them (layer 1, layer 2, the
  // cluster product: ActStager), their stores interleaved with that chain's MFMAs instead of a store phase after
  // the item's products; hat and the Qh / Kh / T rows at the end
  constexpr bool STAGED = !BF;
  // unstaged d = 96 (java dims, 256 VGPRs): h1 leaves right after layer 1 has consumed it instead of being held to
  // the item's end with h2 / po / hat (the held h1 spilled 18 VGPRs)
  constexpr bool H1E = !STAGED && D == 96;
  float* const blk = p.Act ? p.Act + ((int64_t)bh * (p.NQB + p.NKB) + r) * ABLK : nullptr;
  const bool on = blk != nullptr;
  const __amdgpu_buffer_rsrc_t ars = make_rsrc(blk, on ? ABLK * 4 : 0);
  // layer 1's side work: h1's staged stores and layer 1's dropout words
  DropWords<D, PD> dw1(p, 1, row, bh, isK);
  struct Side1 {
    ActStager<D / 32> st;
    DropWords<D, PD>* dw;
    __device__ __forceinline__ void operator()(int g) {
      if constexpr (STAGED) st(g);
      dw->gen(g);
    }
  };
  struct Side {
    ActStager<D / 32> st;
    __device__ __forceinline__ void operator()(int g) { if constexpr (STAGED) st(g); }
  };
  mlp_layer0<D, FL, BF, PD>(p, F.W[0], F.b[0], x, h1, row, bh, isK);
  PHF(0)
  mlp_layer<D, FL, BF>(F.W[1], F.b[1], h1, h2, Side1{{ars, 0, scr, h1, {}}, &dw1});
  if (H1E && on) {
    if (ABF && p.kp <= 16) store_act_lds_bf<D / 32>(blk, h1, scr);
    else store_act_lds<D / 32>(blk, h1, scr);
  }
  PHF(1)
  dw1.apply(p, h2);
  PHF(2)
  mlp_layer<D, FL, BF>(F.W[2], F.b[2], h2, po, Side{{ars, 32 * D * 4, scr, h2, {}}});
  PHF(3)
  // po is not saved when k_proj_bwd_s forms dC from h2 (h2c_path): its stager is skipped (wave-uniform branch)
  struct SideIf {
    ActStager<D / 32> st;
    bool run;
    __device__ __forceinline__ void operator()(int g) { if constexpr (STAGED) { if (run) st(g); } }
  };
  cluster_hat<D, KT, FL, BF>(p, F.C, po, hat, SideIf{{ars, 64 * D * 4, scr, po, {}}, !(h2c_path(D, KT, BF) && p.kp <= 16)});
  PHF(4)
  if (isK) small_mm<KT, FL>(F.S, hat, t);
  next();
  PHF(5)
  if (on) {  // save the activations for k_proj_bwd (item r of this (b,h): Q blocks, then K blocks)
    if constexpr (!STAGED) {
      if (ABF && p.kp <= 16) {
        if (!H1E) store_act_lds_bf<D / 32>(blk, h1, scr);
        store_act_lds_bf<D / 32>(blk + 32 * D, h2, scr);
        store_act_lds_bf<D / 32>(blk + 64 * D, po, scr);
      } else {
        if (!H1E) store_act_lds<D / 32>(blk, h1, scr);
        store_act_lds<D / 32>(blk + 32 * D, h2, scr);
        store_act_lds<D / 32>(blk + 64 * D, po, scr);
      }
    }
    bool hat16 = false;
    if constexpr (KT == 1) {
      if ((D == 64 || D == 96) && p.kp <= 16) {  // k_proj_bwd_s reads hat from the Qh / Kh rows stored below
        hat16 = true;
      }
    }
    if (!hat16) store_act_lds<KT>(blk + 96 * D, hat, scr);
  }
  if (!isK) {
    store_rows<KT>(p.Qh + ((int64_t)bh * p.N + row) * p.kp, p.kp, p.kp, hat, rv);
  } else {
    store_rows<KT>(p.Kh + ((int64_t)bh * p.M + row) * p.kp, p.kp, p.kp, hat, rv);
    store_rows<KT>(p.T + ((int64_t)bh * p.M + row) * p.kp, p.kp, p.kp, t, rv);
  }
  PHF(6)
#undef PHF
  (void)lane; (void)h;
}

// ------------------------------------------------------------------------------------
// F2: per 32-row block of Q or K: Qh = sigmoid(MLP(Q) C^T); Kh likewise and T = Kh S^T.
// grid (NQB + NKB, B*H), one wave per block; weight fragments read from L2.
// ------------------------------------------------------------------------------------
template <int D, int KT>
__global__ __launch_bounds__(64) void k_proj_fwd(const KArgs p) {
  __shared__ __attribute__((aligned(16))) float scr[1024];  // activation store staging (store_act_lds)
  const int bh = blockIdx.y, hd = bh % p.H;
  const FwdFrags F{{p.Wf[0], p.Wf[1], p.Wf[2]}, p.Cf + (size_t)hd * 32 * KT * D, p.Sf + (size_t)hd * 1024 * KT * KT,
                   {p.pb[0], p.pb[1], p.pb[2]}};
  float x[D / 2];
  load_item_x<D>(p, bh / p.H, hd, blockIdx.x, x);
  proj_fwd_item<D, KT, false>(p, F, bh / p.H, hd, blockIdx.x, x, scr, [] {});
}

// F2 with the weight fragments in LDS: grid (G, H), NW waves per workgroup. The workgroup copies the three
// d x d layers and head hd's cluster / S fragments (operand-major, unchanged) into LDS once, then its waves
// run the head's items i_lo + w, i_lo + w + NW, ... of [i_lo, i_hi) (item = b * (NQB + NKB) + block).
// Same results as k_proj_fwd (identical MFMA chains); one L2 fragment fetch per workgroup instead of
// one per item.
template <int D, int KT>
struct ProjFwdLds {
  static constexpr int WB = D * D * 4, CB = 32 * KT * D * 4, SB = 1024 * KT * KT * 4;  // bytes
  static constexpr int NW = D == 64 ? 4 : 8;  // d = 64: two workgroups per CU; d = 96: one of 8 waves
  static constexpr int PIECES = (3 * WB + CB + SB) / 1024;
  static constexpr size_t FBYTES = 3 * WB + CB + SB;
  static constexpr size_t BBYTES = (3 * D * 4 + 15) / 16 * 16;  // the three biases
  static constexpr size_t BYTES = FBYTES + NW * 4096 + BBYTES;   // + a 4 KiB activation staging scratch per wave
  static_assert((3 * WB + CB + SB) % 1024 == 0, "whole 1 KiB DMA pieces");
};

// BF: CSA_DTYPE_BF16 (MLP and cluster projection on bf16 MFMA; T = Kh S^T stays fp32)
template <int D, int KT, bool BF = false, bool PD = true>
__global__ __launch_bounds__((64 * ProjFwdLds<D, KT>::NW)) void k_proj_fwd_l(const KArgs p) {
  using LY = ProjFwdLds<D, KT>;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int hd = blockIdx.y, g = blockIdx.x, G = gridDim.x;
  const uint32_t L0 = lds_offset(lds);
  for (int pc = w; pc < LY::PIECES; pc += LY::NW) {  // 1 KiB pieces: W0 | W1 | W2 | C_hd | S_hd
    const int byte = pc * 1024;
    const float* src;
    int off;
    if (byte < 3 * LY::WB) { src = p.Wf[byte / LY::WB]; off = byte % LY::WB; }
    else if (byte < 3 * LY::WB + LY::CB) { src = p.Cf + (size_t)hd * 32 * KT * D; off = byte - 3 * LY::WB; }
    else { src = p.Sf + (size_t)hd * 1024 * KT * KT; off = byte - 3 * LY::WB - LY::CB; }
    __builtin_amdgcn_raw_ptr_buffer_load_lds(make_rsrc(src, 0x7fffffff), lds_at(L0 + byte), 16, lane_id() * 16, off, 0, 0);
  }
  float* bias = lds + (LY::FBYTES + LY::NW * 4096) / 4;
  for (int e = threadIdx.x; e < 3 * D; e += 64 * LY::NW) bias[e] = p.pb[e / D][e % D];
  const int per_b = p.NQB + p.NKB;
  const int i_lo = (int)((int64_t)g * p.B * per_b / G), i_hi = (int)((int64_t)(g + 1) * p.B * per_b / G);
  float x[D / 2];
  if (i_lo + w < i_hi) load_item_x<D>(p, (i_lo + w) / per_b, hd, (i_lo + w) % per_b, x);
  wait_vm_all();
  __syncthreads();
  const FwdFrags F{{lds, lds + D * D, lds + 2 * D * D}, lds + 3 * D * D, lds + 3 * D * D + 32 * KT * D,
                   {bias, bias + D, bias + 2 * D}};
  float* scr = lds + LY::FBYTES / 4 + 1024 * w;
  for (int it = i_lo + w; it < i_hi; it += LY::NW) {
    const int nx = it + LY::NW;
    auto nextf = [&] {
      if (nx < i_hi) load_item_x<D>(p, nx / per_b, hd, nx % per_b, x);
    };
    proj_fwd_item<D, KT, true, decltype(nextf), BF, PD>(p, F, it / per_b, hd, it % per_b, x, scr, nextf);
  }
}

// fp32: k_attn_bwd_kv runs the elementwise backward once per element and hands the ds / G tiles to
// k_attn_bwd_qg (which then recomputes neither S nor dP). bf16 mode: recomputing S and dP on the 16x faster bf16
// MFMA costs less than moving the tiles through HBM, so k_attn_bwd_qr recomputes them (the round-3 design).
// Same-box A/B (profiles/r04_ab_handoff.txt): fp32 layer step 1.329 (recompute) -> 1.275 ms (handoff); saving the
// forward's S tiles for k_attn_bwd_kv as well measured 1.290 ms (+23 us forward stores, -22 us backward): not kept.
// One-plane handoff (no upstream map gradients): the key side stores w = dM P for an edge (A = 1) and the bit
// pattern W_NO_EDGE (a signalling NaN, which no arithmetic produces) for a non-edge, so the query side rebuilds
//   ds = ((A ? w : 0) - rho P) / sqrt(d),  G = A ? hardtanh(w + csp) : 0
// from one float per element: rho = [n < eps] gamma is 0 on every row whose normaliser is not degenerate, and
// only tiles holding a row with rho != 0 also store P (in the second plane). Half the handoff bytes of the
// two-plane ds | G format, which the map-gradient variant (DG: per-element dgraph / dattn terms) keeps.
constexpr uint32_t W_NO_EDGE = 0x7f800001u;

template <bool BF>
constexpr bool bwd_handoff() {
  return !BF;
}

// ------------------------------------------------------------------------------------
// F3: attention forward, one wave per (b, h, 32-query block), S^T orientation
// (keys = accumulator rows, queries = lanes). Online softmax with two running sums:
//   Z = sum e, Zg = sum e*A; X = (sum e*A*r V) / (Z * max(Zg/Z, 1e-12))
// which equals F.normalize(softmax(s) * graph, p=1) @ dropout (sbm_attn.py:59-63).
// ------------------------------------------------------------------------------------
// Bit-pack one tile's sampled graph / keep mask: ballot r holds key crow(r,0)'s 32 query bits in its
// low word and key crow(r,1)'s in its high word; v_writelane drops each word into its key's lane
// (no per-lane masks or selects). Measured on gfx950: a v_writelane reading an SGPR that a v_cmp wrote
// just before gets stale data, and the hazard recognizer does not look inside inline asm; the 16
// ballots are taken first and written in two batches of 8, each led by one s_nop 4.
template <int R0>
__device__ __forceinline__ uint32_t writelane_batch(uint32_t dst, const unsigned long long (&b)[16]) {
  static_assert(R0 == 0 || R0 == 8, "two batches of 8 ballots");
#define CSA_WL_OPS                                                                                        \
  : "+v"(dst)                                                                                            \
  : "s"((uint32_t)b[R0]), "s"((uint32_t)(b[R0] >> 32)), "s"((uint32_t)b[R0 + 1]),                        \
    "s"((uint32_t)(b[R0 + 1] >> 32)), "s"((uint32_t)b[R0 + 2]), "s"((uint32_t)(b[R0 + 2] >> 32)),        \
    "s"((uint32_t)b[R0 + 3]), "s"((uint32_t)(b[R0 + 3] >> 32)), "s"((uint32_t)b[R0 + 4]),                \
    "s"((uint32_t)(b[R0 + 4] >> 32)), "s"((uint32_t)b[R0 + 5]), "s"((uint32_t)(b[R0 + 5] >> 32)),        \
    "s"((uint32_t)b[R0 + 6]), "s"((uint32_t)(b[R0 + 6] >> 32)), "s"((uint32_t)b[R0 + 7]),                \
    "s"((uint32_t)(b[R0 + 7] >> 32))
  if constexpr (R0 == 0)
    asm("s_nop 4\n\t"
      "v_writelane_b32 %0, %1, 0\n\t"
      "v_writelane_b32 %0, %2, 4\n\t"
      "v_writelane_b32 %0, %3, 1\n\t"
      "v_writelane_b32 %0, %4, 5\n\t"
      "v_writelane_b32 %0, %5, 2\n\t"
      "v_writelane_b32 %0, %6, 6\n\t"
      "v_writelane_b32 %0, %7, 3\n\t"
      "v_writelane_b32 %0, %8, 7\n\t"
      "v_writelane_b32 %0, %9, 8\n\t"
      "v_writelane_b32 %0, %10, 12\n\t"
      "v_writelane_b32 %0, %11, 9\n\t"
      "v_writelane_b32 %0, %12, 13\n\t"
      "v_writelane_b32 %0, %13, 10\n\t"
      "v_writelane_b32 %0, %14, 14\n\t"
      "v_writelane_b32 %0, %15, 11\n\t"
      "v_writelane_b32 %0, %16, 15"
        CSA_WL_OPS);
  else
    asm("s_nop 4\n\t"
      "v_writelane_b32 %0, %1, 16\n\t"
      "v_writelane_b32 %0, %2, 20\n\t"
      "v_writelane_b32 %0, %3, 17\n\t"
      "v_writelane_b32 %0, %4, 21\n\t"
      "v_writelane_b32 %0, %5, 18\n\t"
      "v_writelane_b32 %0, %6, 22\n\t"
      "v_writelane_b32 %0, %7, 19\n\t"
      "v_writelane_b32 %0, %8, 23\n\t"
      "v_writelane_b32 %0, %9, 24\n\t"
      "v_writelane_b32 %0, %10, 28\n\t"
      "v_writelane_b32 %0, %11, 25\n\t"
      "v_writelane_b32 %0, %12, 29\n\t"
      "v_writelane_b32 %0, %13, 26\n\t"
      "v_writelane_b32 %0, %14, 30\n\t"
      "v_writelane_b32 %0, %15, 27\n\t"
      "v_writelane_b32 %0, %16, 31"
        CSA_WL_OPS);
#undef CSA_WL_OPS
  return dst;
}

// 16 ballots -> the bit word of each key lane (lanes 0..31: key c of the tile, bit = query row)
__device__ __forceinline__ uint32_t pack_bits(const bool (&v)[16]) {
  unsigned long long b[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) b[r] = __ballot(v[r]);
  uint32_t w = 0;
  w = writelane_batch<0>(w, b);
  return writelane_batch<8>(w, b);
}

template <int D, int KPH>
struct AttnFwdLds {
  static constexpr bool SWZ = (D == 64);                        // x4 DMA into swizzled unpadded tiles
  static constexpr int DP = D + 4, KP = 2 * KPH;
  static constexpr int KV_BYTES = SWZ ? 32 * 64 * 4 : 32 * DP * 4;  // one K or V image
  static constexpr int T_BYTES = 32 * KP * 4;
  static constexpr int KOFF = 0, VOFF = KV_BYTES, TOFF = 2 * KV_BYTES, BOFF = TOFF + T_BYTES;
  // K image | V image | T image | key bias row (Mpad floats: 0 = valid key, -inf = padded / beyond M)
  __host__ __device__ static size_t bytes(int Mpad) { return (size_t)BOFF + 4 * (size_t)Mpad; }
};

// Key bias row (0 for a valid unmasked key, -inf otherwise: sbm_attn.py:61 masked_fill) in two halves so the
// mask loads of the first KB_UNROLL x 64 keys are in flight together with the prologue's other loads and DMAs
// (a runtime-trip-count loop of load -> store would serialize one memory latency per 64 keys).
constexpr int KB_UNROLL = 4;
struct KeyMask { float v[KB_UNROLL]; };
__device__ __forceinline__ KeyMask key_mask_load(const KArgs& p, int b) {
  const float* mk = p.mask ? p.mask + b * p.mask_sb : nullptr;
  KeyMask km;
#pragma unroll
  for (int u = 0; u < KB_UNROLL; ++u) {
    const int j = lane_id() + 64 * u;
    km.v[u] = (mk && j < p.NKB * 32) ? mk[imin(j, p.M - 1)] : 0.f;
  }
  return km;
}
__device__ __forceinline__ void key_bias_store(float* bias, const KArgs& p, int b, const KeyMask& km) {
#pragma unroll
  for (int u = 0; u < KB_UNROLL; ++u) {
    const int j = lane_id() + 64 * u;
    if (j < p.NKB * 32) bias[j] = (j < p.M && km.v[u] == 0.f) ? 0.f : NEG_INF;
  }
  const float* mk = p.mask ? p.mask + b * p.mask_sb : nullptr;
  for (int j = lane_id() + 64 * KB_UNROLL; j < p.NKB * 32; j += 64) {  // M > 256 only
    const float mv = mk ? mk[imin(j, p.M - 1)] : 0.f;
    bias[j] = (j < p.M && mv == 0.f) ? 0.f : NEG_INF;
  }
}

// Key mask of batch b into registers without a value select (a select right after a load would make the
// compiler wait for it there): clamped addresses, validity applied when the bias row is written.
__device__ __forceinline__ KeyMask key_mask_load_raw(const KArgs& p, int b) {
  KeyMask km;
#pragma unroll
  for (int u = 0; u < KB_UNROLL; ++u) km.v[u] = 0.f;
  if (p.mask) {
    const float* mk = p.mask + b * p.mask_sb;
#pragma unroll
    for (int u = 0; u < KB_UNROLL; ++u) km.v[u] = mk[imin(lane_id() + 64 * u, p.M - 1)];
  }
  return km;
}

// DROP: attention dropout on (keep <=> 16-bit uniform >= drop_thr). HAS_U: STE uniforms supplied by
// the caller (bit-exact parity path, fp32 compare as torch.bernoulli); otherwise 16-bit Philox
// uniforms u16 / 65536 (STE.py:13 draws u < p with p = clamp(expA, .01, .99)).
// One (b, h, 32-query block) item of the forward on the wave's LDS images at lds (zero_images: first use of the
// images; later items find rows past M holding earlier items' finite data, which their -inf key bias masks).
template <int D, int KPH, bool DENSE, bool HAS_U, bool DROP, bool BF>
__device__ __forceinline__ void attn_fwd_item(const KArgs& p, float* __restrict__ lds, int bh, int qb, bool zero_images) {
  using LY = AttnFwdLds<D, KPH>;
  constexpr int DT = D / 32, NS = D / 2, DP = LY::DP, KP = LY::KP;
  constexpr bool SWZ = LY::SWZ;
  constexpr int KPN = KP > 0 ? KP : 16;  // T image width (unused when DENSE)
  const uint32_t Kl = lds_offset(lds), Vl = Kl + LY::VOFF, Tl = Kl + LY::TOFF;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const int b = bh / p.H, hd = bh % p.H;
  const int i = qb * 32 + c;
  const bool iv = i < p.N;
  const int ic = imin(i, p.N - 1);
  const int kld = (int)p.k_sn * 4, vld = (int)p.v_sn * 4;
  // SWZ descriptors span exactly the M valid rows (rows >= M are out of range, never fetched)
  const __amdgpu_buffer_rsrc_t kr = make_rsrc(p.K + b * p.k_sb + hd * p.k_sh, SWZ ? (p.M - 1) * kld + D * 4 : 0x7fffffff);
  const __amdgpu_buffer_rsrc_t vr = make_rsrc(p.V + b * p.v_sb + hd * p.v_sh, SWZ ? (p.M - 1) * vld + D * 4 : 0x7fffffff);
  const __amdgpu_buffer_rsrc_t tr = make_rsrc(DENSE ? p.K : p.T + (int64_t)bh * p.M * p.kp, p.M * p.kp * 4);
  if (zero_images) {
    if constexpr (SWZ) lds_zero<(2 * LY::KV_BYTES + LY::T_BYTES) / 4>(lds);
    else if constexpr (!DENSE) lds_zero<LY::T_BYTES / 4>(lds + LY::TOFF / 4);
  }
  const DmaPat kpat = dma_pat(SW_ROW, kld), vpat = dma_pat(SW_COL, vld);
#define CSA_ISSUE_FWD(row0)                                   \
  do {                                                        \
    if constexpr (SWZ) {                                      \
      dma64(Kl, kr, kpat, kld, (row0));               \
      dma64(Vl, vr, vpat, vld, (row0));               \
    } else {                                                  \
      dma_rows<D>(Kl, kr, kld, (row0), p.M);                  \
      dma_rows<D>(Vl, vr, vld, (row0), p.M);                  \
    }                                                         \
    if constexpr (!DENSE) dma_narrow(Tl, tr, (row0), KPN); \
  } while (0)
  // Prologue: nothing waits on a load before the first tile (s_memtime stamps, profiles/r05_stamps.txt: a prologue
  // that scaled qh and selected the query rows right after their loads waited out one memory latency before
  // issuing tile 0's DMA and another at the first tile, 19% of a wave's life). Issue order (vmcnt retires in
  // issue order): the key mask, whose bias row is written as soon as it lands while the rest is in flight; tile 0's
  // images; the query operands. Query rows past N read row N-1 (finite; their results are never stored).
  const KeyMask km = key_mask_load_raw(p, b);
  CSA_ISSUE_FWD(0);
  float q[NS];
  load_run<NS>(q, p.Q + b * p.q_sb + hd * p.q_sh + (int64_t)ic * p.q_sn + h * NS, true);
  float qh[KPH > 0 ? KPH : 1];
  if constexpr (!DENSE) load_run<KPH>(qh, p.Qh + ((int64_t)bh * p.N + ic) * p.kp + h * KPH, true);
  // Philox STE compares u16 < 65536 p: E is computed 65536x scaled (qh scaled by a power of two, exact, at tile 0)
  constexpr float ESC = HAS_U ? 1.f : 65536.f;
  key_bias_store(lds + LY::BOFF / 4, p, b, km);
  const int kbase = SWZ ? row_base64(c, h) : 4 * (c * DP + NS * h);
  const int tbase = DENSE ? 0 : LY::TOFF + narrow_base<KPN>(c, (KPH / 4) * h);
  int vb[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) vb[t] = LY::VOFF + (SWZ ? col_base64(t, c, h) : 4 * (32 * t + c) + 16 * DP * h);
  const uint32_t qmask = (uint32_t)__ballot(iv);  // valid query bits of a packed word
  // Loop-invariant scalars the tile loop uses, pinned in VGPRs (the opaque asm): the SGPR file is full in the
  // dropout variant, and left to the compiler they spill to VGPR lanes and are re-read (v_readlane) every tile.
  typedef __attribute__((address_space(1))) uint32_t gu32;  // global (not flat) stores
  gu32* abp = (gu32*)(p.Abits + ((int64_t)bh * p.NQB + qb) * p.Mpad + c);  // this lane's packed-word columns
  gu32* rbp = (gu32*)(p.Rbits + ((int64_t)bh * p.NQB + qb) * p.Mpad + c);
  uint32_t ctr_bh = (uint32_t)bh, ctr_ste = (RNG_STE << 28) ^ p.off, ctr_drop = (RNG_ATTN_DROP << 28) ^ p.off;
  uint32_t drop_thr = p.drop_thr;
  float scale = p.scale, e_lo = 0.01f * ESC, e_hi = 0.99f * ESC;
  asm volatile("" : "+v"(abp), "+v"(rbp), "+v"(ctr_bh), "+v"(ctr_ste), "+v"(ctr_drop), "+v"(drop_thr));
  asm volatile("" : "+v"(scale), "+v"(e_lo), "+v"(e_hi));
  float m_run = NEG_INF, zp = 0.f, zgp = 0.f;
  f32x16 o[DT];
#pragma unroll
  for (int t = 0; t < DT; ++t) o[t] = zero16();
  uint32_t cntl = 0;
  // Key tiles whose every key is masked (padded ASTs, sbm_attn.py:61) contribute exactly nothing to the softmax sums
  // and to X (their P is 0), so after the live tiles (ascending, the softmax order of a full pass) they run a light
  // body: expA, sampling and the bit words only (the graph counts padded positions, sbm_attn.py:64, and the backward's
  // STE term reads them), no K / V images, no S or PV products. Tile 0, whose images the prologue loads, is always
  // processed as live. More than 64 key tiles: every tile live.
  uint64_t rem_live = 0, rem_dead = 0, dead = 0;
  const bool tmask = p.NKB <= 64;
  int kt = 0;
  // Philox words of tile kt (they depend only on (query, tile, head))
  auto philox_tile = [&](int kt_, u32x4 (&r_ste)[2], u32x4 (&r_drop)[2], bool with_drop = true) {
    uint32_t sk0 = p.seed_lo, sk1 = p.seed_hi;  // opaque per tile: round keys are not held across the loop
    asm volatile("" : "+s"(sk0), "+s"(sk1));
#pragma unroll
    for (int gp = 0; gp < 2; ++gp) {
      if constexpr (!DENSE && !HAS_U)
        r_ste[gp] = philox4x32(u32x4{(uint32_t)i, (uint32_t)(8 * kt_ + 4 * gp + h), ctr_bh, ctr_ste}, sk0, sk1);
      if constexpr (DROP)
        if (with_drop)
          r_drop[gp] = philox4x32(u32x4{(uint32_t)i, (uint32_t)(8 * kt_ + 4 * gp + h), ctr_bh, ctr_drop}, sk0, sk1);
    }
  };
  // expA^T = T Qh^T (sbm_attn.py:55) of the tile in the T image
  auto echain = [&](int toff) {  // toff: the T image's offset from LY::TOFF (a dead-tile slot)
    f32x16 eacc = zero16();
    if constexpr (!DENSE) {
#pragma unroll
      for (int j = 0; j < KPH / 4; ++j) {
        const f32x4 tv = lds_f4(lds, (tbase + toff) ^ (16 * j));
#pragma unroll
        for (int e = 0; e < 4; ++e) eacc = mfma(tv[e], qh[4 * j + e], eacc);
      }
    }
    return eacc;
  };
  uint32_t myA = 0u, myR = 0u;
  // the sampled graph and the dropout keep mask of a tile (16 + 16 compares; pack_bits makes the bit words)
  auto sample_all = [&](int j0_, const f32x16& eacc, const u32x4 (&r_ste)[2], const u32x4 (&r_drop)[2],
                        bool (&av)[16], bool (&keep)[16]) {
#pragma unroll
    for (int r = 0; r < 16; ++r) { av[r] = true; keep[r] = true; }
    if constexpr (!DENSE) {
      if constexpr (HAS_U) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int j = j0_ + crow(r, h);
          const float v = p.U[((int64_t)bh * p.N + ic) * p.M + imin(j, p.M - 1)];
          const float uu = (iv && j < p.M) ? v : 2.f;
          av[r] = uu < fminf(fmaxf(eacc[r], 0.01f), 0.99f);  // STE.py:11-13
        }
      } else {
#pragma unroll
        for (int r = 0; r < 16; ++r) av[r] = (float)u16_of(r_ste[r >> 3], r & 7) < __builtin_amdgcn_fmed3f(eacc[r], e_lo, e_hi);
      }
    }
    if constexpr (DROP)
#pragma unroll
      for (int r = 0; r < 16; ++r) keep[r] = u16_of(r_drop[r >> 3], r & 7) >= drop_thr;
  };
  // the tile's bit words out, its sampled edges counted
  auto store_abits = [&](int j0_) {
    if constexpr (!DENSE) {
      const uint32_t aw = j0_ + c < p.M ? myA : 0u;  // keys past M: no sampled edge (k_attn_bwd_qg reads dead tiles' words)
      if (h == 0) abp[j0_] = aw;
      cntl += __popc(aw & qmask);  // sampled edges inside [0,N) x [0,M)
    }
  };
  auto store_bits = [&](int j0_) {
    store_abits(j0_);
    if constexpr (DROP) if (h == 0) rbp[j0_] = myR;
  };
  // the live tile after the current one (-1: none), taken off the remaining set
  auto next_live = [&](int kt_) {
    if (!tmask) return kt_ + 1 < p.NKB ? kt_ + 1 : -1;
    if (rem_live) {
      const int nx = __builtin_ctzll(rem_live);
      rem_live &= rem_live - 1;
      return nx;
    }
    return -1;
  };
  for (int idx = 0; idx < p.NKB; ++idx) {
    wait_vm_all();  // tile kt's K/V/T images (at idx = 0 also the query operands) have landed
    if (idx == 0) {
      if constexpr (!DENSE && !HAS_U)
#pragma unroll
        for (int e = 0; e < KPH; ++e) qh[e] *= ESC;
      if (tmask) {  // dead tiles from the key bias row (written before the loop)
        for (int u = 0; 2 * u < p.NKB; ++u) {
          const int jj = imin(64 * u + lane, p.NKB * 32 - 1);  // (a missing odd tile reads the last key)
          const uint64_t bl = __builtin_amdgcn_ballot_w64(lds_f1(lds, LY::BOFF + 4 * jj) == NEG_INF);
          if ((uint32_t)bl == 0xffffffffu) dead |= 1ull << (2 * u);
          if ((uint32_t)(bl >> 32) == 0xffffffffu && 2 * u + 1 < p.NKB) dead |= 1ull << (2 * u + 1);
        }
        const uint64_t all = p.NKB == 64 ? ~0ull : (1ull << p.NKB) - 1;
        dead &= ~1ull;  // tile 0 runs as live (its images are loaded)
        rem_live = all & ~dead & ~1ull;
        rem_dead = dead;
        if (hd == 0 && qb == 0 && lane == 0) p.tdead[b] = dead;  // for the backward's query side
      }
    }
    const int j0 = kt * 32;
    u32x4 r_ste[2], r_drop[2];
    float w[16];
    {
      // the tile's Philox words depend only on (query, tile, head): computed first, so their VALU work can
      // interleave with the S / expA MFMA chains below instead of waiting behind them
      philox_tile(kt, r_ste, r_drop);
      // S^T = K Q^T : A operand = K rows from the image (row c, lin-perm chunks of half h)
      f32x16 sacc = zero16();
      if constexpr (BF) {
#pragma unroll
        for (int j2 = 0; j2 < NS / 8; ++j2) {
          const f32x4 k0 = lds_f4(lds, SWZ ? (kbase ^ (32 * j2)) : kbase + 32 * j2);
          const f32x4 k1 = lds_f4(lds, SWZ ? (kbase ^ (32 * j2 + 16)) : kbase + 32 * j2 + 16);
          sacc = mfma_bf(pack8(k0, k1), pack8(&q[8 * j2]), sacc);
        }
      } else {
#pragma unroll
        for (int j = 0; j < NS / 4; ++j) {
          const f32x4 kv = lds_f4(lds, SWZ ? (kbase ^ (16 * j)) : kbase + 16 * j);
#pragma unroll
          for (int e = 0; e < 4; ++e) sacc = mfma(kv[e], q[4 * j + e], sacc);
        }
      }
      const f32x16 eacc = echain(0);
      // V^T operand values for this tile's PV: lane (d = 32t + c) reads V[key crow(r,h)][d]
      float vt[DT][16];
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) vt[t][r] = lds_f1(lds, vb[t] + (SWZ ? 256 * crow(r, 0) : 4 * DP * crow(r, 0)));
      f32x4 bz[4];  // key bias of registers 4g..4g+3 (keys j0 + 8g + 4h + e)
#pragma unroll
      for (int g = 0; g < 4; ++g) bz[g] = lds_f4(lds, LY::BOFF + 4 * (j0 + 8 * g + 4 * h));
      // all of tile kt is in registers: start the next tile's DMA (overlaps the softmax and PV below)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const int nx = next_live(kt);
      if (nx >= 0) CSA_ISSUE_FWD(nx * 32);
      float s[16];
      float tmax = NEG_INF;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        s[r] = fmaf(sacc[r], scale, bz[r >> 2][r & 3]);
        tmax = fmaxf(tmax, s[r]);
      }
      bool av[16], keep[16];
      sample_all(j0, eacc, r_ste, r_drop, av, keep);
      if constexpr (!DENSE) myA = pack_bits(av);
      if constexpr (DROP) myR = pack_bits(keep);
      store_bits(j0);
      // online softmax update (exp(-inf - m) = 0 covers masked keys; m_use keeps an all-masked prefix finite)
      tmax = xhalf_max(tmax);
      const float m_new = fmaxf(m_run, tmax);
      const float m_use = (m_new == NEG_INF) ? 0.f : m_new;
      const float alpha = __expf(m_run - m_use);
      zp *= alpha;
      zgp *= alpha;
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) o[t][r] *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float e = __expf(s[r] - m_use);
        zp += e;
        const float wa = av[r] ? e : 0.f;
        zgp += wa;
        w[r] = keep[r] ? wa : 0.f;
      }
      m_run = m_new;
      // O^T += V^T W^T (keys beyond M carry w = 0)
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
      if (nx < 0) break;
      kt = nx;
    }
  }
  // Dead tiles (every key masked, after the live ones): P = 0, so no softmax / PV work, and no dropout bits (nothing
  // reads the keep bits of a masked key); expA, the STE draws and the graph's bit words only. Their T images come in
  // chunks of up to DCH into the free K / V / T image space, with one wait per chunk: one tile at a time, each tile
  // would wait out a memory round trip for a few hundred cycles of work.
  if constexpr (!DENSE) {
    constexpr int DCH0 = (LY::TOFF + LY::T_BYTES - LY::KOFF) / LY::T_BYTES, DCH = DCH0 < 8 ? DCH0 : 8;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    while (rem_dead) {
      int kts[DCH];
#pragma unroll
      for (int u = 0; u < DCH; ++u) {
        kts[u] = -1;
        if (rem_dead) {
          kts[u] = __builtin_ctzll(rem_dead);
          rem_dead &= rem_dead - 1;
          dma_narrow(Kl + u * LY::T_BYTES, tr, kts[u] * 32, KPN);
        }
      }
      wait_vm_all();
#pragma unroll
      for (int u = 0; u < DCH; ++u) {
        if (kts[u] < 0) break;
        const int j0 = kts[u] * 32;
        u32x4 r_ste[2], r_drop[2];
        philox_tile(kts[u], r_ste, r_drop, false);
        const f32x16 eacc = echain(u * LY::T_BYTES - LY::TOFF);
        bool av[16], keep[16];
        sample_all(j0, eacc, r_ste, r_drop, av, keep);
        myA = pack_bits(av);
        store_abits(j0);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the chunk's images read out before the next one lands
    }
  }
  const float Z = xhalf_sum(zp), Zg = xhalf_sum(zgp);
  const float n = Zg / Z;
  const float Dn = fmaxf(n, NORM_EPS);
  const float dscale = DROP ? 1.f / (1.f - p.attn_p) : 1.f;  // dropout's 1/(1-p), applied once per row
  const float inv = dscale / (Z * Dn);
  if (iv) {
    float* xo = p.X + b * p.x_sb + hd * p.x_sh + (int64_t)i * p.x_sn;
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      f32x16 v = o[t];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] *= inv;
      o[t] = v;
    }
    store_rows<DT>(xo, D, D, o, true);
    if (h == 0) {
      f32x4 st;
      st[0] = m_run + logf(Z);   // lse: P = exp(s - lse)
      st[1] = 1.f / Dn;          // 1 / max(n, eps)
      st[2] = (n >= NORM_EPS) ? 1.f : 0.f;
      st[3] = 0.f;               // gamma, filled by the backward
      *reinterpret_cast<f32x4*>(p.stats + ((int64_t)bh * p.N + i) * 4) = st;
    }
  }
#undef CSA_ISSUE_FWD
  if constexpr (!DENSE) {
    cntl = (h == 0) ? cntl : 0u;
#pragma unroll
    for (int o2 = 32; o2 >= 1; o2 >>= 1) cntl += __shfl_xor(cntl, o2, 64);
    // one plain store per wave, summed by k_sparsity_finish (10240 atomic adds on the 8 counters of one cache line
    // serialised in that L2 channel: 11 us of the headline forward, 64 us with 4 of 5 key tiles masked,
    // profiles/r06_ab_sparsity_atomic.txt)
    if (lane == 0) p.cnt[(int64_t)bh * p.NQB + qb] = cntl;
  }
}

template <int D, int KPH, bool DENSE, bool HAS_U, bool DROP, bool BF>
__global__ __launch_bounds__(64, (D <= 64 && KPH <= 16) ? 2 : 1) void k_attn_fwd(const KArgs p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const BhBlock xb = xcd_block(p.NQB, p.B * p.H);
  if (!xb.valid) return;
  attn_fwd_item<D, KPH, DENSE, HAS_U, DROP, BF>(p, lds, xb.bh, xb.blk, true);
}

// one workgroup per head: the head's B * NQB per-wave counts summed exactly (integers: any order gives the same total)
__global__ __launch_bounds__(256) void k_sparsity_finish(const uint32_t* __restrict__ cnt, float* __restrict__ sp,
                                                         int H, int B, int NQB, float bnm) {
  __shared__ unsigned long long red[4];
  const int hd = blockIdx.x, t = threadIdx.x;
  unsigned long long s = 0;
  for (int e = t; e < B * NQB; e += 256) s += cnt[((int64_t)(e / NQB) * H + hd) * NQB + e % NQB];
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((t & 63) == 0) red[t >> 6] = s;
  __syncthreads();
  if (t == 0) sp[hd] = (float)((red[0] + red[1]) + (red[2] + red[3])) / bnm;  // torch.sum(graph)/(b*n*m), sbm_attn.py:64
}

// ------------------------------------------------------------------------------------
// F4: optional maps: attn (B,H,N,M) and graph (B,H,N,M) fp32, S orientation (key = lane)
// ------------------------------------------------------------------------------------
template <int D, bool DENSE>
__global__ __launch_bounds__(64) void k_maps(const KArgs p, float* __restrict__ graph, float* __restrict__ attn) {
  constexpr int NS = D / 2;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const BhBlock xb = xcd_block(p.NQB, p.B * p.H);
  if (!xb.valid) return;
  const int qb = xb.blk, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const int i0 = qb * 32;
  float q[NS];
  load_run<NS>(q, p.Q + b * p.q_sb + hd * p.q_sh + (int64_t)imin(i0 + c, p.N - 1) * p.q_sn + h * NS, i0 + c < p.N);
  float lse[16], invD[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int ii = imin(i0 + crow(r, h), p.N - 1);
    lse[r] = p.stats[((int64_t)bh * p.N + ii) * 4 + 0];
    invD[r] = p.stats[((int64_t)bh * p.N + ii) * 4 + 1];
  }
  const float* kb = p.K + b * p.k_sb + hd * p.k_sh;
  const float* mk = p.mask ? p.mask + b * p.mask_sb : nullptr;
  for (int kt = 0; kt < p.NKB; ++kt) {
    const int j = kt * 32 + c;
    const bool jv = j < p.M;
    const int jc = imin(j, p.M - 1);
    float kr[NS];
    load_run<NS>(kr, kb + (int64_t)jc * p.k_sn + h * NS, jv);
    f32x16 sacc = zero16();
#pragma unroll
    for (int s = 0; s < NS; ++s) sacc = mfma(q[s], kr[s], sacc);
    const float mval = mk ? mk[jc] : 0.f;
    const bool kval = jv && mval == 0.f;
    const uint32_t word = DENSE ? 0xffffffffu : p.Abits[((int64_t)bh * p.NQB + qb) * p.Mpad + j];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ii = i0 + crow(r, h);
      if (ii < p.N && jv) {
        const bool a = (word >> crow(r, h)) & 1u;
        const float pv = kval ? __expf(sacc[r] * p.scale - lse[r]) : 0.f;
        const int64_t o = ((int64_t)bh * p.N + ii) * p.M + j;
        if (attn) attn[o] = a ? pv * invD[r] : 0.f;
        if (graph) graph[o] = a ? 1.f : 0.f;
      }
    }
  }
}

// gx[b,h,i] = sum_j dattn[b,h,i,j] * attn[b,h,i,j] for an upstream gradient of the returned attn map
// (sbm_attn.py:62 F.normalize backward needs sum_j G_ij attn_ij over the TOTAL gradient G of attn; the
// dX V^T part is rowsum(dX * X), computed by k_attn_rowprep). Recomputes attn like k_maps (S orientation:
// keys on lanes, queries in registers), one wave per (b, h, 32 queries); lane sums, then one reduction.
template <int D, bool DENSE>
__global__ __launch_bounds__(64) void k_attn_gx(const KArgs p) {
  constexpr int NS = D / 2;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const BhBlock xb = xcd_block(p.NQB, p.B * p.H);
  if (!xb.valid) return;
  const int qb = xb.blk, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const int i0 = qb * 32;
  float q[NS];
  load_run<NS>(q, p.Q + b * p.q_sb + hd * p.q_sh + (int64_t)imin(i0 + c, p.N - 1) * p.q_sn + h * NS, i0 + c < p.N);
  float lse[16], invD[16], acc[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int ii = imin(i0 + crow(r, h), p.N - 1);
    lse[r] = p.stats[((int64_t)bh * p.N + ii) * 4 + 0];
    invD[r] = p.stats[((int64_t)bh * p.N + ii) * 4 + 1];
    acc[r] = 0.f;
  }
  const float* kb = p.K + b * p.k_sb + hd * p.k_sh;
  const float* mk = p.mask ? p.mask + b * p.mask_sb : nullptr;
  for (int kt = 0; kt < p.NKB; ++kt) {
    const int j = kt * 32 + c;
    const bool jv = j < p.M;
    const int jc = imin(j, p.M - 1);
    float kr[NS];
    load_run<NS>(kr, kb + (int64_t)jc * p.k_sn + h * NS, jv);
    f32x16 sacc = zero16();
#pragma unroll
    for (int s2 = 0; s2 < NS; ++s2) sacc = mfma(q[s2], kr[s2], sacc);
    const float mval = mk ? mk[jc] : 0.f;
    const bool kval = jv && mval == 0.f;
    const uint32_t word = DENSE ? 0xffffffffu : p.Abits[((int64_t)bh * p.NQB + qb) * p.Mpad + j];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ii = i0 + crow(r, h);
      const bool in = ii < p.N && jv;
      const bool a = (word >> crow(r, h)) & 1u;
      const float pv = kval ? __expf(sacc[r] * p.scale - lse[r]) : 0.f;
      const float at = (a && in) ? pv * invD[r] : 0.f;
      acc[r] = fmaf(ldz(p.dattn, ((int64_t)bh * p.N + imin(ii, p.N - 1)) * p.M + jc, INT64_MAX, in), at, acc[r]);
    }
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float v = half_sum32(acc[r]);
    const int ii = i0 + crow(r, h);
    if (c == 0 && ii < p.N) p.gx[(int64_t)bh * p.N + ii] = v;
  }
}

// Per query row of the backward (sbm_attn.py:59-63 autograd, oracle/closed_form.py), the row constants of
// k_attn_bwd_kv's elementwise backward, so that per element it runs
//   P = exp2(s log2e / sqrt(d) + c0 + kbias), dM = (keep ? dP : 0) u + v (the dM of an edge, A = 1),
//   ds = ((A ? dM : 0) - rho) P / sqrt(d), G = A ? hardtanh(dM P + csp) : 0, attw = (A & keep) ? P u : 0
// with gamma = rowsum(dX * X) (+ sum_j dattn attn, k_attn_gx) the F.normalize term and n = Zg / Z the row's
// L1 norm of softmax * graph:
//   c0 = -lse log2e, u = dscale / max(n, eps), v = -[n >= eps] gamma / max(n, eps), rho = [n < eps] gamma.
// Rows past N (up to the query block's end) get c0 = -inf, u = v = rho = 0: P = 0, so they add nothing.
// LPR lanes per row (16 for d = 64, 32 for d = 96), one 16-B chunk of dX and of X each: a wave-instruction
// reads whole rows (1 KiB contiguous at d = 64) instead of 64 lanes each on its own 128-B line; the dot
// product's partial sums meet by lane shuffles, and the row's first lane writes its record. A wave covers
// RPW rows (4 instructions per operand in flight). HBM-bound: 2 x 4d B per row.
template <int D>
__global__ __launch_bounds__(256) void k_attn_rowprep(const KArgs p) {
  constexpr int CPR = D / 4, LPR = CPR <= 16 ? 16 : 32, RPI = 64 / LPR, RPW = 4 * RPI;
  const int lane = lane_id(), sub = lane % LPR;
  const int64_t NP = (int64_t)p.NQB * 32, total = (int64_t)p.B * p.H * NP;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) * RPW + lane / LPR;
  float part[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int64_t rc = r0 + u * RPI < total ? r0 + u * RPI : total - 1;
    const int i = (int)(rc % NP), bh = (int)(rc / NP), b = bh / p.H, hd = bh % p.H;
    const bool ld = i < p.N && sub < CPR;
    const int ic = imin(i, p.N - 1), ch = imin(sub, CPR - 1);
    const f32x4 dx = *reinterpret_cast<const f32x4*>(p.dX + b * p.dx_sb + hd * p.dx_sh + (int64_t)ic * p.dx_sn + 4 * ch);
    const f32x4 xr = *reinterpret_cast<const f32x4*>(p.X + b * p.x_sb + hd * p.x_sh + (int64_t)ic * p.x_sn + 4 * ch);
    const float v = fmaf(dx[0], xr[0], fmaf(dx[1], xr[1], fmaf(dx[2], xr[2], dx[3] * xr[3])));
    part[u] = ld ? v : 0.f;
  }
  const float dscale = p.attn_p > 0.f ? 1.f / (1.f - p.attn_p) : 1.f;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    float g = part[u];
#pragma unroll
    for (int o = 1; o < LPR; o <<= 1) g += __shfl_xor(g, o, 64);
    const int64_t row = r0 + u * RPI;
    if (sub == 0 && row < total) {
      const int i = (int)(row % NP), bh = (int)(row / NP);
      const bool iv = i < p.N;
      const int ic = imin(i, p.N - 1);
      const f32x4 st = *reinterpret_cast<const f32x4*>(p.stats + ((int64_t)bh * p.N + ic) * 4);  // lse, 1/D, [n>=eps]
      float gamma = g;
      if (p.dattn) gamma += p.gx[(int64_t)bh * p.N + ic];
      f32x4 rec;
      rec[0] = iv ? -st[0] * LOG2E : NEG_INF;
      rec[1] = iv ? dscale * st[1] : 0.f;
      rec[2] = (iv && st[2] != 0.f) ? -gamma * st[1] : 0.f;
      rec[3] = (iv && st[2] == 0.f) ? gamma : 0.f;
      *reinterpret_cast<f32x4*>(p.brow + row * 4) = rec;
    }
  }
}

// ------------------------------------------------------------------------------------
// Backward elementwise core for one (query i, key j) element (see oracle/closed_form.py)
// ------------------------------------------------------------------------------------
struct Elem { float ds, g, attw; };

// kbias: 0 for a valid key, -inf for a padded one (P = exp(s * scale + kbias - lse) = 0). Branch-free:
// elements outside [0,N) x [0,M) are computed from finite stand-in operands and selected to zero.
__device__ __forceinline__ Elem bwd_elem(float s_raw, float kbias, float dpp, bool a, bool keep, bool inside,
                                         float lse, float invD, float big, float gamma, float scale, float dscale,
                                         float csp, float dgr, float dam) {
  Elem r;
  const float P = __expf(fmaf(s_raw, scale, kbias) - lse);
  const float rm = keep ? dscale : 0.f;
  const float dattn = dpp * rm + dam;  // dropout backward of dX V^T, plus the attn map's own gradient
  const bool mpos = a && (P > 0.f);
  const float dM = (dattn - ((big != 0.f && mpos) ? gamma : 0.f)) * invD;
  const float dPm = a ? dM : 0.f;
  const float rho = (big != 0.f) ? 0.f : gamma;
  const bool ain = a && inside;
  r.ds = inside ? P * (dPm - rho) * scale : 0.f;
  const float dA = dM * P + csp + dgr;
  r.g = ain ? fminf(fmaxf(dA, -1.f), 1.f) : 0.f;  // STE.py:19 hardtanh(A * grad)
  r.attw = ain ? P * invD * rm : 0.f;              // dropout(attn) weight for dV
  return r;
}

// ------------------------------------------------------------------------------------
// B2/B1 shared LDS layout
// ------------------------------------------------------------------------------------
template <int D, int KPH>
struct AttnBwdShape {
  static constexpr bool SWZ = (D == 64);  // x4 DMA into SW_BOTH / SW_ROW swizzled tiles (else padded rows)
  static constexpr int DP = D + 4, KP = 2 * KPH, KPN = KP > 0 ? KP : 16;
  static constexpr int KT = KPH == 0 ? 0 : (KP <= 32 ? 1 : KP / 32), KTA = KT > 0 ? KT : 1;
  static constexpr int IMG = SWZ ? 32 * 64 * 4 : 32 * DP * 4;  // one 32 x D image
  static constexpr int NIMG = 32 * KPN * 4;                    // one 32 x KP narrow image
  // bwd_qg: K | T
  static constexpr int GK = 0, GT = IMG;
  static constexpr size_t G_BYTES = (size_t)IMG + NIMG;
  // bwd_qr: K | V | T | key bias row (Mpad floats)
  static constexpr int QK = 0, QV = IMG, QT = 2 * IMG, QB = 2 * IMG + NIMG;
  static size_t r_bytes(int Mpad) { return (size_t)QB + 4 * (size_t)Mpad; }
  // bwd_kv: Q | dX | Qh | row constants (32 rows x 4, k_attn_rowprep)
  static constexpr int KQ = 0, KX = IMG, KH = 2 * IMG, KS = 2 * IMG + NIMG;
  static constexpr size_t KV_BYTES = (size_t)KS + 32 * 16;
};

// key bias row in LDS: 0 for a valid key, -inf for a padded one or one beyond M (sbm_attn.py:61)

// kp = 16 (k <= 16): the dQh / dT products run on mfma4b with the cluster index on the 16 lanes of a block
// instead of 32x32 tiles with 16 (of 32) padded cluster rows: half the MFMA cycles. Lane (c, h) feeds the
// blocks b = 2h + (c >> 4) with the operand values it holds anyway (row crow(r, h), its own column c); blocks
// b and b + 2 then hold the two lane halves' partial sums for columns 16 b .. 16 b + 15.
// Rows 16 b + (l & 15) (b = 0, 1) of a 32-row block, clusters 4 (l >> 4) .. + 3: the two halves added, stored
// as one f32x4 per lane and block (rows >= nrows are skipped).
__device__ __forceinline__ void store_mb4(float* __restrict__ out, int nrows, int kp, const f32x16& d) {
  const int l = lane_id(), rr = l & 15, cl = 4 * (l >> 4);
#pragma unroll
  for (int b = 0; b < 2; ++b) {
    const int row = 16 * b + rr;
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = d[4 * b + e] + d[8 + 4 * b + e];
    if (row < nrows) *reinterpret_cast<f32x4*>(out + (int64_t)row * kp + cl) = v;
  }
}

// ------------------------------------------------------------------------------------
// B2 (bf16 mode): per (b,h, query block), S^T orientation: recompute S = QK^T and dP = dX V^T on bf16 MFMA,
// the elementwise backward with the row constants of k_attn_rowprep (one record per lane: its query), then
// dQ (attention path) = ds K, dQh = G T. The round-3 design, kept where recomputing is cheaper than the
// k_attn_bwd_qg tile handoff (see bwd_handoff).
// ------------------------------------------------------------------------------------
// DG: an upstream gradient of the graph and / or attn output is present (p.dgraph, p.dattn)
template <int D, int KPH, bool DENSE, bool DROP, bool DG, bool BF>
__global__ __launch_bounds__(64, (D <= 64 && KPH <= 16) ? 2 : 1) void k_attn_bwd_qr(const KArgs p) {
  using SH = AttnBwdShape<D, KPH>;
  constexpr int DT = D / 32, NS = D / 2, DP = SH::DP, KP = SH::KP, KPN = SH::KPN, KTA = SH::KTA;
  constexpr bool SWZ = SH::SWZ;
  constexpr bool MB4 = !DENSE && KP == 16;  // dQh on mfma4b (store_mb4)
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const uint32_t L0 = lds_offset(lds), Kl = L0 + SH::QK, Vl = L0 + SH::QV, Tl = L0 + SH::QT;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const BhBlock xb = xcd_block(p.NQB, p.B * p.H);
  if (!xb.valid) return;
  const int qb = xb.blk, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const int i = qb * 32 + c;
  const bool iv = i < p.N;
  const int ic = imin(i, p.N - 1);
  const int kld = (int)p.k_sn * 4, vld = (int)p.v_sn * 4;
  const __amdgpu_buffer_rsrc_t kr = make_rsrc(p.K + b * p.k_sb + hd * p.k_sh, SWZ ? (p.M - 1) * kld + D * 4 : 0x7fffffff);
  const __amdgpu_buffer_rsrc_t vr = make_rsrc(p.V + b * p.v_sb + hd * p.v_sh, SWZ ? (p.M - 1) * vld + D * 4 : 0x7fffffff);
  const __amdgpu_buffer_rsrc_t tr = make_rsrc(DENSE ? p.K : p.T + (int64_t)bh * p.M * p.kp, p.M * p.kp * 4);
  // rows past M are never fetched: zero the images once so they only ever hold finite data
  if constexpr (SWZ) lds_zero<(2 * SH::IMG + SH::NIMG) / 4>(lds);
  else if constexpr (!DENSE) lds_zero<SH::NIMG / 4>(lds + SH::QT / 4);
  const DmaPat kpat = dma_pat(SW_BOTH, kld), vpat = dma_pat(SW_ROW, vld);
#define CSA_ISSUE_BQ(row0)                          \
  do {                                              \
    if constexpr (SWZ) {                            \
      dma64(Kl, kr, kpat, kld, (row0));             \
      dma64(Vl, vr, vpat, vld, (row0));             \
    } else {                                        \
      dma_rows<D>(Kl, kr, kld, (row0), p.M);        \
      dma_rows<D>(Vl, vr, vld, (row0), p.M);        \
    }                                               \
    if constexpr (!DENSE) dma_narrow(Tl, tr, (row0), KPN); \
  } while (0)
  const KeyMask km = key_mask_load(p, b);
  CSA_ISSUE_BQ(0);
  key_bias_store(lds + SH::QB / 4, p, b, km);
  const int64_t wrow = ((int64_t)bh * p.NQB + qb) * p.Mpad + c;
  uint32_t wAn = DENSE ? 0xffffffffu : p.Abits[wrow];
  uint32_t wRn = DROP ? p.Rbits[wrow] : 0xffffffffu;
  float q[NS], dx[NS];
  load_run<NS>(q, p.Q + b * p.q_sb + hd * p.q_sh + (int64_t)ic * p.q_sn + h * NS, iv);
  load_run<NS>(dx, p.dX + b * p.dx_sb + hd * p.dx_sh + (int64_t)ic * p.dx_sn + h * NS, iv);
  // this lane's query row constants (c0, u, v, rho); a query past N has c0 = -inf: P = 0
  const f32x4 rec = *reinterpret_cast<const f32x4*>(p.brow + ((int64_t)bh * p.NQB * 32 + i) * 4);
  const float csp = (!DENSE && p.dsp) ? p.dsp[hd] / ((float)p.B * (float)p.N * (float)p.M) : 0.f;
  const float c1 = p.scale * LOG2E;
  f32x16 dq[DT], dqh[KTA];
#pragma unroll
  for (int t = 0; t < DT; ++t) dq[t] = zero16();
#pragma unroll
  for (int t = 0; t < KTA; ++t) dqh[t] = zero16();
  for (int kt = 0; kt < p.NKB; ++kt) {
    int ln = threadIdx.x;  // opaque per iteration: keeps the per-row LDS addresses out of the prologue
    asm volatile("" : "+v"(ln));
    const int c = ln & 31, h = (ln >> 5) & 1;
    const int j0 = kt * 32;
    wait_vm_all();  // tile kt's K/V/T images and its bit words have landed
    const uint32_t wA = wAn, wR = wRn;
    f32x16 sacc = zero16(), dpacc = zero16();
    const int kb = SWZ ? row_base64(c, h, SW_BOTH) : 4 * (c * DP + NS * h);
    const int vb = SH::QV + (SWZ ? row_base64(c, h, SW_ROW) : 4 * (c * DP + NS * h));
    if constexpr (BF) {
#pragma unroll
      for (int j2 = 0; j2 < NS / 8; ++j2) {
        const f32x4 k0 = lds_f4(lds, SWZ ? (kb ^ (32 * j2)) : kb + 32 * j2);
        const f32x4 k1 = lds_f4(lds, SWZ ? (kb ^ (32 * j2 + 16)) : kb + 32 * j2 + 16);
        sacc = mfma_bf(pack8(k0, k1), pack8(&q[8 * j2]), sacc);
        const f32x4 v0 = lds_f4(lds, SWZ ? (vb ^ (32 * j2)) : vb + 32 * j2);
        const f32x4 v1 = lds_f4(lds, SWZ ? (vb ^ (32 * j2 + 16)) : vb + 32 * j2 + 16);
        dpacc = mfma_bf(pack8(v0, v1), pack8(&dx[8 * j2]), dpacc);
      }
    } else {
#pragma unroll
      for (int j = 0; j < NS / 4; ++j) {
        const f32x4 kv = lds_f4(lds, SWZ ? (kb ^ (16 * j)) : kb + 16 * j);
#pragma unroll
        for (int e = 0; e < 4; ++e) sacc = mfma(kv[e], q[4 * j + e], sacc);
      }
#pragma unroll
      for (int j = 0; j < NS / 4; ++j) {
        const f32x4 vv = lds_f4(lds, SWZ ? (vb ^ (16 * j)) : vb + 16 * j);
#pragma unroll
        for (int e = 0; e < 4; ++e) dpacc = mfma(vv[e], dx[4 * j + e], dpacc);
      }
    }
    // transposed operands of this tile's dQ / dQh products (lane d holds K[key crow(r,h)][d])
    float kT[DT][16], tT[KTA][16];
#pragma unroll
    for (int t = 0; t < DT; ++t) {
      const int tb = SWZ ? both_base64(t, c, h) : 4 * (32 * t + c) + 16 * DP * h;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        kT[t][r] = SWZ ? both_read(lds, tb, r, SH::QK) : lds_f1(lds, tb + 4 * DP * crow(r, 0));
    }
    if constexpr (MB4) {  // lane (c, h): T[key crow(r,h)][cluster c & 15]
#pragma unroll
      for (int r = 0; r < 16; ++r) tT[0][r] = lds_f1(lds, SH::QT + narrow_elem(crow(r, h), c & 15, KPN));
    } else if constexpr (!DENSE) {
#pragma unroll
      for (int at = 0; at < KTA; ++at)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float v = lds_f1(lds, SH::QT + narrow_elem(crow(r, h), imin(32 * at + c, KP - 1), KPN));
          tT[at][r] = (KP >= 32 || c < KP) ? v : 0.f;
        }
    }
    f32x4 bz[4];  // key bias of registers 4g..4g+3
#pragma unroll
    for (int g = 0; g < 4; ++g) bz[g] = lds_f4(lds, SH::QB + 4 * (j0 + 8 * g + 4 * h));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (kt + 1 < p.NKB) {  // tile kt+1 streams in under the elementwise work and the products below
      CSA_ISSUE_BQ(j0 + 32);
      if constexpr (!DENSE) wAn = p.Abits[wrow + j0 + 32];
      if constexpr (DROP) wRn = p.Rbits[wrow + j0 + 32];
    }
    // Elementwise backward (k_attn_rowprep's formulas). A key past M has P = 0 (bias -inf) and A = 0.
    float dsv[16], gv[16];
    const int nvk = p.M - j0 - 4 * h;  // key crow(r,h) = j0 + crow(r,0) + 4h is < M iff crow(r,0) < nvk
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int jj = crow(r, h), j = j0 + jj;
      const uint32_t a_w = DENSE ? 0xffffffffu : (uint32_t)__shfl((int)wA, jj, 64);
      const uint32_t r_w = DROP ? (uint32_t)__shfl((int)wR, jj, 64) : 0xffffffffu;
      const bool a = ((a_w >> c) & 1u) && crow(r, 0) < nvk;
      const bool kp = (r_w >> c) & 1u;
      const float P = __builtin_amdgcn_exp2f(fmaf(sacc[r], c1, bz[r >> 2][r & 3] + rec[0]));
      float dM = fmaf(kp ? dpacc[r] : 0.f, rec[1], rec[2]);
      float cg = csp;
      if constexpr (DG) {
        const bool inside = iv && (j < p.M);
        const int64_t me = ((int64_t)bh * p.N + ic) * p.M + imin(j, p.M - 1);
        if (p.dgraph) cg += ldz(p.dgraph, me, INT64_MAX, inside);
        if (p.dattn) dM = fmaf(ldz(p.dattn, me, INT64_MAX, inside), rec[1] * (1.f - p.attn_p), dM);
      }
      dsv[r] = ((a ? dM : 0.f) - rec[3]) * (P * p.scale);
      gv[r] = a ? __builtin_amdgcn_fmed3f(fmaf(dM, P, cg), -1.f, 1.f) : 0.f;  // STE.py:19 hardtanh(A * grad)
    }
    // dQ^T += K^T ds^T ; dQh^T += T^T G^T  (keys beyond M carry ds = G = 0)
    if constexpr (BF) {
      const bf16x8 s0 = pack8(&dsv[0]), s1 = pack8(&dsv[8]);
#pragma unroll
      for (int t = 0; t < DT; ++t) {
        dq[t] = mfma_bf(pack8(&kT[t][0]), s0, dq[t]);
        dq[t] = mfma_bf(pack8(&kT[t][8]), s1, dq[t]);
      }
    } else {
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) dq[t] = mfma(kT[t][r], dsv[r], dq[t]);
    }
    if constexpr (MB4) {
#pragma unroll
      for (int r = 0; r < 16; ++r) dqh[0] = mfma4b(tT[0][r], gv[r], dqh[0]);
    } else if constexpr (!DENSE) {
#pragma unroll
      for (int at = 0; at < KTA; ++at)
#pragma unroll
        for (int r = 0; r < 16; ++r) dqh[at] = mfma(tT[at][r], gv[r], dqh[at]);
    }
  }
#undef CSA_ISSUE_BQ
  store_rows<DT>(p.dQ + b * p.dq_sb + hd * p.dq_sh + (int64_t)i * p.dq_sn, D, D, dq, iv);
  if constexpr (MB4) store_mb4(p.dQh + ((int64_t)bh * p.N + qb * 32) * p.kp, p.N - qb * 32, p.kp, dqh[0]);
  else if constexpr (!DENSE) store_rows<KTA>(p.dQh + ((int64_t)bh * p.N + i) * p.kp, p.kp, p.kp, dqh, iv);
}

// ------------------------------------------------------------------------------------
// B2: per (b,h, query block), S^T orientation (keys = accumulator K-steps, queries = lanes):
//   dQ (attention path) = ds K, dQh = G T
// from the ds / G tiles k_attn_bwd_kv computed in S orientation (Layout::w_dsg, [key][query] per tile), so
// neither S = QK^T nor dP = dX V^T is recomputed here and the elementwise backward runs once per element.
// Lane (c, h) reads its query's 16 values of a tile (keys crow(r,h)) with coalesced dword loads; the K tile
// (SW_COL image: column reads only) and T tile arrive by LDS-DMA. The kernel streams 8 KB of ds / G per
// tile from HBM against 48 MFMAs, so it runs four waves per SIMD (d = 64, k <= 16: <= 128 VGPRs, 10 KB of
// LDS per wave): the ds / G registers are refilled right behind the MFMAs that read them and the K / T
// operands are read from LDS just before their MFMAs, and the other waves' MFMAs cover the load latency.
// ------------------------------------------------------------------------------------
template <int D, int KPH, bool DENSE, bool BF, bool W1>
__global__ __launch_bounds__(64, (D <= 64 && KPH <= 8) ? 4 : 2) void k_attn_bwd_qg(const KArgs p) {
  using SH = AttnBwdShape<D, KPH>;
  constexpr int DT = D / 32, DP = SH::DP, KP = SH::KP, KPN = SH::KPN, KTA = SH::KTA;
  constexpr bool SWZ = SH::SWZ;
  constexpr bool MB4 = !DENSE && KP == 16;  // dQh on mfma4b (store_mb4)
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const uint32_t L0 = lds_offset(lds), Kl = L0 + SH::GK, Tl = L0 + SH::GT;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const BhBlock xb = xcd_block(p.NQB, p.B * p.H);
  if (!xb.valid) return;
  const int qb = xb.blk, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const int i = qb * 32 + c;
  const bool iv = i < p.N;
  const int kld = (int)p.k_sn * 4;
  const __amdgpu_buffer_rsrc_t kr = make_rsrc(p.K + b * p.k_sb + hd * p.k_sh, SWZ ? (p.M - 1) * kld + D * 4 : 0x7fffffff);
  const __amdgpu_buffer_rsrc_t tr = make_rsrc(DENSE ? p.K : p.T + (int64_t)bh * p.M * p.kp, p.M * p.kp * 4);
  // rows past M are never fetched: zero the images once so they only ever hold finite data (those keys carry
  // ds = G = 0 in the tiles)
  if constexpr (SWZ) lds_zero<(SH::IMG + SH::NIMG) / 4>(lds);
  else if constexpr (!DENSE) lds_zero<SH::NIMG / 4>(lds + SH::GT / 4);
  const DmaPat kpat = dma_pat(SW_COL, kld);
#define CSA_ISSUE_BQ(row0)                                  \
  do {                                                      \
    if constexpr (SWZ) dma64(Kl, kr, kpat, kld, (row0));    \
    else dma_rows<D>(Kl, kr, kld, (row0), p.M);             \
    if constexpr (!DENSE) dma_narrow(Tl, tr, (row0), KPN);  \
  } while (0)
  // element (key crow(r,h), query c) of tile kt: tb + kt * 1024 + 32 crow(r,h)
  const float* tb = p.dsg + ((int64_t)bh * p.NQB + qb) * p.NKB * 1024 + c;
  float dsv[16], gv[16];  // W1: dsv holds the tile's w values until the top of its iteration
  auto load_tile = [&](int kt) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      dsv[r] = tb[kt * 1024 + 32 * crow(r, h)];
      if constexpr (!DENSE && !W1) gv[r] = tb[p.gplane + kt * 1024 + 32 * crow(r, h)];
    }
  };
  // W1, a fully masked key tile: k_attn_bwd_kv stores no w tile for it (w = dM P = 0 on every element), so the
  // sampled bits come from the forward's bit words instead (word of key crow(r, h), bit = this lane's query: the
  // words of registers 4g .. 4g + 3 are keys 8g + 4h + 0..3, one 16-B broadcast load per half-wave), parked in dsv
  // until the top of the tile's iteration
  const uint32_t* abw = p.Abits + ((int64_t)bh * p.NQB + qb) * p.Mpad + 4 * h;
  auto load_bits = [&](int kt) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(abw + kt * 32 + 8 * g);
#pragma unroll
      for (int e = 0; e < 4; ++e) dsv[4 * g + e] = v[e];
    }
  };
  // W1: this lane's rho (k_attn_rowprep) and the STE term; ds is summed unscaled and dQ scaled at the end
  const float rho = W1 ? p.brow[(((int64_t)bh * p.NQB + qb) * 32 + c) * 4 + 3] : 0.f;
  const float csp = (W1 && p.dsp) ? p.dsp[hd] / ((float)p.B * (float)p.N * (float)p.M) : 0.f;
  // key tiles whose every key is masked (the forward's record): their ds is 0 (P = 0), so no dQ products and no K
  // image; the T image and the tile (its A bits carry the STE term into dQh) still stream in
  const uint64_t tdead = (p.mask && p.NKB <= 64) ? p.tdead[b] : 0ull;
  CSA_ISSUE_BQ(0);
  load_tile(0);
  f32x16 dq[DT], dqh[KTA];
#pragma unroll
  for (int t = 0; t < DT; ++t) dq[t] = zero16();
#pragma unroll
  for (int t = 0; t < KTA; ++t) dqh[t] = zero16();
  // the tile loop twice: without dead tiles (every unpadded batch: tdead is 0) the compiler folds the skips away and
  // the body stays one scheduling region
  if (tdead) {
    for (int kt = 0; kt < p.NKB; ++kt) {
      int ln = threadIdx.x;  // opaque per iteration: keeps the per-row LDS addresses out of the prologue
      asm volatile("" : "+v"(ln));
      const int c = ln & 31, h = (ln >> 5) & 1;
      const bool more = kt + 1 < p.NKB;
      wait_vm_all();  // tile kt's K / T images and ds / G values (dead: bit words) have landed
      if constexpr (W1) {  // k_attn_bwd_kv's expressions (W_NO_EDGE)
        if ((tdead >> kt) & 1ull) {  // STE term only: G = A ? hardtanh(csp) : 0
  #pragma unroll
          for (int r = 0; r < 16; ++r) {
            const bool a = (__float_as_uint(dsv[r]) >> c) & 1u;  // (the forward stores no bit for keys past M)
            gv[r] = a ? __builtin_amdgcn_fmed3f(0.f + csp, -1.f, 1.f) : 0.f;
            dsv[r] = 0.f;
          }
        } else {
  #pragma unroll
          for (int r = 0; r < 16; ++r) {
            const bool a = __float_as_uint(dsv[r]) != W_NO_EDGE;
            const float w = a ? dsv[r] : 0.f;
            gv[r] = a ? __builtin_amdgcn_fmed3f(w + csp, -1.f, 1.f) : 0.f;
            dsv[r] = w;
          }
          if (rho != 0.f) {  // rare: a degenerate row (n < eps) also takes -rho P from the second plane
  #pragma unroll
            for (int r = 0; r < 16; ++r) dsv[r] = fmaf(-rho, tb[p.gplane + kt * 1024 + 32 * crow(r, h)], dsv[r]);
          }
        }
      }
      // dQ^T += K^T ds^T (lane d holds K[key crow(r,h)][d], read from the SW_COL / padded image per K-step)
  #pragma unroll
      for (int t = 0; t < (((tdead >> kt) & 1ull) ? 0 : DT); ++t) {
        const int cb = SH::GK + (SWZ ? col_base64(t, c, h) : 4 * (32 * t + c) + 16 * DP * h);
        float kT[16];
  #pragma unroll
        for (int r = 0; r < 16; ++r) kT[r] = lds_f1(lds, cb + (SWZ ? 256 * crow(r, 0) : 4 * DP * crow(r, 0)));
        if constexpr (BF) {
          dq[t] = mfma_bf(pack8(&kT[0]), pack8(&dsv[0]), dq[t]);
          dq[t] = mfma_bf(pack8(&kT[8]), pack8(&dsv[8]), dq[t]);
        } else {
  #pragma unroll
          for (int r = 0; r < 16; ++r) dq[t] = mfma(kT[r], dsv[r], dq[t]);
        }
      }
      // dQh^T += T^T G^T
      if constexpr (MB4) {  // lane (c, h): T[key crow(r,h)][cluster c & 15]
        float tT[16];
  #pragma unroll
        for (int r = 0; r < 16; ++r) tT[r] = lds_f1(lds, SH::GT + narrow_elem(crow(r, h), c & 15, KPN));
  #pragma unroll
        for (int r = 0; r < 16; ++r) dqh[0] = mfma4b(tT[r], gv[r], dqh[0]);
      } else if constexpr (!DENSE) {
  #pragma unroll
        for (int at = 0; at < KTA; ++at) {
          float tT[16];
  #pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float v = lds_f1(lds, SH::GT + narrow_elem(crow(r, h), imin(32 * at + c, KP - 1), KPN));
            tT[r] = (KP >= 32 || c < KP) ? v : 0.f;
          }
  #pragma unroll
          for (int r = 0; r < 16; ++r) dqh[at] = mfma(tT[r], gv[r], dqh[at]);
        }
      }
      if (more) {  // images read out and ds / G consumed by the MFMAs above: tile kt+1 streams in
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if ((tdead >> (kt + 1)) & 1ull) {
          if constexpr (!DENSE) dma_narrow(Tl, tr, kt * 32 + 32, KPN);
          if constexpr (W1) load_bits(kt + 1);
          else load_tile(kt + 1);
        } else {
          CSA_ISSUE_BQ(kt * 32 + 32);
          load_tile(kt + 1);
        }
      }
    }
  } else {
    const uint64_t tdead = 0;
    for (int kt = 0; kt < p.NKB; ++kt) {
      int ln = threadIdx.x;  // opaque per iteration: keeps the per-row LDS addresses out of the prologue
      asm volatile("" : "+v"(ln));
      const int c = ln & 31, h = (ln >> 5) & 1;
      const bool more = kt + 1 < p.NKB;
      wait_vm_all();  // tile kt's K / T images and ds / G values (dead: bit words) have landed
      if constexpr (W1) {  // k_attn_bwd_kv's expressions (W_NO_EDGE)
        if ((tdead >> kt) & 1ull) {  // STE term only: G = A ? hardtanh(csp) : 0
  #pragma unroll
          for (int r = 0; r < 16; ++r) {
            const bool a = (__float_as_uint(dsv[r]) >> c) & 1u;  // (the forward stores no bit for keys past M)
            gv[r] = a ? __builtin_amdgcn_fmed3f(0.f + csp, -1.f, 1.f) : 0.f;
            dsv[r] = 0.f;
          }
        } else {
  #pragma unroll
          for (int r = 0; r < 16; ++r) {
            const bool a = __float_as_uint(dsv[r]) != W_NO_EDGE;
            const float w = a ? dsv[r] : 0.f;
            gv[r] = a ? __builtin_amdgcn_fmed3f(w + csp, -1.f, 1.f) : 0.f;
            dsv[r] = w;
          }
          if (rho != 0.f) {  // rare: a degenerate row (n < eps) also takes -rho P from the second plane
  #pragma unroll
            for (int r = 0; r < 16; ++r) dsv[r] = fmaf(-rho, tb[p.gplane + kt * 1024 + 32 * crow(r, h)], dsv[r]);
          }
        }
      }
      // dQ^T += K^T ds^T (lane d holds K[key crow(r,h)][d], read from the SW_COL / padded image per K-step)
  #pragma unroll
      for (int t = 0; t < (((tdead >> kt) & 1ull) ? 0 : DT); ++t) {
        const int cb = SH::GK + (SWZ ? col_base64(t, c, h) : 4 * (32 * t + c) + 16 * DP * h);
        float kT[16];
  #pragma unroll
        for (int r = 0; r < 16; ++r) kT[r] = lds_f1(lds, cb + (SWZ ? 256 * crow(r, 0) : 4 * DP * crow(r, 0)));
        if constexpr (BF) {
          dq[t] = mfma_bf(pack8(&kT[0]), pack8(&dsv[0]), dq[t]);
          dq[t] = mfma_bf(pack8(&kT[8]), pack8(&dsv[8]), dq[t]);
        } else {
  #pragma unroll
          for (int r = 0; r < 16; ++r) dq[t] = mfma(kT[r], dsv[r], dq[t]);
        }
      }
      // dQh^T += T^T G^T
      if constexpr (MB4) {  // lane (c, h): T[key crow(r,h)][cluster c & 15]
        float tT[16];
  #pragma unroll
        for (int r = 0; r < 16; ++r) tT[r] = lds_f1(lds, SH::GT + narrow_elem(crow(r, h), c & 15, KPN));
  #pragma unroll
        for (int r = 0; r < 16; ++r) dqh[0] = mfma4b(tT[r], gv[r], dqh[0]);
      } else if constexpr (!DENSE) {
  #pragma unroll
        for (int at = 0; at < KTA; ++at) {
          float tT[16];
  #pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float v = lds_f1(lds, SH::GT + narrow_elem(crow(r, h), imin(32 * at + c, KP - 1), KPN));
            tT[r] = (KP >= 32 || c < KP) ? v : 0.f;
          }
  #pragma unroll
          for (int r = 0; r < 16; ++r) dqh[at] = mfma(tT[r], gv[r], dqh[at]);
        }
      }
      if (more) {  // images read out and ds / G consumed by the MFMAs above: tile kt+1 streams in
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if ((tdead >> (kt + 1)) & 1ull) {
          if constexpr (!DENSE) dma_narrow(Tl, tr, kt * 32 + 32, KPN);
          if constexpr (W1) load_bits(kt + 1);
          else load_tile(kt + 1);
        } else {
          CSA_ISSUE_BQ(kt * 32 + 32);
          load_tile(kt + 1);
        }
      }
    }
  }
#undef CSA_ISSUE_BQ
  if constexpr (W1) {
#pragma unroll
    for (int t = 0; t < DT; ++t)
#pragma unroll
      for (int e = 0; e < 16; ++e) dq[t][e] *= p.scale;
  }
  store_rows<DT>(p.dQ + b * p.dq_sb + hd * p.dq_sh + (int64_t)i * p.dq_sn, D, D, dq, iv);
  if constexpr (MB4) store_mb4(p.dQh + ((int64_t)bh * p.N + qb * 32) * p.kp, p.N - qb * 32, p.kp, dqh[0]);
  else if constexpr (!DENSE) store_rows<KTA>(p.dQh + ((int64_t)bh * p.N + i) * p.kp, p.kp, p.kp, dqh, iv);
}

// ------------------------------------------------------------------------------------
// B1: per (b,h, key block), S orientation (queries = acc rows, keys = lanes): dK, dV, dT
// ------------------------------------------------------------------------------------
// SW_BOTH pair read for the d = 2m + t accumulator mapping (d = 64): columns 2c, 2c + 1 of row crow(r, h), one b64.
// Address = 256 row + 16 ((c >> 1) ^ swz(row)) + 8 (c & 1); swz(crow(r, h)) = (12h) ^ ((r & 3) | 8 bit2(r)), so the
// lane part (pair_base64) XORs with a per-register constant, as both_read's does.
__device__ __forceinline__ int pair_base64(int c, int h) { return 1024 * h + 8 * (c & 1) + 16 * ((c >> 1) ^ (12 * h)); }
__device__ __forceinline__ float2 pair_read(const float* lds, int base, int r, int off) {
  const int kr = 16 * ((r & 3) | (8 * ((r >> 2) & 1)));
  return *reinterpret_cast<const float2*>(reinterpret_cast<const char*>(lds) + off + 256 * crow(r, 0) + (base ^ kr));
}

template <int D, int KPH, bool DENSE, bool DROP, bool DG, bool BF>
__global__ __launch_bounds__(64, (D <= 64 && KPH <= 16) ? 2 : 1) void k_attn_bwd_kv(const KArgs p) {
  using SH = AttnBwdShape<D, KPH>;
  constexpr int DT = D / 32, NS = D / 2, DP = SH::DP, KP = SH::KP, KPN = SH::KPN, KTA = SH::KTA;
  constexpr bool SWZ = SH::SWZ;
  constexpr bool MB4 = !DENSE && KP == 16;  // dT on mfma4b (store_mb4)
  constexpr bool HO = bwd_handoff<BF>();    // ds / G tiles out for k_attn_bwd_qg (else k_attn_bwd_qr recomputes)
  constexpr bool W1 = HO && !DENSE && !DG;  // one-plane w tiles (W_NO_EDGE)
  constexpr bool PAIR = SWZ && !BF;  // dK / dV rows as d = 2m + t (b64 operand reads, pair_read)
  // FG (every variant without map gradients): the row constants are formed here from the forward's row statistics
  // and gamma = rowsum(dX * X), computed per query block from the dX image and the lane's X row; the key block 0
  // waves store them for the query-side kernel. With map gradients (DG) gamma also takes k_attn_gx's term and
  // k_attn_rowprep forms them before this kernel.
  constexpr bool FG = !DG;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const uint32_t L0 = lds_offset(lds), Ql = L0 + SH::KQ, Xl = L0 + SH::KX, Hl = L0 + SH::KH, Sl = L0 + SH::KS;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const BhBlock xb = xcd_block_rev(p.NKB, p.B * p.H);  // reverse of the forward's walk (L2 reuse of X, bit words)
  if (!xb.valid) return;
  const int kbi = xb.blk, bh = xb.bh, b = bh / p.H, hd = bh % p.H;
  const int j = kbi * 32 + c;
  const bool jv = j < p.M;
  const int jc = imin(j, p.M - 1);
  const int qld = (int)p.q_sn * 4, xld = (int)p.dx_sn * 4;
  const __amdgpu_buffer_rsrc_t qr_ = make_rsrc(p.Q + b * p.q_sb + hd * p.q_sh, SWZ ? (p.N - 1) * qld + D * 4 : 0x7fffffff);
  const __amdgpu_buffer_rsrc_t xr_ = make_rsrc(p.dX + b * p.dx_sb + hd * p.dx_sh, SWZ ? (p.N - 1) * xld + D * 4 : 0x7fffffff);
  const __amdgpu_buffer_rsrc_t hr_ = make_rsrc(DENSE ? p.dX : p.Qh + (int64_t)bh * p.N * p.kp, p.N * p.kp * 4);
  // row-constant image source: the forward's (lse, 1 / max(n, eps), [n >= eps], 0) rows (FG; rows >= N out of range)
  // or k_attn_rowprep's (c0, u, v, rho) records
  const __amdgpu_buffer_rsrc_t sr_ = FG ? make_rsrc(p.stats + (int64_t)bh * p.N * 4, p.N * 16)
                                        : make_rsrc(p.brow + (int64_t)bh * p.NQB * 128, p.NQB * 512);
  // FG: this lane's half of X row (query i0 + c, clamped): NS floats at columns NS h .., one f32x4 per dP K-group
  const float* xrow = p.X + b * p.x_sb + hd * p.x_sh + NS * h;
  f32x4 xv4[NS / 4];
  auto load_x = [&](int i0) {
    if constexpr (FG) {
      const float* xp = xrow + (int64_t)imin(i0 + (lane & 31), p.N - 1) * p.x_sn;
#pragma unroll
      for (int s4 = 0; s4 < NS / 4; ++s4) xv4[s4] = *reinterpret_cast<const f32x4*>(xp + 4 * s4);
    }
  };
  // rows past N are never fetched: zero the images once so they only ever hold finite data
  if constexpr (SWZ) lds_zero<(int)(SH::KV_BYTES / 4)>(lds);
  else lds_zero<(SH::NIMG + 512) / 4>(lds + SH::KH / 4);
  const DmaPat qpat = dma_pat(SW_BOTH, qld), xpat = dma_pat(SW_BOTH, xld);
  if constexpr (SWZ) {
    dma64(Ql, qr_, qpat, qld, 0);
    dma64(Xl, xr_, xpat, xld, 0);
  } else {
    dma_rows<D>(Ql, qr_, qld, 0, p.N);
    dma_rows<D>(Xl, xr_, xld, 0, p.N);
  }
  if constexpr (!DENSE) dma_narrow(Hl, hr_, 0, KPN);
  dma_tile_contig<4>(Sl, sr_, 0);
  const int64_t wcol = (int64_t)bh * p.NQB * p.Mpad + j;
  uint32_t wAn = DENSE ? 0xffffffffu : p.Abits[wcol];
  uint32_t wRn = DROP ? p.Rbits[wcol] : 0xffffffffu;
  // Nothing waits on these loads before the first tile (the prologue used to select on the key rows and the mask
  // value right after loading them: a memory latency exposed per wave, profiles/r05_stamps.txt). A key past M reads
  // row M-1 (finite); its A bits, P (kbias = -inf) and stored rows are masked.
  const float* mk = p.mask ? p.mask + b * p.mask_sb : nullptr;
  const float mval = mk ? mk[jc] : 0.f;
  const float dspv = (!DENSE && p.dsp) ? p.dsp[hd] : 0.f;
  const uint32_t kvm = jv ? 0xffffffffu : 0u;  // a key past M counts as not sampled: its G is stored as 0
  // this lane's row (key j) of the ds / G tiles handed to k_attn_bwd_qg, tile (qb, kbi) at + qb * NKB * 1024
  float* dsw = p.dsg + ((int64_t)bh * p.NQB * p.NKB + kbi) * 1024 + c * 32 + 4 * h;
  float kr[NS], vr[NS];
  load_run<NS>(kr, p.K + b * p.k_sb + hd * p.k_sh + (int64_t)jc * p.k_sn + h * NS, true);
  load_run<NS>(vr, p.V + b * p.v_sb + hd * p.v_sh + (int64_t)jc * p.v_sn + h * NS, true);
  const float dscale = DROP ? 1.f / (1.f - p.attn_p) : 1.f;
  const float c1 = p.scale * LOG2E;
  f32x16 dv[DT], dk[DT], dtt[KTA];
#pragma unroll
  for (int t = 0; t < DT; ++t) { dv[t] = zero16(); dk[t] = zero16(); }
#pragma unroll
  for (int t = 0; t < KTA; ++t) dtt[t] = zero16();
  // A key block whose every key is masked (padded ASTs, sbm_attn.py:61): P = 0 on all its elements, so dK = dV = 0
  // and its only gradient is the STE term G = A ? hardtanh(csp (+ dgraph)) : 0 (STE.py:17-19), into dT here and into
  // the query side's dQh, which in the one-plane format reads the tile's A bits from the forward's bit words (no w
  // tile is stored: those stores, a partial line per lane, cost more than the full loop, profiles/r06_dead_kv.txt).
  // Key block 0 always runs the full loop (with FG it forms the row constants the query side reads).
  bool dead = false;
  if (mk && kbi > 0 && p.NKB <= 64) {  // (the forward's dead-tile record, which k_attn_bwd_qg reads, spans 64 tiles)
    wait_vm_all();
    dead = __builtin_amdgcn_ballot_w64(jv && mval == 0.f) == 0;
  }
  if (dead) {
    // Latency-bound otherwise (a round trip per query block, nothing to hide it under): the Qh images and bit words
    // of up to CH query blocks are fetched together into the free Q / dX / Qh image space, then processed with no
    // wait in between (the prologue's loads have landed: the wait above).
    constexpr int CH0 = (int)((SH::KS) / SH::NIMG), CH = CH0 < 8 ? CH0 : 8;
    const float csp = dspv / ((float)p.B * (float)p.N * (float)p.M);
    for (int q0 = 0; q0 < p.NQB; q0 += CH) {
      const int nq = imin(CH, p.NQB - q0);
      uint32_t wA[CH];
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the previous chunk's images read out
#pragma unroll
      for (int u = 0; u < CH; ++u)
        if (u < nq) {
          if constexpr (!DENSE) {
            dma_narrow(L0 + u * SH::NIMG, hr_, (q0 + u) * 32, KPN);
            wA[u] = p.Abits[wcol + (int64_t)(q0 + u) * p.Mpad];
          } else {
            wA[u] = 0u;
          }
        }
      wait_vm_all();
#pragma unroll
      for (int u = 0; u < CH; ++u) {
        if (u >= nq) break;
        const int qb = q0 + u, i0 = qb * 32;
        const int hb = u * SH::NIMG;  // this block's Qh image
        const uint32_t qvm = p.N - i0 >= 32 ? 0xffffffffu : (1u << (p.N - i0)) - 1u;
        const uint32_t wAs = (wA[u] & qvm & kvm) >> (4 * h);
#pragma unroll
        for (int half = 0; half < 2; ++half) {
          float gv[8];
#pragma unroll
          for (int rr = 0; rr < 8; ++rr) {
            const int r = 8 * half + rr;
            const bool a = !DENSE && ((wAs >> crow(r, 0)) & 1u);
            float cg = csp;
            if constexpr (DG) {
              const int ii = i0 + crow(r, h);
              const int64_t me = ((int64_t)bh * p.N + imin(ii, p.N - 1)) * p.M + jc;
              if (p.dgraph) cg += ldz(p.dgraph, me, INT64_MAX, (ii < p.N) && jv);
            }
            gv[rr] = a ? __builtin_amdgcn_fmed3f(0.f + cg, -1.f, 1.f) : 0.f;  // w = dM P = 0
          }
          // one-plane format (W1): no w tile at all, k_attn_bwd_qg reads the tile's bits from the forward's words
          // (its tdead record); two planes: ds = 0 and G
          if constexpr (HO && !W1) {
            float* const w = dsw + (int64_t)qb * p.NKB * 1024 + 16 * half;
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
            {
              *reinterpret_cast<f32x4*>(w) = z;  // plain stores, as the live tiles' (partial rows per lane)
              *reinterpret_cast<f32x4*>(w + 8) = z;
              if constexpr (!DENSE) {
                *reinterpret_cast<f32x4*>(w + p.gplane) = f32x4{gv[0], gv[1], gv[2], gv[3]};
                *reinterpret_cast<f32x4*>(w + p.gplane + 8) = f32x4{gv[4], gv[5], gv[6], gv[7]};
              }
            }
          }
          if constexpr (MB4) {
#pragma unroll
            for (int rr = 0; rr < 8; ++rr)
              dtt[0] = mfma4b(lds_f1(lds, hb + narrow_elem(crow(8 * half + rr, h), c & 15, KPN)), gv[rr], dtt[0]);
          } else if constexpr (!DENSE) {
#pragma unroll
            for (int at = 0; at < KTA; ++at)
#pragma unroll
              for (int rr = 0; rr < 8; ++rr) {
                const int r = 8 * half + rr;
                const float v = lds_f1(lds, hb + narrow_elem(crow(r, h), imin(32 * at + c, KP - 1), KPN));
                dtt[at] = mfma((KP >= 32 || c < KP) ? v : 0.f, gv[rr], dtt[at]);
              }
          }
        }
      }
    }
  }
  for (int qb = 0; qb < (dead ? 0 : p.NQB); ++qb) {
    int ln = threadIdx.x;  // opaque per iteration: keeps the per-row LDS addresses out of the prologue
    asm volatile("" : "+v"(ln));
    const int c = ln & 31, h = (ln >> 5) & 1;
    const int i0 = qb * 32;
    const bool more = qb + 1 < p.NQB;
    wait_vm_all();  // query block qb's Q / dX / Qh / row-constant images and bit words have landed
    float mvl = mval, dsl = dspv;  // opaque per tile: their uses stay behind the wait above
    asm volatile("" : "+v"(mvl), "+v"(dsl));
    const float kbias = (jv && mvl == 0.f) ? 0.f : NEG_INF;  // this lane's key (sbm_attn.py:61)
    const float csp = dsl / ((float)p.B * (float)p.N * (float)p.M);
    // FG: this block's X rows are loaded here, behind the wait (their latency hides under the S chain), and the row
    // constants formed after it (form_rec), before the elementwise reads them
    load_x(i0);
    bool rho_any = false;  // W1: does a row of this query block have rho != 0 (its query side then needs P as well)?
    auto form_rec = [&]() {
      if constexpr (FG) {
        // gamma of query i0 + c = rowsum(dX * X): this lane's half from the dX image row and its X registers, then
        // the two halves added; the row constants as k_attn_rowprep forms them
        const int xb0 = SWZ ? row_base64(c, h, SW_BOTH) : 4 * (c * DP + NS * h);
        float gp = 0.f;
#pragma unroll
        for (int s4 = 0; s4 < NS / 4; ++s4) {
          const f32x4 dx4 = lds_f4(lds, SH::KX + (SWZ ? (xb0 ^ (16 * s4)) : xb0 + 16 * s4));
          gp = fmaf(dx4[0], xv4[s4][0], fmaf(dx4[1], xv4[s4][1], fmaf(dx4[2], xv4[s4][2], fmaf(dx4[3], xv4[s4][3], gp))));
        }
        const float gamma = xhalf_sum(gp);
        const bool iv = i0 + c < p.N;
        const f32x4 st = lds_f4(lds, SH::KS + 16 * c);  // lse, 1 / max(n, eps), [n >= eps] (finite data past N)
        f32x4 rec;
        rec[0] = iv ? -st[0] * LOG2E : NEG_INF;
        rec[1] = iv ? dscale * st[1] : 0.f;
        rec[2] = (iv && st[2] != 0.f) ? -gamma * st[1] : 0.f;
        rec[3] = (iv && st[2] == 0.f) ? gamma : 0.f;
        if (h == 0) {
          *reinterpret_cast<f32x4*>(lds + SH::KS / 4 + 4 * c) = rec;
          if (kbi == 0) *reinterpret_cast<f32x4*>(p.brow + (((int64_t)bh * p.NQB + qb) * 32 + c) * 4) = rec;
        }
        rho_any = W1 && __builtin_amdgcn_ballot_w64(rec[3] != 0.f) != 0;
      } else {
        rho_any = W1 && __builtin_amdgcn_ballot_w64(lds_f1(lds, SH::KS + 16 * c + 12) != 0.f) != 0;
      }
    };
    // sampled / keep bits shifted so that register r's query is bit crow(r, 0); queries past N and keys past M
    // count as not sampled
    const uint32_t qvm = p.N - i0 >= 32 ? 0xffffffffu : (1u << (p.N - i0)) - 1u;
    const uint32_t wAs = (wAn & qvm & kvm) >> (4 * h), wRs = wRn >> (4 * h);
    if (more) {
      if constexpr (!DENSE) wAn = p.Abits[wcol + (int64_t)(qb + 1) * p.Mpad];
      if constexpr (DROP) wRn = p.Rbits[wcol + (int64_t)(qb + 1) * p.Mpad];
    }
    f32x16 sacc = zero16(), dpacc = zero16();
    const int qrb = SWZ ? row_base64(c, h, SW_BOTH) : 4 * (c * DP + NS * h);
    if constexpr (BF) {
#pragma unroll
      for (int j2 = 0; j2 < NS / 8; ++j2) {
        const f32x4 q0 = lds_f4(lds, SH::KQ + (SWZ ? (qrb ^ (32 * j2)) : qrb + 32 * j2));
        const f32x4 q1 = lds_f4(lds, SH::KQ + (SWZ ? (qrb ^ (32 * j2 + 16)) : qrb + 32 * j2 + 16));
        sacc = mfma_bf(pack8(q0, q1), pack8(&kr[8 * j2]), sacc);
        const f32x4 x0 = lds_f4(lds, SH::KX + (SWZ ? (qrb ^ (32 * j2)) : qrb + 32 * j2));
        const f32x4 x1 = lds_f4(lds, SH::KX + (SWZ ? (qrb ^ (32 * j2 + 16)) : qrb + 32 * j2 + 16));
        dpacc = mfma_bf(pack8(x0, x1), pack8(&vr[8 * j2]), dpacc);
      }
      form_rec();
    } else {
#pragma unroll
      for (int s4 = 0; s4 < NS / 4; ++s4) {
        const f32x4 qv = lds_f4(lds, SH::KQ + (SWZ ? (qrb ^ (16 * s4)) : qrb + 16 * s4));
#pragma unroll
        for (int e = 0; e < 4; ++e) sacc = mfma(qv[e], kr[4 * s4 + e], sacc);
      }
      form_rec();  // (between the chains: the X registers die before dP's accumulator is live)
#pragma unroll
      for (int s4 = 0; s4 < NS / 4; ++s4) {
        const f32x4 xv = lds_f4(lds, SH::KX + (SWZ ? (qrb ^ (16 * s4)) : qrb + 16 * s4));
#pragma unroll
        for (int e = 0; e < 4; ++e) dpacc = mfma(xv[e], vr[4 * s4 + e], dpacc);
      }
    }
    // column read of element (query crow(r,h), d = 32t + c) of the Q / dX image at byte offset off
    int cb[DT];
#pragma unroll
    for (int t = 0; t < DT; ++t) cb[t] = SWZ ? both_base64(t, c, h) : 4 * (32 * t + c) + 16 * DP * h;
    auto colv = [&](int off, int t, int r) {
      return SWZ ? both_read(lds, cb[t], r, off) : lds_f1(lds, off + cb[t] + 4 * DP * crow(r, 0));
    };
    // Two halves of the query block (registers r = 8 half .. 8 half + 7 = rows 16 half .. 16 half + 15):
    // elementwise, then the dV / dK / dT K-steps of those rows; query block qb+1's images are DMA'd in
    // after the second half.
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      // Elementwise backward, once per element (k_attn_rowprep's row constants; scalar fp32: packed v_pk_* beside
      // the MFMAs cost more issue cycles than they save). A query past N has c0 = -inf (P = 0) and A = 0; a key
      // past M has kbias = -inf and A = 0; so every element outside [0,N) x [0,M) stores ds = G = attw = 0.
      float dsv[8], gv[8], awv[8], wv[4];
      // this half's queries 16 half + 4 h + (0..3) and + 8 of the tile: two f32x4 per plane
      float* const wst = dsw + (int64_t)qb * p.NKB * 1024 + 16 * half;
#pragma unroll
      for (int rr = 0; rr < 8; ++rr) {
        const int r = 8 * half + rr;
        const f32x4 rec = lds_f4(lds, SH::KS + 16 * crow(r, h));  // (c0, u, v, rho) of query crow(r, h)
        const bool a = (wAs >> crow(r, 0)) & 1u;
        const bool kp = !DROP || ((wRs >> crow(r, 0)) & 1u);
        const float P = __builtin_amdgcn_exp2f(fmaf(sacc[r], c1, rec[0] + kbias));
        float dM = fmaf(kp ? dpacc[r] : 0.f, rec[1], rec[2]);
        float cg = csp;
        if constexpr (DG) {  // upstream gradients of the returned graph / attn maps
          const int ii = i0 + crow(r, h);
          const bool inside = (ii < p.N) && jv;
          const int64_t me = ((int64_t)bh * p.N + imin(ii, p.N - 1)) * p.M + jc;
          if (p.dgraph) cg += ldz(p.dgraph, me, INT64_MAX, inside);
          if (p.dattn) dM = fmaf(ldz(p.dattn, me, INT64_MAX, inside), rec[1] * (1.f - p.attn_p), dM);
        }
        if constexpr (W1) {  // the query side's expressions exactly (k_attn_bwd_qg)
          const float w = dM * P;
          wv[rr & 3] = __uint_as_float(a ? __float_as_uint(w) : W_NO_EDGE);
          dsv[rr] = fmaf(-rec[3], P, a ? w : 0.f) * p.scale;
          gv[rr] = a ? __builtin_amdgcn_fmed3f(w + cg, -1.f, 1.f) : 0.f;
        } else {
          dsv[rr] = ((a ? dM : 0.f) - rec[3]) * (P * p.scale);
          gv[rr] = a ? __builtin_amdgcn_fmed3f(fmaf(dM, P, cg), -1.f, 1.f) : 0.f;  // STE.py:19 hardtanh(A * grad)
        }
        awv[rr] = (a && kp) ? P * rec[1] : 0.f;  // dropout(attn) weight for dV
        if constexpr (W1) {  // stored as soon as four are ready (fewer live registers); plain stores, see below
          if ((rr & 3) == 3)
            *reinterpret_cast<f32x4*>(wst + 2 * (rr & 4)) = f32x4{wv[0], wv[1], wv[2], wv[3]};
        }
      }
      if constexpr (HO) {  // queries 16 half + 4 h + (0..3) and + 8: two f32x4 per tile, for ds and for G
        float* const w = wst;
        // Plain (write-back) stores: a lane writes 16 B of its key's 128-B tile row per instruction, so a row is
        // completed by four instructions; non-temporal stores sent each 32-B piece on its own (round 6, same box:
        // k_attn_bwd_kv 356 -> 345 us, k_attn_bwd_qg unchanged, profiles/r06_ab_wtile_store.txt; round 4 had measured
        // non-temporal stores faster for the two-plane tiles, k_attn_bwd_qg 157 -> 134 us, before the one-plane format)
#define CSA_ST4(ptr, val) (*reinterpret_cast<f32x4*>(ptr) = (val))
        if constexpr (W1) {  // (the w values are stored in the elementwise loop)
          if (rho_any) {  // rare (a degenerate row): P of the half's elements, recomputed, into the second plane
            float pv[8];
#pragma unroll
            for (int rr = 0; rr < 8; ++rr) {
              const f32x4 rec = lds_f4(lds, SH::KS + 16 * crow(8 * half + rr, h));
              pv[rr] = __builtin_amdgcn_exp2f(fmaf(sacc[8 * half + rr], c1, rec[0] + kbias));
            }
            CSA_ST4(w + p.gplane, (f32x4{pv[0], pv[1], pv[2], pv[3]}));
            CSA_ST4(w + p.gplane + 8, (f32x4{pv[4], pv[5], pv[6], pv[7]}));
          }
        } else {
          CSA_ST4(w, (f32x4{dsv[0], dsv[1], dsv[2], dsv[3]}));
          CSA_ST4(w + 8, (f32x4{dsv[4], dsv[5], dsv[6], dsv[7]}));
        }
        if constexpr (!DENSE && !W1) {
          CSA_ST4(w + p.gplane, (f32x4{gv[0], gv[1], gv[2], gv[3]}));
          CSA_ST4(w + p.gplane + 8, (f32x4{gv[4], gv[5], gv[6], gv[7]}));
        }
#undef CSA_ST4
      }
      // dV^T += dX^T attw ; dK^T += Q^T ds ; dT^T += Qh^T G  (queries beyond N carry zeros)
      if constexpr (BF) {
        const bf16x8 aw8 = pack8(awv), ds8 = pack8(dsv);
#pragma unroll
        for (int t = 0; t < DT; ++t) {
          float xc[8], qc[8];
#pragma unroll
          for (int rr = 0; rr < 8; ++rr) { xc[rr] = colv(SH::KX, t, 8 * half + rr); qc[rr] = colv(SH::KQ, t, 8 * half + rr); }
          dv[t] = mfma_bf(pack8(xc), aw8, dv[t]);
          dk[t] = mfma_bf(pack8(qc), ds8, dk[t]);
        }
      } else if constexpr (PAIR) {  // d = 2m + t: the two tiles' operands of a K-step are one b64 read
        const int pb = pair_base64(c, h);
#pragma unroll
        for (int rr = 0; rr < 8; ++rr) {
          const float2 xv = pair_read(lds, pb, 8 * half + rr, SH::KX), qv2 = pair_read(lds, pb, 8 * half + rr, SH::KQ);
          dv[0] = mfma(xv.x, awv[rr], dv[0]);
          dv[1] = mfma(xv.y, awv[rr], dv[1]);
          dk[0] = mfma(qv2.x, dsv[rr], dk[0]);
          dk[1] = mfma(qv2.y, dsv[rr], dk[1]);
          if ((rr & 1) == 1) __builtin_amdgcn_sched_barrier(0);  // at most two K-steps of operands in flight
        }
      } else {
#pragma unroll
        for (int t = 0; t < DT; ++t)
#pragma unroll
          for (int rr = 0; rr < 8; ++rr) dv[t] = mfma(colv(SH::KX, t, 8 * half + rr), awv[rr], dv[t]);
#pragma unroll
        for (int t = 0; t < DT; ++t)
#pragma unroll
          for (int rr = 0; rr < 8; ++rr) dk[t] = mfma(colv(SH::KQ, t, 8 * half + rr), dsv[rr], dk[t]);
      }
      if constexpr (MB4) {  // lane (c, h): Qh[query crow(r,h)][cluster c & 15]
#pragma unroll
        for (int rr = 0; rr < 8; ++rr)
          dtt[0] = mfma4b(lds_f1(lds, SH::KH + narrow_elem(crow(8 * half + rr, h), c & 15, KPN)), gv[rr], dtt[0]);
      } else if constexpr (!DENSE) {
#pragma unroll
        for (int at = 0; at < KTA; ++at)
#pragma unroll
          for (int rr = 0; rr < 8; ++rr) {
            const int r = 8 * half + rr;
            const float v = lds_f1(lds, SH::KH + narrow_elem(crow(r, h), imin(32 * at + c, KP - 1), KPN));
            dtt[at] = mfma((KP >= 32 || c < KP) ? v : 0.f, gv[rr], dtt[at]);
          }
      }
      if (more) {
        // the whole refill after the second half: no mid-tile wait on the first half's reads, so the second
        // half's elementwise can be scheduled among the first half's MFMAs (a per-half rolling refill measured
        // 4 us slower, profiles/r04_ab_kv_refill.txt)
        if constexpr (SWZ) {
          if (half == 1) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            dma64(Xl, xr_, xpat, xld, i0 + 32);
            dma64(Ql, qr_, qpat, qld, i0 + 32);
            if constexpr (!DENSE) dma_narrow(Hl, hr_, i0 + 32, KPN);
            dma_tile_contig<4>(Sl, sr_, i0 + 32);
          }
        } else if (half == 1) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          dma_rows<D>(Xl, xr_, xld, i0 + 32, p.N);
          dma_rows<D>(Ql, qr_, qld, i0 + 32, p.N);
          if constexpr (!DENSE) dma_narrow(Hl, hr_, i0 + 32, KPN);
          dma_tile_contig<4>(Sl, sr_, i0 + 32);
        }
      }
    }
  }
  if constexpr (PAIR) {  // d = 2 crow(r, h) + t: registers 4g .. 4g + 3 of both tiles are d = 16g + 8h .. + 7
    if (jv) {
      float* dkp = p.dK + b * p.dk_sb + hd * p.dk_sh + (int64_t)j * p.dk_sn + 8 * h;
      float* dvp = p.dV + b * p.dv_sb + hd * p.dv_sh + (int64_t)j * p.dv_sn + 8 * h;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        *reinterpret_cast<f32x4*>(dkp + 16 * g) = f32x4{dk[0][4 * g], dk[1][4 * g], dk[0][4 * g + 1], dk[1][4 * g + 1]};
        *reinterpret_cast<f32x4*>(dkp + 16 * g + 4) =
            f32x4{dk[0][4 * g + 2], dk[1][4 * g + 2], dk[0][4 * g + 3], dk[1][4 * g + 3]};
        *reinterpret_cast<f32x4*>(dvp + 16 * g) = f32x4{dv[0][4 * g], dv[1][4 * g], dv[0][4 * g + 1], dv[1][4 * g + 1]};
        *reinterpret_cast<f32x4*>(dvp + 16 * g + 4) =
            f32x4{dv[0][4 * g + 2], dv[1][4 * g + 2], dv[0][4 * g + 3], dv[1][4 * g + 3]};
      }
    }
  } else {
    store_rows<DT>(p.dK + b * p.dk_sb + hd * p.dk_sh + (int64_t)j * p.dk_sn, D, D, dk, jv);
    store_rows<DT>(p.dV + b * p.dv_sb + hd * p.dv_sh + (int64_t)j * p.dv_sn, D, D, dv, jv);
  }
  if constexpr (MB4) store_mb4(p.dT + ((int64_t)bh * p.M + kbi * 32) * p.kp, p.M - kbi * 32, p.kp, dtt[0]);
  else if constexpr (!DENSE) store_rows<KTA>(p.dT + ((int64_t)bh * p.M + j) * p.kp, p.kp, p.kp, dtt, jv);
}

// ------------------------------------------------------------------------------------
// B3: projection backward. Workgroup = 4 waves, grid (G, H): head hd, batch chunk g.
// Each wave takes one 32-row item (Q or K block) per group of 4. Per item the saved activations
// (k_proj_fwd) replace any forward recompute. Five weight-gradient products
//   dS_h += dT^T Kh, dC_h += dZ^T po, dW2 += dp^T h2, dW1 += dh2^T h1, dW0 += dh1^T x
// reduce over the group's 128 rows. Both operands are staged in LDS in the activation-block
// layout (one 32-row region per wave): DS from the wave's registers, IN by LDS-DMA of the saved
// block, issued as soon as the region is free so it lands under the chain MFMAs. The output tiles
// are dealt round-robin to the waves (tile g -> wave g % 4). When they fit (REGACC: <= 8 tiles per
// wave) each wave accumulates its tiles in registers over all its items and writes its part of
// the WG's slab exactly once. Otherwise it read-modify-writes the slab once per group. Neither
// path uses atomics, so the result is deterministic.
// ------------------------------------------------------------------------------------
template <int D, int KT>
struct ProjBwdShape {
  static constexpr int DT = D / 32, NS = D / 2, KP32 = 32 * KT;
  static constexpr int F = (D > KP32 ? D : KP32);  // feature rows per staging region
  static constexpr int REG = F * 32;                // floats per wave region
  static constexpr size_t LDS_BYTES = sizeof(float) * 8 * REG;  // DS regions, then IN regions
  static constexpr int ABLK = (3 * D + KP32) * 32;  // activation block floats per item
  // output tiles in stage order dS | dC | dW2 | dW1 | dW0
  static constexpr int G_S = 0, G_C = KT * KT, G_W2 = G_C + KT * DT, G_W1 = G_W2 + DT * DT, G_W0 = G_W1 + DT * DT,
                       NTILE = G_W0 + DT * DT;
  static constexpr int NACC = (NTILE + 3) / 4;
  // up to 8 accumulator tiles per wave (128 registers: the kernel runs one wave per SIMD for d = 96 or
  // KT > 1, so the unified VGPR/AGPR file has room); d = 96 has 31 tiles = 8 per wave. Beyond that the
  // slab is read-modify-written once per group.
  static constexpr bool REGACC = NACC <= 8;
};

// act_off(32t + crow(r,h), c) split into a lane base and a compile-time offset: for these features
// (f>>1)&7 = K(r) ^ (h<<1) with K(r) = ((r>>1)&1) | ((r>>2)&1)<<2, so only 4 lane bases exist
// (K in {0,1,4,5}); the rest, 32*(32t + (r&3) + 8(r>>2)), folds into the ds instruction offset.
struct AccLanes { int base[4]; };
__device__ __forceinline__ AccLanes acc_lanes(int lane) {
  asm volatile("" : "+v"(lane));  // per call: no address survives across helpers
  const int c = lane & 31, h = lane >> 5, q = (c >> 2) ^ (h << 1);
  AccLanes L;
  const int kv[4] = {0, 1, 4, 5};
#pragma unroll
  for (int i = 0; i < 4; ++i) L.base[i] = 128 * h + 4 * (q ^ kv[i]) + (c & 3);
  return L;
}
__device__ __forceinline__ constexpr int acc_kidx(int r) { return ((r >> 1) & 1) | (((r >> 2) & 1) << 1); }
__device__ __forceinline__ constexpr int acc_coff(int t, int r) { return 32 * (32 * t + (r & 3) + 8 * (r >> 2)); }

// acc tiles (feature rows 32t + crow(r,h), data row c) -> own staging region; features >= nvalid are 0
template <int NT>
__device__ __forceinline__ void stage_ds(float* __restrict__ reg, const f32x16 (&a)[NT], int nvalid, int lane) {
  const AccLanes L = acc_lanes(lane);
  const int h = lane >> 5;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int f = 32 * t + crow(r, h);
      reg[L.base[acc_kidx(r)] + acc_coff(t, r)] = (f < nvalid) ? a[t][r] : 0.f;
    }
}

// own region -> acc tiles (lane c = data row)
template <int NT>
__device__ __forceinline__ void read_act(f32x16 (&a)[NT], const float* __restrict__ reg, int lane) {
  const AccLanes L = acc_lanes(lane);
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) a[t][r] = reg[L.base[acc_kidx(r)] + acc_coff(t, r)];
}

// acc += sum over the 128 staged rows of DS[32ot + i][row] * IN[32it + j][row]
// K-step s of half h takes rows 64h + s: region 2h + s/32, chunk (s%32)/4.
// BF: on bf16 MFMA, K-groups s4 = 2 s8, 2 s8 + 1 (8 consecutive staged rows) per instruction
template <int REG, bool BF = false>
__device__ __forceinline__ f32x16 outer_tile(const float* __restrict__ ds, const float* __restrict__ in, int ot, int it,
                                             f32x16 acc, int lane) {
  asm volatile("" : "+v"(lane));
  const int c = lane & 31, h = lane >> 5, sw = (c >> 1) & 7;
  const float* a = ds + 2 * h * REG + (32 * ot + c) * 32;
  const float* b = in + 2 * h * REG + (32 * it + c) * 32;
  if constexpr (BF) {
#pragma unroll
    for (int s8 = 0; s8 < 8; ++s8) {
      f32x4 av[2], bv[2];
#pragma unroll
      for (int u = 0; u < 2; ++u) {
        const int s4 = 2 * s8 + u, off = (s4 >> 3) * REG + 4 * ((s4 & 7) ^ sw);
        av[u] = *reinterpret_cast<const f32x4*>(a + off);
        bv[u] = *reinterpret_cast<const f32x4*>(b + off);
      }
      acc = mfma_bf(pack8(av[0], av[1]), pack8(bv[0], bv[1]), acc);
    }
    return acc;
  }
#pragma unroll
  for (int s4 = 0; s4 < 16; ++s4) {
    const int off = (s4 >> 3) * REG + 4 * ((s4 & 7) ^ sw);
    const f32x4 av = *reinterpret_cast<const f32x4*>(a + off);
    const f32x4 bv = *reinterpret_cast<const f32x4*>(b + off);
#pragma unroll
    for (int e = 0; e < 4; ++e) acc = mfma(av[e], bv[e], acc);
  }
  return acc;
}

// feature f's sum over the 128 staged rows (fixed order)
template <int REG>
__device__ __forceinline__ float region_rowsum(const float* __restrict__ ds, int f) {
  asm volatile("" : "+v"(f));
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    float sw = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(ds + w * REG + act_off(f, 4 * k));
      sw += (v[0] + v[1]) + (v[2] + v[3]);
    }
    s += sw;
  }
  return s;
}

// destination of output tile g inside a WG slab
template <int D, int KT>
struct TileDst { float* base; int ldo, orows, icols, ot, it; };
template <int D, int KT>
__device__ __forceinline__ TileDst<D, KT> tile_dst(float* slab, int g) {
  using Sh = ProjBwdShape<D, KT>;
  constexpr int DT = Sh::DT, KP32 = Sh::KP32;
  float* sC = slab + 3 * D * D + 3 * D;
  float* sS = sC + KP32 * D;
  TileDst<D, KT> t;
  if (g < Sh::G_C) { t.base = sS; t.ldo = KP32; t.orows = KP32; t.icols = KP32; t.ot = g / KT; t.it = g % KT; }
  else if (g < Sh::G_W2) { const int q = g - Sh::G_C; t.base = sC; t.ldo = D; t.orows = KP32; t.icols = D; t.ot = q / DT; t.it = q % DT; }
  else {
    const int l = g < Sh::G_W1 ? 2 : g < Sh::G_W0 ? 1 : 0;
    const int q = g - (l == 2 ? Sh::G_W2 : l == 1 ? Sh::G_W1 : Sh::G_W0);
    t.base = slab + l * D * D; t.ldo = D; t.orows = D; t.icols = D; t.ot = q / DT; t.it = q % DT;
  }
  return t;
}

template <int NTILE>
__device__ __forceinline__ void tile_store(float* __restrict__ base, int ldo, int orows, int icols, int ot, int it,
                                           const f32x16& v, bool accumulate, int lane) {
  const int c = lane & 31, h = lane >> 5;
  const int col = 32 * it + c;
  if (col >= icols) return;
  float old[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = 32 * ot + crow(r, h);
    old[r] = (accumulate && row < orows) ? base[row * ldo + col] : 0.f;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = 32 * ot + crow(r, h);
    if (row < orows) base[row * ldo + col] = old[r] + v[r];
  }
}

// One product stage: tiles g0 .. g0 + nto*nti - 1 (tile g -> wave g % 4)
template <int D, int KT, int G0, int NTO, int NTI>
__device__ __forceinline__ void outer_stage(const float* ds, const float* in, f32x16 (&acc)[ProjBwdShape<D, KT>::NACC],
                                            float* slab, int w, int lane) {
  using Sh = ProjBwdShape<D, KT>;
  if constexpr (Sh::REGACC) {
#pragma unroll
    for (int g = G0; g < G0 + NTO * NTI; ++g)
      if ((g & 3) == w) acc[g >> 2] = outer_tile<Sh::REG>(ds, in, (g - G0) / NTI, (g - G0) % NTI, acc[g >> 2], lane);
  } else {
    for (int g = G0 + ((w - G0) & 3); g < G0 + NTO * NTI; g += 4) {
      const f32x16 v = outer_tile<Sh::REG>(ds, in, (g - G0) / NTI, (g - G0) % NTI, zero16(), lane);
      const TileDst<D, KT> t = tile_dst<D, KT>(slab, g);
      tile_store<0>(t.base, t.ldo, t.orows, t.icols, t.ot, t.it, v, true, lane);
    }
  }
}

// out^T = Wfrag^T-style product: out[it] = sum_s frag[it][s] * in[s/16][s%16] (acc-perm input)
// (S4MAX < NSTEP/4: only the first 4 S4MAX K-steps, for inputs known to be zero beyond them.)
template <int NTO, int NTI, int S4MAX = 4 * NTI, int LA = 1>
__device__ __forceinline__ void mm_acc(const float* __restrict__ frag, const f32x16 (&in)[NTI], f32x16 (&out)[NTO]) {
#pragma unroll
  for (int t = 0; t < NTO; ++t) out[t] = zero16();
  frag_chain<NTO, S4MAX, LA>(frag, 16 * NTI, out, [&](int s) { return in[s / 16][s % 16]; });
}

// mm_acc over fragments held in LDS (FL) or global memory; NSTEP = the K-steps of the stored layout
// (8 for the compacted k <= 16 cluster fragments: only K-groups 0 and 1 of each tile are copied).
template <int NTO, int NTI, int S4MAX, int NSTEP, bool FL, bool BF = false>
__device__ __forceinline__ void mm_acc_f(const float* __restrict__ frag, const f32x16 (&in)[NTI], f32x16 (&out)[NTO]) {
#pragma unroll
  for (int t = 0; t < NTO; ++t) out[t] = zero16();
  // L2 fragments two K-groups ahead (measured 2% faster k_proj_bwd_s<64> than one), LDS fragments one
  frag_chain<NTO, S4MAX, S4MAX < 4 ? 1 : (FL ? FL_LA : 2), FL, BF>(frag, NSTEP, out,
                                                                  [&](int s) { return in[s / 16][s % 16]; });
}

template <int D, int KT>
__global__ __launch_bounds__(256, (D <= 64 && KT <= 1 ? 2 : 1)) void k_proj_bwd(const KArgs p) {
  using Sh = ProjBwdShape<D, KT>;
  constexpr int DT = Sh::DT, NS = Sh::NS, KP32 = Sh::KP32, REG = Sh::REG, ABLK = Sh::ABLK, NACC = Sh::NACC;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* DS = lds;
  float* IN = lds + 4 * REG;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int hd = blockIdx.y, g = blockIdx.x, G = gridDim.x;
  const int per_b = p.NQB + p.NKB;
  const int i_lo = (int)((int64_t)g * p.B * per_b / G), i_hi = (int)((int64_t)(g + 1) * p.B * per_b / G);
  const int n_items = i_hi - i_lo;  // this workgroup's items: i_lo .. i_hi - 1 of the head
  float* slab = p.slab + ((int64_t)hd * G + g) * p.slab_floats;
  const float ks = p.proj_p > 0.f ? 1.f / (1.f - p.proj_p) : 1.f;
  const float* CfT = p.CfT + (size_t)hd * KP32 * D;
  const float* SfT = p.SfT + (size_t)hd * KP32 * KP32;
  float* DSw = DS + w * REG;
  float* INw = IN + w * REG;
  const uint32_t INl = lds_offset(IN) + 4 * REG * w;
  f32x16 acc[NACC];
#pragma unroll
  for (int i = 0; i < NACC; ++i) acc[i] = zero16();
  float dbacc[3] = {0.f, 0.f, 0.f};

  // per-wave item of group grp (wave-uniform scalars)
  struct Item { int b, r, isK, rb, nrows; bool has; };
  auto item_of = [&](int grp) {
    Item it;
    const int item = grp * 4 + w;
    it.has = item < n_items;
    it.b = it.has ? (i_lo + item) / per_b : 0;
    it.r = it.has ? (i_lo + item) % per_b : 0;
    it.isK = it.r >= p.NQB;
    it.rb = it.isK ? it.r - p.NQB : it.r;
    it.nrows = it.isK ? p.M : p.N;
    return it;
  };
  auto act_rsrc = [&](const Item& it) {
    return make_rsrc(p.Act + ((int64_t)(it.b * p.H + hd) * per_b + it.r) * ABLK, ABLK * 4);
  };
  // group 0's first operands: hat -> IN, dT / dQh -> registers
  f32x16 gin[KT];
  {
    const Item it = item_of(0);
    dma_block16<KP32 * 128>(INl, act_rsrc(it), 96 * D * 4);
    const int row = it.rb * 32 + c, rowc = imin(row, it.nrows - 1), bh = it.b * p.H + hd;
    load_rows<KT>(gin, (it.isK ? p.dT + ((int64_t)bh * p.M + rowc) * p.kp : p.dQh + ((int64_t)bh * p.N + rowc) * p.kp),
                  p.kp, it.has && row < it.nrows);
  }

  for (int grp = 0; grp * 4 < n_items; ++grp) {
    int tid = threadIdx.x;  // opaque: per-lane addresses are recomputed in the loop, not hoisted
    asm volatile("" : "+v"(tid));
    const int ln = tid & 63;
    const Item it = item_of(grp);
    const int row = it.rb * 32 + c;
    const bool rv = it.has && row < it.nrows;
    const int rowc = imin(row, it.nrows - 1);
    const int bh = it.b * p.H + hd;
    const __amdgpu_buffer_rsrc_t ar = act_rsrc(it);
    // ---- dS_h += sum_rows dT^T Kh^T (K items; Q items stage zeros)
    wait_vm_all();
    f32x16 hat[KT];
    read_act<KT>(hat, INw, ln);
    stage_ds<KT>(DSw, gin, it.isK ? KP32 : 0, ln);
    __syncthreads();
    outer_stage<D, KT, Sh::G_S, KT, KT>(DS, IN, acc, slab, w, ln);
    __syncthreads();
    // ---- dC_h += sum_rows dZ^T p^T
    dma_block16<D * 128>(INl, ar, 64 * D * 4);  // po
    f32x16 dz[KT];
    if (it.isK) {
      mm_acc<KT, KT>(SfT, gin, dz);  // dKh^T = S^T dT^T
    } else {
#pragma unroll
      for (int t = 0; t < KT; ++t) dz[t] = gin[t];
    }
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) dz[t][r] = dz[t][r] * hat[t][r] * (1.f - hat[t][r]);
    stage_ds<KT>(DSw, dz, KP32, ln);
    wait_vm_all();
    __syncthreads();
    outer_stage<D, KT, Sh::G_C, KT, DT>(DS, IN, acc, slab, w, ln);
    __syncthreads();
    // ---- layer 2 (proj.6): dW2 += dp^T h2 ; db2 ; dh2 = W2^T dp
    dma_block16<D * 128>(INl, ar, 32 * D * 4);  // h2
    f32x16 dcur[DT];
    mm_acc<DT, KT>(CfT, dz, dcur);  // dp^T = C^T dZ^T
    stage_ds<DT>(DSw, dcur, D, ln);
    wait_vm_all();
    __syncthreads();
    outer_stage<D, KT, Sh::G_W2, DT, DT>(DS, IN, acc, slab, w, ln);
    if (tid < D) {
      const float sred = region_rowsum<REG>(DS, tid);
      if constexpr (Sh::REGACC) dbacc[2] += sred; else slab[3 * D * D + 2 * D + tid] += sred;
    }
    __syncthreads();
    {
      f32x16 hv[DT], dh[DT];
      read_act<DT>(hv, INw, ln);  // own h2 (relu mask)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      dma_block16<D * 128>(INl, ar, 0);  // h1
      mm_acc<DT, DT>(p.WfT[2], dcur, dh);
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) dcur[t][r] = (hv[t][r] > 0.f) ? dh[t][r] * ks : 0.f;
    }
    // ---- layer 1 (proj.3): dW1 += dh2^T h1 ; db1 ; dh1 = W1^T dh2
    stage_ds<DT>(DSw, dcur, D, ln);
    float x[NS];
    {
      const float* X = it.isK ? p.K + it.b * p.k_sb + hd * p.k_sh + (int64_t)rowc * p.k_sn
                              : p.Q + it.b * p.q_sb + hd * p.q_sh + (int64_t)rowc * p.q_sn;
      load_run<NS>(x, X + h * NS, rv);
    }
    wait_vm_all();
    __syncthreads();
    outer_stage<D, KT, Sh::G_W1, DT, DT>(DS, IN, acc, slab, w, ln);
    if (tid < D) {
      const float sred = region_rowsum<REG>(DS, tid);
      if constexpr (Sh::REGACC) dbacc[1] += sred; else slab[3 * D * D + D + tid] += sred;
    }
    __syncthreads();
    {
      f32x16 hv[DT], dh[DT];
      read_act<DT>(hv, INw, ln);  // own h1 (relu mask)
      // layer 0 input x (lin-perm rows) -> own IN region, feature s + NS*h
#pragma unroll
      for (int s = 0; s < NS; ++s) INw[act_off(s + NS * h, c)] = x[s];
      mm_acc<DT, DT>(p.WfT[1], dcur, dh);
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) dcur[t][r] = (hv[t][r] > 0.f) ? dh[t][r] * ks : 0.f;
    }
    // ---- layer 0 (proj.0): dW0 += dh1^T x ; db0
    stage_ds<DT>(DSw, dcur, D, ln);
    __syncthreads();
    outer_stage<D, KT, Sh::G_W0, DT, DT>(DS, IN, acc, slab, w, ln);
    if (tid < D) {
      const float sred = region_rowsum<REG>(DS, tid);
      if constexpr (Sh::REGACC) dbacc[0] += sred; else slab[3 * D * D + tid] += sred;
    }
    __syncthreads();
    // next group's hat / dT operands stream in under the dx chain
    if ((grp + 1) * 4 < n_items) {
      const Item nx = item_of(grp + 1);
      dma_block16<KP32 * 128>(INl, act_rsrc(nx), 96 * D * 4);
      const int nrow = nx.rb * 32 + c, nrowc = imin(nrow, nx.nrows - 1), nbh = nx.b * p.H + hd;
      load_rows<KT>(gin, (nx.isK ? p.dT + ((int64_t)nbh * p.M + nrowc) * p.kp : p.dQh + ((int64_t)nbh * p.N + nrowc) * p.kp),
                    p.kp, nx.has && nrow < nx.nrows);
    }
    {
      f32x16 dxm[DT];
      mm_acc<DT, DT>(p.WfT[0], dcur, dxm);
      if (rv) {  // second-path gradient: dQ/dK += MLP backward
        float* dst = it.isK ? p.dK + it.b * p.dk_sb + hd * p.dk_sh + (int64_t)row * p.dk_sn
                            : p.dQ + it.b * p.dq_sb + hd * p.dq_sh + (int64_t)row * p.dq_sn;
#pragma unroll
        for (int t = 0; t < DT; ++t)
#pragma unroll
          for (int g4 = 0; g4 < 4; ++g4) {
            const int c0 = 32 * t + 8 * g4 + 4 * h;
            f32x4 v = *reinterpret_cast<f32x4*>(dst + c0);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] += dxm[t][4 * g4 + e];
            *reinterpret_cast<f32x4*>(dst + c0) = v;
          }
      }
    }
  }
  if constexpr (Sh::REGACC) {  // this wave's tiles and (wave 0/1) bias sums: written exactly once
#pragma unroll
    for (int gt = 0; gt < Sh::NTILE; ++gt)
      if ((gt & 3) == w) {
        const TileDst<D, KT> t = tile_dst<D, KT>(slab, gt);
        tile_store<0>(t.base, t.ldo, t.orows, t.icols, t.ot, t.it, acc[gt >> 2], false, lane);
      }
    const int tid = threadIdx.x;
    if (tid < D) {
      slab[3 * D * D + tid] = dbacc[0];
      slab[3 * D * D + D + tid] = dbacc[1];
      slab[3 * D * D + 2 * D + tid] = dbacc[2];
    }
  }
}

// ------------------------------------------------------------------------------------
// B3s: projection backward for k <= 16 clusters and d = 64 or 96 (config/python.py and config/java.py).
// Same math and slab layout as k_proj_bwd. Differences:
//  * dS_h and dC_h are k x k and k x d: each wave accumulates them over its OWN items with 16x16x4
//    MFMAs (dT^T Kh from a global-load operand and the hat block; dZ^T po through a wave-private
//    transpose), so these two small products need no barriers; the 4 wave partials are summed in a
//    fixed order once per workgroup.
//  * only the three d x d products dW2, dW1, dW0 go through the shared staging, split evenly over the
//    4 waves (d = 64: one 32x32 tile each; d = 96: 9 tiles x 4 K-quarters = 36 units, 9 per wave, see
//    outer_stage96), and each wave's next chain product runs between the two barriers of a stage:
//    6 barriers per group of 4 items instead of 10, no idle waves.
//  * bias sums: each wave sums its own staged rows (8 LDS reads per feature), the 4 wave partials are
//    combined once at the end.
//  * chain products over the cluster index stop at K = 16.
// ------------------------------------------------------------------------------------
template <int D>
struct ProjBwdSmallShape {
  static constexpr int DT = D / 32, NS = D / 2, REG = D * 32;
  static constexpr int NSL = D == 64 ? 1 : 3;               // dW tile slots per wave per stage
  static constexpr int HATF = 16 * 32;                       // hat block: 16 features x 32 rows
  static constexpr int GINF = 32 * 16;                       // dT / dQh rows of the item: 32 rows x 16
  static constexpr int PARTF = 256 + 16 * D + 3 * D + 16;    // end-of-kernel wave partial: dS | dC | db | sum dZ
  // d = 96 (one workgroup per CU anyway): weight fragments in LDS. WF holds the d x d layer of the next
  // chain product (W2, W1, W0 in turn, DMA'd a stage ahead); CF / SF the head's cluster fragments
  // (K-groups 0, 1 only: k <= 16), loaded once.
  // d = 64 keeps two workgroups per CU within 80 KiB: the hat / gin blocks go into the wave's own DS region
  // (free from B6 to the stage of layer 2, so they are DMA'd right after B6) and the small cluster chains
  // read their fragments from L2 (LCS = 0). (Round 1's d = 64 LW with the d = 96 layout, 102 KiB, one
  // workgroup per CU, measured no faster: 0.404 vs 0.402 ms.)
  static constexpr bool LW = true, LCS = D == 96, HIN_DS = D == 64;
  static constexpr int WF = 8 * REG + (HIN_DS ? 0 : 4 * HATF + 4 * GINF), WFF = LW ? D * D : 0;
  static constexpr int CF = WF + WFF, CFF = LCS ? D / 32 * 512 : 0, SF = CF + CFF, SFF = LCS ? 512 : 0;
  // d = 64: 80 KiB (2 workgroups per CU); d = 96: 156 KiB
  static_assert(!HIN_DS || 512 + HATF + GINF <= REG, "dZ scratch | hat | gin fit the wave's DS region");
  static constexpr size_t LDS_BYTES = sizeof(float) * (SF + SFF);
  static_assert(4 * PARTF + (D == 96 ? 9 * 1024 : 0) <= 8 * REG, "end-of-kernel partials fit the staging");
};

// One K-quarter (s4 = 4q .. 4q+3: 32 of the 128 staged rows, 16 MFMAs) of a staged outer product:
// operand reads and the MFMAs, split so the next quarter's reads can be issued first.
template <int REG>
__device__ __forceinline__ void quarter_load(const float* __restrict__ a, const float* __restrict__ b, int q, int sw,
                                             f32x4 (&av)[4], f32x4 (&bv)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int off = (q >> 1) * REG + 4 * ((4 * (q & 1) + i) ^ sw);
    av[i] = *reinterpret_cast<const f32x4*>(a + off);
    bv[i] = *reinterpret_cast<const f32x4*>(b + off);
  }
}

// d = 96 stage: the 9 output tiles x 4 K-quarters are 36 units; wave w takes units 9w .. 9w+8 in
// tile-major order, i.e. tiles t = 2w + j (ot = t / 3, it = t % 3) over the quarters [w, 4), [0, 4),
// [0, w] for j = 0, 1, 2. Slot 0 of wave w > 0 and slot 2 of wave w < 3 are the two halves of one tile,
// combined in a fixed order at the end. The operand reads of the next position are issued before the
// current position's MFMAs (unconditionally: every read is in bounds), so only the MFMA blocks sit
// under the wave-uniform activity branches.
template <int REG, bool BF = false>
__device__ __forceinline__ void outer_stage96(const float* __restrict__ ds, const float* __restrict__ in,
                                              f32x16 (&acc)[3], int w, int lane) {
  asm volatile("" : "+v"(lane));
  const int c = lane & 31, h = lane >> 5, sw = (c >> 1) & 7;
  const float* a[3];
  const float* b[3];
#pragma unroll
  for (int j = 0; j < 3; ++j) {
    const int t = 2 * w + j, ot = t / 3, it = t - 3 * ot;
    a[j] = ds + 2 * h * REG + (32 * ot + c) * 32;
    b[j] = in + 2 * h * REG + (32 * it + c) * 32;
  }
  f32x4 av[2][4], bv[2][4];
  quarter_load<REG>(a[0], b[0], 0, sw, av[0], bv[0]);
#pragma unroll
  for (int P = 0; P < 12; ++P) {
    const int j = P >> 2, q = P & 3;
    if (P + 1 < 12) quarter_load<REG>(a[(P + 1) >> 2], b[(P + 1) >> 2], (P + 1) & 3, sw, av[(P + 1) & 1], bv[(P + 1) & 1]);
    if (j == 1 || (j == 0 ? q >= w : q <= w)) {
      if constexpr (BF) {
#pragma unroll
        for (int i = 0; i < 4; i += 2)
          acc[j] = mfma_bf(pack8(av[P & 1][i], av[P & 1][i + 1]), pack8(bv[P & 1][i], bv[P & 1][i + 1]), acc[j]);
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[j] = mfma(av[P & 1][i][e], bv[P & 1][i][e], acc[j]);
      }
    }
    fence_sched();
  }
}

template <int D, bool BF = false>
__device__ __forceinline__ void outer_stage_s(const float* __restrict__ ds, const float* __restrict__ in,
                                              f32x16 (&acc)[ProjBwdSmallShape<D>::NSL], int w, int lane) {
  if constexpr (D == 64) acc[0] = outer_tile<ProjBwdSmallShape<D>::REG, BF>(ds, in, w >> 1, w & 1, acc[0], lane);
  else outer_stage96<ProjBwdSmallShape<D>::REG, BF>(ds, in, acc, w, lane);
}

// bias-gradient partial of this wave: sums of its own staged rows, feature lane (and lane + 64 for d = 96).
// (Batching the reads, or moving them under the chain / outer MFMAs as side work, pushed d = 96 into
// spills or measured no faster on one box: tools/ab_multi.sh.)
template <int D>
__device__ __forceinline__ void own_rowsum(const float* __restrict__ dsw, float (&db)[2], int lane) {
  asm volatile("" : "+v"(lane));
#pragma unroll
  for (int u = 0; u < (D + 63) / 64; ++u) {
    const int f = lane + 64 * u;
    if (f < D) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const f32x4 v = *reinterpret_cast<const f32x4*>(dsw + act_off(f, 4 * k));
        s += (v[0] + v[1]) + (v[2] + v[3]);
      }
      db[u] += s;
    }
  }
}

// BF: CSA_DTYPE_BF16 (the C^T dZ chain, the three W^T chains and the three d x d weight-gradient outer products on
// bf16 MFMA; the S^T dT chain, dS, dC, the bias sums and every elementwise step stay fp32)
template <int D, bool BF = false>
__global__ __launch_bounds__(256, ProjBwdSmallShape<D>::LCS ? 1 : 2) void k_proj_bwd_s(const KArgs p) {
  static_assert(D == 64 || D == 96, "d x d stages split over 4 waves for d = 64 and 96");
  using Sh = ProjBwdSmallShape<D>;
  using Sf = ProjBwdShape<D, 1>;  // slab layout
  constexpr int DT = Sh::DT, NS = Sh::NS, REG = Sh::REG, NSL = Sh::NSL, ABLK = Sf::ABLK;
  constexpr bool LW = Sh::LW, LCS = Sh::LCS, HIN_DS = Sh::HIN_DS;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  float* DS = lds;
  float* IN = lds + 4 * REG;
  const int lane = lane_id(), c = lane & 31, h = lane >> 5, c16 = lane & 15, g4 = lane >> 4;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int hd = blockIdx.y;
  const int per_b = p.NQB + p.NKB;
  // this workgroup's item kind, its index among the workgroups of that kind and their count, its slab
  int kind = p.pb_kind, g = blockIdx.x, G = gridDim.x, gs = p.pb_goff + g;
  if (kind == 3) {
    const bool key = g < p.pb_gk;
    kind = key ? 1 : 2; gs = g; G = key ? p.pb_gk : G - p.pb_gk; g = key ? g : g - p.pb_gk;
  }
  // items of the head, per batch element: all (Q blocks, then K blocks), or one kind only
  const int ipb = kind == 1 ? p.NKB : kind == 2 ? p.NQB : per_b, roff = kind == 1 ? p.NQB : 0;
  const int i_lo = (int)((int64_t)g * p.B * ipb / G), i_hi = (int)((int64_t)(g + 1) * p.B * ipb / G);
  const int n_items = i_hi - i_lo;  // this workgroup's items: i_lo .. i_hi - 1 of its kind's items
  float* slab = p.slab + ((int64_t)hd * p.G + gs) * p.slab_floats;
  const float ks = p.proj_p > 0.f ? 1.f / (1.f - p.proj_p) : 1.f;
  const float* CfT = p.CfT + (size_t)hd * 32 * D;
  const float* SfT = p.SfT + (size_t)hd * 32 * 32;
  const float* WFs = lds + Sh::WF;  // LW: weight fragments of the next chain product
  const float* CFs = lds + Sh::CF;  // LW: cluster fragments (K-groups 0, 1)
  const float* SFs = lds + Sh::SF;
  float* DSw = DS + w * REG;
  float* INw = IN + w * REG;
  // hat / gin blocks: HIN_DS: floats [512, 1536) of the wave's DS region (after the dZ scratch)
  const int hat_f = HIN_DS ? w * REG + 512 : 8 * REG + w * Sh::HATF;
  const int gin_f = HIN_DS ? w * REG + 512 + Sh::HATF : 8 * REG + 4 * Sh::HATF + w * Sh::GINF;
  float* HATw = lds + hat_f;
  const uint32_t INl = lds_offset(IN) + 4 * REG * w, HATl = lds_offset(lds) + 4 * hat_f;
  const float* GINw = lds + gin_f;
  const uint32_t GINl = lds_offset(lds) + 4 * gin_f;
  f32x16 acc[3][NSL];  // this wave's dW2 | dW1 | dW0 tile slots (outer_stage_s)
#pragma unroll
  for (int l = 0; l < 3; ++l)
#pragma unroll
    for (int j = 0; j < NSL; ++j) acc[l][j] = zero16();
  constexpr bool H2C = h2c_path(D, 1, BF);  // dC from h2 (see h2c_path); this kernel runs for k <= 16 only
  f32x4 accS = {0.f, 0.f, 0.f, 0.f}, accC[D / 16], accZ = accS;
#pragma unroll
  for (int t = 0; t < D / 16; ++t) accC[t] = accS;
  float dbp[3][2] = {{0.f, 0.f}, {0.f, 0.f}, {0.f, 0.f}};  // db0 | db1 | db2 partials (own_rowsum)

  struct Item { int b, r, isK, rb, nrows; bool has; };
  auto item_of = [&](int grp) {
    Item it;
    const int item = grp * 4 + w;
    it.has = item < n_items;
    it.b = it.has ? (i_lo + item) / ipb : 0;
    it.r = it.has ? roff + (i_lo + item) % ipb : 0;
    it.isK = it.r >= p.NQB;
    it.rb = it.isK ? it.r - p.NQB : it.r;
    it.nrows = it.isK ? p.M : p.N;
    return it;
  };
  auto act_rsrc = [&](const Item& it) {
    return make_rsrc(p.Act + ((int64_t)(it.b * p.H + hd) * per_b + it.r) * ABLK, ABLK * 4);
  };
  // per-item operands DMA'd into LDS one group ahead (register-free, so they are issued early):
  // the hat block and the item's 32 dT / dQh rows, read at the top of the group both in the acc
  // orientation (lane = row) and as the 16x16x4 A operand (lane (c16, g4), step s: dT[row 4s + g4][c16]).
  // the item's hat block: its rows of Qh / Kh as k_proj_fwd_l stored them for the attention kernels ([row][16],
  // rows past the item's last row not fetched), so the forward saves no second copy in the activation block
  // (HAT_ACT: the activation block's feature-major copy, the round-4 form)
  constexpr bool HQK = true;
  auto prefetch_hat = [&](const Item& it) {
    if constexpr (HQK) {
      const int bh = it.b * p.H + hd, row0 = it.rb * 32;
      const float* src = it.isK ? p.Kh + ((int64_t)bh * p.M + row0) * p.kp : p.Qh + ((int64_t)bh * p.N + row0) * p.kp;
      dma_block16<2048>(HATl, make_rsrc(src, imin(32, it.nrows - row0) * p.kp * 4), 0);
    } else {
      dma_block16<2048>(HATl, act_rsrc(it), 96 * D * 4);
    }
  };
  // element (row, cluster f < 16) of the wave's hat block
  auto hat_at = [&](int row, int f) { return HQK ? HATw[row * 16 + f] : HATw[act_off(f, row)]; };
  auto prefetch = [&](const Item& it) {
    const int bh = it.b * p.H + hd, row0 = it.rb * 32;
    const float* src = it.isK ? p.dT + ((int64_t)bh * p.M + row0) * p.kp : p.dQh + ((int64_t)bh * p.N + row0) * p.kp;
    // rows past the item's last row are outside the descriptor: not fetched (values masked below)
    dma_block16<2048>(GINl, make_rsrc(src, imin(32, it.nrows - row0) * p.kp * 4), 0);
  };
  // LW: layer l's d x d fragments (36 KiB) -> WF, a quarter per wave (visible after a vmcnt wait + barrier)
  auto load_wf = [&](int l) {
    dma_block16<D * D>(lds_offset(lds) + 4 * Sh::WF + D * D * w, make_rsrc(p.WfT[l], 4 * D * D), D * D * w);
  };
  if constexpr (LCS) {  // the head's cluster fragments, K-groups 0 and 1 of each tile (2 KiB pieces)
    if (w < DT) dma_block16<2048>(lds_offset(lds) + 4 * (Sh::CF + 512 * w), make_rsrc(CfT, 4 * 32 * D), 4096 * w);
    else if (w == 3) dma_block16<2048>(lds_offset(lds) + 4 * Sh::SF, make_rsrc(SfT, 4 * 32 * 32), 0);
    wait_vm_all();
    __syncthreads();
  }
  if constexpr (HQK) {  // rows past an item's last row are never fetched: they only ever hold finite data
#pragma unroll
    for (int e = 0; e < Sh::HATF / 64; ++e) HATw[lane + 64 * e] = 0.f;
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  prefetch_hat(item_of(0));
  prefetch(item_of(0));
  if constexpr (LW) load_wf(2);
#define PHASE(i)

  for (int grp = 0; grp * 4 < n_items; ++grp) {
    int tid = threadIdx.x;  // opaque: per-lane addresses are recomputed in the loop, not hoisted
    asm volatile("" : "+v"(tid));
    const int ln = tid & 63;
    const Item it = item_of(grp);
    const int row = it.rb * 32 + c;
    const bool rv = it.has && row < it.nrows;
    const int rowc = imin(row, it.nrows - 1);
    const int bh = it.b * p.H + hd;
    const __amdgpu_buffer_rsrc_t ar = act_rsrc(it);
    // hat block, gin, dTt (LW: the W2 fragments, D*D/1024 DMAs issued after them, may be in flight)
    if constexpr (LW) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D * D / 1024) : "memory");
    else wait_vm_all();
    PHASE(0);
    if constexpr (BF) dma_block16<D * 64>(INl + 2 * REG, ar, 64 * D * 4);  // bf16 po -> upper half (widened below)
    else if constexpr (H2C) dma_block16<D * 128>(INl, ar, 32 * D * 4);  // h2 -> own IN region (free since B6): the dC
    else dma_block16<D * 128>(INl, ar, 64 * D * 4);  // product below, then layer 2's stage (po -> IN otherwise)
    f32x16 gin[1];
    float dTt[8];
#pragma unroll
    for (int g2 = 0; g2 < 2; ++g2) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(GINw + c * 16 + 8 * g2 + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) gin[0][4 * g2 + e] = rv ? v[e] : 0.f;
    }
#pragma unroll
    for (int r = 8; r < 16; ++r) gin[0][r] = 0.f;  // clusters >= 16
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float v = GINw[(4 * s + g4) * 16 + c16];
      dTt[s] = (it.has && it.isK && it.rb * 32 + 4 * s + g4 < p.M) ? v : 0.f;
    }
    // ---- dS_h += dT^T Kh (K items), private 16x16x4: B = Kh[row 4s + g4][cluster c16] from the hat block
    if (it.isK) {
#pragma unroll
      for (int s = 0; s < 8; ++s) accS = mfma16(dTt[s], hat_at(4 * s + g4, c16), accS);
    }
    // ---- hat (acc orientation, clusters >= 16 are zero) and dZ = (S^T dT | dQh) * hat (1 - hat)
    f32x16 hat;
#pragma unroll
    for (int r = 0; r < 16; ++r) hat[r] = r < 8 ? hat_at(c, crow(r, h)) : 0.f;
    if constexpr (HQK) {  // registers 0-3 / 4-7 are clusters 4h .. 4h+3 / 8+4h .. of row c: two b128 reads
      const f32x4 h0 = *reinterpret_cast<const f32x4*>(HATw + c * 16 + 4 * h);
      const f32x4 h1 = *reinterpret_cast<const f32x4*>(HATw + c * 16 + 8 + 4 * h);
#pragma unroll
      for (int e = 0; e < 4; ++e) { hat[e] = h0[e]; hat[4 + e] = h1[e]; }
    }
    f32x16 dz[1];
    if (it.isK) {
      mm_acc_f<1, 1, 2, LCS ? 8 : 16, LCS>(LCS ? SFs : SfT, gin, dz);  // dKh^T = S^T dT^T (clusters < 16)
    } else {
      dz[0] = gin[0];
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) dz[0][r] = r < 8 ? dz[0][r] * hat[r] * (1.f - hat[r]) : 0.f;
    // dZ -> wave-private transpose scratch in the (free) DS region: [row][cluster], 16 clusters per row
#pragma unroll
    for (int g2 = 0; g2 < 2; ++g2) {
      f32x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = dz[0][4 * g2 + e];
      *reinterpret_cast<f32x4*>(DSw + c * 16 + 8 * g2 + 4 * h) = v;
    }
    // ---- dp^T = C^T dZ^T (clusters < 16)
    f32x16 dcur[DT];
    mm_acc_f<DT, 1, 2, LCS ? 8 : 16, LCS, BF>(LCS ? CFs : CfT, dz, dcur);
    wait_vm_all();  // po (LW: and the W2 fragments)
    if constexpr (BF) widen_act_bf<REG>(INw, ln);
    // ---- dC_h += dZ^T po, private 16x16x4: A = dZ[row 4s + g4][cluster c16], B = po[row 4s + g4][16t + c16]
    //      (H2C: dZ^T h2, and accZ[e] = sum over rows of dZ[.][cluster 4 g4 + e], B = 1)
#pragma unroll
    for (int s = 0; s < 8; ++s) {
      const float a = DSw[(4 * s + g4) * 16 + c16];
#pragma unroll
      for (int t = 0; t < D / 16; ++t) accC[t] = mfma16(a, INw[act_off(16 * t + c16, 4 * s + g4)], accC[t]);
      if constexpr (H2C) accZ = mfma16(a, 1.f, accZ);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    PHASE(1);
    // ---- layer 2 (proj.6): stage dp, h2 -> IN; dh2_pre = W2^T dp under the DMA
    stage_ds<DT>(DSw, dcur, D, ln);
    if constexpr (LW) __syncthreads();  // B0: every wave's quarter of the W2 fragments landed
    if constexpr (BF) dma_block16<D * 64>(INl + 2 * REG, ar, 32 * D * 4);  // bf16 h2 -> upper half
    else if constexpr (!H2C) dma_block16<D * 128>(INl, ar, 32 * D * 4);  // h2 (H2C: in IN since the group top)
    f32x16 dh[DT];
    mm_acc_f<DT, DT, 4 * DT, 16 * DT, LW, BF>(LW ? WFs : p.WfT[2], dcur, dh);
    wait_vm_all();
    if constexpr (BF) widen_act_bf<REG>(INw, ln);
    PHASE(7);
    __syncthreads();  // B1: dp, h2 of every wave staged
    PHASE(2);
    if constexpr (LW) load_wf(1);  // every wave is past its W2 chain
    outer_stage_s<D, BF>(DS, IN, acc[0], w, ln);
    own_rowsum<D>(DSw, dbp[2], ln);
    {
      f32x16 hv[DT];
      read_act<DT>(hv, INw, ln);  // own h2 (relu mask)
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) dcur[t][r] = (hv[t][r] > 0.f) ? dh[t][r] * ks : 0.f;
    }
    if constexpr (LW) wait_vm_all();  // W1 fragments
    PHASE(3);
    __syncthreads();  // B2: stage dW2 read out
    PHASE(2);
    // ---- layer 1 (proj.3): stage dh2, h1 -> IN and x rows under dh1_pre = W1^T dh2
    stage_ds<DT>(DSw, dcur, D, ln);
    if constexpr (BF) dma_block16<D * 64>(INl + 2 * REG, ar, 0);  // bf16 h1 -> upper half
    else dma_block16<D * 128>(INl, ar, 0);  // h1
    f32x4 x4[NS / 4];  // raw (clamped-row) loads: the row mask is applied when x is staged, so the
    {                  // loads do not wait here
      const float* X = it.isK ? p.K + it.b * p.k_sb + hd * p.k_sh + (int64_t)rowc * p.k_sn
                              : p.Q + it.b * p.q_sb + hd * p.q_sh + (int64_t)rowc * p.q_sn;
#pragma unroll
      for (int j = 0; j < NS / 4; ++j) x4[j] = *reinterpret_cast<const f32x4*>(X + h * NS + 4 * j);
    }
    mm_acc_f<DT, DT, 4 * DT, 16 * DT, LW, BF>(LW ? WFs : p.WfT[1], dcur, dh);
    wait_vm_all();
    if constexpr (BF) widen_act_bf<REG>(INw, ln);
    PHASE(4);
    __syncthreads();  // B3
    PHASE(2);
    if constexpr (LW) load_wf(0);  // every wave is past its W1 chain
    outer_stage_s<D, BF>(DS, IN, acc[1], w, ln);
    own_rowsum<D>(DSw, dbp[1], ln);
    {
      f32x16 hv[DT];
      read_act<DT>(hv, INw, ln);  // own h1 (relu mask)
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) dcur[t][r] = (hv[t][r] > 0.f) ? dh[t][r] * ks : 0.f;
    }
    PHASE(3);
    __syncthreads();  // B4
    PHASE(2);
    // ---- layer 0 (proj.0): stage dh1, x -> IN; this item's dQ / dK rows load under the last stage
    stage_ds<DT>(DSw, dcur, D, ln);
#pragma unroll
    for (int s = 0; s < NS; ++s) INw[act_off(s + NS * h, c)] = rv ? x4[s >> 2][s & 3] : 0.f;
    float* dst = it.isK ? p.dK + it.b * p.dk_sb + hd * p.dk_sh + (int64_t)rowc * p.dk_sn
                        : p.dQ + it.b * p.dq_sb + hd * p.dq_sh + (int64_t)rowc * p.dq_sn;
    f32x4 old[2 * DT], old2[2 * DT];
    const bool more = (grp + 1) * 4 < n_items;
    auto load_old = [&]() {
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int g2 = 0; g2 < 4; g2 += 2) old[2 * t + g2 / 2] = *reinterpret_cast<const f32x4*>(dst + 32 * t + 8 * g2 + 4 * h);
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int g2 = 1; g2 < 4; g2 += 2) old2[2 * t + g2 / 2] = *reinterpret_cast<const f32x4*>(dst + 32 * t + 8 * g2 + 4 * h);
    };
    auto prefetch_next = [&]() {
      if (more) {  // private hat / gin regions are free again: next group's operands stream in now
        prefetch_hat(item_of(grp + 1));
        prefetch(item_of(grp + 1));
      }
    };
    if constexpr (LW) {
      wait_vm_all();  // W0 fragments
    } else {
      load_old();
      prefetch_next();
    }
    PHASE(5);
    __syncthreads();  // B5
    PHASE(2);
    if constexpr (LW && !HIN_DS) prefetch_next();  // (after the W0 wait above)
    outer_stage_s<D, BF>(DS, IN, acc[2], w, ln);
    own_rowsum<D>(DSw, dbp[0], ln);
    if constexpr (LW) load_old();  // LW: the dQ / dK rows load under the dx chain (fewer live registers)
    PHASE(3);
    f32x16 dxm[DT];
    mm_acc_f<DT, DT, 4 * DT, 16 * DT, LW, BF>(LW ? WFs : p.WfT[0], dcur, dxm);  // second-path dx = W0^T dh1
    if (rv) {  // dQ / dK += MLP backward
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int g2 = 0; g2 < 4; ++g2) {
          f32x4 v = (g2 & 1) ? old2[2 * t + g2 / 2] : old[2 * t + g2 / 2];
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] += dxm[t][4 * g2 + e];
          *reinterpret_cast<f32x4*>(dst + 32 * t + 8 * g2 + 4 * h) = v;
        }
    }
    PHASE(6);
    __syncthreads();  // B6: DS / IN free for the next group (LW: WF too)
    PHASE(2);
    if constexpr (LW) {
      if constexpr (HIN_DS) prefetch_next();  // DS regions are free: hat / gin first (the next group top
      if (more) load_wf(2);                   // waits for them with the W2 fragments still in flight)
    }
  }
#undef PHASE
  // ---- slab, written once: dW tiles, bias sums and dS / dC, wave partials combined in a fixed order
  float* part = lds + w * Sh::PARTF;  // [dS 16 x 16 | dC 16 x D | db0 | db1 | db2] of this wave
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    part[(4 * g4 + e) * 16 + c16] = accS[e];
#pragma unroll
    for (int t = 0; t < D / 16; ++t) part[256 + (4 * g4 + e) * D + 16 * t + c16] = accC[t][e];
    if (H2C && c16 == 0) part[256 + 19 * D + 4 * g4 + e] = accZ[e];
  }
#pragma unroll
  for (int l = 0; l < 3; ++l)
#pragma unroll
    for (int u = 0; u < (D + 63) / 64; ++u)
      if (lane + 64 * u < D) part[256 + 16 * D + l * D + lane + 64 * u] = dbp[l][u];
  float* shr = lds + 4 * Sh::PARTF;  // d = 96: slot-2 halves of the shared tiles, [stage][wave < 3]
  if constexpr (NSL == 3) {
    if (w < 3) {
#pragma unroll
      for (int l = 0; l < 3; ++l)
#pragma unroll
        for (int r = 0; r < 16; ++r) shr[(3 * l + w) * 1024 + 64 * r + lane] = acc[l][2][r];
    }
  }
  __syncthreads();
#pragma unroll
  for (int l = 0; l < 3; ++l) {
    const int g0 = l == 0 ? Sf::G_W2 : l == 1 ? Sf::G_W1 : Sf::G_W0;
    if constexpr (NSL == 1) {
      const TileDst<D, 1> t = tile_dst<D, 1>(slab, g0 + w);
      tile_store<0>(t.base, t.ldo, t.orows, t.icols, t.ot, t.it, acc[l][0], false, lane);
    } else {
      f32x16 v = acc[l][0];
      if (w > 0) {  // tile 2w: quarters [0, w) from wave w - 1, then [w, 4) from this wave
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = shr[(3 * l + w - 1) * 1024 + 64 * r + lane] + v[r];
      }
      const TileDst<D, 1> t0 = tile_dst<D, 1>(slab, g0 + 2 * w);
      tile_store<0>(t0.base, t0.ldo, t0.orows, t0.icols, t0.ot, t0.it, v, false, lane);
      const TileDst<D, 1> t1 = tile_dst<D, 1>(slab, g0 + 2 * w + 1);
      tile_store<0>(t1.base, t1.ldo, t1.orows, t1.icols, t1.ot, t1.it, acc[l][1], false, lane);
      if (w == 3) {
        const TileDst<D, 1> t2 = tile_dst<D, 1>(slab, g0 + 8);
        tile_store<0>(t2.base, t2.ldo, t2.orows, t2.icols, t2.ot, t2.it, acc[l][2], false, lane);
      }
    }
  }
  const int tid = threadIdx.x;
  for (int e = tid; e < 3 * D; e += 256) {
    float v = 0.f;
#pragma unroll
    for (int ww = 0; ww < 4; ++ww) v += lds[ww * Sh::PARTF + 256 + 16 * D + e];
    slab[3 * D * D + e] = v;  // db0 | db1 | db2
  }
  float* sC = slab + 3 * D * D + 3 * D;  // (32 x D), rows >= 16 zero
  float* sS = sC + 32 * D;               // (32 x 32), rows / cols >= 16 zero
  for (int e = tid; e < 32 * D + 32 * 32; e += 256) {
    float v = 0.f;
    if (e < 32 * D) {
      const int a = e / D, f = e % D;
      if (a < 16) {
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) v += lds[ww * Sh::PARTF + 256 + a * D + f];
      } else if (H2C && a == 16 && f < 16) {  // H2C: row 16 holds sum dZ per cluster f (k_cluster_grad)
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) v += lds[ww * Sh::PARTF + 256 + 19 * D + f];
      }
      sC[e] = v;
    } else {
      const int q = e - 32 * D, a = q / 32, bb = q % 32;
      if (a < 16 && bb < 16) {
#pragma unroll
        for (int ww = 0; ww < 4; ++ww) v += lds[ww * Sh::PARTF + a * 16 + bb];
      }
      sS[q] = v;
    }
  }
}

// ------------------------------------------------------------------------------------
// B4: fixed-order reduction of the partial slabs
//   out dW, db (sum over H x G slabs); dC_h, dS_h (sum over the head's G slabs) -> workspace
// One workgroup per 64 consecutive outputs: lane l owns output e0 + l, wave w sums the slabs
// w, w+4, w+8, ... with 8 independent accumulators (8 loads in flight per lane, each wave load a
// coalesced 256 B row of one slab), then the 4 wave partials are combined in a fixed order.
// The summation order depends only on (H, G), never on timing -> bitwise deterministic.
// ------------------------------------------------------------------------------------
// 16 waves per 64 slab elements: the shared weight elements sum H x G slabs each (432 at B = 256), and with
// four waves only ~200 workgroups (one per CU) held the whole 20 MB of their reads in flight.
constexpr int RS_WAVES = 16;
__global__ __launch_bounds__(64 * RS_WAVES) void k_reduce_slabs(const KArgs p, int D, int KP32, float* __restrict__ dW0,
                                                      float* __restrict__ dW1, float* __restrict__ dW2,
                                                      float* __restrict__ db0, float* __restrict__ db1,
                                                      float* __restrict__ db2, float* __restrict__ dS_ws,
                                                      float* __restrict__ dC_ws) {
  __shared__ float red[RS_WAVES][64];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * 64 + l;
  const int G = p.G;
  const int64_t nW = 3LL * D * D + 3LL * D;
  const int64_t nC = (int64_t)p.H * KP32 * D, nS = (int64_t)p.H * KP32 * KP32;
  int64_t off = 0;
  int s0 = 0, ns = 0;
  if (e < nW) {
    off = e; s0 = 0; ns = p.H * G;
  } else if (e < nW + nC) {
    const int64_t f = e - nW;
    off = nW + f % (KP32 * D); s0 = (int)(f / (KP32 * D)) * G; ns = G;
  } else if (e < nW + nC + nS) {
    const int64_t f = e - nW - nC;
    off = nW + (int64_t)KP32 * D + f % (KP32 * KP32); s0 = (int)(f / (KP32 * KP32)) * G; ns = G;
  }
  const float* src = p.slab + (int64_t)s0 * p.slab_floats + off;
  float acc[8];
#pragma unroll
  for (int a = 0; a < 8; ++a) acc[a] = 0.f;
  int i = w;
  for (; i + RS_WAVES * 7 < ns; i += RS_WAVES * 8) {
#pragma unroll
    for (int a = 0; a < 8; ++a) acc[a] += src[(int64_t)(i + RS_WAVES * a) * p.slab_floats];
  }
#pragma unroll
  for (int a = 0; a < 8; ++a)
    if (i + RS_WAVES * a < ns) acc[a] += src[(int64_t)(i + RS_WAVES * a) * p.slab_floats];
  red[w][l] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (w != 0 || ns == 0) return;
  float s = 0.f;  // the waves' partials in wave order (fixed: deterministic)
#pragma unroll
  for (int v = 0; v < RS_WAVES; ++v) s += red[v][l];
  if (e < nW) {
    const int64_t DD = (int64_t)D * D;
    if (e < DD) dW0[e] = s;
    else if (e < 2 * DD) dW1[e - DD] = s;
    else if (e < 3 * DD) dW2[e - 2 * DD] = s;
    else if (e < 3 * DD + D) db0[e - 3 * DD] = s;
    else if (e < 3 * DD + 2 * D) db1[e - 3 * DD - D] = s;
    else db2[e - 3 * DD - 2 * D] = s;
  } else if (e < nW + nC) {
    dC_ws[e - nW] = s;
  } else {
    dS_ws[e - nW - nC] = s;
  }
}

// dC_h = dC_ws[h] + (dD + dD^T) C_h, dD = S o (dS - <S, dS>)   (softmax over k^2, sbm_attn.py:39)
// One workgroup per (cluster row a, head): the k coefficients dD(a,b) + dD(b,a) go to LDS once and
// the D outputs of row a are k-term fmaf chains over coalesced rows of C (b ascending; the <S, dS>
// reduction is a fixed-order tree), so the result is deterministic.
// h2c (h2c_path): dC_ws rows 0..15 hold sum dZ^T h2 and row 16 sum dZ per cluster; the po product is formed here,
// once per head: sum_f dZ^T h2[a][f] W2[t][f] + sumdZ[a] b2[t] (fixed order)
__global__ __launch_bounds__(128) void k_cluster_grad(const float* __restrict__ S, const float* __restrict__ dS_ws,
                                                      const float* __restrict__ dC_ws, const float* __restrict__ C,
                                                      float* __restrict__ dC, int k, int D, int KP32,
                                                      const float* __restrict__ W2, const float* __restrict__ b2,
                                                      int h2c) {
  const int a = blockIdx.x, hd = blockIdx.y, tid = threadIdx.x;
  __shared__ float red[128];
  __shared__ float coef[128];
  __shared__ float arow[256];  // h2c: row a of sum dZ^T h2 (D <= 256)
  if (h2c)
    for (int f = tid; f < D; f += 128) arow[f] = dC_ws[((size_t)hd * KP32 + a) * D + f];
  // h2c: this thread's row t = tid of W2, loaded before the softmax backward so its latency overlaps it
  const bool w4 = h2c && ((uintptr_t)W2 & 15) == 0 && (D & 3) == 0 && D <= 128;
  f32x4 wv[32];
  if (w4 && tid < D) {
    const f32x4* wr = reinterpret_cast<const f32x4*>(W2 + (size_t)tid * D);
#pragma unroll
    for (int j = 0; j < 32; ++j)
      if (4 * j < D) wv[j] = wr[j];
  }
  const float* Sh = S + (size_t)hd * KP32 * KP32;
  const float* dSh = dS_ws + (size_t)hd * KP32 * KP32;
  float acc = 0.f;
  for (int e = tid; e < k * k; e += 128) {
    const int r = e / k, c = e % k;
    acc += Sh[r * KP32 + c] * dSh[r * KP32 + c];
  }
  red[tid] = acc;
  __syncthreads();
  for (int s = 64; s > 0; s >>= 1) {
    if (tid < s) red[tid] += red[tid + s];
    __syncthreads();
  }
  const float dot = red[0];
  if (tid < k)
    coef[tid] = Sh[a * KP32 + tid] * (dSh[a * KP32 + tid] - dot) + Sh[tid * KP32 + a] * (dSh[tid * KP32 + a] - dot);
  __syncthreads();
  const float* Ch = C + (size_t)hd * k * D;
  const float* Ah = dC_ws + (size_t)hd * KP32 * D;
  for (int t = tid; t < D; t += 128) {
    float s;
    if (h2c) {  // row t of W2 (w4: preloaded in 16-B pieces, t = tid); f ascending (fixed order)
      s = 0.f;
      if (w4) {
#pragma unroll
        for (int j = 0; j < 32; ++j)
          if (4 * j < D)
#pragma unroll
            for (int e = 0; e < 4; ++e) s = fmaf(arow[4 * j + e], wv[j][e], s);
      } else {
        for (int f = 0; f < D; ++f) s = fmaf(arow[f], W2[(size_t)t * D + f], s);
      }
      s = fmaf(Ah[16 * D + a], b2[t], s);
    } else {
      s = Ah[a * D + t];
    }
    for (int b = 0; b < k; ++b) s = fmaf(coef[b], Ch[b * D + t], s);
    dC[((size_t)hd * k + a) * D + t] = s;
  }
}

__global__ void k_ste_sample(const float* __restrict__ pr, const float* __restrict__ u, float* __restrict__ A,
                             int64_t n, float lo, float hi) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
    A[e] = (u[e] < fminf(fmaxf(pr[e], lo), hi)) ? 1.f : 0.f;
}

__global__ void k_ste_backward(const float* __restrict__ A, const float* __restrict__ g, float* __restrict__ out,
                               int64_t n) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256)
    out[e] = fminf(fmaxf(A[e] * g[e], -1.f), 1.f);
}

// ------------------------------------------------------------------------------------
// Host side
// ------------------------------------------------------------------------------------

struct Stage {  // records caller-owned events around one stage (no-op when prof is NULL)
  const csa_prof* pf; int s; hipStream_t st;
  Stage(const csa_prof* pf_, int s_, hipStream_t st_) : pf(pf_), s(s_), st(st_) {
    if (pf && pf->start[s]) (void)hipEventRecord((hipEvent_t)pf->start[s], st);
  }
  ~Stage() {
    if (pf && pf->stop[s]) (void)hipEventRecord((hipEvent_t)pf->stop[s], st);
  }
};

csa_status fail(csa_status s, const char* msg) {
  csa::set_error("%s", msg);
  return s;
}

// a HIP runtime call (not a launch) failed: report the thread's last HIP error
csa_status fail_hip(const char* what) {
  const hipError_t e = hipGetLastError();
  csa::set_error("%s: %s", what, hipGetErrorString(e));
  return CSA_LAUNCH_FAILED;
}

csa_status check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    csa::set_error("%s: %s", what, hipGetErrorString(e));
    return CSA_LAUNCH_FAILED;
  }
  return CSA_OK;
}

bool supported(int64_t d, int64_t k, uint32_t flags) {
  if (d != 64 && d != 96) return false;
  if (flags & CSA_FLAG_DENSE) return true;
  return k >= 1 && k <= (d == 64 ? 128 : 32);  // d=64: cluster sweep up to 128 (BASELINE config 5)
}

KArgs make_kargs(const csa_sbm_fwd_args* a, const Layout& L) {
  KArgs p;
  memset(&p, 0, sizeof(p));
  p.B = (int)a->B; p.H = (int)a->H; p.N = (int)a->N; p.M = (int)a->M; p.k = (int)L.k; p.kp = (int)L.kp;
  p.NQB = (int)L.NQB; p.NKB = (int)L.NKB; p.Mpad = (int)L.Mpad;
  p.Q = a->Q; p.K = a->K; p.V = a->V;
  p.q_sb = a->q_sb; p.q_sh = a->q_sh; p.q_sn = a->q_sn;
  p.k_sb = a->k_sb; p.k_sh = a->k_sh; p.k_sn = a->k_sn;
  p.v_sb = a->v_sb; p.v_sh = a->v_sh; p.v_sn = a->v_sn;
  p.mask = a->key_mask; p.mask_sb = a->mask_sb;
  p.bf16 = a->dtype == CSA_DTYPE_BF16;
  for (int l = 0; l < 3; ++l) p.pb[l] = a->proj_b[l];
  void* st = a->state;
  for (int l = 0; l < 3; ++l) {
    p.Wf[l] = (const float*)((char*)st + L.Wf[l]);
    p.WfT[l] = (const float*)((char*)st + L.WfT[l]);
  }
  p.Cf = (const float*)((char*)st + L.Cf); p.CfT = (const float*)((char*)st + L.CfT);
  p.Sf = (const float*)((char*)st + L.Sf); p.SfT = (const float*)((char*)st + L.SfT);
  p.S = (const float*)((char*)st + L.S);
  p.Qh = (float*)((char*)st + L.Qh); p.Kh = (float*)((char*)st + L.Kh); p.T = (float*)((char*)st + L.T);
  p.stats = (float*)((char*)st + L.stats);
  p.Act = (a->flags & CSA_FLAG_FWD_ONLY) ? nullptr : (float*)((char*)st + L.Act);
  p.Abits = (uint32_t*)((char*)st + L.Abits); p.Rbits = (uint32_t*)((char*)st + L.Rbits);
  p.cnt = (uint32_t*)((char*)st + L.cnt);
  p.tdead = (unsigned long long*)((char*)st + L.tdead);
  p.U = a->uniforms;
  p.seed_lo = (uint32_t)a->seed; p.seed_hi = (uint32_t)(a->seed >> 32); p.off = (uint32_t)a->offset;
  p.attn_p = a->attn_dropout; p.proj_p = a->proj_dropout;
  p.drop_thr = (uint32_t)ceil((double)a->attn_dropout * 65536.0);
  p.pdrop_thr = (uint32_t)ceil((double)a->proj_dropout * 65536.0);
  p.scale = 1.f / sqrtf((float)a->d);
  p.X = a->X;
  const bool xc = a->x_sb == 0 && a->x_sh == 0 && a->x_sn == 0;  // zero triple: (B,H,N,d) contiguous
  p.x_sb = xc ? a->H * a->N * a->d : a->x_sb;
  p.x_sh = xc ? a->N * a->d : a->x_sh;
  p.x_sn = xc ? a->d : a->x_sn;
  return p;
}

// (b, h, row) element strides of a (B,H,R,d) operand; the zero triple means contiguous
struct Str3 { int64_t sb, sh, sn; };
inline Str3 strides_or_contig(int64_t sb, int64_t sh, int64_t sn, int64_t H, int64_t R, int64_t d) {
  if (sb == 0 && sh == 0 && sn == 0) return Str3{H * R * d, R * d, d};
  return Str3{sb, sh, sn};
}

csa_status validate_fwd(const csa_sbm_fwd_args* a) {
  if (!a) return fail(CSA_INVALID_ARG, "null args");
  if (a->dtype != CSA_DTYPE_F32 && a->dtype != CSA_DTYPE_BF16) return fail(CSA_INVALID_ARG, "dtype must be CSA_DTYPE_F32 or CSA_DTYPE_BF16");
  if (a->dtype == CSA_DTYPE_BF16 && !(a->flags & CSA_FLAG_DENSE) && a->k > 16)
    return fail(CSA_UNSUPPORTED_SHAPE, "bf16 SBM attention is instantiated for k <= 16");
  const bool dense = a->flags & CSA_FLAG_DENSE;
  if (a->B < 1 || a->H < 1 || a->N < 1 || a->M < 1) return fail(CSA_INVALID_ARG, "B, H, N, M must be >= 1");
  if (!a->Q || !a->K || !a->V || !a->X || !a->state) return fail(CSA_INVALID_ARG, "null Q/K/V/X/state");
  if (!supported(a->d, a->k, a->flags)) return fail(CSA_UNSUPPORTED_SHAPE, "unsupported (d, k): d=64 with k in [1,128], or d=96 with k in [1,32]");
  if (!dense) {
    if (!a->cluster_w || !a->sparsity) return fail(CSA_INVALID_ARG, "null cluster_w/sparsity");
    for (int l = 0; l < 3; ++l)
      if (!a->proj_w[l] || !a->proj_b[l]) return fail(CSA_INVALID_ARG, "null proj weight/bias");
  }
  if (a->attn_dropout < 0.f || a->attn_dropout >= 1.f || a->proj_dropout < 0.f || a->proj_dropout >= 1.f)
    return fail(CSA_INVALID_ARG, "dropout p must be in [0,1)");
  auto al16 = [](const void* ptr, int64_t sb, int64_t sh, int64_t sn) {
    return (((uintptr_t)ptr) % 16 == 0) && sb % 4 == 0 && sh % 4 == 0 && sn % 4 == 0;
  };
  if (!al16(a->Q, a->q_sb, a->q_sh, a->q_sn) || !al16(a->K, a->k_sb, a->k_sh, a->k_sn) ||
      !al16(a->V, a->v_sb, a->v_sh, a->v_sn))
    return fail(CSA_INVALID_ARG, "Q/K/V must be 16-byte aligned with strides multiple of 4 elements");
  if (!al16(a->X, a->x_sb, a->x_sh, a->x_sn))
    return fail(CSA_INVALID_ARG, "X must be 16-byte aligned with strides multiple of 4 elements");
  return CSA_OK;
}

template <int D, int KPH, bool DENSE, bool BF>
void launch_attn_fwd(const KArgs& p, int BH, const Layout& L, bool has_u, bool drop, hipStream_t st) {
  const size_t lds_bytes = AttnFwdLds<D, KPH>::bytes((int)L.Mpad);
  const dim3 grid(xcd_grid((int)L.NQB, BH));
  if (lds_bytes > 64 * 1024) {
    set_dyn_lds((const void*)k_attn_fwd<D, KPH, DENSE, false, false, BF>, (int)lds_bytes);
    set_dyn_lds((const void*)k_attn_fwd<D, KPH, DENSE, false, true, BF>, (int)lds_bytes);
    set_dyn_lds((const void*)k_attn_fwd<D, KPH, DENSE, !DENSE, false, BF>, (int)lds_bytes);
    set_dyn_lds((const void*)k_attn_fwd<D, KPH, DENSE, !DENSE, true, BF>, (int)lds_bytes);
  }
  if (!DENSE && has_u) {
    if (drop) hipLaunchKernelGGL((k_attn_fwd<D, KPH, DENSE, !DENSE, true, BF>), grid, dim3(64), lds_bytes, st, p);
    else hipLaunchKernelGGL((k_attn_fwd<D, KPH, DENSE, !DENSE, false, BF>), grid, dim3(64), lds_bytes, st, p);
  } else {
    if (drop) hipLaunchKernelGGL((k_attn_fwd<D, KPH, DENSE, false, true, BF>), grid, dim3(64), lds_bytes, st, p);
    else hipLaunchKernelGGL((k_attn_fwd<D, KPH, DENSE, false, false, BF>), grid, dim3(64), lds_bytes, st, p);
  }
}

// bf16 instantiations exist for the shapes BASELINE runs (k <= 16, and the dense ablation) only
template <int D, int KPH, bool DENSE>
void launch_attn_fwd_any(const KArgs& p, int BH, const Layout& L, bool has_u, bool drop, hipStream_t st) {
  if constexpr (KPH <= 8) {
    if (p.bf16) return launch_attn_fwd<D, KPH, DENSE, true>(p, BH, L, has_u, drop, st);
  }
  launch_attn_fwd<D, KPH, DENSE, false>(p, BH, L, has_u, drop, st);
}

template <int D, int KPH, int KT>
csa_status launch_fwd(const csa_sbm_fwd_args* a, const Layout& L, hipStream_t st) {
  KArgs p = make_kargs(a, L);
  const int BH = (int)(a->B * a->H);
  if constexpr (KPH > 0) {
    const int KP32 = 32 * KT;
    float* S = (float*)((char*)a->state + L.S);
    {
    Stage sg(a->prof, CSA_STAGE_PREP, st);
    FragJobs J;
    memset(&J, 0, sizeof(J));
    int n = 0;
    J.j[n++] = FragJob{S, (float*)p.Sf, KP32, KP32, KP32, 0, 1, KT, 16 * KT, (int)a->H, (int64_t)KP32 * KP32,
                       (int64_t)KP32 * KP32};
    J.j[n++] = FragJob{S, (float*)p.SfT, KP32, KP32, KP32, 1, 1, KT, 16 * KT, (int)a->H, (int64_t)KP32 * KP32,
                       (int64_t)KP32 * KP32};
    const int nS = n;  // S_h's fragments: laid out by the head's softmax block
    for (int l = 0; l < 3; ++l) {  // forward weights: A[o][i] = W[o][i]; l=0 lin-perm, else acc-perm
      J.j[n++] = FragJob{a->proj_w[l], (float*)p.Wf[l], D, D, D, 0, l == 0 ? 0 : 1, D / 32, D / 2, 1, 0, 0};
    }
    for (int l = 0; l < 3; ++l) {  // transposed (backward): A[i][o] = W[o][i], acc-perm over o
      J.j[n++] = FragJob{a->proj_w[l], (float*)p.WfT[l], D, D, D, 1, 1, D / 32, D / 2, 1, 0, 0};
    }
    J.j[n++] = FragJob{a->cluster_w, (float*)p.Cf, (int)a->k, D, D, 0, 1, KT, D / 2, (int)a->H, a->k * D,
                       (int64_t)KP32 * D};
    J.j[n++] = FragJob{a->cluster_w, (float*)p.CfT, D, (int)a->k, D, 1, 1, D / 32, 16 * KT, (int)a->H, a->k * D,
                       (int64_t)KP32 * D};
    J.n = n;
    const int kk = (int)(a->k * a->k);
    auto prep = kk <= 256 ? k_prep<1> : kk <= 1024 ? k_prep<4> : kk <= 4096 ? k_prep<16> : k_prep<64>;
    hipLaunchKernelGGL(prep, dim3((unsigned)a->H + 128), dim3(256), 0, st, a->cluster_w, S, (int)a->k, D, KP32,
                       (int)a->H, J, nS);
    }
    {
      Stage sg(a->prof, CSA_STAGE_PROJ_FWD, st);
      bool done = false;
      if constexpr (KT == 1) {  // k <= 32: weight fragments in LDS
        using PL = ProjFwdLds<D, KT>;
        {
          const int64_t items = a->B * (L.NQB + L.NKB), slots = (D == 64 && PL::NW == 4 ? 2 : 1) * 256LL;
          const int G = (int)std::max<int64_t>(1, std::min<int64_t>(slots / a->H, (items + PL::NW - 1) / PL::NW));
          // (PD: the projection dropout's Philox words are drawn; without dropout they are not)
#define CSA_PF_LAUNCH(BFV, PDV)                                                                         \
  do {                                                                                                  \
    set_dyn_lds((const void*)k_proj_fwd_l<D, KT, BFV, PDV>, (int)PL::BYTES);                            \
    hipLaunchKernelGGL((k_proj_fwd_l<D, KT, BFV, PDV>), dim3(G, a->H), dim3(64 * PL::NW), PL::BYTES, st, p); \
  } while (0)
          const bool pd = a->proj_dropout > 0.f;
          if (p.bf16) {  // CSA_DTYPE_BF16: MLP + cluster projection on bf16 MFMA
            if (pd) CSA_PF_LAUNCH(true, true);
            else CSA_PF_LAUNCH(true, false);
          } else {
            if (pd) CSA_PF_LAUNCH(false, true);
            else CSA_PF_LAUNCH(false, false);
          }
#undef CSA_PF_LAUNCH
          done = true;
        }
      }
      if (!done) hipLaunchKernelGGL((k_proj_fwd<D, KT>), dim3(L.NQB + L.NKB, BH), dim3(64), 0, st, p);
    }
    {
      Stage sg(a->prof, CSA_STAGE_ATTN_FWD, st);
      launch_attn_fwd_any<D, KPH, false>(p, BH, L, a->uniforms != nullptr, a->attn_dropout > 0.f, st);
    }
    hipLaunchKernelGGL(k_sparsity_finish, dim3((unsigned)a->H), dim3(256), 0, st, (const uint32_t*)p.cnt, a->sparsity,
                       (int)a->H, (int)a->B, (int)L.NQB, (float)a->B * (float)a->N * (float)a->M);
  } else {
    Stage sg(a->prof, CSA_STAGE_ATTN_FWD, st);
    launch_attn_fwd_any<D, 0, true>(p, BH, L, false, a->attn_dropout > 0.f, st);
  }
  return check_launch("csa_sbm_fwd");
}

// the row constants, then k_attn_bwd_kv (the elementwise backward; ds / G tiles out), then k_attn_bwd_qg, in
// stream order (bf16 mode: k_attn_bwd_qr recomputes the query side instead of reading tiles, bwd_handoff).
// mid(): enqueued between the key half and the query half (the concurrent schedule forks the projection
// backward's key-block items there).
template <int D, int KPH, bool DENSE, bool DROP, bool DG, bool BF, typename MID>
void launch_attn_bwd_v(const KArgs& p, int BH, const Layout& L, const csa_prof* pf, hipStream_t st, MID mid) {
  using SH = AttnBwdShape<D, KPH>;
  if constexpr (DG) {  // (otherwise k_attn_bwd_kv forms the row constants itself)
    Stage sg(pf, CSA_STAGE_ATTN_ROWPREP, st);
    constexpr int RPW = 4 * (64 / (D / 4 <= 16 ? 16 : 32));  // rows per wave (k_attn_rowprep)
    const int64_t rows = (int64_t)BH * L.NQB * 32, per_block = 4LL * RPW;
    hipLaunchKernelGGL(k_attn_rowprep<D>, dim3((unsigned)((rows + per_block - 1) / per_block)), dim3(256), 0, st, p);
  }
  {
    Stage sg(pf, CSA_STAGE_ATTN_BWD_KV, st);
    hipLaunchKernelGGL((k_attn_bwd_kv<D, KPH, DENSE, DROP, DG, BF>), dim3(xcd_grid((int)L.NKB, BH)), dim3(64),
                       SH::KV_BYTES, st, p);
  }
  mid();
  Stage sg(pf, CSA_STAGE_ATTN_BWD_Q, st);
  if constexpr (bwd_handoff<BF>()) {
    hipLaunchKernelGGL((k_attn_bwd_qg<D, KPH, DENSE, BF, !DENSE && !DG>), dim3(xcd_grid((int)L.NQB, BH)), dim3(64), SH::G_BYTES,
                       st, p);
  } else {
    const size_t r_lds = SH::r_bytes((int)L.Mpad);
    if (r_lds > 64 * 1024) set_dyn_lds((const void*)k_attn_bwd_qr<D, KPH, DENSE, DROP, DG, BF>, (int)r_lds);
    hipLaunchKernelGGL((k_attn_bwd_qr<D, KPH, DENSE, DROP, DG, BF>), dim3(xcd_grid((int)L.NQB, BH)), dim3(64), r_lds,
                       st, p);
  }
}

template <int D, int KPH, bool DENSE, bool BF, typename MID>
void launch_attn_bwd_b(const KArgs& p, int BH, const Layout& L, bool drop, const csa_prof* pf, hipStream_t st, MID mid) {
  const bool dg = p.dgraph != nullptr || p.dattn != nullptr;
  if (p.dattn)  // sum_j dattn_ij attn_ij per query row, added to gamma by k_attn_rowprep
    hipLaunchKernelGGL((k_attn_gx<D, DENSE>), dim3(xcd_grid((int)L.NQB, BH)), dim3(64), 0, st, p);
  if (drop) {
    if (dg) return launch_attn_bwd_v<D, KPH, DENSE, true, true, BF>(p, BH, L, pf, st, mid);
    return launch_attn_bwd_v<D, KPH, DENSE, true, false, BF>(p, BH, L, pf, st, mid);
  }
  if (dg) return launch_attn_bwd_v<D, KPH, DENSE, false, true, BF>(p, BH, L, pf, st, mid);
  return launch_attn_bwd_v<D, KPH, DENSE, false, false, BF>(p, BH, L, pf, st, mid);
}

template <int D, int KPH, bool DENSE, typename MID>
void launch_attn_bwd(const KArgs& p, int BH, const Layout& L, bool drop, const csa_prof* pf, hipStream_t st, MID mid) {
  if constexpr (KPH <= 8) {
    if (p.bf16) return launch_attn_bwd_b<D, KPH, DENSE, true>(p, BH, L, drop, pf, st, mid);
  }
  return launch_attn_bwd_b<D, KPH, DENSE, false>(p, BH, L, drop, pf, st, mid);
}

// k_proj_bwd_s over items of `kind` (KArgs::pb_kind) with G workgroups per head, on stream s
template <int D>
void launch_proj_bwd_s(KArgs p, int kind, int G, int goff, int gk, int Gtot, int H, hipStream_t s) {
  using Ss = ProjBwdSmallShape<D>;
  p.pb_kind = kind; p.pb_goff = goff; p.pb_gk = gk; p.G = Gtot;
  if (p.bf16) {  // CSA_DTYPE_BF16: projection contractions on bf16 MFMA
    set_dyn_lds((const void*)k_proj_bwd_s<D, true>, (int)Ss::LDS_BYTES);
    hipLaunchKernelGGL((k_proj_bwd_s<D, true>), dim3(G, H), dim3(256), Ss::LDS_BYTES, s, p);
  } else {
    set_dyn_lds((const void*)k_proj_bwd_s<D>, (int)Ss::LDS_BYTES);
    hipLaunchKernelGGL((k_proj_bwd_s<D>), dim3(G, H), dim3(256), Ss::LDS_BYTES, s, p);
  }
}

template <int D, int KPH>
constexpr bool SPLIT_H2C() { return (D == 64 || D == 96) && KPH == 8 && h2c_path(D, 1, false); }

template <int D, int KPH, int KT>
csa_status launch_bwd(const csa_sbm_bwd_args* b, const Layout& L, hipStream_t st) {
  const csa_sbm_fwd_args* a = b->fwd;
  KArgs p = make_kargs(a, L);
  const bool dense = a->flags & CSA_FLAG_DENSE;
  p.dX = b->dX; p.dsp = b->dsparsity; p.dgraph = b->dgraph; p.dattn = b->dattn;
  p.gx = b->workspace ? (float*)((char*)b->workspace + L.w_gx) : nullptr;
  p.dQ = b->dQ; p.dK = b->dK; p.dV = b->dV;
  {
    const Str3 x = strides_or_contig(b->dx_sb, b->dx_sh, b->dx_sn, a->H, a->N, a->d);
    const Str3 q = strides_or_contig(b->dq_sb, b->dq_sh, b->dq_sn, a->H, a->N, a->d);
    const Str3 k = strides_or_contig(b->dk_sb, b->dk_sh, b->dk_sn, a->H, a->M, a->d);
    const Str3 v = strides_or_contig(b->dv_sb, b->dv_sh, b->dv_sn, a->H, a->M, a->d);
    p.dx_sb = x.sb; p.dx_sh = x.sh; p.dx_sn = x.sn;
    p.dq_sb = q.sb; p.dq_sh = q.sh; p.dq_sn = q.sn;
    p.dk_sb = k.sb; p.dk_sh = k.sh; p.dk_sn = k.sn;
    p.dv_sb = v.sb; p.dv_sh = v.sh; p.dv_sn = v.sn;
  }
  p.dQh = (float*)((char*)b->workspace + L.w_dQh);
  p.dT = (float*)((char*)b->workspace + L.w_dT);
  p.slab = (float*)((char*)b->workspace + L.w_slab);
  p.G = (int)L.G; p.slab_floats = L.slab_floats;
  p.dsg = (float*)((char*)b->workspace + L.w_dsg); p.gplane = L.w_dsg_plane;
  p.brow = (float*)((char*)b->workspace + L.w_brow);
  const int BH = (int)(a->B * a->H);
  (void)dense;
  const csa_prof* pf = b->prof;
  if constexpr (KT > 0) {
    // Concurrent schedule (k <= 16): the projection backward's key-block items need only dT and dK, which the
    // key half has written, so they run on the caller's side stream beside k_attn_bwd_qg (HBM / latency bound)
    // and the query-block items follow it on this stream. Separate slab sets, summed in a fixed order: the
    // results are bitwise those of the in-order schedule. Only on an explicit CSA_SCHED_CONCURRENT: AUTO runs in
    // order, measured 0.06 ms per step faster at the headline shape (the two kernels contend for the same CUs;
    // profiles/r04_ab_concurrent.txt).
    constexpr bool SPLIT = (D == 64 || D == 96) && KPH == 8;
    const bool conc = SPLIT && b->side_stream && b->side_fork && b->side_join && b->schedule == CSA_SCHED_CONCURRENT;
    const SideLane lane{(hipStream_t)b->side_stream, (hipEvent_t)b->side_fork, (hipEvent_t)b->side_join};
    const int Gtot = (int)(L.G_K + L.G_Q);
    bool forked = false;
    auto mid = [&]() {
      if (!conc || !lane.fork(st)) return;
      forked = true;
      Stage sg(pf, CSA_STAGE_PROJ_BWD_K, lane.s);
      if constexpr (SPLIT) launch_proj_bwd_s<D>(p, 1, (int)L.G_K, 0, 0, Gtot, (int)a->H, lane.s);
    };
    launch_attn_bwd<D, KPH, false>(p, BH, L, a->attn_dropout > 0.f, pf, st, mid);
    if (conc && !forked) return fail_hip("csa_sbm_bwd: side-stream fork");
    using Sh = ProjBwdShape<D, KT>;
    if (!Sh::REGACC && hipMemsetAsync(p.slab, 0, sizeof(float) * a->H * L.G * L.slab_floats, st) != hipSuccess)
      return check_launch("memset slabs");
    {
      Stage sg(pf, CSA_STAGE_PROJ_BWD, st);
      if constexpr (SPLIT) {  // k <= 16: the same workgroup items and slab sets on every schedule
        // in order: both kinds in one launch, each workgroup's items and slab as in the concurrent form
        if (forked) launch_proj_bwd_s<D>(p, 2, (int)L.G_Q, (int)L.G_K, 0, Gtot, (int)a->H, st);
        else launch_proj_bwd_s<D>(p, 3, Gtot, 0, (int)L.G_K, Gtot, (int)a->H, st);
      } else {
        set_dyn_lds((const void*)k_proj_bwd<D, KT>, (int)Sh::LDS_BYTES);
        hipLaunchKernelGGL((k_proj_bwd<D, KT>), dim3(L.G, a->H), dim3(256), Sh::LDS_BYTES, st, p);
      }
    }
    if (forked && !lane.join(st)) return fail_hip("csa_sbm_bwd: side-stream join");
    if constexpr (SPLIT) p.G = Gtot;  // the reduction sums both launches' slabs
    Stage sr(pf, CSA_STAGE_REDUCE, st);
    const int KP32 = 32 * KT;
    float* dS_ws = (float*)((char*)b->workspace + L.w_dS);
    float* dC_ws = (float*)((char*)b->workspace + L.w_dC);
    const int64_t total = 3LL * D * D + 3LL * D + (int64_t)a->H * KP32 * D + (int64_t)a->H * KP32 * KP32;
    hipLaunchKernelGGL(k_reduce_slabs, dim3((unsigned)((total + 63) / 64)), dim3(64 * RS_WAVES), 0, st, p, D, KP32,
                       b->dproj_w[0], b->dproj_w[1], b->dproj_w[2], b->dproj_b[0], b->dproj_b[1], b->dproj_b[2],
                       dS_ws, dC_ws);
    const int h2c = (SPLIT_H2C<D, KPH>() && !p.bf16) ? 1 : 0;  // k_proj_bwd_s formed dC from h2
    hipLaunchKernelGGL(k_cluster_grad, dim3((unsigned)a->k, (unsigned)a->H), dim3(128), 0, st, p.S, (const float*)dS_ws,
                       (const float*)dC_ws, a->cluster_w, b->dcluster_w, (int)a->k, D, KP32, a->proj_w[2],
                       a->proj_b[2], h2c);
  } else {
    launch_attn_bwd<D, 0, true>(p, BH, L, a->attn_dropout > 0.f, pf, st, [] {});
  }
  return check_launch("csa_sbm_bwd");
}

}  // namespace

extern "C" {

int csa_abi_version(void) { return CSA_ABI_VERSION; }

const char* csa_status_str(csa_status s) {
  switch (s) {
    case CSA_OK: return "CSA_OK";
    case CSA_INVALID_ARG: return "CSA_INVALID_ARG";
    case CSA_UNSUPPORTED_SHAPE: return "CSA_UNSUPPORTED_SHAPE";
    case CSA_LAUNCH_FAILED: return "CSA_LAUNCH_FAILED";
  }
  return "CSA_UNKNOWN";
}

const char* csa_last_error_str(void) { return csa::get_error(); }

int csa_sbm_supported(int64_t d, int64_t k, uint32_t flags) { return supported(d, k, flags) ? 1 : 0; }

size_t csa_sbm_state_bytes(int64_t B, int64_t H, int64_t N, int64_t M, int64_t d, int64_t k, uint32_t flags) {
  return make_layout(B, H, N, M, d, k, flags).total;
}

size_t csa_sbm_bwd_workspace_bytes(int64_t B, int64_t H, int64_t N, int64_t M, int64_t d, int64_t k, uint32_t flags) {
  return make_layout(B, H, N, M, d, k, flags).w_total;
}

csa_status csa_sbm_fwd(const csa_sbm_fwd_args* a, void* stream) {
  csa_status s = validate_fwd(a);
  if (s != CSA_OK) return s;
  const Layout L = make_layout(a->B, a->H, a->N, a->M, a->d, a->k, a->flags);
  hipStream_t st = (hipStream_t)stream;
  const DeviceGuard guard(st);
  const bool dense = a->flags & CSA_FLAG_DENSE;
  if (a->d == 64) {
    if (dense) return launch_fwd<64, 0, 1>(a, L, st);
    switch (L.kp) {
      case 16: return launch_fwd<64, 8, 1>(a, L, st);
      case 32: return launch_fwd<64, 16, 1>(a, L, st);
      case 64: return launch_fwd<64, 32, 2>(a, L, st);
      default: return launch_fwd<64, 64, 4>(a, L, st);
    }
  }
  if (dense) return launch_fwd<96, 0, 1>(a, L, st);
  return L.kp <= 16 ? launch_fwd<96, 8, 1>(a, L, st) : launch_fwd<96, 16, 1>(a, L, st);
}

csa_status csa_sbm_maps(const csa_sbm_fwd_args* a, float* graph, float* attn, void* stream) {
  csa_status s = validate_fwd(a);
  if (s != CSA_OK) return s;
  if (!graph && !attn) return CSA_OK;
  const bool dense = a->flags & CSA_FLAG_DENSE;
  const Layout L = make_layout(a->B, a->H, a->N, a->M, a->d, a->k, a->flags);
  KArgs p = make_kargs(a, L);
  hipStream_t st = (hipStream_t)stream;
  const DeviceGuard guard(st);
  const dim3 grid(xcd_grid((int)L.NQB, (int)(a->B * a->H)));
  if (a->d == 64) {
    if (dense) hipLaunchKernelGGL((k_maps<64, true>), grid, dim3(64), 0, st, p, graph, attn);
    else hipLaunchKernelGGL((k_maps<64, false>), grid, dim3(64), 0, st, p, graph, attn);
  } else {
    if (dense) hipLaunchKernelGGL((k_maps<96, true>), grid, dim3(64), 0, st, p, graph, attn);
    else hipLaunchKernelGGL((k_maps<96, false>), grid, dim3(64), 0, st, p, graph, attn);
  }
  return check_launch("csa_sbm_maps");
}

csa_status csa_sbm_bwd(const csa_sbm_bwd_args* b, void* stream) {
  if (!b || !b->fwd) return fail(CSA_INVALID_ARG, "null args");
  csa_status s = validate_fwd(b->fwd);
  if (s != CSA_OK) return s;
  const csa_sbm_fwd_args* a = b->fwd;
  const bool dense = a->flags & CSA_FLAG_DENSE;
  if (!b->dX || !b->dQ || !b->dK || !b->dV || !b->workspace) return fail(CSA_INVALID_ARG, "null dX/dQ/dK/dV/workspace");
  {
    auto al16 = [](const void* ptr, int64_t sb, int64_t sh, int64_t sn) {
      return (((uintptr_t)ptr) % 16 == 0) && sb % 4 == 0 && sh % 4 == 0 && sn % 4 == 0;
    };
    if (!al16(b->dX, b->dx_sb, b->dx_sh, b->dx_sn) || !al16(b->dQ, b->dq_sb, b->dq_sh, b->dq_sn) ||
        !al16(b->dK, b->dk_sb, b->dk_sh, b->dk_sn) || !al16(b->dV, b->dv_sb, b->dv_sh, b->dv_sn))
      return fail(CSA_INVALID_ARG, "dX/dQ/dK/dV must be 16-byte aligned with strides multiple of 4 elements");
  }
  if (!dense && (!b->dcluster_w || !b->dproj_w[0] || !b->dproj_w[1] || !b->dproj_w[2] || !b->dproj_b[0] ||
                 !b->dproj_b[1] || !b->dproj_b[2]))
    return fail(CSA_INVALID_ARG, "null parameter-gradient output");
  if (b->schedule > CSA_SCHED_CONCURRENT) return fail(CSA_INVALID_ARG, "schedule must be a CSA_SCHED_* value");
  if (a->flags & CSA_FLAG_FWD_ONLY) return fail(CSA_INVALID_ARG, "the forward ran with CSA_FLAG_FWD_ONLY: no backward state");
  if ((a->flags & CSA_FLAG_BF16_WS) && a->dtype != CSA_DTYPE_BF16)
    return fail(CSA_INVALID_ARG, "CSA_FLAG_BF16_WS sizes the workspace of a CSA_DTYPE_BF16 call only");
  // bf16 mode recomputes on the query side (bwd_handoff<true>() == false): no handoff tiles in its workspace
  const Layout L = make_layout(a->B, a->H, a->N, a->M, a->d, a->k,
                               a->flags | ((a->dtype == CSA_DTYPE_BF16 && !bwd_handoff<true>()) ? CSA_FLAG_BF16_WS : 0u));
  hipStream_t st = (hipStream_t)stream;
  const DeviceGuard guard(st);
  if (a->d == 64) {
    if (dense) return launch_bwd<64, 0, 0>(b, L, st);
    switch (L.kp) {
      case 16: return launch_bwd<64, 8, 1>(b, L, st);
      case 32: return launch_bwd<64, 16, 1>(b, L, st);
      case 64: return launch_bwd<64, 32, 2>(b, L, st);
      default: return launch_bwd<64, 64, 4>(b, L, st);
    }
  }
  if (dense) return launch_bwd<96, 0, 0>(b, L, st);
  return L.kp <= 16 ? launch_bwd<96, 8, 1>(b, L, st) : launch_bwd<96, 16, 1>(b, L, st);
}

csa_status csa_ste_sample(const float* pr, const float* u, float* A, int64_t n, float lo, float hi, void* stream) {
  if (!pr || !u || !A || n < 0) return fail(CSA_INVALID_ARG, "null pointer or negative n");
  if (n == 0) return CSA_OK;
  const unsigned grid = (unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  const DeviceGuard guard((hipStream_t)stream);
  hipLaunchKernelGGL(k_ste_sample, dim3(grid), dim3(256), 0, (hipStream_t)stream, pr, u, A, n, lo, hi);
  return check_launch("csa_ste_sample");
}

csa_status csa_ste_backward(const float* A, const float* g, float* out, int64_t n, void* stream) {
  if (!A || !g || !out || n < 0) return fail(CSA_INVALID_ARG, "null pointer or negative n");
  if (n == 0) return CSA_OK;
  const unsigned grid = (unsigned)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  const DeviceGuard guard((hipStream_t)stream);
  hipLaunchKernelGGL(k_ste_backward, dim3(grid), dim3(256), 0, (hipStream_t)stream, A, g, out, n);
  return check_launch("csa_ste_backward");
}

// FullAttention (module/sbm_attn.py:77-87): csa_sbm_fwd / csa_sbm_bwd with CSA_FLAG_DENSE set (k, cluster_w,
// proj_*, uniforms and sparsity are ignored)
csa_status csa_dense_attn_fwd(const csa_sbm_fwd_args* a, void* stream) {
  if (!a) return fail(CSA_INVALID_ARG, "null args");
  csa_sbm_fwd_args d = *a;
  d.flags |= CSA_FLAG_DENSE;
  d.k = 0;
  return csa_sbm_fwd(&d, stream);
}

csa_status csa_dense_attn_bwd(const csa_sbm_bwd_args* b, void* stream) {
  if (!b || !b->fwd) return fail(CSA_INVALID_ARG, "null args");
  csa_sbm_fwd_args d = *b->fwd;
  d.flags |= CSA_FLAG_DENSE;
  d.k = 0;
  csa_sbm_bwd_args e = *b;
  e.fwd = &d;
  return csa_sbm_bwd(&e, stream);
}

}  // extern "C"
