// torch.ops.csa.* for the attention hot path, implemented in C++ (TORCH_LIBRARY_IMPL): the thin shim of
// SURVEY.md §7 step 2. Each op validates its inputs, allocates outputs / state / workspace with the torch
// caching allocator, takes the current HIP stream and calls the extern "C" entry points of libcsa_hip.so
// (include/csa_hip.h). No kernels and no compute here; a failing status raises (TORCH_CHECK) with the
// library's message. The autograd Functions and the drop-in modules above it are Python
// (csa_amd/ops.py, csa_amd/rel_ops.py); their fake (meta) implementations are registered there.
//
// Ops (schemas in csa_amd/ops.py _SCHEMAS, the round-2 Python registrations, so callers are unchanged):
//   sbm_fwd / sbm_maps / sbm_bwd    SBMAttention and FullAttention (module/sbm_attn.py:32-87)
//   ste_sample / ste_backward       SampleGraphSparseGraph (module/STE.py:8-19)
//   rel_attn_fwd / rel_attn_bwd     DisentangledAttn.rel_attn (module/disentangled_attn.py:44-65)
#include <ATen/ATen.h>
#include <ATen/DeviceGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include <memory>
#include <mutex>
#include <vector>

#include "../../include/csa_hip.h"

namespace {

using at::Tensor;
using c10::optional;

// per-stage profiling records (bench.py): caller-owned csa_prof structs, installed from Python
const csa_prof* g_prof_fwd = nullptr;
const csa_prof* g_prof_bwd = nullptr;
const csa_prof* g_prof_rel_fwd = nullptr;  // ABI v9: CSE relation attention (CSA_REL_STAGE_*)
const csa_prof* g_prof_rel_bwd = nullptr;

void check(csa_status s, const char* what) {
  TORCH_CHECK(s == CSA_OK, what, " failed: ", csa_status_str(s), ": ", csa_last_error_str());
}

// The current stream of t's device. PyTorch's default stream has a null handle, which the library resolves to
// the calling thread's current device: every op therefore opens a device guard on its first tensor
// (OptionalDeviceGuard below) before it reads the stream, as codegen'd ATen ops do.
void* cur_stream(const Tensor& t) { return (void*)c10::hip::getCurrentHIPStream(t.device().index()).stream(); }

void require_gpu(const Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), "csa ops run only on the GPU (HIP); ", name, " is on ", t.device());
}

// (B,H,N,d) fp32 view usable by the kernels: last dim contiguous, 16-B aligned, strides % 4 == 0, no zero
// leading stride (a broadcast, e.g. the gradient of X.sum((0,1,2)): the ABI reads an all-zero stride triple
// as "contiguous"). Non-contiguous split_heads views (sbm_attn.py:137-140) pass through without a copy.
Tensor bhnd(Tensor t) {
  if (t.scalar_type() != at::kFloat) t = t.to(at::kFloat);
  bool ok = t.dim() == 4 && t.stride(3) == 1 && (reinterpret_cast<uintptr_t>(t.data_ptr()) % 16) == 0;
  for (int i = 0; ok && i < 3; ++i) ok = t.stride(i) > 0 && t.stride(i) % 4 == 0;
  return ok ? t : t.contiguous();
}
Tensor f32c(const Tensor& t) { return t.to(at::kFloat).contiguous(); }
const float* fp(const Tensor& t) { return t.data_ptr<float>(); }
float* fpw(Tensor& t) { return t.data_ptr<float>(); }

// (B,H,N,d) view of a (B,N,H,d) buffer: combine_heads of it is a free view (sbm_attn.py:143-146)
Tensor head_major_out(int64_t B, int64_t H, int64_t N, int64_t d, const at::TensorOptions& o) {
  return at::empty({B, N, H, d}, o).transpose(1, 2);
}

// caller-owned side lane of a device (ABI v5): one non-blocking stream and two timing-free events, created
// on first use and kept for the process lifetime, plus the mutex a call holds from its fork to its join (two
// host threads sharing a device's lane could otherwise interleave their event records)
struct Lane { void* s; void* fork; void* join; std::mutex* mu; };
Lane side_lane(int dev) {
  static std::mutex mu;
  static std::vector<Lane> lanes;
  static std::vector<std::unique_ptr<std::mutex>> call_mu;
  std::lock_guard<std::mutex> lock(mu);
  if ((int)lanes.size() <= dev) lanes.resize(dev + 1, Lane{nullptr, nullptr, nullptr, nullptr});
  Lane& l = lanes[dev];
  if (!l.s) {
    int prev = -1;
    TORCH_CHECK(hipGetDevice(&prev) == hipSuccess && hipSetDevice(dev) == hipSuccess, "csa side lane: hipSetDevice");
    hipStream_t s = nullptr;
    hipEvent_t f = nullptr, j = nullptr;
    const bool ok = hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess &&
                    hipEventCreateWithFlags(&f, hipEventDisableTiming) == hipSuccess &&
                    hipEventCreateWithFlags(&j, hipEventDisableTiming) == hipSuccess;
    (void)hipSetDevice(prev);
    TORCH_CHECK(ok, "csa side lane: stream / event creation failed");
    call_mu.emplace_back(new std::mutex());
    l = Lane{(void*)s, (void*)f, (void*)j, call_mu.back().get()};
  }
  return l;
}
// Hands the device's side lane to b unless the schedule is in order; the returned lock (empty when no lane
// is handed over) must be held until the library call that uses the lane has returned.
template <typename Args>
std::unique_lock<std::mutex> set_side_lane(Args& b, const Tensor& t, int64_t schedule) {
  b.schedule = (uint32_t)schedule;
  if (schedule == CSA_SCHED_IN_ORDER) return {};
  const Lane l = side_lane(t.device().index());
  b.side_stream = l.s; b.side_fork = l.fork; b.side_join = l.join;
  return std::unique_lock<std::mutex>(*l.mu);
}

// ------------------------------------------------------------------------------------------------
// SBM / dense attention
// ------------------------------------------------------------------------------------------------
struct SbmIn {
  Tensor Q, K, V, mask, cw, u;
  std::vector<Tensor> pw, pb;
};
SbmIn sbm_prep(const Tensor& Q, const Tensor& K, const Tensor& V, const optional<Tensor>& mask,
               const optional<Tensor>& cluster_w, at::TensorList proj_w, at::TensorList proj_b,
               const optional<Tensor>& uniforms) {
  require_gpu(Q, "Q"); require_gpu(K, "K"); require_gpu(V, "V");
  SbmIn r;
  r.Q = bhnd(Q); r.K = bhnd(K); r.V = bhnd(V);
  if (mask) r.mask = mask->to(Q.device(), at::kFloat).contiguous();
  if (uniforms) r.u = uniforms->to(Q.device(), at::kFloat).contiguous();
  if (cluster_w) r.cw = f32c(*cluster_w);
  for (const Tensor& w : proj_w) r.pw.push_back(f32c(w));
  for (const Tensor& b : proj_b) r.pb.push_back(f32c(b));
  return r;
}

csa_sbm_fwd_args fwd_struct(const SbmIn& in, int64_t k, int64_t seed, int64_t offset, double attn_p, double proj_p,
                            bool dense, bool bf16) {
  csa_sbm_fwd_args a;
  memset(&a, 0, sizeof(a));
  a.B = in.Q.size(0); a.H = in.Q.size(1); a.N = in.Q.size(2); a.M = in.K.size(2); a.d = in.Q.size(3);
  a.k = dense ? 0 : k;
  a.Q = fp(in.Q); a.q_sb = in.Q.stride(0); a.q_sh = in.Q.stride(1); a.q_sn = in.Q.stride(2);
  a.K = fp(in.K); a.k_sb = in.K.stride(0); a.k_sh = in.K.stride(1); a.k_sn = in.K.stride(2);
  a.V = fp(in.V); a.v_sb = in.V.stride(0); a.v_sh = in.V.stride(1); a.v_sn = in.V.stride(2);
  if (in.mask.defined()) { a.key_mask = fp(in.mask); a.mask_sb = in.mask.stride(0); }
  if (!dense) {
    TORCH_CHECK(in.cw.defined() && in.pw.size() == 3 && in.pb.size() == 3, "csa::sbm: cluster / projection weights");
    a.cluster_w = fp(in.cw);
    for (int i = 0; i < 3; ++i) { a.proj_w[i] = fp(in.pw[i]); a.proj_b[i] = fp(in.pb[i]); }
  }
  if (in.u.defined()) a.uniforms = fp(in.u);
  a.seed = (uint64_t)seed; a.offset = (uint64_t)offset;
  a.attn_dropout = (float)attn_p; a.proj_dropout = (float)proj_p;
  a.flags = dense ? CSA_FLAG_DENSE : 0u;
  a.dtype = bf16 ? CSA_DTYPE_BF16 : CSA_DTYPE_F32;
  return a;
}

std::tuple<Tensor, Tensor, Tensor> sbm_fwd(const Tensor& Q, const Tensor& K, const Tensor& V,
                                           const optional<Tensor>& mask, const optional<Tensor>& cluster_w,
                                           at::TensorList proj_w, at::TensorList proj_b,
                                           const optional<Tensor>& uniforms, int64_t k, int64_t seed,
                                           int64_t offset, double attn_p, double proj_p, bool dense, bool bf16,
                                           bool fwd_only) {
  const at::OptionalDeviceGuard guard(at::device_of(Q));
  const SbmIn in = sbm_prep(Q, K, V, mask, cluster_w, proj_w, proj_b, uniforms);
  const int64_t B = in.Q.size(0), H = in.Q.size(1), N = in.Q.size(2), d = in.Q.size(3), M = in.K.size(2);
  const uint32_t flags = (dense ? CSA_FLAG_DENSE : 0u) | (fwd_only ? CSA_FLAG_FWD_ONLY : 0u);
  TORCH_CHECK(csa_sbm_supported(d, k, flags), "csa::sbm_fwd: unsupported head_dim=", d, " / num_clusters=", k);
  const auto o = in.Q.options().dtype(at::kFloat);
  Tensor X = head_major_out(B, H, N, d, o);
  Tensor sp = at::empty({dense ? 0 : H}, o);
  Tensor state = at::empty({(int64_t)csa_sbm_state_bytes(B, H, N, M, d, k, flags)}, o.dtype(at::kByte));
  csa_sbm_fwd_args a = fwd_struct(in, k, seed, offset, attn_p, proj_p, dense, bf16);
  a.flags = flags;
  a.X = fpw(X); a.x_sb = X.stride(0); a.x_sh = X.stride(1); a.x_sn = X.stride(2);
  if (!dense) a.sparsity = fpw(sp);
  a.state = state.data_ptr();
  a.prof = g_prof_fwd;
  check(csa_sbm_fwd(&a, cur_stream(in.Q)), "csa_sbm_fwd");
  return {X, sp, state};
}

// The (graph, attn) maps SBMAttention returns (sbm_attn.py:57,62), from a forward's state.
std::tuple<Tensor, Tensor> sbm_maps(const Tensor& Q, const Tensor& K, const Tensor& V, const optional<Tensor>& mask,
                                    const Tensor& state, int64_t k, bool dense) {
  const at::OptionalDeviceGuard guard(at::device_of(Q));
  const SbmIn in = sbm_prep(Q, K, V, mask, c10::nullopt, {}, {}, c10::nullopt);
  const int64_t B = in.Q.size(0), H = in.Q.size(1), N = in.Q.size(2), M = in.K.size(2);
  Tensor graph = at::empty({B, H, N, M}, in.Q.options().dtype(at::kFloat));
  Tensor attn = at::empty_like(graph);
  csa_sbm_fwd_args a = fwd_struct(in, k, 0, 0, 0.0, 0.0, true, false);
  a.flags = dense ? CSA_FLAG_DENSE : 0u;
  a.k = dense ? 0 : k;
  a.X = const_cast<float*>(a.Q);  // unused by the maps; a valid aligned pointer for validation
  if (!dense) {  // the validation of non-dense args needs these non-null (unused by the maps kernel)
    a.cluster_w = a.Q; a.sparsity = const_cast<float*>(a.Q);
    for (int i = 0; i < 3; ++i) { a.proj_w[i] = a.Q; a.proj_b[i] = a.Q; }
  }
  a.state = const_cast<void*>(state.data_ptr());
  check(csa_sbm_maps(&a, fpw(graph), fpw(attn), cur_stream(in.Q)), "csa_sbm_maps");
  return {graph, attn};
}

// Backward of sbm_fwd: [dQ, dK, dV] (+ [dcluster_w, dW0, db0, dW1, db1, dW2, db2] unless dense). packed: [dQ, dK, dV]
// is ONE packed (B, N, 3, H, d) tensor (the gradient of a fused QKV projection, written in place).
std::vector<Tensor> sbm_bwd(const Tensor& Q, const Tensor& K, const Tensor& V, const optional<Tensor>& mask,
                            const optional<Tensor>& cluster_w, at::TensorList proj_w, at::TensorList proj_b,
                            int64_t k, double attn_p, double proj_p, int64_t seed, int64_t offset, bool dense,
                            const Tensor& state, const Tensor& X, const Tensor& dX_,
                            const optional<Tensor>& dsparsity, const optional<Tensor>& dgraph, bool bf16,
                            bool packed, const optional<Tensor>& dattn, int64_t schedule) {
  const at::OptionalDeviceGuard guard(at::device_of(Q));
  const SbmIn in = sbm_prep(Q, K, V, mask, cluster_w, proj_w, proj_b, c10::nullopt);
  const int64_t B = in.Q.size(0), H = in.Q.size(1), N = in.Q.size(2), d = in.Q.size(3), M = in.K.size(2);
  const uint32_t flags = dense ? CSA_FLAG_DENSE : 0u;
  const auto o = in.Q.options().dtype(at::kFloat);
  Tensor sp = at::empty({dense ? 0 : H}, o);
  csa_sbm_fwd_args a = fwd_struct(in, k, seed, offset, attn_p, proj_p, dense, bf16);
  a.X = const_cast<float*>(X.data_ptr<float>());
  if (X.dim() == 4) { a.x_sb = X.stride(0); a.x_sh = X.stride(1); a.x_sn = X.stride(2); }
  if (!dense) a.sparsity = fpw(sp);
  a.state = const_cast<void*>(state.data_ptr());
  const Tensor dX = bhnd(dX_);  // strided (e.g. the combine_heads view's gradient) without a copy
  std::vector<Tensor> outs;
  Tensor dQ, dK, dV;
  if (packed) {
    Tensor P = at::empty({B, N, 3, H, d}, o);
    dQ = P.select(2, 0).transpose(1, 2); dK = P.select(2, 1).transpose(1, 2); dV = P.select(2, 2).transpose(1, 2);
    outs.push_back(P);
  } else {
    dQ = at::empty({B, H, N, d}, o); dK = at::empty({B, H, M, d}, o); dV = at::empty_like(dK);
    outs = {dQ, dK, dV};
  }
  csa_sbm_bwd_args b;
  memset(&b, 0, sizeof(b));
  b.fwd = &a;
  b.dX = fp(dX); b.dQ = fpw(dQ); b.dK = fpw(dK); b.dV = fpw(dV);
  b.dx_sb = dX.stride(0); b.dx_sh = dX.stride(1); b.dx_sn = dX.stride(2);
  b.dq_sb = dQ.stride(0); b.dq_sh = dQ.stride(1); b.dq_sn = dQ.stride(2);
  b.dk_sb = dK.stride(0); b.dk_sh = dK.stride(1); b.dk_sn = dK.stride(2);
  b.dv_sb = dV.stride(0); b.dv_sh = dV.stride(1); b.dv_sn = dV.stride(2);
  Tensor ws, da, dsp, dg;
  ws = at::empty({(int64_t)csa_sbm_bwd_workspace_bytes(B, H, N, M, d, k, flags | (a.dtype == CSA_DTYPE_BF16 ? CSA_FLAG_BF16_WS : 0u))},
                 o.dtype(at::kByte));
  b.workspace = ws.data_ptr();
  if (dattn) { da = f32c(*dattn); b.dattn = fp(da); }
  if (!dense) {
    if (dsparsity) { dsp = f32c(*dsparsity); b.dsparsity = fp(dsp); }
    if (dgraph) { dg = f32c(*dgraph); b.dgraph = fp(dg); }
    Tensor dC = at::empty_like(in.cw);
    b.dcluster_w = fpw(dC);
    outs.push_back(dC);
    for (int i = 0; i < 3; ++i) {
      Tensor dw = at::empty_like(in.pw[i]), db = at::empty_like(in.pb[i]);
      b.dproj_w[i] = fpw(dw); b.dproj_b[i] = fpw(db);
      outs.push_back(dw); outs.push_back(db);
    }
  }
  b.prof = g_prof_bwd;
  {
    const std::unique_lock<std::mutex> lane_lock = set_side_lane(b, in.Q, schedule);
    check(csa_sbm_bwd(&b, cur_stream(in.Q)), "csa_sbm_bwd");
  }
  return outs;
}

// STE.py:10-15: A = (u < clamp(p, lo, hi)) as fp32 {0,1}.
Tensor ste_sample(const Tensor& p_, const Tensor& u_, double lo, double hi) {
  const at::OptionalDeviceGuard guard(at::device_of(p_));
  require_gpu(p_, "p"); require_gpu(u_, "u");
  const Tensor p = f32c(p_), u = f32c(u_);
  TORCH_CHECK(p.numel() == u.numel(), "csa::ste_sample: p and u differ in size");
  Tensor A = at::empty_like(p);
  check(csa_ste_sample(fp(p), fp(u), fpw(A), p.numel(), (float)lo, (float)hi, cur_stream(p)), "csa_ste_sample");
  return A;
}

// STE.py:17-19: hardtanh(A * grad).
Tensor ste_backward(const Tensor& A_, const Tensor& g_) {
  const at::OptionalDeviceGuard guard(at::device_of(g_));
  require_gpu(A_, "A"); require_gpu(g_, "g");
  const Tensor A = f32c(A_), g = f32c(g_);
  TORCH_CHECK(A.numel() == g.numel(), "csa::ste_backward: A and g differ in size");
  Tensor out = at::empty_like(g);
  check(csa_ste_backward(fp(A), fp(g), fpw(out), g.numel(), cur_stream(g)), "csa_ste_backward");
  return out;
}

// ------------------------------------------------------------------------------------------------
// CSE relation attention
// ------------------------------------------------------------------------------------------------
csa_rel_attn_args rel_args(const Tensor& q, const Tensor& k, const Tensor& v, const Tensor& lq, const Tensor& lk,
                           const Tensor& rel, const Tensor& mask, int64_t group, bool bf16) {
  csa_rel_attn_args a;
  memset(&a, 0, sizeof(a));
  a.B = q.size(0); a.H = q.size(1); a.N = q.size(2); a.L = lq.size(1); a.d = q.size(3);
  a.q = fp(q); a.q_sb = q.stride(0); a.q_sh = q.stride(1); a.q_sn = q.stride(2);
  a.k = fp(k); a.k_sb = k.stride(0); a.k_sh = k.stride(1); a.k_sn = k.stride(2);
  a.v = fp(v); a.v_sb = v.stride(0); a.v_sh = v.stride(1); a.v_sn = v.stride(2);
  a.lq = fp(lq); a.lk = fp(lk);
  TORCH_CHECK(rel.scalar_type() == at::kByte && mask.scalar_type() == at::kByte && rel.is_contiguous() &&
              mask.is_contiguous() && rel.dim() == 4 && mask.dim() == 4,
              "csa::rel_attn: rel / mask must be contiguous uint8 (B,P,N,N) planes");
  a.rel = rel.data_ptr<uint8_t>(); a.rel_sb = rel.stride(0); a.rel_sh = rel.stride(1);
  a.mask = mask.data_ptr<uint8_t>(); a.mask_sb = mask.stride(0); a.mask_sh = mask.stride(1);
  a.rel_head_group = group;
  a.dtype = bf16 ? CSA_DTYPE_BF16 : CSA_DTYPE_F32;
  a.prof = g_prof_rel_fwd;
  return a;
}

// [out (B,H,N,d), row_stats (B,H,N,2), state (uint8)]; d_k = 64: out is a (B,H,N,d) view of (B,N,H,d) memory
std::vector<Tensor> rel_attn_fwd(const Tensor& q_, const Tensor& k_, const Tensor& v_, const Tensor& lq_,
                                 const Tensor& lk_, const Tensor& rel, const Tensor& mask, int64_t group, bool bf16) {
  const at::OptionalDeviceGuard guard(at::device_of(q_));
  require_gpu(q_, "q"); require_gpu(k_, "k"); require_gpu(v_, "v"); require_gpu(lq_, "lq"); require_gpu(lk_, "lk");
  require_gpu(rel, "rel"); require_gpu(mask, "mask");
  const Tensor q = bhnd(q_), k = bhnd(k_), v = bhnd(v_), lq = f32c(lq_), lk = f32c(lk_);
  const int64_t B = q.size(0), H = q.size(1), N = q.size(2), d = q.size(3), L = lq.size(1);
  const auto o = q.options().dtype(at::kFloat);
  Tensor out = d == 64 ? head_major_out(B, H, N, d, o) : at::empty({B, H, N, d}, o);
  Tensor lse = at::empty({B, H, N, 2}, o);  // (row max, 1/row sum)
  Tensor state = at::empty({(int64_t)csa_rel_attn_state_bytes(B, H, N, L, d)}, o.dtype(at::kByte));
  csa_rel_attn_args a = rel_args(q, k, v, lq, lk, rel, mask, group, bf16);
  a.out = fpw(out); a.row_stats = fpw(lse); a.state = state.data_ptr();
  a.o_sb = out.stride(0); a.o_sh = out.stride(1); a.o_sn = out.stride(2);
  check(csa_rel_attn_fwd(&a, cur_stream(q)), "csa_rel_attn_fwd");
  return {out, lse, state};
}

// [dq, dk, dv, dlq (H,L,d), dlk (H,L,d)]; packed (d_k = 64): [dq, dk, dv] is ONE packed (B, N, 3, H, d) tensor
std::vector<Tensor> rel_attn_bwd(const Tensor& q_, const Tensor& k_, const Tensor& v_, const Tensor& lq_,
                                 const Tensor& lk_, const Tensor& rel, const Tensor& mask, int64_t group,
                                 const Tensor& out, const Tensor& lse, const Tensor& state, const Tensor& dout_,
                                 bool bf16, bool packed, int64_t schedule) {
  const at::OptionalDeviceGuard guard(at::device_of(q_));
  const Tensor q = bhnd(q_), k = bhnd(k_), v = bhnd(v_), lq = f32c(lq_), lk = f32c(lk_);
  const int64_t B = q.size(0), H = q.size(1), N = q.size(2), d = q.size(3), L = lq.size(1);
  const Tensor dout = d == 64 ? bhnd(dout_) : f32c(dout_);
  const auto o = q.options().dtype(at::kFloat);
  csa_rel_attn_args a = rel_args(q, k, v, lq, lk, rel, mask, group, bf16);
  a.out = const_cast<float*>(out.data_ptr<float>()); a.row_stats = const_cast<float*>(lse.data_ptr<float>());
  a.state = const_cast<void*>(state.data_ptr());
  a.o_sb = out.stride(0); a.o_sh = out.stride(1); a.o_sn = out.stride(2);
  Tensor P, dq, dk, dv;
  if (packed) {
    P = at::empty({B, N, 3, H, d}, o);
    dq = P.select(2, 0).transpose(1, 2); dk = P.select(2, 1).transpose(1, 2); dv = P.select(2, 2).transpose(1, 2);
  } else {
    dq = at::empty({B, H, N, d}, o); dk = at::empty({B, H, N, d}, o); dv = at::empty({B, H, N, d}, o);
  }
  Tensor dlq = at::empty_like(lq), dlk = at::empty_like(lk);
  Tensor ws = at::empty({(int64_t)csa_rel_attn_bwd_workspace_bytes(B, H, N, L, d)}, o.dtype(at::kByte));
  csa_rel_attn_bwd_args b;
  memset(&b, 0, sizeof(b));
  b.fwd = &a;
  b.dout = fp(dout); b.dq = fpw(dq); b.dk = fpw(dk); b.dv = fpw(dv);
  b.do_sb = dout.stride(0); b.do_sh = dout.stride(1); b.do_sn = dout.stride(2);
  if (packed) {  // contiguous outputs leave the triples zero (= contiguous)
    b.dq_sb = dq.stride(0); b.dq_sh = dq.stride(1); b.dq_sn = dq.stride(2);
    b.dk_sb = dk.stride(0); b.dk_sh = dk.stride(1); b.dk_sn = dk.stride(2);
    b.dv_sb = dv.stride(0); b.dv_sh = dv.stride(1); b.dv_sn = dv.stride(2);
  }
  b.dlq = fpw(dlq); b.dlk = fpw(dlk); b.workspace = ws.data_ptr();
  b.prof = g_prof_rel_bwd;
  a.prof = nullptr;  // the forward's stages are not re-run by the backward
  {
    const std::unique_lock<std::mutex> lane_lock = set_side_lane(b, q, schedule);
    check(csa_rel_attn_bwd(&b, cur_stream(q)), "csa_rel_attn_bwd");
  }
  if (packed) return {P, dlq, dlk};
  return {dq, dk, dv, dlq, dlk};
}

}  // namespace

extern "C" {
// bench.py's per-stage HIP-event profiling: csa_prof structs the caller owns (NULL = off)
void csa_torch_set_stage_profiler(const csa_prof* fwd, const csa_prof* bwd) {
  g_prof_fwd = fwd;
  g_prof_bwd = bwd;
}
// the same for the CSE relation attention (ABI v9 CSA_REL_STAGE_* slots)
void csa_torch_set_rel_profiler(const csa_prof* fwd, const csa_prof* bwd) {
  g_prof_rel_fwd = fwd;
  g_prof_rel_bwd = bwd;
}
}

// The schemas are defined by csa_amd/ops.py (torch.library.define, with the fake implementations), so the
// package imports and traces without this library; loading it registers the GPU implementations.
TORCH_LIBRARY_IMPL(csa, CUDA, m) {
  m.impl("sbm_fwd", &sbm_fwd);
  m.impl("sbm_maps", &sbm_maps);
  m.impl("sbm_bwd", &sbm_bwd);
  m.impl("ste_sample", &ste_sample);
  m.impl("ste_backward", &ste_backward);
  m.impl("rel_attn_fwd", &rel_attn_fwd);
  m.impl("rel_attn_bwd", &rel_attn_bwd);
}
