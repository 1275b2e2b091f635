// AdamW step of script/optimizer.py:49-106 (HF-style AdamW, used with correct_bias=False by
// script/train.py:80) as ONE multi-tensor kernel on gfx950.
//
// The reference walks the parameters in Python and issues 7 elementwise ops per tensor
// (mul_, add_, mul_, addcmul_, sqrt, add_, addcdiv_ [+ add_ for weight decay]), i.e. ~200 tensors x
// 7 launches and 7 read/write passes over the optimizer state per step. Here every element is read
// once (param, grad, exp_avg, exp_avg_sq) and written once (param, exp_avg, exp_avg_sq): 28 B per
// parameter, HBM-bound.
//
// Mixed precision: GradScaler hands the optimizer its scale and found_inf as device tensors
// (_step_supports_amp_scaling), so unscaling and the skip-on-inf happen here, with no host sync.
//
// Work decomposition: each tensor is cut into CSA_ADAMW_CHUNK-element chunks; one 256-thread
// workgroup per chunk; chunk_tensor[] / chunk_start[] (built once per parameter layout by the
// caller) map a chunk to its tensor and offset without a search.
#include "csa_common.hpp"
#include "../../include/csa_hip.h"

using csa::f32x4;

namespace {

struct AdamElem {
  float b1, b2, om_b1, om_b2, eps, neg_step, neg_decay;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamElem& c) {
  m = fmaf(c.om_b1, g, m * c.b1);               // exp_avg.mul_(beta1).add_(grad, alpha=1-beta1)
  v = fmaf(c.om_b2 * g, g, v * c.b2);           // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1-beta2)
  const float den = __builtin_sqrtf(v) + c.eps;  // exp_avg_sq.sqrt().add_(eps)
  p = fmaf(c.neg_step, m / den, p);             // p.addcdiv_(exp_avg, denom, value=-step_size)
  p = fmaf(c.neg_decay, p, p);                  // p.add_(p, alpha=-lr*weight_decay)  (0: no-op)
}

__global__ __launch_bounds__(256) void k_adamw(const csa_adamw_tensor* __restrict__ tensors,
                                               const int32_t* __restrict__ chunk_tensor,
                                               const int64_t* __restrict__ chunk_start, AdamElem c,
                                               const float* __restrict__ grad_scale,
                                               const float* __restrict__ found_inf) {
  if (found_inf != nullptr && *found_inf != 0.f) return;  // GradScaler: skip the step on inf/NaN grads
  const float inv = grad_scale != nullptr ? (float)(1.0 / (double)*grad_scale) : 1.f;
  const int64_t chunk = blockIdx.x;
  const int t = chunk_tensor[chunk];
  const csa_adamw_tensor T = tensors[t];
  const int64_t base = (chunk - chunk_start[t]) * CSA_ADAMW_CHUNK;
  const int64_t rem = T.numel - base;
  const int n = (int)(rem < CSA_ADAMW_CHUNK ? rem : CSA_ADAMW_CHUNK);
  float* __restrict__ p = T.param + base;
  const float* __restrict__ g = T.grad + base;
  float* __restrict__ m = T.exp_avg + base;
  float* __restrict__ v = T.exp_avg_sq + base;
  const bool vec = ((((uintptr_t)p) | ((uintptr_t)g) | ((uintptr_t)m) | ((uintptr_t)v)) & 15) == 0;
  if (vec) {
    for (int i = 4 * (int)threadIdx.x; i < n; i += 4 * 256) {
      if (i + 4 <= n) {
        f32x4 pv = *reinterpret_cast<const f32x4*>(p + i);
        const f32x4 gv = *reinterpret_cast<const f32x4*>(g + i);
        f32x4 mv = *reinterpret_cast<const f32x4*>(m + i);
        f32x4 vv = *reinterpret_cast<const f32x4*>(v + i);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float pe = pv[e], me = mv[e], ve = vv[e];
          adam_elem(pe, gv[e] * inv, me, ve, c);
          pv[e] = pe; mv[e] = me; vv[e] = ve;
        }
        *reinterpret_cast<f32x4*>(p + i) = pv;
        *reinterpret_cast<f32x4*>(m + i) = mv;
        *reinterpret_cast<f32x4*>(v + i) = vv;
      } else {
        for (int e = i; e < n; ++e) adam_elem(p[e], g[e] * inv, m[e], v[e], c);
      }
    }
  } else {
    for (int i = threadIdx.x; i < n; i += 256) adam_elem(p[i], g[i] * inv, m[i], v[i], c);
  }
}

}  // namespace

extern "C" csa_status csa_adamw_step(const csa_adamw_args* a, void* stream) {
  if (!a) {
    csa::set_error("csa_adamw_step: null args");
    return CSA_INVALID_ARG;
  }
  if (a->ntensors < 0 || a->nchunks < 0 || a->nchunks > 0x7fffffff) {
    csa::set_error("csa_adamw_step: bad ntensors/nchunks");
    return CSA_INVALID_ARG;
  }
  if (a->nchunks == 0) return CSA_OK;
  if (!a->tensors || !a->chunk_tensor || !a->chunk_start) {
    csa::set_error("csa_adamw_step: null tensor table");
    return CSA_INVALID_ARG;
  }
  if (!(a->beta1 >= 0.f && a->beta1 < 1.f && a->beta2 >= 0.f && a->beta2 < 1.f && a->eps >= 0.f)) {
    csa::set_error("csa_adamw_step: invalid beta/eps");
    return CSA_INVALID_ARG;
  }
  AdamElem c;
  c.b1 = a->beta1; c.b2 = a->beta2; c.om_b1 = a->one_minus_beta1; c.om_b2 = a->one_minus_beta2;
  c.eps = a->eps; c.neg_step = -a->step_size; c.neg_decay = -a->decay;
  const csa::DeviceGuard guard((hipStream_t)stream);
  hipLaunchKernelGGL(k_adamw, dim3((unsigned)a->nchunks), dim3(256), 0, (hipStream_t)stream, a->tensors,
                     a->chunk_tensor, a->chunk_start, c, a->grad_scale, a->found_inf);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    csa::set_error("csa_adamw_step: %s", hipGetErrorString(e));
    return CSA_LAUNCH_FAILED;
  }
  return CSA_OK;
}
