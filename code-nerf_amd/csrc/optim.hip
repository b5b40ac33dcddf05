// The training step's optimiser: torch.optim.AdamW.step as
// the reference runs it (train.py:113 over the param groups of utils/util.py:159-164), on
// ONE flat fp32 buffer holding every parameter of every group, with the gradient and both
// moments in three more flat buffers of the same layout.  The host cuts the buffer into
// segments of equal (lr, weight_decay, step) -- normally one per param group -- and one
// launch updates up to kMaxSegs of them; a parameter without a gradient lies in no
// segment and is not touched (torch skips it too).
//
// Per element, torch's _single_tensor_adam (decoupled weight decay, amsgrad / maximize
// off), every op rounded to fp32 as torch's separate CPU kernels round it:
//   p = p * (1 - lr wd)
//   m = fma(1 - b1, g - m, m)              exp_avg.lerp_(grad, 1 - b1) (CPU lerp = fmadd)
//   v = v * b2;  v = v + ((1 - b2) g) g    exp_avg_sq.mul_(b2).addcmul_(grad, grad, 1 - b2)
//   p = p + ((-lr / (1 - b1^t)) m) / (sqrt(v) / sqrt(1 - b2^t) + eps)      addcdiv_
// The scalar factors are folded on the host in double, as the Python code computes them.
// HBM-bound: 16 B read + 12 B written per parameter.
#include <cmath>

#include "cn_common.h"

namespace cn {
namespace optim {

constexpr int kMaxSegs = 8;

struct AdamWArgs {
  int64_t begin[kMaxSegs], end[kMaxSegs];  // float4 ranges
  float decay[kMaxSegs];                   // 1 - lr * weight_decay
  float step_neg[kMaxSegs];                // -lr / (1 - beta1^step)
  float bc2_sqrt[kMaxSegs];                // (1 - beta2^step) ** 0.5
  int64_t lo, hi;                          // float4 span of all segments
  int n_segs;
  int lerp_small;                          // |1 - beta1| < 0.5: torch's lerp branch
  float w1, beta2, w2, eps;                // 1 - beta1, beta2, 1 - beta2, eps
  const float* dyn;                        // non-null: {decay, step_neg, bc2_sqrt} per segment in
                                           // device memory (graph replays: the host refreshes them)
};

// The per-segment scalar factors, folded in double as the Python optimiser computes them.
inline void fold_scalars(double lr, double wd, int64_t step, double beta1, double beta2, float* out) {
  const double t = static_cast<double>(step);
  out[0] = static_cast<float>(1.0 - lr * wd);
  out[1] = static_cast<float>(-(lr / (1.0 - std::pow(beta1, t))));
  out[2] = static_cast<float>(std::pow(1.0 - std::pow(beta2, t), 0.5));
}

__device__ __forceinline__ void adamw_elem(float& p, float g, float& m, float& v, float decay, float sn, float bc2,
                                           const AdamWArgs& a) {
  p = __fmul_rn(p, decay);
  const float d = __fsub_rn(g, m);
  m = a.lerp_small ? fmaf(a.w1, d, m) : fmaf(__fsub_rn(a.w1, 1.0f), d, g);
  v = __fmul_rn(v, a.beta2);
  v = __fadd_rn(v, __fmul_rn(__fmul_rn(a.w2, g), g));
  const float den = __fadd_rn(__fdiv_rn(__fsqrt_rn(v), bc2), a.eps);
  p = __fadd_rn(p, __fdiv_rn(__fmul_rn(sn, m), den));
}

__global__ __launch_bounds__(256) void adamw_kernel(float4* __restrict__ param, const float4* __restrict__ grad,
                                                    float4* __restrict__ exp_avg, float4* __restrict__ exp_avg_sq,
                                                    AdamWArgs a) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = a.lo + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.hi; i += stride) {
    bool hit = false;
    float decay = 1.0f, sn = 0.0f, bc2 = 1.0f;
#pragma unroll
    for (int k = 0; k < kMaxSegs; ++k) {
      if (k < a.n_segs && i >= a.begin[k] && i < a.end[k]) {
        hit = true;
        decay = a.dyn ? a.dyn[3 * k] : a.decay[k];
        sn = a.dyn ? a.dyn[3 * k + 1] : a.step_neg[k];
        bc2 = a.dyn ? a.dyn[3 * k + 2] : a.bc2_sqrt[k];
      }
    }
    if (!hit) continue;
    float4 p = param[i], m = exp_avg[i], v = exp_avg_sq[i];
    const float4 g = grad[i];
    adamw_elem(p.x, g.x, m.x, v.x, decay, sn, bc2, a);
    adamw_elem(p.y, g.y, m.y, v.y, decay, sn, bc2, a);
    adamw_elem(p.z, g.z, m.z, v.z, decay, sn, bc2, a);
    adamw_elem(p.w, g.w, m.w, v.w, decay, sn, bc2, a);
    param[i] = p;
    exp_avg[i] = m;
    exp_avg_sq[i] = v;
  }
}

}  // namespace optim
}  // namespace cn

// AdamW step over flat buffers: see include/codenerf.h.
extern "C" int cn_adamw_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n_segments,
                             const int64_t* seg_begin, const int64_t* seg_end, const double* lr,
                             const double* weight_decay, const int64_t* step, double beta1, double beta2, double eps,
                             cn_stream_t stream) {
  using namespace cn;
  CN_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && seg_begin && seg_end && lr && weight_decay && step);
  CN_CHECK_ARG(n_segments >= 1 && beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0);
  const void* bufs[4] = {param, grad, exp_avg, exp_avg_sq};
  for (const void* q : bufs) CN_CHECK_ARG(reinterpret_cast<uintptr_t>(q) % 16 == 0);
  for (int64_t k = 0; k < n_segments; ++k) {
    CN_CHECK_ARG(seg_begin[k] >= 0 && seg_begin[k] < seg_end[k] && seg_begin[k] % 4 == 0 && seg_end[k] % 4 == 0);
    CN_CHECK_ARG(k == 0 || seg_begin[k] >= seg_end[k - 1]);
    CN_CHECK_ARG(step[k] >= 1 && lr[k] >= 0.0 && weight_decay[k] >= 0.0);
  }
  hipStream_t st = as_stream(stream);
  for (int64_t k0 = 0; k0 < n_segments; k0 += optim::kMaxSegs) {
    optim::AdamWArgs a = {};
    a.n_segs = static_cast<int>(n_segments - k0 < optim::kMaxSegs ? n_segments - k0 : optim::kMaxSegs);
    a.w1 = static_cast<float>(1.0 - beta1);
    a.lerp_small = std::fabs(a.w1) < 0.5f ? 1 : 0;
    a.beta2 = static_cast<float>(beta2);
    a.w2 = static_cast<float>(1.0 - beta2);
    a.eps = static_cast<float>(eps);
    for (int j = 0; j < a.n_segs; ++j) {
      const int64_t k = k0 + j;
      a.begin[j] = seg_begin[k] / 4;
      a.end[j] = seg_end[k] / 4;
      float f[3];
      optim::fold_scalars(lr[k], weight_decay[k], step[k], beta1, beta2, f);
      a.decay[j] = f[0];
      a.step_neg[j] = f[1];
      a.bc2_sqrt[j] = f[2];
    }
    a.lo = a.begin[0];
    a.hi = a.end[a.n_segs - 1];
    hipLaunchKernelGGL(optim::adamw_kernel, dim3(elementwise_grid(a.hi - a.lo, 256)), dim3(256), 0, st,
                       reinterpret_cast<float4*>(param), reinterpret_cast<const float4*>(grad),
                       reinterpret_cast<float4*>(exp_avg), reinterpret_cast<float4*>(exp_avg_sq), a);
    const int rc = launch_status();
    if (rc != CN_OK) return rc;
  }
  return CN_OK;
}

extern "C" int cn_adamw_scalars(int64_t n_segments, const double* lr, const double* weight_decay, const int64_t* step,
                                double beta1, double beta2, float* out) {
  CN_CHECK_ARG(n_segments >= 1 && lr && weight_decay && step && out && beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 &&
               beta2 < 1.0);
  for (int64_t k = 0; k < n_segments; ++k) {
    CN_CHECK_ARG(step[k] >= 1 && lr[k] >= 0.0 && weight_decay[k] >= 0.0);
    cn::optim::fold_scalars(lr[k], weight_decay[k], step[k], beta1, beta2, out + 3 * k);
  }
  return CN_OK;
}

extern "C" int cn_adamw_step_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                                 int64_t n_segments, const int64_t* seg_begin, const int64_t* seg_end,
                                 const float* scalars, double beta1, double beta2, double eps, cn_stream_t stream) {
  using namespace cn;
  CN_CHECK_ARG(param && grad && exp_avg && exp_avg_sq && seg_begin && seg_end && scalars);
  CN_CHECK_ARG(n_segments >= 1 && beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0);
  const void* bufs[4] = {param, grad, exp_avg, exp_avg_sq};
  for (const void* q : bufs) CN_CHECK_ARG(reinterpret_cast<uintptr_t>(q) % 16 == 0);
  for (int64_t k = 0; k < n_segments; ++k) {
    CN_CHECK_ARG(seg_begin[k] >= 0 && seg_begin[k] < seg_end[k] && seg_begin[k] % 4 == 0 && seg_end[k] % 4 == 0);
    CN_CHECK_ARG(k == 0 || seg_begin[k] >= seg_end[k - 1]);
  }
  hipStream_t st = as_stream(stream);
  for (int64_t k0 = 0; k0 < n_segments; k0 += optim::kMaxSegs) {
    optim::AdamWArgs a = {};
    a.n_segs = static_cast<int>(n_segments - k0 < optim::kMaxSegs ? n_segments - k0 : optim::kMaxSegs);
    a.w1 = static_cast<float>(1.0 - beta1);
    a.lerp_small = std::fabs(a.w1) < 0.5f ? 1 : 0;
    a.beta2 = static_cast<float>(beta2);
    a.w2 = static_cast<float>(1.0 - beta2);
    a.eps = static_cast<float>(eps);
    a.dyn = scalars + 3 * k0;
    for (int j = 0; j < a.n_segs; ++j) {
      a.begin[j] = seg_begin[k0 + j] / 4;
      a.end[j] = seg_end[k0 + j] / 4;
    }
    a.lo = a.begin[0];
    a.hi = a.end[a.n_segs - 1];
    hipLaunchKernelGGL(optim::adamw_kernel, dim3(elementwise_grid(a.hi - a.lo, 256)), dim3(256), 0, st,
                       reinterpret_cast<float4*>(param), reinterpret_cast<const float4*>(grad),
                       reinterpret_cast<float4*>(exp_avg), reinterpret_cast<float4*>(exp_avg_sq), a);
    const int rc = launch_status();
    if (rc != CN_OK) return rc;
  }
  return CN_OK;
}
