// The step's scalar loss, fused (train.py:103-108, eval.py:157-163):
//   loss = mse(rgb_coarse[:, :3], target[:, :3]) + mse(rgb_fine[:, :3], target[:, :3])
//        + lambda * (||z_s|| + ||z_t||)
// The reference spends ~15 small aten launches on this and on its backward (two sub/pow/
// mean chains, two norms of expanded code tensors, the adds, and their grads).  Here one
// single-workgroup reduction forward (double accumulation) and one elementwise backward.
// ||z|| of a code row expanded over E rays (eval: z_s.expand(R, -1)) is sqrt(E * sum z^2);
// with E = 1 the code tensor is taken whole (train: the full embedding tables, .data, no
// gradient -- train.py:106-107 through model.py:113-120).
#include <algorithm>

#include "cn_common.h"

namespace {

constexpr int kThreads = 1024;

__device__ __forceinline__ double block_sum(double v, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < kThreads / 64; ++i) s += red[i];
  return s;  // valid on thread 0
}

// out: [loss_coarse, loss_fine, regulariser, total, ||z_s||, ||z_t||]
__global__ __launch_bounds__(kThreads) void render_loss_kernel(const float* __restrict__ rgb_c,
                                                               const float* __restrict__ rgb_f,
                                                               const float* __restrict__ target, int64_t ldt,
                                                               int64_t n_rays, const float* __restrict__ zs,
                                                               const float* __restrict__ zt, int64_t n_code,
                                                               double expand, float lambda, float* __restrict__ out) {
  __shared__ double red[kThreads / 64];
  double sc = 0.0, sf = 0.0, ss = 0.0, st = 0.0;
  const int64_t n = n_rays * 3;
  for (int64_t i = threadIdx.x; i < n; i += kThreads) {
    const int64_t r = i / 3, c = i - 3 * r;
    const float t = target[r * ldt + c];
    if (rgb_c) {
      const float d = rgb_c[i] - t;
      sc += static_cast<double>(d) * d;
    }
    if (rgb_f) {
      const float d = rgb_f[i] - t;
      sf += static_cast<double>(d) * d;
    }
  }
  for (int64_t i = threadIdx.x; i < n_code; i += kThreads) {
    if (zs) ss += static_cast<double>(zs[i]) * zs[i];
    if (zt) st += static_cast<double>(zt[i]) * zt[i];
  }
  sc = block_sum(sc, red);
  sf = block_sum(sf, red);
  ss = block_sum(ss, red);
  st = block_sum(st, red);
  if (threadIdx.x == 0) {
    const float lc = static_cast<float>(sc / static_cast<double>(n));
    const float lf = static_cast<float>(sf / static_cast<double>(n));
    const float ns = static_cast<float>(sqrt(ss * expand)), nt = static_cast<float>(sqrt(st * expand));
    const float reg = lambda * (ns + nt);
    out[0] = lc;
    out[1] = lf;
    out[2] = reg;
    out[3] = (lc + lf) + reg;
    out[4] = ns;
    out[5] = nt;
  }
}

// d loss_total / d rgb = g * 2 (rgb - t) / (3R) (mse 'mean'); d / d z_row = g * lambda * E z / ||z||
// (the expanded rows' gradients summed onto the row); g = *grad (device scalar).
__global__ void render_loss_backward_kernel(const float* __restrict__ rgb_c, const float* __restrict__ rgb_f,
                                            const float* __restrict__ target, int64_t ldt, int64_t n_rays,
                                            const float* __restrict__ zs, const float* __restrict__ zt,
                                            int64_t n_code, float expand, float lambda,
                                            const float* __restrict__ stats, const float* __restrict__ grad,
                                            float* __restrict__ d_rgb_c, float* __restrict__ d_rgb_f,
                                            float* __restrict__ d_zs, float* __restrict__ d_zt) {
  const float g = *grad;
  const int64_t n = n_rays * 3;
  const float k = __fdiv_rn(2.0f, static_cast<float>(n));
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / 3, c = i - 3 * r;
    const float t = target[r * ldt + c];
    if (d_rgb_c) d_rgb_c[i] = g * (k * (rgb_c[i] - t));
    if (d_rgb_f) d_rgb_f[i] = g * (k * (rgb_f[i] - t));
  }
  // torch's norm backward is 0 at a zero norm
  const float ks = stats[4] > 0.0f ? g * lambda * expand / stats[4] : 0.0f;
  const float kt = stats[5] > 0.0f ? g * lambda * expand / stats[5] : 0.0f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n_code; i += (int64_t)gridDim.x * blockDim.x) {
    if (d_zs) d_zs[i] = ks * zs[i];
    if (d_zt) d_zt[i] = kt * zt[i];
  }
}

}  // namespace

extern "C" int cn_render_loss(const float* rgb_coarse, const float* rgb_fine, const float* target,
                              int64_t target_stride, int64_t n_rays, const float* z_s, const float* z_t,
                              int64_t n_code, int64_t expand, float regularizer_lambda, float* out,
                              cn_stream_t stream) {
  CN_CHECK_ARG(n_rays > 0 && target && target_stride >= 3 && out && (rgb_coarse || rgb_fine));
  CN_CHECK_ARG(n_code >= 0 && expand >= 1 && (n_code == 0 || (z_s && z_t)));
  hipLaunchKernelGGL(render_loss_kernel, dim3(1), dim3(kThreads), 0, cn::as_stream(stream), rgb_coarse, rgb_fine,
                     target, target_stride, n_rays, z_s, z_t, n_code, static_cast<double>(expand),
                     regularizer_lambda, out);
  return cn::launch_status();
}

extern "C" int cn_render_loss_backward(const float* rgb_coarse, const float* rgb_fine, const float* target,
                                       int64_t target_stride, int64_t n_rays, const float* z_s, const float* z_t,
                                       int64_t n_code, int64_t expand, float regularizer_lambda, const float* stats,
                                       const float* grad_total, float* d_rgb_coarse, float* d_rgb_fine,
                                       float* d_z_s, float* d_z_t, cn_stream_t stream) {
  CN_CHECK_ARG(n_rays > 0 && target && target_stride >= 3 && stats && grad_total);
  CN_CHECK_ARG((!d_rgb_coarse || rgb_coarse) && (!d_rgb_fine || rgb_fine));
  CN_CHECK_ARG((!d_z_s && !d_z_t) || (z_s && z_t && n_code > 0 && expand >= 1));
  const int64_t n = std::max<int64_t>(n_rays * 3, n_code);
  hipLaunchKernelGGL(render_loss_backward_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0,
                     cn::as_stream(stream), rgb_coarse, rgb_fine, target, target_stride, n_rays, z_s, z_t, n_code,
                     static_cast<float>(expand), regularizer_lambda, stats, grad_total, d_rgb_coarse, d_rgb_fine,
                     d_z_s, d_z_t);
  return cn::launch_status();
}
