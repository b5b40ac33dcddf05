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

// Large code tensors (train: the whole embedding tables, 2 x 2458 x 256): per-block partial sums
// of squares (double) into partials[2 b], [2 b + 1]; the loss kernel adds them up.
constexpr int kPartThreads = 256;
// code values per partial block: 1024 (4 per thread, one float4 each) -- 615 blocks for the C3
// tables instead of 77 blocks looping 32 times (11 -> ~3 us; the loss kernel adds the partials)
constexpr int64_t kPartElems = 1024;

__global__ __launch_bounds__(kPartThreads) void code_sq_partials_kernel(const float* __restrict__ zs,
                                                                        const float* __restrict__ zt, int64_t n_code,
                                                                        double* __restrict__ partials) {
  __shared__ double red[2][kPartThreads / 64];
  double ss = 0.0, st = 0.0;
  const int64_t b0 = blockIdx.x * kPartElems, b1 = min(b0 + kPartElems, n_code);
  // all of a thread's loads first, then the products (four values per thread)
  float vs[kPartElems / kPartThreads], vt[kPartElems / kPartThreads];
#pragma unroll
  for (int k = 0; k < kPartElems / kPartThreads; ++k) {
    const int64_t i = b0 + threadIdx.x + k * kPartThreads;
    vs[k] = i < b1 ? zs[i] : 0.0f;
    vt[k] = i < b1 ? zt[i] : 0.0f;
  }
#pragma unroll
  for (int k = 0; k < kPartElems / kPartThreads; ++k) {
    ss += static_cast<double>(vs[k]) * vs[k];
    st += static_cast<double>(vt[k]) * vt[k];
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ss += __shfl_xor(ss, o);
    st += __shfl_xor(st, o);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = ss;
    red[1][threadIdx.x >> 6] = st;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0.0, b = 0.0;
    for (int w = 0; w < kPartThreads / 64; ++w) {
      a += red[0][w];
      b += red[1][w];
    }
    partials[2 * blockIdx.x] = a;
    partials[2 * blockIdx.x + 1] = b;
  }
}

// out: [loss_coarse, loss_fine, regulariser, total, ||z_s||, ||z_t||].  n_part > 0: the code sums
// come from the n_part partial pairs instead of z_s / z_t.
__global__ __launch_bounds__(kThreads) void render_loss_kernel(const float* __restrict__ rgb_c,
                                                               const float* __restrict__ rgb_f,
                                                               const float* __restrict__ target, int64_t ldt,
                                                               int64_t n_rays, const float* __restrict__ zs,
                                                               const float* __restrict__ zt, int64_t n_code,
                                                               const double* __restrict__ partials, int n_part,
                                                               double expand, float lambda, float* __restrict__ out,
                                                               double* __restrict__ psnr) {
  __shared__ double red[kThreads / 64];
  double sc = 0.0, sf = 0.0, ss = 0.0, st = 0.0;
  const int64_t n = n_rays * 3;
  // four elements per thread and round, their loads issued together (one at a time the 12 rounds of
  // a 4096-ray chunk were 12 serial memory latencies); the same per-thread summation order
  constexpr int kU = 4;
  for (int64_t i0 = threadIdx.x; i0 < n; i0 += kU * kThreads) {
    float t[kU], c[kU], f[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = i0 + u * kThreads;
      const bool ok = i < n;
      const int64_t ii = ok ? i : 0;
      const int64_t r = ii / 3, cc = ii - 3 * r;
      t[u] = target[r * ldt + cc];
      c[u] = rgb_c ? rgb_c[ii] : 0.0f;
      f[u] = rgb_f ? rgb_f[ii] : 0.0f;
      if (!ok) t[u] = c[u] = f[u] = 0.0f;
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const float dc = c[u] - t[u], df = f[u] - t[u];
      if (rgb_c) sc += static_cast<double>(dc) * dc;
      if (rgb_f) sf += static_cast<double>(df) * df;
    }
  }
  if (n_part > 0) {
    for (int i = threadIdx.x; i < n_part; i += kThreads) {
      ss += partials[2 * i];
      st += partials[2 * i + 1];
    }
  } else {
    for (int64_t i = threadIdx.x; i < n_code; i += kThreads) {
      if (zs) ss += static_cast<double>(zs[i]) * zs[i];
      if (zt) st += static_cast<double>(zt[i]) * zt[i];
    }
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
    if (psnr) {  // mse2psnr (util.py:216-227) of the fine loss, float64
      const double m = static_cast<double>(rgb_f ? lf : lc);
      psnr[0] = -10.0 * log10(m == 0.0 ? 1e-5 : m);
    }
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
                                            float* __restrict__ d_zs, float* __restrict__ d_zt, int accumulate_z) {
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
    if (accumulate_z) {
      if (d_zs) d_zs[i] += ks * zs[i];
      if (d_zt) d_zt[i] += kt * zt[i];
    } else {
      if (d_zs) d_zs[i] = ks * zs[i];
      if (d_zt) d_zt[i] = kt * zt[i];
    }
  }
}

}  // namespace

extern "C" int64_t cn_render_loss_workspace_doubles(int64_t n_code) {
  if (n_code < 0) return -1;
  return n_code <= 2 * kPartElems ? 0 : 2 * cn::ceil_div(n_code, kPartElems);
}

extern "C" int cn_render_loss(const float* rgb_coarse, const float* rgb_fine, const float* target,
                              int64_t target_stride, int64_t n_rays, const float* z_s, const float* z_t,
                              int64_t n_code, int64_t expand, float regularizer_lambda, double* workspace,
                              float* out, cn_stream_t stream) {
  return cn_render_loss_psnr(rgb_coarse, rgb_fine, target, target_stride, n_rays, z_s, z_t, n_code, expand,
                             regularizer_lambda, workspace, out, nullptr, stream);
}

extern "C" int cn_render_loss_psnr(const float* rgb_coarse, const float* rgb_fine, const float* target,
                                   int64_t target_stride, int64_t n_rays, const float* z_s, const float* z_t,
                                   int64_t n_code, int64_t expand, float regularizer_lambda, double* workspace,
                                   float* out, double* psnr, cn_stream_t stream) {
  CN_CHECK_ARG(n_rays > 0 && target && target_stride >= 3 && out && (rgb_coarse || rgb_fine));
  CN_CHECK_ARG(n_code >= 0 && expand >= 1 && (n_code == 0 || (z_s && z_t)));
  const int64_t ws = cn_render_loss_workspace_doubles(n_code);
  CN_CHECK_ARG(ws == 0 || workspace);
  const int n_part = static_cast<int>(ws / 2);
  if (n_part > 0)
    hipLaunchKernelGGL(code_sq_partials_kernel, dim3(n_part), dim3(kPartThreads), 0, cn::as_stream(stream), z_s, z_t,
                       n_code, workspace);
  hipLaunchKernelGGL(render_loss_kernel, dim3(1), dim3(kThreads), 0, cn::as_stream(stream), rgb_coarse, rgb_fine,
                     target, target_stride, n_rays, z_s, z_t, n_code, workspace, n_part, static_cast<double>(expand),
                     regularizer_lambda, out, psnr);
  return cn::launch_status();
}

extern "C" int cn_render_loss_backward(const float* rgb_coarse, const float* rgb_fine, const float* target,
                                       int64_t target_stride, int64_t n_rays, const float* z_s, const float* z_t,
                                       int64_t n_code, int64_t expand, float regularizer_lambda, const float* stats,
                                       const float* grad_total, float* d_rgb_coarse, float* d_rgb_fine,
                                       float* d_z_s, float* d_z_t, int accumulate_z, cn_stream_t stream) {
  CN_CHECK_ARG(n_rays > 0 && target && target_stride >= 3 && stats && grad_total);
  CN_CHECK_ARG(accumulate_z == 0 || accumulate_z == 1);
  CN_CHECK_ARG((!d_rgb_coarse || rgb_coarse) && (!d_rgb_fine || rgb_fine));
  CN_CHECK_ARG((!d_z_s && !d_z_t) || (z_s && z_t && n_code > 0 && expand >= 1));
  const int64_t n = std::max<int64_t>(n_rays * 3, n_code);
  hipLaunchKernelGGL(render_loss_backward_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0,
                     cn::as_stream(stream), rgb_coarse, rgb_fine, target, target_stride, n_rays, z_s, z_t, n_code,
                     static_cast<float>(expand), regularizer_lambda, stats, grad_total, d_rgb_coarse, d_rgb_fine,
                     d_z_s, d_z_t, accumulate_z);
  return cn::launch_status();
}
