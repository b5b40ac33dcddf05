// Ray generation: RaySampler (view_synthesis/nerf/ray_sampler.py).
//
// Memory-bound and tiny (24 B/ray written); one lane per pixel / ray with the
// 3-float records read and written by consecutive lanes.
#include "cn_common.h"

namespace {

// ray_sampler.py:35-51 — meshgrid(indexing='xy'): pixel p = h*W + w,
// dir = ((w - cx)/f, -(h - cy)/f, -1); no +0.5 centre (quirk Q3).
__global__ void ray_directions_kernel(int64_t height, int64_t width, float focal, float cx,
                                      float cy, float* __restrict__ dirs) {
  const int64_t n = height * width;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n;
       p += (int64_t)gridDim.x * blockDim.x) {
    const float w = static_cast<float>(p % width);
    const float h = static_cast<float>(p / width);
    dirs[3 * p + 0] = __fdiv_rn(__fsub_rn(w, cx), focal);
    dirs[3 * p + 1] = __fdiv_rn(-__fsub_rn(h, cy), focal);
    dirs[3 * p + 2] = -1.0f;
  }
}

// ray_sampler.py:95-98 — rd[b,p,:] = R_b d_p (einsum 'hwij,bji->bhwj'),
// ro[b,p,:] = t_b.
__global__ void ray_bundle_kernel(const float* __restrict__ dirs, int64_t hw,
                                  const float* __restrict__ c2w, int64_t batch,
                                  float* __restrict__ ro, float* __restrict__ rd) {
  const int64_t n = hw * batch;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = q / hw, p = q % hw;
    const float* T = c2w + 16 * b;
    const float d0 = dirs[3 * p], d1 = dirs[3 * p + 1], d2 = dirs[3 * p + 2];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float acc = __fmul_rn(d0, T[4 * j + 0]);
      acc = __fadd_rn(acc, __fmul_rn(d1, T[4 * j + 1]));
      acc = __fadd_rn(acc, __fmul_rn(d2, T[4 * j + 2]));
      rd[3 * q + j] = acc;
      ro[3 * q + j] = T[4 * j + 3];
    }
  }
}

// ray_sampler.py:77-80 — per-image fancy-index gather.  Indices out of
// [0, hw) produce NaN rays (the host wrapper validates them first).
__global__ void gather_rays_kernel(const float* __restrict__ ro, const float* __restrict__ rd,
                                   int64_t batch, int64_t hw,
                                   const int64_t* __restrict__ sel, int64_t s,
                                   float* __restrict__ ro_out, float* __restrict__ rd_out) {
  const int64_t n = batch * s;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = q / s;
    const int64_t p = sel[q];
    const bool ok = p >= 0 && p < hw;
    const int64_t src = (b * hw + (ok ? p : 0)) * 3;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      ro_out[3 * q + j] = ok ? ro[src + j] : __int_as_float(0x7fc00000);
      rd_out[3 * q + j] = ok ? rd[src + j] : __int_as_float(0x7fc00000);
    }
  }
}

}  // namespace

extern "C" int cn_ray_directions(int64_t height, int64_t width, float focal, float cx,
                                 float cy, float* dirs, cn_stream_t stream) {
  CN_CHECK_ARG(height > 0 && width > 0 && dirs != nullptr && focal != 0.0f);
  const int64_t n = height * width;
  hipLaunchKernelGGL(ray_directions_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0,
                     cn::as_stream(stream), height, width, focal, cx, cy, dirs);
  return cn::launch_status();
}

extern "C" int cn_ray_bundle(const float* dirs, int64_t hw, const float* c2w, int64_t batch,
                             float* ro, float* rd, cn_stream_t stream) {
  CN_CHECK_ARG(hw > 0 && batch > 0 && dirs && c2w && ro && rd);
  const int64_t n = hw * batch;
  hipLaunchKernelGGL(ray_bundle_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0,
                     cn::as_stream(stream), dirs, hw, c2w, batch, ro, rd);
  return cn::launch_status();
}

extern "C" int cn_gather_rays(const float* ro, const float* rd, int64_t batch, int64_t hw,
                              const int64_t* select_inds, int64_t sample_size, float* ro_out,
                              float* rd_out, cn_stream_t stream) {
  CN_CHECK_ARG(batch > 0 && hw > 0 && sample_size > 0 && sample_size <= hw);
  CN_CHECK_ARG(ro && rd && select_inds && ro_out && rd_out);
  const int64_t n = batch * sample_size;
  hipLaunchKernelGGL(gather_rays_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0,
                     cn::as_stream(stream), ro, rd, batch, hw, select_inds, sample_size, ro_out,
                     rd_out);
  return cn::launch_status();
}

// ---------------------------------------------------------------- backward
namespace {

// get_bundle backward (ray_sampler.py:97-98): d R_b[j][i] = sum_p g_rd[b,p,j] d_p[i],
// d t_b[j] = sum_p g_ro[b,p,j] into d_c2w (B,4,4) rows 0..2 (row 3 untouched).
// One block per image, one reduction of 12 sums over its pixels.
__global__ __launch_bounds__(256) void ray_bundle_backward_kernel(const float* __restrict__ dirs, int64_t hw,
                                                                  const float* __restrict__ g_ro,
                                                                  const float* __restrict__ g_rd,
                                                                  float* __restrict__ d_c2w) {
  __shared__ float red[12][256];
  const int64_t b = blockIdx.x;
  float acc[12] = {0};
  for (int64_t p = threadIdx.x; p < hw; p += blockDim.x) {
    const float d0 = dirs[3 * p], d1 = dirs[3 * p + 1], d2 = dirs[3 * p + 2];
    const int64_t q = b * hw + p;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const float g = g_rd ? g_rd[3 * q + j] : 0.0f;
      acc[4 * j + 0] += g * d0;
      acc[4 * j + 1] += g * d1;
      acc[4 * j + 2] += g * d2;
      acc[4 * j + 3] += g_ro ? g_ro[3 * q + j] : 0.0f;
    }
  }
#pragma unroll
  for (int k = 0; k < 12; ++k) red[k][threadIdx.x] = acc[k];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s)
#pragma unroll
      for (int k = 0; k < 12; ++k) red[k][threadIdx.x] += red[k][threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x < 12) d_c2w[16 * b + threadIdx.x] += red[threadIdx.x][0];
}

// sample gather backward (ray_sampler.py:77-80): indices within an image are a
// permutation prefix (unique), so the scatter is a plain store into zeroed grads.
__global__ void gather_rays_backward_kernel(const float* __restrict__ g_o, const float* __restrict__ g_d,
                                            int64_t batch, int64_t hw, const int64_t* __restrict__ sel, int64_t s,
                                            float* __restrict__ d_ro, float* __restrict__ d_rd) {
  const int64_t n = batch * s;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = q / s, p = sel[q];
    if (p < 0 || p >= hw) continue;
    const int64_t dst = (b * hw + p) * 3;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      if (d_ro && g_o) d_ro[dst + j] += g_o[3 * q + j];
      if (d_rd && g_d) d_rd[dst + j] += g_d[3 * q + j];
    }
  }
}

}  // namespace

extern "C" int cn_ray_bundle_backward(const float* dirs, int64_t hw, int64_t batch, const float* g_ro,
                                      const float* g_rd, float* d_c2w, cn_stream_t stream) {
  CN_CHECK_ARG(dirs && d_c2w && hw > 0 && batch > 0 && batch < (1ll << 31) && (g_ro || g_rd));
  hipLaunchKernelGGL(ray_bundle_backward_kernel, dim3(static_cast<unsigned>(batch)), dim3(256), 0,
                     cn::as_stream(stream), dirs, hw, g_ro, g_rd, d_c2w);
  return cn::launch_status();
}

extern "C" int cn_gather_rays_backward(const float* g_ro, const float* g_rd, int64_t batch, int64_t hw,
                                       const int64_t* select_inds, int64_t sample_size, float* d_ro, float* d_rd,
                                       cn_stream_t stream) {
  CN_CHECK_ARG(batch > 0 && hw > 0 && sample_size > 0 && sample_size <= hw && select_inds);
  const int64_t n = batch * sample_size;
  hipLaunchKernelGGL(gather_rays_backward_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0,
                     cn::as_stream(stream), g_ro, g_rd, batch, hw, select_inds, sample_size, d_ro, d_rd);
  return cn::launch_status();
}
