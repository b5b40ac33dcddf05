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
