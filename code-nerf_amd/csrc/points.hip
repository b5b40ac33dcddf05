// Point sampling: PointSampler (view_synthesis/nerf/point_sampler.py).
//
// sample_uniform is a pure stream (12 B ray + 4 B bin in, 16 B per sample out).
// sample_pdf gives one wavefront to one ray: the ray's cdf, bins and merged
// depth list live in LDS, the cdf is a wave scan (exact in double, so the
// sequential loop's bits), searchsorted is a binary search there, and the
// final sort a bitonic network over (value, position) keys in the wave's
// registers -- the stable sort of the unsorted perturbed fine samples, ties
// included.
#include "cn_common.h"

namespace {

// point_sampler.py:60-70.  z = lower + (upper - lower) * t (perturb) or z_bins;
// pts = ro + rd * z, each op rounded separately as torch does.
__global__ void sample_uniform_kernel(const float* __restrict__ ro, const float* __restrict__ rd,
                                      int64_t n_rays, const float* __restrict__ zb,
                                      const float* __restrict__ lower,
                                      const float* __restrict__ upper, int64_t nc,
                                      const float* __restrict__ t_rand, float* __restrict__ z_out,
                                      float* __restrict__ pts_out) {
  const int64_t n = n_rays * nc;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = q / nc, i = q % nc;
    float z;
    if (t_rand) {
      z = __fadd_rn(lower[i], __fmul_rn(__fsub_rn(upper[i], lower[i]), t_rand[q]));
    } else {
      z = zb[i];
    }
    z_out[q] = z;
    if (pts_out) {
#pragma unroll
      for (int j = 0; j < 3; ++j) pts_out[3 * q + j] = cn::mul_add_rn(rd[3 * r + j], z, ro[3 * r + j]);
    }
  }
}

// The same for nc % 4 == 0 (every config: 32 / 64 coarse samples) and 16-B aligned buffers: one
// lane per 4 consecutive samples of a ray -- 16-B loads of the bins / bounds / draws and 16-B stores
// of z (a wave stores 1 KiB per instruction; pts as 3 x 16 B per lane, 3 KiB contiguous per wave),
// 32-bit index math (n_rays * nc / 4 < 2^32, checked by the host) instead of a 64-bit divide per
// sample, and one pass over a grid that covers the work (no grid-stride loop).  Bitwise the same
// arithmetic per sample.
__global__ __launch_bounds__(256) void sample_uniform4_kernel(const float* __restrict__ ro, const float* __restrict__ rd,
                                                              unsigned n4, unsigned nc4, const float4* __restrict__ zb,
                                                              const float4* __restrict__ lower,
                                                              const float4* __restrict__ upper,
                                                              const float4* __restrict__ t_rand, float4* __restrict__ z_out,
                                                              float4* __restrict__ pts_out) {
  const unsigned q = blockIdx.x * 256u + threadIdx.x;
  if (q >= n4) return;
  const unsigned r = q / nc4, i4 = q - r * nc4;
  float4 z;
  if (t_rand) {
    const float4 lo = lower[i4], up = upper[i4], t = t_rand[q];
    z.x = __fadd_rn(lo.x, __fmul_rn(__fsub_rn(up.x, lo.x), t.x));
    z.y = __fadd_rn(lo.y, __fmul_rn(__fsub_rn(up.y, lo.y), t.y));
    z.z = __fadd_rn(lo.z, __fmul_rn(__fsub_rn(up.z, lo.z), t.z));
    z.w = __fadd_rn(lo.w, __fmul_rn(__fsub_rn(up.w, lo.w), t.w));
  } else {
    z = zb[i4];
  }
  z_out[q] = z;
  if (pts_out) {
    const float o0 = ro[3 * r], o1 = ro[3 * r + 1], o2 = ro[3 * r + 2];
    const float d0 = rd[3 * r], d1 = rd[3 * r + 1], d2 = rd[3 * r + 2];
    float4* po = pts_out + 3 * static_cast<size_t>(q);
    po[0] = make_float4(cn::mul_add_rn(d0, z.x, o0), cn::mul_add_rn(d1, z.x, o1), cn::mul_add_rn(d2, z.x, o2),
                        cn::mul_add_rn(d0, z.y, o0));
    po[1] = make_float4(cn::mul_add_rn(d1, z.y, o1), cn::mul_add_rn(d2, z.y, o2), cn::mul_add_rn(d0, z.z, o0),
                        cn::mul_add_rn(d1, z.z, o1));
    po[2] = make_float4(cn::mul_add_rn(d2, z.z, o2), cn::mul_add_rn(d0, z.w, o0), cn::mul_add_rn(d1, z.w, o1),
                        cn::mul_add_rn(d2, z.w, o2));
  }
}

// pts = ro[..., None, :] + rd[..., None, :] * z[..., :, None] (point_sampler.py:70, :118).
__global__ void ray_points_kernel(const float* __restrict__ ro, const float* __restrict__ rd,
                                  const float* __restrict__ z, int64_t n_rays, int64_t s,
                                  float* __restrict__ pts) {
  const int64_t n = n_rays * s * 3;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = q / 3, j = q - 3 * e, r = e / s;
    pts[q] = cn::mul_add_rn(rd[3 * r + j], z[e], ro[3 * r + j]);
  }
}

constexpr int kPdfWaves = 4;       // rays per 256-thread block
constexpr int kPdfMaxN = 512;      // nc + nf

// torch.linspace(0, 1, n) on the CPU (RangeFactoriesKernel: symmetric halves).
__device__ __forceinline__ float linspace01(int i, int n) {
  if (n == 1) return 0.0f;
  const float step = __fdiv_rn(1.0f, static_cast<float>(n - 1));
  if (i < n / 2) return __fmul_rn(step, static_cast<float>(i));
  return __fsub_rn(1.0f, __fmul_rn(step, static_cast<float>(n - 1 - i)));
}

// torch.sum over a contiguous fp32 row on the CPU (aten SumKernel.cpp): rows
// shorter than 8 use the scalar 4-way ILP row_sum; longer rows accumulate
// 8-wide vectors in 4 ILP partials, fold them, add the scalar tail first and
// then the 8 lanes in order.  Exact for n < 512 (no cascade level is taken).
__device__ float torch_cpu_row_sum(const float* x, int n) {
  if (n < 8) {
    float p[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    const int s = n / 4;
    for (int i = 0; i < s; ++i)
      for (int k = 0; k < 4; ++k) p[k] = __fadd_rn(p[k], x[4 * i + k]);
    for (int i = 4 * s; i < n; ++i) p[0] = __fadd_rn(p[0], x[i]);
    return __fadd_rn(__fadd_rn(__fadd_rn(p[0], p[1]), p[2]), p[3]);
  }
  const int nv = n / 8, s = nv / 4;
  float fin = 0.0f;
  for (int k = 8 * nv; k < n; ++k) fin = __fadd_rn(fin, x[k]);
  for (int k = 0; k < 8; ++k) {
    float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int i = 0; i < s; ++i)
      for (int j = 0; j < 4; ++j) a[j] = __fadd_rn(a[j], x[(4 * i + j) * 8 + k]);
    float p = a[0];
    for (int i = 4 * s; i < nv; ++i) p = __fadd_rn(p, x[8 * i + k]);
    p = __fadd_rn(__fadd_rn(__fadd_rn(p, a[1]), a[2]), a[3]);
    fin = __fadd_rn(fin, p);
  }
  return fin;
}

// torch_cpu_row_sum for one wave (every lane returns it): the eight column chains of the n >= 8 path
// run in lanes 0..7, every lane then folds the scalar tail and the eight chains in torch's order.
__device__ float torch_cpu_row_sum_wave(const float* x, int n, int lane) {
  if (n < 8) return torch_cpu_row_sum(x, n);
  const int nv = n / 8, s = nv / 4;
  float p = 0.0f;
  if (lane < 8) {
    const int k = lane;
    float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int i = 0; i < s; ++i)
      for (int j = 0; j < 4; ++j) a[j] = __fadd_rn(a[j], x[(4 * i + j) * 8 + k]);
    p = a[0];
    for (int i = 4 * s; i < nv; ++i) p = __fadd_rn(p, x[8 * i + k]);
    p = __fadd_rn(__fadd_rn(__fadd_rn(p, a[1]), a[2]), a[3]);
  }
  float fin = 0.0f;
  for (int k = 8 * nv; k < n; ++k) fin = __fadd_rn(fin, x[k]);
  for (int k = 0; k < 8; ++k) fin = __fadd_rn(fin, __shfl(p, k));
  return fin;
}

// sort(cat(z, samples)) (:116) of one ray in its wave's registers: a bitonic network over N2 (value,
// position) keys, element e = lane + 64 h in lane `lane`, slot h; keys past n are +inf at positions past
// n, so ties order by position -- the stable sort.  Partners 64 or more apart sit in the same lane
// (a register exchange), nearer ones in lane ^ j (a cross-lane shuffle): no LDS, no barrier.  Then the
// sorted depths (and points) stored in order, coalesced.
template <int N2>
__device__ __forceinline__ void sort_store(const float* val, int n, int lane, float* __restrict__ zo,
                                           float* __restrict__ po, const float* o, const float* d) {
  constexpr int E = N2 / 64;
  float v[E];
  int ix[E];
#pragma unroll
  for (int h = 0; h < E; ++h) {
    const int e = lane + 64 * h;
    v[h] = e < n ? val[e] : __builtin_inff();
    ix[h] = e;
  }
#pragma unroll
  for (int k = 2; k <= N2; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
#pragma unroll
        for (int h = 0; h < E; ++h) {
          const int hp = h ^ (j >> 6);
          if (hp > h) {
            const bool up = ((lane + 64 * h) & k) == 0;
            const bool after = v[h] > v[hp] || (v[h] == v[hp] && ix[h] > ix[hp]);
            if (after == up) {
              const float tv = v[h];
              const int ti = ix[h];
              v[h] = v[hp];
              ix[h] = ix[hp];
              v[hp] = tv;
              ix[hp] = ti;
            }
          }
        }
      } else {
#pragma unroll
        for (int h = 0; h < E; ++h) {
          const float pv = __shfl_xor(v[h], j);
          const int pi = __shfl_xor(ix[h], j);
          const bool up = ((lane + 64 * h) & k) == 0, lower = (lane & j) == 0;
          const bool after = v[h] > pv || (v[h] == pv && ix[h] > pi);
          if (after == (lower == up)) {      // the lower slot of an ascending pair keeps the smaller key
            v[h] = pv;
            ix[h] = pi;
          }
        }
      }
    }
  }
#pragma unroll
  for (int h = 0; h < E; ++h) {
    const int e = lane + 64 * h;
    if (e < n) {
      zo[e] = v[h];
      if (po) {
#pragma unroll
        for (int j = 0; j < 3; ++j) po[3 * e + j] = cn::mul_add_rn(d[j], v[h], o[j]);
      }
    }
  }
}

// point_sampler.py:84-118, one wave per ray.
//   pdf / cdf: torch's CPU cumsum adds the fp32 pdf in double and rounds every prefix.  When every
//   nonzero |pdf| >= 2^-28 (so all are multiples of 2^-51) and sum |pdf| < 1.5 (every prefix below
//   2^2), each double prefix is EXACT -- whatever the order of the additions -- so a wave scan gives
//   the sequential loop's bits; a ray outside those bounds takes the sequential loop in lane 0.
//   sort(cat(z, samples)) (:116): sort_store, a bitonic network in registers.
__global__ __launch_bounds__(256) void sample_pdf_kernel(
    const float* __restrict__ ro, const float* __restrict__ rd, const float* __restrict__ weights,
    int64_t w_stride, const float* __restrict__ z, int64_t n_rays, int nc, int nf,
    const float* __restrict__ u_in, int64_t u_stride, float* __restrict__ z_out,
    float* __restrict__ pts_out) {
  __shared__ float s_cdf[kPdfWaves][256];
  __shared__ float s_mid[kPdfWaves][256];
  __shared__ float s_val[kPdfWaves][kPdfMaxN];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t r_raw = blockIdx.x * (int64_t)kPdfWaves + wv;
  const bool valid = r_raw < n_rays;       // wave-uniform; every wave reaches each barrier
  const int64_t r = valid ? r_raw : n_rays - 1;
  float* cdf = s_cdf[wv];
  float* mid = s_mid[wv];
  float* val = s_val[wv];
  const float* zr = z + r * nc;
  const float* wr = weights + r * w_stride;
  const int nw = nc - 2;      // pdf entries
  const int ncdf = nc - 1;    // cdf / bins entries
  const int n = nc + nf;
  int n2 = 64;
  while (n2 < n) n2 <<= 1;

  // bins = 0.5 * (z[1:] + z[:-1]) (:85); coarse depths into the merge list
  for (int j = lane; j < ncdf; j += 64) mid[j] = __fmul_rn(0.5f, __fadd_rn(zr[j + 1], zr[j]));
  for (int j = lane; j < nc; j += 64) val[j] = zr[j];

  // w = weights + 1e-5 (:86), staged in cdf[1..nw]
  for (int j = lane; j < nw; j += 64) cdf[j + 1] = __fadd_rn(wr[j], 1e-5f);
  __syncthreads();
  {
    // pdf = w / sum(w) (:87), cdf = [0, cumsum(pdf)] (:88-89)
    const float total = torch_cpu_row_sum_wave(cdf + 1, nw, lane);
    float pdf[4];            // entries lane + 64 q (nw <= 254)
    bool ok = true;
    float asum = 0.0f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = lane + 64 * q;
      pdf[q] = j < nw ? __fdiv_rn(cdf[j + 1], total) : 0.0f;
      const float a = fabsf(pdf[q]);
      ok = ok && (a == 0.0f || a >= 0x1p-28f);     // false for NaN
      asum += a;
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) asum += __shfl_xor(asum, off);
    ok = __all(ok) && asum < 1.5f;
    if (ok) {
      double carry = 0.0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (64 * q >= nw) break;                    // wave-uniform
        const int j = lane + 64 * q;
        double v = static_cast<double>(pdf[q]);
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
          const double t = __shfl_up(v, off);
          if (lane >= off) v += t;
        }
        v += carry;
        if (j < nw) cdf[j + 1] = static_cast<float>(v);
        carry = __shfl(v, 63);
      }
      if (lane == 0) cdf[0] = 0.0f;
    } else if (lane == 0) {
      double acc = 0.0;
      cdf[0] = 0.0f;
      for (int j = 1; j <= nw; ++j) {
        acc += static_cast<double>(__fdiv_rn(cdf[j], total));
        cdf[j] = static_cast<float>(acc);
      }
    }
  }
  __syncthreads();

  // invert the cdf (:92-113)
  for (int i = lane; i < nf; i += 64) {
    const float u = u_in ? u_in[r * u_stride + i] : linspace01(i, nf);
    int lo = 0, hi = ncdf;  // searchsorted(right=True): first j with cdf[j] > u
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (cdf[m] <= u) lo = m + 1; else hi = m;
    }
    const int below = lo - 1 > 0 ? lo - 1 : 0;
    const int above = lo < ncdf - 1 ? lo : ncdf - 1;
    const float c0 = cdf[below], c1 = cdf[above];
    float denom = __fsub_rn(c1, c0);
    if (denom < 1e-5f) denom = 1.0f;
    const float t = __fdiv_rn(__fsub_rn(u, c0), denom);
    const float b0 = mid[below], b1 = mid[above];
    val[nc + i] = __fadd_rn(b0, __fmul_rn(t, __fsub_rn(b1, b0)));
  }
  __syncthreads();
  if (!valid) return;                       // no barrier below
  float* zo = z_out + r * n;
  const float* o = pts_out ? ro + 3 * r : nullptr;
  const float* d = pts_out ? rd + 3 * r : nullptr;
  switch (n2) {
    case 64: sort_store<64>(val, n, lane, zo, pts_out ? pts_out + r * n * 3 : nullptr, o, d); break;
    case 128: sort_store<128>(val, n, lane, zo, pts_out ? pts_out + r * n * 3 : nullptr, o, d); break;
    case 256: sort_store<256>(val, n, lane, zo, pts_out ? pts_out + r * n * 3 : nullptr, o, d); break;
    default: sort_store<512>(val, n, lane, zo, pts_out ? pts_out + r * n * 3 : nullptr, o, d); break;
  }
}

}  // namespace

extern "C" int cn_sample_uniform(const float* ro, const float* rd, int64_t n_rays,
                                 const float* z_bins, const float* lower, const float* upper,
                                 int64_t nc, const float* t_rand, float* z_out, float* pts_out,
                                 cn_stream_t stream) {
  CN_CHECK_ARG(n_rays > 0 && nc > 0 && z_out);
  CN_CHECK_ARG(t_rand ? (lower && upper) : (z_bins != nullptr));
  CN_CHECK_ARG(!pts_out || (ro && rd));
  const int64_t n = n_rays * nc;
  auto al16 = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (nc % 4 == 0 && n / 4 < (int64_t(1) << 32) - 256 && al16(z_out) && al16(pts_out) &&
      (t_rand ? (al16(t_rand) && al16(lower) && al16(upper)) : al16(z_bins))) {
    const unsigned n4 = static_cast<unsigned>(n / 4);
    hipLaunchKernelGGL(sample_uniform4_kernel, dim3(static_cast<unsigned>(cn::ceil_div(n / 4, 256))), dim3(256), 0,
                       cn::as_stream(stream), ro, rd, n4, static_cast<unsigned>(nc / 4),
                       reinterpret_cast<const float4*>(z_bins), reinterpret_cast<const float4*>(lower),
                       reinterpret_cast<const float4*>(upper), reinterpret_cast<const float4*>(t_rand),
                       reinterpret_cast<float4*>(z_out), reinterpret_cast<float4*>(pts_out));
    return cn::launch_status();
  }
  hipLaunchKernelGGL(sample_uniform_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0,
                     cn::as_stream(stream), ro, rd, n_rays, z_bins, lower, upper, nc, t_rand,
                     z_out, pts_out);
  return cn::launch_status();
}

extern "C" int cn_sample_pdf(const float* ro, const float* rd, const float* weights,
                             int64_t w_stride, const float* z, int64_t n_rays, int64_t nc,
                             int64_t nf, const float* u, int64_t u_stride, float* z_out,
                             float* pts_out, cn_stream_t stream) {
  CN_CHECK_ARG(n_rays > 0 && nc >= 3 && nc <= 256 && nf > 0 && nc + nf <= kPdfMaxN);
  CN_CHECK_ARG(weights && z && z_out && w_stride >= nc - 2);
  CN_CHECK_ARG(!pts_out || (ro && rd));
  CN_CHECK_ARG(!u || u_stride == 0 || u_stride >= nf);
  const unsigned grid = static_cast<unsigned>(cn::ceil_div(n_rays, kPdfWaves));
  hipLaunchKernelGGL(sample_pdf_kernel, dim3(grid), dim3(64 * kPdfWaves), 0,
                     cn::as_stream(stream), ro, rd, weights, w_stride, z, n_rays,
                     static_cast<int>(nc), static_cast<int>(nf), u, u_stride, z_out, pts_out);
  return cn::launch_status();
}

extern "C" int cn_ray_points(const float* ro, const float* rd, const float* z, int64_t n_rays,
                             int64_t n_samples, float* pts, cn_stream_t stream) {
  CN_CHECK_ARG(ro && rd && z && pts && n_rays > 0 && n_samples > 0);
  const int64_t n = n_rays * n_samples * 3;
  hipLaunchKernelGGL(ray_points_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0,
                     cn::as_stream(stream), ro, rd, z, n_rays, n_samples, pts);
  return cn::launch_status();
}
