// Volume integration: volume_render (view_synthesis/nerf/volumetric_render.py:36-66).
//
// The exclusive prefix of sigma*delta -- transmittance = exp(-[0, cumsum(sigma*delta)[:-1]]) --
// is a scan over the lanes' run totals followed by the in-run prefix (layout below).
#include "cn_common.h"

namespace {

// L lanes per ray: 16 (one DPP row; 4 rays per wave, 16 per 256-thread block) for S <= 128, 64
// (the whole wave; 4 rays per block) above, so a lane's run stays <= 8 samples in registers at
// every S <= 512.  Lane i of a ray owns the contiguous run of samples [i run, (i + 1) run),
// run = ceil(S / L) <= K; its next sample's depth (z[j + 1] past the run) comes from lane i + 1 by
// DPP (a lane shuffle when L = 64) instead of a second load; the exclusive prefix of sigma*delta
// over the lanes' run totals is a 4-step DPP row scan (in double, as torch's CPU cumsum
// accumulates, Q13) plus, for L = 64, the earlier rows' totals read back as scalars; the per-ray
// sums are DPP row reductions (plus the row totals for L = 64) -- no LDS traffic in any
// cross-lane step.
// Algorithmic bytes per ray: 12 (rd) + 20*S in (raw + z), 4*S + 20 out.
constexpr int kMaxRun = 8;
constexpr int kMaxSamples = 64 * kMaxRun;  // 512

// Raw rows, depths and weights cross the kernel once: non-temporal 16-B loads and stores (streamed
// past the caches) -- the C2 launch 91 -> 86 us alone, 83 -> 74 us with the grouped launch (r04,
// tools/volume_timing.py, HIP-event medians).
typedef float nt_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 nt_load4(const float4* p) {
  const nt_f4 v = __builtin_nontemporal_load(reinterpret_cast<const nt_f4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nt_store4(float4 v, float4* p) {
  __builtin_nontemporal_store(nt_f4{v.x, v.y, v.z, v.w}, reinterpret_cast<nt_f4*>(p));
}

template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ double dppd(double x) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(v & 0xffffffff), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(v >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}
// Inclusive prefix over the 16 lanes of the row (row_shr: lane i reads lane i - n, 0 below the row).
__device__ __forceinline__ double row_inclusive_scan(double x) {
  x += dppd<0x111>(x);
  x += dppd<0x112>(x);
  x += dppd<0x114>(x);
  x += dppd<0x118>(x);
  return x;
}
// Inclusive suffix over the row (row_shl: lane i reads lane i + n, 0 past the row).
__device__ __forceinline__ float row_inclusive_suffix(float x) {
  x += dppf<0x101>(x);
  x += dppf<0x102>(x);
  x += dppf<0x104>(x);
  x += dppf<0x108>(x);
  return x;
}
// Sum over the row's 16 lanes, valid in lane 15.
__device__ __forceinline__ float row_sum(float x) {
  x += dppf<0x111>(x);
  x += dppf<0x112>(x);
  x += dppf<0x114>(x);
  x += dppf<0x118>(x);
  return x;
}

__device__ __forceinline__ float lanef(float x, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), l));
}
__device__ __forceinline__ double laned(double x, int l) {
  const long long v = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_readlane(static_cast<int>(v & 0xffffffff), l);
  const int hi = __builtin_amdgcn_readlane(static_cast<int>(v >> 32), l);
  return __longlong_as_double((static_cast<long long>(hi) << 32) | static_cast<unsigned>(lo));
}

// The ray-level cross-lane steps over its L lanes.  L = 16: the row steps.  L = 64 (one ray per
// wave): the row step, then the other rows' totals -- uniform, read back by readlane -- added in
// a fixed order.
template <int L>
__device__ __forceinline__ double ray_exclusive_scan(double v) {
  const double x = row_inclusive_scan(v);
  if constexpr (L == 16) {
    return x - v;
  } else {
    const int row = (threadIdx.x & 63) >> 4;
    const double t0 = laned(x, 15), t1 = laned(x, 31), t2 = laned(x, 47);
    double off = 0.0;
    if (row > 0) off += t0;
    if (row > 1) off += t1;
    if (row > 2) off += t2;
    return (x - v) + off;
  }
}
template <int L>
__device__ __forceinline__ float ray_exclusive_suffix(float v) {
  const float x = row_inclusive_suffix(v);
  if constexpr (L == 16) {
    return x - v;
  } else {  // row totals: the inclusive suffix in each row's lane 0
    const int row = (threadIdx.x & 63) >> 4;
    const float t1 = lanef(x, 16), t2 = lanef(x, 32), t3 = lanef(x, 48);
    float off = 0.0f;
    if (row < 3) off += t3;
    if (row < 2) off += t2;
    if (row < 1) off += t1;
    return (x - v) + off;
  }
}
// The ray's sum over its L lanes: valid in lane 15 of the row (L = 16) / every lane (L = 64).
template <int L>
__device__ __forceinline__ float ray_sum(float x) {
  x = row_sum(x);
  if constexpr (L == 64) x = ((lanef(x, 15) + lanef(x, 31)) + lanef(x, 47)) + lanef(x, 63);
  return x;
}
// ... valid in every lane of the ray.
template <int L>
__device__ __forceinline__ float ray_sum_all(float x) {
  if constexpr (L == 16) return __shfl(row_sum(x), (threadIdx.x & 63) | 15);
  else return ray_sum<64>(x);
}
// Lane + 1's value (the next run's first depth); 0 (L = 16) or the lane's own value (L = 64) past
// the ray's last lane, where it is never used.
template <int L>
__device__ __forceinline__ float next_lane(float x) {
  if constexpr (L == 16) return dppf<0x101>(x);
  else return __shfl_down(x, 1);
}

// Load this lane's run of depths (zero past S): 16-B vector loads when the run is a multiple of
// 4 aligned to 16 B (every S % 4 == 0 with run % 4 == 0: S = 64, 128 -- the C2 / C3 shapes),
// element loads otherwise.
template <int K>
__device__ __forceinline__ void load_depths(const float* zr, int j0, int run, int S_in, float (&zz)[K]) {
  if (K % 4 == 0 && run % 4 == 0 && (S_in & 3) == 0 && j0 + run <= S_in) {
#pragma unroll
    for (int q = 0; q < K / 4; ++q) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (4 * q < run) v = nt_load4(reinterpret_cast<const float4*>(zr + j0) + q);
      zz[4 * q] = v.x;
      zz[4 * q + 1] = v.y;
      zz[4 * q + 2] = v.z;
      zz[4 * q + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int i = 0; i < K; ++i) zz[i] = (i < run && j0 + i < S_in) ? zr[j0 + i] : 0.0f;
  }
}

template <int K>
__device__ __forceinline__ void load_run(const float* zr, const float4* rr, int j0, int run, int S_in, float (&zz)[K],
                                         float4 (&rv)[K]) {
  load_depths<K>(zr, j0, run, S_in, zz);
#pragma unroll
  for (int i = 0; i < K; ++i)
    rv[i] = (i < run && j0 + i < S_in) ? rr[j0 + i] : make_float4(0.f, 0.f, 0.f, 0.f);
}

// Raw rows through LDS: a lane's run of float4 samples is 16 run bytes apart from its
// neighbour's, so per-lane loads of it touch every cache line run times.  The wave's rays' rows
// (64 / L of them) are ONE contiguous (64 / L) S float4 block: lane l copies quads l + 64 t with
// coalesced 16-B loads into LDS slot pad(q) = q + q / 4 (a padding quad after every four: runs of
// four then sit 5 quads apart, conflict-free across a 16-lane group), and each lane then reads
// its own run from there.  The backward stores d raw back the same way.  <= 64 K quads per wave.
__device__ __forceinline__ int pad4(int q) { return q + (q >> 2); }


template <int K>
__device__ __forceinline__ void stage_rows_in(const float4* __restrict__ src, int nq, float4* sl, int lane) {
#pragma unroll
  for (int t = 0; t < K; ++t) {
    const int q = lane + 64 * t;
    if (q < nq) sl[pad4(q)] = nt_load4(src + q);
  }
}

template <int K>
__device__ __forceinline__ void stage_rows_out(float4* __restrict__ dst, int nq, const float4* sl, int lane) {
#pragma unroll
  for (int t = 0; t < K; ++t) {
    const int q = lane + 64 * t;
    if (q < nq) dst[q] = sl[pad4(q)];
  }
}

// This lane's run of raw rows from the wave's LDS copy (q0: the run's first quad in the wave block).
template <int K>
__device__ __forceinline__ void load_raw_lds(const float4* sl, int q0, int j0, int run, int S_in, float4 (&rv)[K]) {
#pragma unroll
  for (int i = 0; i < K; ++i) rv[i] = (i < run && j0 + i < S_in) ? sl[pad4(q0 + i)] : make_float4(0.f, 0.f, 0.f, 0.f);
}

// One lane's part of a ray (lane sub of its L): the run's depths zz and raw rows rv loaded, |rd| = nrm.
template <int K, bool FULL, int L>
__device__ __forceinline__ void render_run(const float (&zz)[K], const float4 (&rv)[K], int S_in, int64_t r, float nrm,
                                           float* __restrict__ rgb, float* __restrict__ disp, float* __restrict__ acc,
                                           float* __restrict__ weights, float* __restrict__ depth) {
  const int sub = threadIdx.x & (L - 1);
  // S == 1: the reference's dists = cat(z[1:] - z[:-1], full_like(that[..., :1], 1e10))
  // is EMPTY (both pieces are 0 wide), so no sample contributes (rgb = acc = depth = 0,
  // disp = NaN, weights (R, 0)).  Reproduced by treating the ray as sample-free.
  // FULL (S_in == 16 K: every lane's run is K samples): the run / bounds tests fold away
  const int S = FULL ? L * K : (S_in == 1 ? 0 : S_in);
  const int run = FULL ? K : (S_in + L - 1) / L;
  const int j0 = sub * run;
  float sd[K], wv[K];
  const float znext = next_lane<L>(zz[0]);  // the first depth of lane sub + 1's run
  double run_sum = 0.0;  // sum of this run's sigma*delta that feeds later transmittances
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int j = j0 + i;
    sd[i] = 0.0f;
    if (i < run && j < S) {
      // dists = [z[1:] - z[:-1], 1e10] (:41-44), delta = dists * |rd| (:45)
      const float zn = (i + 1 < run) ? zz[(i + 1) % K] : znext;
      const float dist = (j + 1 < S) ? __fsub_rn(zn, zz[i]) : 1e10f;
      const float sigma = cn::softplus20(__fsub_rn(rv[i].w, 1.0f));  // shifted_softplus (:32)
      sd[i] = __fmul_rn(sigma, __fmul_rn(dist, nrm));
      if (j + 1 < S) run_sum += static_cast<double>(sd[i]);
    }
  }
  double prefix = ray_exclusive_scan<L>(run_sum);

  float cr = 0.f, cg = 0.f, cb = 0.f, dep = 0.f, ac = 0.f;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int j = j0 + i;
    wv[i] = 0.0f;
    if (i < run && j < S) {
      const float trans = expf(-static_cast<float>(prefix));      // (:54-57)
      const float alpha = __fsub_rn(1.0f, expf(-sd[i]));           // (:58)
      const float w = __fmul_rn(alpha, trans);                     // (:59)
      // widened_sigmoid (:28): sigmoid(x) * 1.002 - 0.001
      const float c0 = __fsub_rn(__fmul_rn(cn::sigmoid_hw(rv[i].x), 1.002f), 0.001f);
      const float c1 = __fsub_rn(__fmul_rn(cn::sigmoid_hw(rv[i].y), 1.002f), 0.001f);
      const float c2 = __fsub_rn(__fmul_rn(cn::sigmoid_hw(rv[i].z), 1.002f), 0.001f);
      cr += w * c0;
      cg += w * c1;
      cb += w * c2;
      dep += w * zz[i];
      ac += w;
      wv[i] = w;
      if (j + 1 < S) prefix += static_cast<double>(sd[i]);
    }
  }
  if (weights) {  // this lane's run of weights: 16-B stores where the run is aligned (see load_depths)
    float* wr = weights + r * S_in;
    if (K % 4 == 0 && run % 4 == 0 && (S_in & 3) == 0 && j0 + run <= S_in && S > 0) {
#pragma unroll
      for (int q = 0; q < K / 4; ++q)
        if (4 * q < run)
          nt_store4(make_float4(wv[4 * q], wv[4 * q + 1], wv[4 * q + 2], wv[4 * q + 3]),
                                      reinterpret_cast<float4*>(wr + j0) + q);
    } else {
#pragma unroll
      for (int i = 0; i < K; ++i)
        if (i < run && j0 + i < S) wr[j0 + i] = wv[i];
    }
  }
  cr = ray_sum<L>(cr);
  cg = ray_sum<L>(cg);
  cb = ray_sum<L>(cb);
  dep = ray_sum<L>(dep);
  ac = ray_sum<L>(ac);
  if (sub == (L == 16 ? 15 : 63)) {
    rgb[3 * r] = cr;
    rgb[3 * r + 1] = cg;
    rgb[3 * r + 2] = cb;
    depth[r] = dep;
    acc[r] = ac;
    // (:63) torch.max propagates NaN: disp is NaN when acc == 0
    const float q = dep / ac;
    disp[r] = (q != q) ? q : 1.0f / fmaxf(1e-10f, q);
  }
}

template <int K, bool FULL, int L>
__global__ __launch_bounds__(256) void volume_render_kernel(
    const float* __restrict__ raw, const float* __restrict__ z, const float* __restrict__ rd,
    int64_t n_rays, int S_in, float* __restrict__ rgb, float* __restrict__ disp,
    float* __restrict__ acc, float* __restrict__ weights, float* __restrict__ depth) {
  static_assert(K <= kMaxRun && (L == 16 || L == 64) && (!FULL || L == 16), "instance");
  if (FULL) S_in = L * K;  // the host dispatches FULL only for S == 16 K: lets every bound fold
  __shared__ float4 slds[4 * 80 * K];  // per wave: <= 64 K quads, padded 5 / 4
  const int sub = threadIdx.x & (L - 1), lane = threadIdx.x & 63;
  const int64_t r = ((int64_t)blockIdx.x * 256 + threadIdx.x) / L;
  const int64_t rw0 = r - lane / L;  // the wave's first ray
  float4* sl = slds + (threadIdx.x >> 6) * 80 * K;
  if (rw0 < n_rays)
    stage_rows_in<K>(reinterpret_cast<const float4*>(raw) + rw0 * S_in,
                     static_cast<int>(min<int64_t>(64 / L, n_rays - rw0)) * S_in, sl, lane);
  // lanes read quads other lanes wrote: keep the staging stores ahead of the reads (no instruction;
  // LDS operations of one wave then execute in program order)
  __builtin_amdgcn_wave_barrier();
  if (r >= n_rays) return;  // whole rays leave together: the cross-lane steps never read an exited lane
  const int run = FULL ? K : (S_in + L - 1) / L;
  const int j0 = sub * run;
  const float* zr = z + r * S_in;
  const float d0 = rd[3 * r], d1 = rd[3 * r + 1], d2 = rd[3 * r + 2];
  const float nrm = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(d0, d0), __fmul_rn(d1, d1)), __fmul_rn(d2, d2)));
  float zz[K];
  float4 rv[K];
  load_depths<K>(zr, j0, run, S_in, zz);
  load_raw_lds<K>(sl, (lane / L) * S_in + j0, j0, run, S_in, rv);
  render_run<K, FULL, L>(zz, rv, S_in, r, nrm, rgb, disp, acc, weights, depth);
}

// S = 16 K with n_rays % 4 == 0 (dispatched for S = 64: the C2 / C3 / C5 coarse launches; at K = 8
// the staged rows would cost the occupancy): wave w renders G groups of 4 rays, groups
// w + g W of the grid's W waves.  Every group's raw rows, depths and directions are loaded up front,
// so the later groups' loads are in flight while the wave integrates the earlier ones.
template <int K, int G>
__global__ __launch_bounds__(256) void volume_render_groups_kernel(
    const float* __restrict__ raw, const float* __restrict__ z, const float* __restrict__ rd, int64_t n_rays,
    float* __restrict__ rgb, float* __restrict__ disp, float* __restrict__ acc, float* __restrict__ weights,
    float* __restrict__ depth) {
  constexpr int L = 16, S = L * K;
  __shared__ float4 slds[4 * 80 * K];
  const int lane = threadIdx.x & 63, sub = lane & 15;
  float4* sl = slds + (threadIdx.x >> 6) * 80 * K;
  const int64_t n_waves = (int64_t)gridDim.x * 4, wave = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  float4 stg[G][K];
  float zz[G][K], dv[G][3];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    // past the end: a copy of the last group (no branch around the loads, so the arrays stay in registers)
    const int64_t rw0 = min(4 * (wave + g * n_waves), n_rays - 4);
    const float4* src = reinterpret_cast<const float4*>(raw) + rw0 * S;
#pragma unroll
    for (int t = 0; t < K; ++t) stg[g][t] = nt_load4(src + lane + 64 * t);
    const int64_t r = rw0 + lane / L;
    float zl[K];
    load_depths<K>(z + r * S, sub * K, K, S, zl);
#pragma unroll
    for (int i = 0; i < K; ++i) zz[g][i] = zl[i];
#pragma unroll
    for (int d = 0; d < 3; ++d) dv[g][d] = rd[3 * r + d];
  }
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int64_t rw0 = 4 * (wave + g * n_waves);
    if (rw0 >= n_rays) continue;  // wave-uniform
#pragma unroll
    for (int t = 0; t < K; ++t) sl[pad4(lane + 64 * t)] = stg[g][t];
    __builtin_amdgcn_wave_barrier();
    float4 rv[K];
    load_raw_lds<K>(sl, (lane / L) * S + sub * K, sub * K, K, S, rv);
    __builtin_amdgcn_wave_barrier();
    float zg[K];
#pragma unroll
    for (int i = 0; i < K; ++i) zg[i] = zz[g][i];
    const float nrm = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(dv[g][0], dv[g][0]), __fmul_rn(dv[g][1], dv[g][1])),
                                           __fmul_rn(dv[g][2], dv[g][2])));
    render_run<K, true, L>(zg, rv, S, rw0 + lane / L, nrm, rgb, disp, acc, weights, depth);
  }
}

}  // namespace

// Instances: S = 64 / 128 (every C2-C5 coarse / merged shape) take the FULL 16-lane ones; other
// S <= 128 the 16-lane ones with run <= 4 / 8; S <= 512 (the 32 + 160 and 64 + 128 merged
// shapes: S = 192) the 64-lane ones with run <= 4 / 8.
#define CN_VOLUME_DISPATCH(KERNEL, S, N, STREAM, ...)                                                      \
  do {                                                                                                      \
    const dim3 g16(static_cast<unsigned>(cn::ceil_div((N), 16))), g64(static_cast<unsigned>(cn::ceil_div((N), 4))); \
    if ((S) == 64) hipLaunchKernelGGL((KERNEL<4, true, 16>), g16, dim3(256), 0, STREAM, __VA_ARGS__);      \
    else if ((S) == 128) hipLaunchKernelGGL((KERNEL<8, true, 16>), g16, dim3(256), 0, STREAM, __VA_ARGS__); \
    else if ((S) <= 64) hipLaunchKernelGGL((KERNEL<4, false, 16>), g16, dim3(256), 0, STREAM, __VA_ARGS__); \
    else if ((S) <= 128) hipLaunchKernelGGL((KERNEL<8, false, 16>), g16, dim3(256), 0, STREAM, __VA_ARGS__); \
    else if ((S) <= 256) hipLaunchKernelGGL((KERNEL<4, false, 64>), g64, dim3(256), 0, STREAM, __VA_ARGS__); \
    else hipLaunchKernelGGL((KERNEL<8, false, 64>), g64, dim3(256), 0, STREAM, __VA_ARGS__);                \
  } while (0)

extern "C" int cn_volume_render(const float* raw, const float* z, const float* rd, int64_t n_rays,
                                int64_t n_samples, float* rgb, float* disp, float* acc,
                                float* weights, float* depth, cn_stream_t stream) {
  CN_CHECK_ARG(raw && z && rd && rgb && disp && acc && depth);
  CN_CHECK_ARG(n_rays > 0 && n_samples > 0 && n_samples <= kMaxSamples);
  CN_CHECK_ARG(cn::aligned16(raw) && cn::aligned16(z) && cn::aligned16(weights));
  if (n_samples == 64 && n_rays % 4 == 0) {  // C2 / C5 coarse: two ray groups per wave
    constexpr int G = 2;
    const int64_t waves = cn::ceil_div(n_rays / 4, G);
    hipLaunchKernelGGL((volume_render_groups_kernel<4, G>), dim3(static_cast<unsigned>(cn::ceil_div(waves, 4))),
                       dim3(256), 0, cn::as_stream(stream), raw, z, rd, n_rays, rgb, disp, acc, weights, depth);
    return cn::launch_status();
  }
  CN_VOLUME_DISPATCH(volume_render_kernel, n_samples, n_rays, cn::as_stream(stream), raw, z, rd, n_rays,
                     static_cast<int>(n_samples), rgb, disp, acc, weights, depth);
  return cn::launch_status();
}

// ---------------------------------------------------------------- backward
// Gradient of volume_render (volumetric_render.py:36-66) w.r.t. raw and rd.
// With sd_i = sigma_i delta_i, T_i = exp(-sum_{j<i} sd_j), w_i = (1 - e^{-sd_i}) T_i:
//   G_i = g_w_i + g_rgb . c_i + g_depth z_i + g_acc          (dL/dw_i)
//   dL/dsd_i = G_i T_i e^{-sd_i} - sum_{j>i} G_j w_j          (reverse ray scan)
//   d raw_i[0:3] = w_i g_rgb 1.002 s(1-s);  d raw_i[3] = dL/dsd_i delta_i softplus'(raw_i[3]-1)
//   d rd = (sum_i dL/dsd_i sigma_i dist_i) rd/|rd|
// g_disp folds into g_depth / g_acc through disp = 1/max(1e-10, depth/acc).
// z is never differentiated (the reference detaches its samples).  Same layout as the forward.
namespace {

template <int K, bool FULL, int L>
__global__ __launch_bounds__(256) void volume_render_backward_kernel(
    const float* __restrict__ raw, const float* __restrict__ z, const float* __restrict__ rd,
    int64_t n_rays, int S_in, const float* __restrict__ g_rgb, const float* __restrict__ g_disp,
    const float* __restrict__ g_acc, const float* __restrict__ g_w, const float* __restrict__ g_depth,
    float* __restrict__ d_raw, float* __restrict__ d_rd, int accumulate_rd) {
  static_assert(K <= kMaxRun && (L == 16 || L == 64) && (!FULL || L == 16), "instance");
  if (FULL) S_in = L * K;  // as in the forward
  __shared__ float4 slds[4 * 80 * K];  // per wave: raw in, then d raw out (forward's layout)
  const int sub = threadIdx.x & (L - 1), lane = threadIdx.x & 63;
  const int64_t r_ = ((int64_t)blockIdx.x * 256 + threadIdx.x) / L;
  const int64_t rw0 = r_ - lane / L;
  if (rw0 >= n_rays) return;  // the whole wave
  const int nq = static_cast<int>(min<int64_t>(64 / L, n_rays - rw0)) * S_in;  // the wave's valid quads
  float4* sl = slds + (threadIdx.x >> 6) * 80 * K;
  stage_rows_in<K>(reinterpret_cast<const float4*>(raw) + rw0 * S_in, nq, sl, lane);
  __builtin_amdgcn_wave_barrier();  // cross-lane LDS reads follow (see the forward)
  // a ray past n_rays (L = 16 only) stays alive as a copy of the last ray, nothing stored, so the
  // wave's coalesced d raw copy-out runs in every lane
  const bool live = r_ < n_rays;
  const int64_t r = live ? r_ : n_rays - 1;
  const int S = FULL ? L * K : (S_in == 1 ? 0 : S_in);  // see the forward: S == 1 has no contributing sample
  const int run = FULL ? K : (S_in + L - 1) / L;
  const int j0 = sub * run;
  const float* zr = z + r * S_in;
  const float4* rr = reinterpret_cast<const float4*>(raw) + r * S_in;
  const float d0 = rd[3 * r], d1 = rd[3 * r + 1], d2 = rd[3 * r + 2];
  const float nrm = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(d0, d0), __fmul_rn(d1, d1)), __fmul_rn(d2, d2)));

  float sd[K], zz[K], dist[K], sig[K], w[K], tr[K];
  float4 rv[K];
  const int q0 = (lane / L) * S_in + j0;  // this run's first quad in the wave block
  load_depths<K>(zr, j0, run, S_in, zz);
  if (live) load_raw_lds<K>(sl, q0, j0, run, S_in, rv);
  else load_run<K>(zr, rr, j0, run, S_in, zz, rv);  // the last ray again (not in this wave's block)
  const float znext = next_lane<L>(zz[0]);
  double run_sum = 0.0;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int j = j0 + i;
    sd[i] = 0.0f;
    dist[i] = 0.0f;
    sig[i] = 0.0f;
    if (i < run && j < S) {
      const float zn = (i + 1 < run) ? zz[(i + 1) % K] : znext;
      dist[i] = (j + 1 < S) ? __fsub_rn(zn, zz[i]) : 1e10f;
      sig[i] = cn::softplus20(__fsub_rn(rv[i].w, 1.0f));
      sd[i] = __fmul_rn(sig[i], __fmul_rn(dist[i], nrm));
      if (j + 1 < S) run_sum += static_cast<double>(sd[i]);
    }
  }
  double prefix = ray_exclusive_scan<L>(run_sum);
  float dep = 0.f, ac = 0.f;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int j = j0 + i;
    w[i] = 0.0f;
    tr[i] = 0.0f;
    if (i < run && j < S) {
      tr[i] = expf(-static_cast<float>(prefix));
      w[i] = __fmul_rn(__fsub_rn(1.0f, expf(-sd[i])), tr[i]);
      dep += w[i] * zz[i];
      ac += w[i];
      if (j + 1 < S) prefix += static_cast<double>(sd[i]);
    }
  }
  // the ray's depth / acc in every lane of the ray
  dep = ray_sum_all<L>(dep);
  ac = ray_sum_all<L>(ac);
  const float gr0 = g_rgb ? g_rgb[3 * r] : 0.f, gr1 = g_rgb ? g_rgb[3 * r + 1] : 0.f;
  const float gr2 = g_rgb ? g_rgb[3 * r + 2] : 0.f;
  float gdep = g_depth ? g_depth[r] : 0.f, gacc = g_acc ? g_acc[r] : 0.f;
  if (g_disp) {
    const float q = dep / ac;
    if (q > 1e-10f) {  // d(1/q)/dq = -1/q^2; below the clamp torch routes the gradient to the constant
      const float gq = -g_disp[r] / (q * q);
      gdep += gq / ac;
      gacc += gq * (-dep / (ac * ac));
    }
  }
  // G_i and the per-sample colour gradients
  float G[K], gw_run = 0.f;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const int j = j0 + i;
    G[i] = 0.0f;
    if (i < run && j < S) {
      const float s0 = cn::sigmoid_hw(rv[i].x), s1 = cn::sigmoid_hw(rv[i].y), s2 = cn::sigmoid_hw(rv[i].z);
      const float c0 = s0 * 1.002f - 0.001f, c1 = s1 * 1.002f - 0.001f, c2 = s2 * 1.002f - 0.001f;
      G[i] = gr0 * c0 + gr1 * c1 + gr2 * c2 + gdep * zz[i] + gacc + (g_w ? g_w[r * S_in + j] : 0.f);
      rv[i].x = w[i] * gr0 * 1.002f * s0 * (1.0f - s0);  // reuse rv for d_raw[0:3]
      rv[i].y = w[i] * gr1 * 1.002f * s1 * (1.0f - s1);
      rv[i].z = w[i] * gr2 * 1.002f * s2 * (1.0f - s2);
      gw_run += G[i] * w[i];
    }
  }
  float suffix = ray_exclusive_suffix<L>(gw_run);  // sum of G_j w_j over later lanes' runs
  float gnorm = 0.f;
#pragma unroll
  for (int i = K - 1; i >= 0; --i) {
    const int j = j0 + i;
    if (i < run && j < S) {
      const float dsd = G[i] * tr[i] * expf(-sd[i]) - suffix;
      suffix += G[i] * w[i];
      const float x = rv[i].w - 1.0f;
      const float dsp = x > 20.0f ? 1.0f : cn::sigmoid_hw(x);
      float4 o = rv[i];
      o.w = dsd * (dist[i] * nrm) * dsp;
      if (live) sl[pad4(q0 + i)] = o;
      gnorm += dsd * sig[i] * dist[i];
    } else if (i < run && j < S_in) {
      if (live) sl[pad4(q0 + i)] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __builtin_amdgcn_wave_barrier();  // the copy-out reads quads other lanes wrote
  stage_rows_out<K>(reinterpret_cast<float4*>(d_raw) + rw0 * S_in, nq, sl, lane);
  gnorm = ray_sum<L>(gnorm);
  if (live && sub == (L == 16 ? 15 : 63) && d_rd) {
    const float inv = nrm > 0.f ? gnorm / nrm : 0.f;
    if (accumulate_rd) {      // one writer per ray: the caller's running sum of the ray's gradients
      d_rd[3 * r] += inv * d0;
      d_rd[3 * r + 1] += inv * d1;
      d_rd[3 * r + 2] += inv * d2;
    } else {
      d_rd[3 * r] = inv * d0;
      d_rd[3 * r + 1] = inv * d1;
      d_rd[3 * r + 2] = inv * d2;
    }
  }
}

}  // namespace

extern "C" int cn_volume_render_backward(const float* raw, const float* z, const float* rd,
                                         int64_t n_rays, int64_t n_samples, const float* g_rgb,
                                         const float* g_disp, const float* g_acc,
                                         const float* g_weights, const float* g_depth,
                                         float* d_raw, float* d_rd, int accumulate_rd, cn_stream_t stream) {
  CN_CHECK_ARG(raw && z && rd && d_raw && (accumulate_rd == 0 || accumulate_rd == 1));
  CN_CHECK_ARG(n_rays > 0 && n_samples > 0 && n_samples <= kMaxSamples);
  CN_CHECK_ARG(cn::aligned16(raw) && cn::aligned16(z) && cn::aligned16(d_raw));
  CN_VOLUME_DISPATCH(volume_render_backward_kernel, n_samples, n_rays, cn::as_stream(stream), raw, z, rd, n_rays,
                     static_cast<int>(n_samples), g_rgb, g_disp, g_acc, g_weights, g_depth, d_raw, d_rd,
                     accumulate_rd);
  return cn::launch_status();
}
