// The pose path of the eval step, fused:
//   eval.py:22-38      pose_spherical(theta, phi, rho) -> c2w
//   ray_sampler.py:53-99  RaySampler.sample: permutation prefix per image, get_bundle, gather
//   eval.py:147-148    target_pixels[..., select_inds, :]
//   eval.py:161-162    pose_error = || SE3.Log(inverse(gt) @ cam) ||  (utils/lieutils.py:453-718)
//
// The reference builds a 4x4 pose from ~20 scalar torch ops, rotates ALL H*W directions,
// then gathers S of them, and differentiates that graph back to (theta, phi, rho) with
// autograd.  Here one launch computes the pose and only the S selected rays (and their
// target pixels); one launch per pose reduces the ray gradients and applies the analytic
// d c2w / d(theta, phi, rho).  The selection is the host numpy permutation (parity mode,
// same RNG calls as the reference) or an on-device Philox draw (cn_random_select).
#include <math.h>

#include "cn_common.h"

namespace {

// eval.py:33-37, each product rounded in the reference's order (left to right).
__device__ __forceinline__ void spherical_pose(float th, float ph, float rho, float* T) {
  const float st = sinf(th), ct = cosf(th), sp = sinf(ph), cp = cosf(ph);
  T[0] = -sp;                T[1] = __fmul_rn(-st, cp); T[2] = __fmul_rn(ct, cp);
  T[3] = __fmul_rn(__fmul_rn(rho, ct), cp);
  T[4] = cp;                 T[5] = __fmul_rn(-st, sp); T[6] = __fmul_rn(ct, sp);
  T[7] = __fmul_rn(__fmul_rn(rho, ct), sp);
  T[8] = 0.0f;               T[9] = ct;                 T[10] = st;
  T[11] = __fmul_rn(rho, st);
  T[12] = 0.0f; T[13] = 0.0f; T[14] = 0.0f; T[15] = 1.0f;
}

// One thread per selected ray: q = b * s + i -> pixel p = sel[q] (or i when sel is NULL:
// the whole bundle, get_bundle).  rd_j = d0 R[j][0] + d1 R[j][1] + d2 R[j][2] in the order
// of cn_ray_bundle (ray_sampler.py:95-98); ro = t; target row gathered with the ray.
__global__ __launch_bounds__(256) void pose_rays_kernel(const float* __restrict__ th_, const float* __restrict__ ph_,
                                                        const float* __restrict__ rho_, const float* __restrict__ c2w_in,
                                                        int64_t batch, const float* __restrict__ dirs, int64_t hw,
                                                        const int64_t* __restrict__ sel, int64_t s,
                                                        const float* __restrict__ target, int64_t ch,
                                                        float* __restrict__ c2w_out, float* __restrict__ ro,
                                                        float* __restrict__ rd, float* __restrict__ tgt_out) {
  const int64_t n = batch * s;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = q / s, i = q - b * s;
    float T[16];
    if (th_) {
      spherical_pose(th_[b], ph_[b], rho_[b], T);
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) T[k] = c2w_in[16 * b + k];
    }
    if (c2w_out && i == 0) {
#pragma unroll
      for (int k = 0; k < 16; ++k) c2w_out[16 * b + k] = T[k];
    }
    const int64_t p = sel ? sel[q] : i;
    const bool ok = p >= 0 && p < hw;
    const int64_t pc = ok ? p : 0;
    const float d0 = dirs[3 * pc], d1 = dirs[3 * pc + 1], d2 = dirs[3 * pc + 2];
    const float nan = __int_as_float(0x7fc00000);
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      float acc = __fmul_rn(d0, T[4 * j + 0]);
      acc = __fadd_rn(acc, __fmul_rn(d1, T[4 * j + 1]));
      acc = __fadd_rn(acc, __fmul_rn(d2, T[4 * j + 2]));
      rd[3 * q + j] = ok ? acc : nan;
      ro[3 * q + j] = ok ? T[4 * j + 3] : nan;
    }
    if (target && tgt_out) {
      const float* src = target + (b * hw + pc) * ch;
      for (int64_t c = 0; c < ch; ++c) tgt_out[q * ch + c] = ok ? src[c] : nan;
    }
  }
}

// One block per pose: G[j][k] = sum_i g_rd[i][j] d[i][k], g_t[j] = sum_i g_ro[i][j] over the
// pose's s rays (the gradient the reference's autograd scatters into the (H, W, 3) bundle and
// contracts in the einsum backward), then the chain rule through eval.py:33-37:
//   d/dtheta: R01 -ct cp, R11 -ct sp, R21 -st, R02 -st cp, R12 -st sp, R22 ct,
//             t0 -rho st cp, t1 -rho st sp, t2 rho ct
//   d/dphi:   R00 -cp, R10 -sp, R01 st sp, R11 -st cp, R02 -ct sp, R12 ct cp,
//             t0 -rho ct sp, t1 rho ct cp
//   d/drho:   t0 ct cp, t1 ct sp, t2 st
// 1024 threads per pose: two rays per thread for the eval step's 2048, every load of a thread's rays
// issued before its FMAs (the index, then the direction gather: two memory round trips in all; the
// 256-thread loop took two per ray, 10.4 us per call).
constexpr int kPoseBwdThreads = 1024;
__global__ __launch_bounds__(kPoseBwdThreads) void pose_rays_backward_kernel(const float* __restrict__ th_,
                                                                 const float* __restrict__ ph_,
                                                                 const float* __restrict__ rho_,
                                                                 const float* __restrict__ dirs, int64_t hw,
                                                                 const int64_t* __restrict__ sel, int64_t s,
                                                                 const float* __restrict__ g_ro,
                                                                 const float* __restrict__ g_rd,
                                                                 float* __restrict__ d_c2w, float* __restrict__ d_th,
                                                                 float* __restrict__ d_ph, float* __restrict__ d_rho) {
  constexpr int kW = kPoseBwdThreads / 64;
  __shared__ float red[12][kW];
  const int64_t b = blockIdx.x;
  float acc[12] = {0};
  constexpr int kU = 2;   // rays per thread and round, loaded together
  for (int64_t i0 = threadIdx.x; i0 < s; i0 += kU * kPoseBwdThreads) {
    int64_t p[kU];
    bool ok[kU];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t i = i0 + u * kPoseBwdThreads;
      ok[u] = i < s;
      p[u] = ok[u] ? (sel ? sel[b * s + i] : i) : 0;
      ok[u] = ok[u] && p[u] >= 0 && p[u] < hw;
    }
    float d[kU][3], gr[kU][3], go[kU][3];
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      const int64_t q = b * s + i0 + u * kPoseBwdThreads, pp = ok[u] ? p[u] : 0;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        d[u][j] = dirs[3 * pp + j];
        gr[u][j] = (ok[u] && g_rd) ? g_rd[3 * q + j] : 0.0f;
        go[u][j] = (ok[u] && g_ro) ? g_ro[3 * q + j] : 0.0f;
      }
    }
#pragma unroll
    for (int u = 0; u < kU; ++u) {
      if (!ok[u]) continue;
#pragma unroll
      for (int j = 0; j < 3; ++j) {
        acc[4 * j + 0] = fmaf(gr[u][j], d[u][0], acc[4 * j + 0]);
        acc[4 * j + 1] = fmaf(gr[u][j], d[u][1], acc[4 * j + 1]);
        acc[4 * j + 2] = fmaf(gr[u][j], d[u][2], acc[4 * j + 2]);
        acc[4 * j + 3] += go[u][j];
      }
    }
  }
  // wave butterfly, then the waves through LDS (a fixed pairwise tree)
#pragma unroll
  for (int k = 0; k < 12; ++k) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) acc[k] += __shfl_xor(acc[k], o);
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 12; ++k) red[k][wave] = acc[k];
  __syncthreads();
  if (threadIdx.x != 0) return;
  float G[12];
#pragma unroll
  for (int k = 0; k < 12; ++k) {
    float t[kW];
#pragma unroll
    for (int w = 0; w < kW; ++w) t[w] = red[k][w];
#pragma unroll
    for (int n = kW / 2; n > 0; n >>= 1)
#pragma unroll
      for (int w = 0; w < n; ++w) t[w] = t[w] + t[w + n];
    G[k] = t[0];
  }
  if (d_c2w) {
#pragma unroll
    for (int k = 0; k < 12; ++k) d_c2w[16 * b + k] = G[k];
#pragma unroll
    for (int k = 12; k < 16; ++k) d_c2w[16 * b + k] = 0.0f;
  }
  if (th_) {
    const float th = th_[b], ph = ph_[b], rho = rho_[b];
    const float st = sinf(th), ct = cosf(th), sp = sinf(ph), cp = cosf(ph);
    // G index: row j, column k -> 4 j + k (k = 3: translation)
    const float dth = G[1] * (-ct * cp) + G[5] * (-ct * sp) + G[9] * (-st) + G[2] * (-st * cp) + G[6] * (-st * sp) +
                      G[10] * ct + G[3] * (-rho * st * cp) + G[7] * (-rho * st * sp) + G[11] * (rho * ct);
    const float dph = G[0] * (-cp) + G[4] * (-sp) + G[1] * (st * sp) + G[5] * (-st * cp) + G[2] * (-ct * sp) +
                      G[6] * (ct * cp) + G[3] * (-rho * ct * sp) + G[7] * (rho * ct * cp);
    const float drho = G[3] * (ct * cp) + G[7] * (ct * sp) + G[11] * st;
    if (d_th) d_th[b] = dth;
    if (d_ph) d_ph[b] = dph;
    if (d_rho) d_rho[b] = drho;
  }
}

// ---------------------------------------------------------------- device selection
// Philox4x32-10 (Salmon et al., SC'11): counter (i, b, offset_lo, offset_hi), key = seed.
__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 k) {
  constexpr uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u, W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = M0 * c.x, hi0 = __umulhi(M0, c.x);
    const uint32_t lo1 = M1 * c.z, hi1 = __umulhi(M1, c.z);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += W0;
    k.y += W1;
  }
  return c;
}

constexpr int kSelThreads = 1024;
constexpr int kSelMax = 16384;  // pixels per image: 128 KiB of 64-bit keys in LDS

// np.random.permutation(hw)[:s] in distribution (ray_sampler.py:41-42): every pixel draws a
// 50-bit Philox key (low 14 bits = its index, so keys are distinct), one workgroup
// bitonic-sorts the image's keys in LDS, and the s smallest -- a uniformly random ordered
// s-subset -- are the selection.  One workgroup per image.
__global__ __launch_bounds__(kSelThreads) void random_select_kernel(int64_t hw, int64_t s, uint64_t seed,
                                                                    uint64_t offset, int n_pad,
                                                                    int64_t* __restrict__ sel) {
  __shared__ uint64_t keys[kSelMax];
  const uint32_t b = blockIdx.x;
  const uint2 k = make_uint2(static_cast<uint32_t>(seed), static_cast<uint32_t>(seed >> 32));
  for (int i = threadIdx.x; i < n_pad; i += kSelThreads) {
    uint64_t key = ~0ull;
    if (i < hw) {
      const uint4 r = philox4x32(make_uint4(static_cast<uint32_t>(i), b, static_cast<uint32_t>(offset),
                                            static_cast<uint32_t>(offset >> 32)), k);
      key = ((static_cast<uint64_t>(r.x) << 32 | r.y) & ~0x3FFFull) | static_cast<uint64_t>(i);
    }
    keys[i] = key;
  }
  __syncthreads();
  const int half = n_pad >> 1;
  for (int kk = 2; kk <= n_pad; kk <<= 1) {
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < half; t += kSelThreads) {
        const int lo = 2 * t - (t & (j - 1));
        const int hi = lo + j;
        const bool up = (lo & kk) == 0;
        const uint64_t x = keys[lo], y = keys[hi];
        if ((x > y) == up) {
          keys[lo] = y;
          keys[hi] = x;
        }
      }
      __syncthreads();
    }
  }
  for (int64_t i = threadIdx.x; i < s; i += kSelThreads)
    sel[static_cast<int64_t>(b) * s + i] = static_cast<int64_t>(keys[i] & 0x3FFFull);
}

// ---------------------------------------------------------------- SE3 pose error
// utils/lieutils.py:41-81 (coeff_A: sin t / t with the Taylor branch below 1e-3)
__device__ __forceinline__ float sin_by_t(float t) {
  if (fabsf(t) < 1e-3f) {
    const float t2 = t * t;
    return 1.0f - t2 / 6.0f * (1.0f - t2 / 20.0f * (1.0f - t2 / 42.0f));
  }
  return sinf(t) / t;
}

// eval.py:161-162: g = inverse(gt) @ cam; twist = SE3.Log(g) (lieutils.py:709-718:
// w = SO3.Log(R) :528-566, v = inv_vecs_Xg_ig(w) p :568-582); err = ||twist||_2.
// One thread per pose.  The inverse is a general 4x4 inverse (torch.inverse) in double.
// SO3.Log's quirks are kept: (tr - 1) / 2 > 1 gives acos = NaN, neither branch applies and
// w = 0.  Its |sin t / t| <= 1e-7 branch (t near pi) raises NameError in the reference
// ("torh.sign", lieutils.py:553); here it computes what that branch intends.
__global__ void pose_error_kernel(const float* __restrict__ gt, const float* __restrict__ cam, int64_t batch,
                                  float* __restrict__ twist, float* __restrict__ err) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= batch) return;
  double m[16], inv[16];
  for (int k = 0; k < 16; ++k) m[k] = gt[16 * b + k];
  // adjugate / determinant
  inv[0] = m[5] * m[10] * m[15] - m[5] * m[11] * m[14] - m[9] * m[6] * m[15] + m[9] * m[7] * m[14] +
           m[13] * m[6] * m[11] - m[13] * m[7] * m[10];
  inv[4] = -m[4] * m[10] * m[15] + m[4] * m[11] * m[14] + m[8] * m[6] * m[15] - m[8] * m[7] * m[14] -
           m[12] * m[6] * m[11] + m[12] * m[7] * m[10];
  inv[8] = m[4] * m[9] * m[15] - m[4] * m[11] * m[13] - m[8] * m[5] * m[15] + m[8] * m[7] * m[13] +
           m[12] * m[5] * m[11] - m[12] * m[7] * m[9];
  inv[12] = -m[4] * m[9] * m[14] + m[4] * m[10] * m[13] + m[8] * m[5] * m[14] - m[8] * m[6] * m[13] -
            m[12] * m[5] * m[10] + m[12] * m[6] * m[9];
  inv[1] = -m[1] * m[10] * m[15] + m[1] * m[11] * m[14] + m[9] * m[2] * m[15] - m[9] * m[3] * m[14] -
           m[13] * m[2] * m[11] + m[13] * m[3] * m[10];
  inv[5] = m[0] * m[10] * m[15] - m[0] * m[11] * m[14] - m[8] * m[2] * m[15] + m[8] * m[3] * m[14] +
           m[12] * m[2] * m[11] - m[12] * m[3] * m[10];
  inv[9] = -m[0] * m[9] * m[15] + m[0] * m[11] * m[13] + m[8] * m[1] * m[15] - m[8] * m[3] * m[13] -
           m[12] * m[1] * m[11] + m[12] * m[3] * m[9];
  inv[13] = m[0] * m[9] * m[14] - m[0] * m[10] * m[13] - m[8] * m[1] * m[14] + m[8] * m[2] * m[13] +
            m[12] * m[1] * m[10] - m[12] * m[2] * m[9];
  inv[2] = m[1] * m[6] * m[15] - m[1] * m[7] * m[14] - m[5] * m[2] * m[15] + m[5] * m[3] * m[14] +
           m[13] * m[2] * m[7] - m[13] * m[3] * m[6];
  inv[6] = -m[0] * m[6] * m[15] + m[0] * m[7] * m[14] + m[4] * m[2] * m[15] - m[4] * m[3] * m[14] -
           m[12] * m[2] * m[7] + m[12] * m[3] * m[6];
  inv[10] = m[0] * m[5] * m[15] - m[0] * m[7] * m[13] - m[4] * m[1] * m[15] + m[4] * m[3] * m[13] +
            m[12] * m[1] * m[7] - m[12] * m[3] * m[5];
  inv[14] = -m[0] * m[5] * m[14] + m[0] * m[6] * m[13] + m[4] * m[1] * m[14] - m[4] * m[2] * m[13] -
            m[12] * m[1] * m[6] + m[12] * m[2] * m[5];
  inv[3] = -m[1] * m[6] * m[11] + m[1] * m[7] * m[10] + m[5] * m[2] * m[11] - m[5] * m[3] * m[10] -
           m[9] * m[2] * m[7] + m[9] * m[3] * m[6];
  inv[7] = m[0] * m[6] * m[11] - m[0] * m[7] * m[10] - m[4] * m[2] * m[11] + m[4] * m[3] * m[10] +
           m[8] * m[2] * m[7] - m[8] * m[3] * m[6];
  inv[11] = -m[0] * m[5] * m[11] + m[0] * m[7] * m[9] + m[4] * m[1] * m[11] - m[4] * m[3] * m[9] -
            m[8] * m[1] * m[7] + m[8] * m[3] * m[5];
  inv[15] = m[0] * m[5] * m[10] - m[0] * m[6] * m[9] - m[4] * m[1] * m[10] + m[4] * m[2] * m[9] +
            m[8] * m[1] * m[6] - m[8] * m[2] * m[5];
  const double det = m[0] * inv[0] + m[1] * inv[4] + m[2] * inv[8] + m[3] * inv[12];
  float g[12];  // rows 0..2 of inverse(gt) @ cam, rounded to fp32 as torch.matmul's output
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 4; ++c) {
      double acc = 0.0;
      for (int k = 0; k < 4; ++k) acc += (inv[4 * r + k] / det) * static_cast<double>(cam[16 * b + 4 * k + c]);
      g[4 * r + c] = static_cast<float>(acc);
    }
  // SO3.Log (lieutils.py:528-566)
  const float tr = (g[0] + g[5]) + g[10];
  const float cth = (tr - 1.0f) / 2.0f;
  const float t = acosf(cth);
  const float sc = sin_by_t(t);
  float w0 = 0.0f, w1 = 0.0f, w2 = 0.0f;
  if (fabsf(sc) > 1e-7f) {
    w0 = (g[9] - g[6]) / (2.0f * sc);   // X[2][1]
    w1 = (g[2] - g[8]) / (2.0f * sc);   // X[0][2]
    w2 = (g[4] - g[1]) / (2.0f * sc);   // X[1][0]
  } else if (fabsf(sc) <= 1e-7f) {
    const float t2 = t * t;
    const float a00 = (g[0] + 1.0f) * t2 / 2.0f, a11 = (g[5] + 1.0f) * t2 / 2.0f, a22 = (g[10] + 1.0f) * t2 / 2.0f;
    const float a02 = g[2] * t2 / 2.0f, a12 = g[6] * t2 / 2.0f;
    float s3 = a02 > 0.0f ? 1.0f : (a02 < 0.0f ? -1.0f : 1.0f);
    float s23 = a12 > 0.0f ? 1.0f : (a12 < 0.0f ? -1.0f : 1.0f);
    w0 = sqrtf(a00);
    w1 = sqrtf(a11) * (s23 * s3);
    w2 = sqrtf(a22) * s3;
  }
  // inv_vecs_Xg_ig (lieutils.py:568-582): H = I - X/2 + eta X^2
  const float tw = sqrtf(w0 * w0 + w1 * w1 + w2 * w2);
  float eta;
  if (fabsf(tw) < 1e-3f) {
    const float t2 = tw * tw;
    eta = ((t2 / 40.0f + 1.0f) * t2 / 42.0f + 1.0f) * t2 / 720.0f + 1.0f / 12.0f;
  } else {
    eta = (1.0f - (tw / 2.0f) / tanf(tw / 2.0f)) / (tw * tw);
  }
  const float X[9] = {0.0f, -w2, w1, w2, 0.0f, -w0, -w1, w0, 0.0f};
  float H[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) {
      float x2 = 0.0f;
      for (int k = 0; k < 3; ++k) x2 += X[3 * r + k] * X[3 * k + c];
      H[3 * r + c] = (r == c ? 1.0f : 0.0f) - 0.5f * X[3 * r + c] + eta * x2;
    }
  float v[3];
  for (int r = 0; r < 3; ++r) v[r] = H[3 * r] * g[3] + H[3 * r + 1] * g[7] + H[3 * r + 2] * g[11];
  const float x[6] = {w0, w1, w2, v[0], v[1], v[2]};
  float ss = 0.0f;
  for (int k = 0; k < 6; ++k) {
    if (twist) twist[6 * b + k] = x[k];
    ss += x[k] * x[k];
  }
  if (err) err[b] = sqrtf(ss);
}

}  // namespace

extern "C" int cn_pose_rays(const float* theta, const float* phi, const float* rho, const float* c2w, int64_t batch,
                            const float* dirs,
                            int64_t hw, const int64_t* select_inds, int64_t sample_size, const float* target,
                            int64_t target_channels, float* c2w_out, float* ro, float* rd, float* target_out,
                            cn_stream_t stream) {
  CN_CHECK_ARG(batch > 0 && hw > 0 && dirs && ro && rd && ((theta && phi && rho) || c2w));
  CN_CHECK_ARG(select_inds ? (sample_size > 0 && sample_size <= hw) : sample_size == hw);
  CN_CHECK_ARG(!target || (target_out && target_channels > 0));
  const int64_t n = batch * sample_size;
  hipLaunchKernelGGL(pose_rays_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0, cn::as_stream(stream),
                     theta && phi && rho ? theta : nullptr, phi, rho, c2w, batch, dirs, hw, select_inds, sample_size, target, target_channels, c2w_out,
                     ro, rd, target_out);
  return cn::launch_status();
}

extern "C" int cn_pose_rays_backward(const float* theta, const float* phi, const float* rho, int64_t batch,
                                     const float* dirs, int64_t hw, const int64_t* select_inds, int64_t sample_size,
                                     const float* g_ro, const float* g_rd, float* d_c2w, float* d_theta,
                                     float* d_phi, float* d_rho, cn_stream_t stream) {
  const bool want_angles = d_theta || d_phi || d_rho;
  CN_CHECK_ARG(batch > 0 && batch < (1ll << 31) && hw > 0 && dirs && (g_ro || g_rd) && (d_c2w || want_angles));
  CN_CHECK_ARG(select_inds ? (sample_size > 0 && sample_size <= hw) : sample_size == hw);
  CN_CHECK_ARG(!want_angles || (theta && phi && rho));
  hipLaunchKernelGGL(pose_rays_backward_kernel, dim3(static_cast<unsigned>(batch)), dim3(kPoseBwdThreads), 0,
                     cn::as_stream(stream), want_angles ? theta : nullptr, phi, rho, dirs, hw, select_inds,
                     sample_size, g_ro, g_rd, d_c2w, d_theta, d_phi, d_rho);
  return cn::launch_status();
}

extern "C" int cn_random_select(int64_t batch, int64_t hw, int64_t sample_size, uint64_t seed, uint64_t offset,
                                int64_t* select_inds, cn_stream_t stream) {
  CN_CHECK_ARG(batch > 0 && batch < (1ll << 31) && select_inds);
  CN_CHECK_ARG(sample_size > 0 && sample_size <= hw);
  if (hw > kSelMax) return CN_EUNSUPPORTED;
  int n_pad = 2;
  while (n_pad < hw) n_pad <<= 1;
  hipLaunchKernelGGL(random_select_kernel, dim3(static_cast<unsigned>(batch)), dim3(kSelThreads), 0,
                     cn::as_stream(stream), hw, sample_size, seed, offset, n_pad, select_inds);
  return cn::launch_status();
}

extern "C" int cn_pose_error(const float* gt_c2w, const float* cam_c2w, int64_t batch, float* twist, float* err,
                             cn_stream_t stream) {
  CN_CHECK_ARG(batch > 0 && gt_c2w && cam_c2w && (twist || err));
  hipLaunchKernelGGL(pose_error_kernel, dim3(static_cast<unsigned>(cn::ceil_div(batch, 64))), dim3(64), 0,
                     cn::as_stream(stream), gt_c2w, cam_c2w, batch, twist, err);
  return cn::launch_status();
}
