// Pieces shared by the fp32 and 3xbf16 field kernels: launch arguments, the
// per-sample input decode (points, Q1 view direction, code row) and the
// positional-encoding feature values each lane half owns.
#pragma once

#include "cn_common.h"
#include "mlp_layout.h"

namespace cn {
namespace mlp {

typedef float floatx16 __attribute__((ext_vector_type(16)));

struct Params {
  const float* p[CN_NUM_PARAMS];
};

enum ParamIdx {
  kWXyz1 = 0, kBXyz1, kWXyz2, kBXyz2, kWOut, kBOut, kWSc1, kBSc1, kWSc2, kBSc2, kWTc1, kBTc1,
  kWDir1, kBDir1, kWDir2, kBDir2, kWRgb, kBRgb
};

enum InputMode { kFromPts = 0, kFromRayZ = 1, kFromEncoded = 2 };

struct FieldArgs {
  const float* packed;
  const float* code_bias;
  const int64_t* code_index;
  int64_t n_codes;
  const float* pts;  // kFromPts: (n_rays*S, 3)
  const float* ro;   // kFromRayZ
  const float* rd;   // view directions (kFromPts / kFromRayZ)
  const float* z;    // kFromRayZ: (n_rays*S)
  const float* x;    // kFromEncoded: (m, 90)
  int64_t n_rays, n_samples, chunk_rows, m;
  float fx[10];
  float fd[4];
  float* raw;
  float* save;  // fp32 kernel only: (5, m, 256) post-activation h1, h2, feat, v1, v2 for the backward
  // 3xbf16 training forward / fused backward (mlp_x3.hip)
  unsigned* masks;       // ReLU masks, kMaskWordsPerTile per 128-sample tile
  const float* d_raw;    // backward: dL/draw (m, 4)
  float* g_code;         // backward: (n_codes, kCbStride) accumulated
  float* d_pts;          // backward: (m, 3) written (kFromPts)
  float* d_ro;           // backward: (n_rays, 3) accumulated (kFromRayZ)
  float* d_rd;           // backward: (n_rays, 3) accumulated
  float* dpre;           // fp32 fused training backward: (5, m, 256) masked layer-input gradients
  float* xenc;           // fp32 training forward: (m, 64) the positional encodings it multiplied (xenc_col)
  // fused eval backward, deterministic form (cn_field_backward_fused_ws: one code row, every wave inside
  // one ray): no float atomics -- partials a fixed-order reduction adds up afterwards
  float* gc_part;        // (blocks x waves, kCbStride): each wave's g_code row
  float* gc_rows;        // fp32: set -> each workgroup's wave rows summed in wave order, one row per workgroup
  float* ray_part;       // (m / wave samples, 6): each wave's d ro, d rd of its ray (the points' part)
  float* q1_part;        // (m, 3): each sample's d rd of its Q1 view-direction ray
  int64_t n_blocks;      // set by the backward launchers: the grid they launched
};

// The most workgroups a fused backward launches in the deterministic form, and its most waves per
// workgroup (gc_part holds kMaxBwdBlocks x kMaxBwdWaves rows).
constexpr int64_t kMaxBwdBlocks = 512, kMaxBwdWaves = 8;

// Column c' of the fp32 training forward's encoding plane (64 floats per sample: lane group g's 16
// k-step values of layer_xyz1 at 16 g + t) -> PositionalEmbedder column (position_embed.py:44-53:
// x_d -> d, sin(f_k x_d) -> 3 + 6k + d, cos -> 6 + 6k + d), or -1 for the padding slot; the field
// kernel's feature map for layer_xyz1's k-steps (mlp_f32.hip col_enc_xyz).
__host__ __device__ constexpr int xenc_col(int cp) {
  const int t = cp & 15, g = cp >> 4, i = t & 7, p = 4 * i + g;
  if (p < 30) return (t < 8 ? 3 : 6) + 6 * (p / 3) + p % 3;
  return t < 8 ? (g == 2 ? 0 : 2) : (g == 2 ? 1 : -1);
}

// v[i] for a lane-varying i in 0..2 by selects: an indexed read of a private array would
// place the whole array (and the struct holding it) in scratch memory.
__device__ __forceinline__ float pick3(const float (&v)[3], int i) {
  return i == 0 ? v[0] : (i == 1 ? v[1] : v[2]);
}
// v[i] += x for a lane-varying i in 0..2, by selects (see pick3).
__device__ __forceinline__ void add3(float (&v)[3], int i, float x) {
  v[0] += i == 0 ? x : 0.0f;
  v[1] += i == 1 ? x : 0.0f;
  v[2] += i == 2 ? x : 0.0f;
}

// sin / cos of an encoding argument without branches, for |x| <= kFastSinBound: Cody-Waite
// reduction by pi/2 in three fp32 parts with FMAs, then the Cephes sinf / cosf polynomials on
// [-pi/4, pi/4] (max 1.5 ulp against float64 sin / cos over |x| <= 2^14, 0.34 ulp mean; ocml's
// sincosf is of the same class but branches into its large-argument path, which keeps the field
// kernels from interleaving the encodings with the first layer's MFMAs).  Callers check the bound
// (positional encodings: |x| 2^(L-1) of scene coordinates; beyond it they take sincosf).
constexpr float kFastSinBound = 16384.0f;
__device__ __forceinline__ void fast_sincosf(float x, float& sn, float& cs) {
  const float j = __builtin_rintf(x * 0.636619772367581343f);
  float r = fmaf(-j, 1.57079637050628662109375f, x);
  r = fmaf(-j, -4.37113900018624283e-8f, r);
  r = fmaf(-j, -1.71512451000591636e-15f, r);
  const float z = r * r;
  const float s = fmaf(r * z, fmaf(z, fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f), -1.6666654611e-1f), r);
  const float c = fmaf(z * z, fmaf(z, fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f), 4.166664568298827e-2f),
                       fmaf(-0.5f, z, 1.0f));
  const int q = static_cast<int>(j) & 3;
  const float s1 = (q & 1) ? c : s, c1 = (q & 1) ? s : c;
  sn = (q & 2) ? -s1 : s1;
  cs = ((q + 1) & 2) ? -c1 : c1;
}

// An encoding's (sin, cos) for the dW kernels that regenerate the encodings: fast_sincosf inside
// its bound -- the arithmetic the field kernels' lazy path used for every in-range wave (and, unlike
// ocml's sincosf, ~20 VALU instructions without a branch) -- ocml's sincosf beyond it, per lane.
__device__ __forceinline__ void enc_sincosf(float x, float& sn, float& cs) {
  if (fabsf(x) <= kFastSinBound) fast_sincosf(x, sn, cs);
  else sincosf(x, &sn, &cs);
}

// One sample's inputs: point, unit Q1 view direction, code row.
struct SampleIn {
  float x[3];
  float vd[3];
  float nrm;        // |rd| of the Q1 direction ray (the backward's d rd scale)
  int64_t code_of;  // ray (or row) whose code applies
};

// Unit view direction of ray dray (rd normalised with the reference's op order); returns |rd|.
__device__ __forceinline__ float view_dir(const FieldArgs& a, int64_t dray, float (&vd)[3]) {
  const float d0 = a.rd[3 * dray], d1 = a.rd[3 * dray + 1], d2 = a.rd[3 * dray + 2];
  const float nrm = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(d0, d0), __fmul_rn(d1, d1)), __fmul_rn(d2, d2)));
  vd[0] = __fdiv_rn(d0, nrm);
  vd[1] = __fdiv_rn(d1, nrm);
  vd[2] = __fdiv_rn(d2, nrm);
  return nrm;
}

template <int MODE>
__device__ __forceinline__ SampleIn decode_sample(const FieldArgs& a, int64_t rc) {
  SampleIn in;
  if constexpr (MODE == kFromEncoded) {
    in.code_of = rc;
  } else {
    const int64_t S = a.n_samples;
    const int64_t ray = rc / S, smp = rc - ray * S;
    if constexpr (MODE == kFromPts) {
      in.x[0] = a.pts[3 * rc]; in.x[1] = a.pts[3 * rc + 1]; in.x[2] = a.pts[3 * rc + 2];
    } else {
      const float zv = a.z[rc];
#pragma unroll
      for (int j = 0; j < 3; ++j) in.x[j] = mul_add_rn(a.rd[3 * ray + j], zv, a.ro[3 * ray + j]);
    }
    // Q1 (nerf/__init__.py:127-128): within a chunk of Rc rays, sample row
    // k = r*S + s takes the view direction of ray k mod Rc.
    const int64_t base = (ray / a.chunk_rows) * a.chunk_rows;
    const int64_t rcnt = min(a.chunk_rows, a.n_rays - base);
    const int64_t dray = base + ((ray - base) * S + smp) % rcnt;
    in.nrm = view_dir(a, dray, in.vd);
    in.code_of = ray;
  }
  return in;
}

__device__ __forceinline__ int64_t code_row(const FieldArgs& a, int64_t code_of) {
  return a.code_index ? a.code_index[code_of] : (a.n_codes == 1 ? 0 : code_of);
}

// sincos of pair q of lane half h: x[d] * f[k] for p = 2q + h, k = p / 3, d = p % 3.
template <int Q, int NF>
__device__ __forceinline__ void enc_pair(const float* x, const float* f, int h, float& sn, float& cs) {
  constexpr int p0 = 2 * Q, p1 = 2 * Q + 1;
  const float a0 = __fmul_rn(x[p0 % 3], f[p0 / 3]);
  const float a1 = (p1 / 3 < NF) ? __fmul_rn(x[p1 % 3], f[p1 / 3]) : 0.0f;
  sincosf(h ? a1 : a0, &sn, &cs);
}

// The 2P+2 encoding values lane half h feeds, in k_from_enc order (mlp_layout.h):
// sines of its P pairs, cosines, then raw inputs (x0, x1 | x2, 0).
template <int P, int NF, int Q = 0>
__device__ __forceinline__ void encode_pairs(const float* x, const float* f, int h, float* out) {
  if constexpr (Q < P) {
    float sn, cs;
    enc_pair<Q, NF>(x, f, h, sn, cs);
    out[Q] = sn;
    out[P + Q] = cs;
    encode_pairs<P, NF, Q + 1>(x, f, h, out);
  } else {
    out[2 * P] = h ? x[2] : x[0];
    out[2 * P + 1] = h ? 0.0f : x[1];
  }
}

// ---------------------------------------------------------------- code bias (model.py:174-192)
// Per code row: the three code layers (model.py:174-177), then the code halves
// of layer_xyz2 / fc_out / fc_rgb plus their biases.  Each code row is spread
// over kCbSlices workgroups so the 1.5 MiB of weight rows are read by many CUs
// at once (one CU per code was latency bound, ~85 us): slice q < 8 forms
// xyz2 rows 32q..32q+31, slices 8..15 fc_out rows (slice 15 also row 256),
// slice 16 the three fc_rgb rows.  Each slice first forms the one code-layer
// vector it consumes (s1, s2 or t1; 256 dots, L2-resident weights after the
// first slice touches them).  Every output is one wave-wide dot product: 64
// lanes read a 256-float weight row as one coalesced float4 each, then a
// butterfly sum.

constexpr int kCbThreads = 512;
constexpr int kCbSlices = 17;

// The dot of a 256-float row with v as 64 lanes x float4 (w, x: this lane's quarter), summed by a
// butterfly: every lane ends with the total.
__device__ __forceinline__ float wave_dot4(float4 a, float4 b) {
  float s = fmaf(a.x, b.x, fmaf(a.y, b.y, fmaf(a.z, b.z, a.w * b.w)));
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  return s;
}

// Workgroup `blk` (= code * kCbSlices + slice) of the code-bias launch (cn_code_bias; also a role of
// the one-launch step preparation, cn_field_prepare).
// act (optional, (n_codes, 768)): the code-layer activations s1 | s2 | t1 (post-ReLU), written by the
// first slice of each layer -- the code backward's ReLU masks and outer-product operands.
__device__ __forceinline__ void code_bias_block(const Params& P, const float* __restrict__ z_s,
                                                const float* __restrict__ z_t, float* __restrict__ out, int64_t blk,
                                                float* __restrict__ act = nullptr) {
  __shared__ __attribute__((aligned(16))) float z[kCode], hv[kCode];
  const int64_t c = blk / kCbSlices;
  const int q = static_cast<int>(blk % kCbSlices), t = threadIdx.x, lane = t & 63, wave = t >> 6;
  constexpr int kW = kCbThreads / 64;
  const int l = q < 8 ? 0 : (q < 16 ? 1 : 2);  // 0: s1 -> xyz2, 1: s2 -> fc_out, 2: t1 -> fc_rgb
  if (t < kCode) z[t] = (l == 2 ? z_t : z_s)[c * kCode + t];
  __syncthreads();
  {
    // rows wave + 8 i: eight rows' loads in flight per round (no branch between them), the lane-0
    // writes after; bias + ReLU once per output below
    const float* W = P.p[l == 0 ? kWSc1 : (l == 1 ? kWSc2 : kWTc1)];
    const float4 zv = reinterpret_cast<const float4*>(z)[lane];
#pragma unroll
    for (int i0 = 0; i0 < kCode / kW; i0 += 8) {
      float4 wv[8];
#pragma unroll
      for (int x = 0; x < 8; ++x) wv[x] = reinterpret_cast<const float4*>(W + (wave + (i0 + x) * kW) * kCode)[lane];
      float d[8];
#pragma unroll
      for (int x = 0; x < 8; ++x) d[x] = wave_dot4(wv[x], zv);
      if (lane == 0)
#pragma unroll
        for (int x = 0; x < 8; ++x) hv[wave + (i0 + x) * kW] = d[x];
    }
  }
  __syncthreads();
  if (t < kCode) {
    const float* B = P.p[l == 0 ? kBSc1 : (l == 1 ? kBSc2 : kBTc1)];
    hv[t] = fmaxf(hv[t] + B[t], 0.f);
    if (act && (q == 0 || q == 8 || q == 16)) act[c * 3 * kCode + l * kCode + t] = hv[t];
  }
  __syncthreads();
  float* o = out + c * kCbStride;
  int r0, nr;
  if (l == 0) { r0 = 32 * q; nr = 32; }
  else if (l == 1) { r0 = 32 * (q - 8); nr = q == 15 ? 33 : 32; }
  else { r0 = 0; nr = 3; }
  // at most 5 rows per wave (33 / 8): all their loads first, then the dots
  const float4 hq = reinterpret_cast<const float4*>(hv)[lane];
  float4 wv[5];
  float bv[5];
  int dst[5];
#pragma unroll
  for (int x = 0; x < 5; ++x) {
    const int r = min(r0 + wave + x * kW, r0 + nr - 1);  // rows past the slice repeat its last (not stored)
    const float* w;
    if (l == 0) {
      w = P.p[kWXyz2] + r * (kHidden + kCode) + kHidden; bv[x] = P.p[kBXyz2][r]; dst[x] = kCbXyz2 + r;
    } else if (l == 1) {
      // slice rows 0..255 map to fc_out rows 1..256 (feat); row 256 -> fc_out row 0 (sigma)
      const int i = r == kCode ? 0 : r + 1;
      w = P.p[kWOut] + i * (kHidden + kCode) + kHidden; bv[x] = P.p[kBOut][i];
      dst[x] = i == 0 ? kCbSigma : kCbFeat + i - 1;
    } else {
      w = P.p[kWRgb] + r * (kHidden + kCode) + kHidden; bv[x] = P.p[kBRgb][r]; dst[x] = kCbRgb + r;
    }
    wv[x] = reinterpret_cast<const float4*>(w)[lane];
  }
#pragma unroll
  for (int x = 0; x < 5; ++x) {
    const float a = wave_dot4(wv[x], hq);
    if (lane == 0 && wave + x * kW < nr) o[dst[x]] = a + bv[x];
  }
  if (l == 2 && t >= 3 && t < kCbStride - kCbRgb) o[kCbRgb + t] = 0.f;  // pad 516..519
}

// 3xbf16 variant (mlp_x3.hip): forward (optionally writing ReLU masks) and the
// fused backward over the transposed pack.
int64_t packed_floats_x3();
int launch_pack_x3(const Params& P, float* packed, hipStream_t st);
int launch_pack_x3t(const Params& P, float* packed, hipStream_t st);
int launch_field_x3(int mode, FieldArgs& a, hipStream_t st);
int64_t mask_words_x3(int64_t m);
int launch_field_x3_bwd(int mode, FieldArgs& a, hipStream_t st);

// fp32 16x16x4 two-waves-per-SIMD variant (mlp_f32.hip): inference forward.
int64_t packed_floats_w16();
int launch_pack_w16(const Params& P, float* packed, hipStream_t st);
int launch_field_w16(int mode, FieldArgs& a, hipStream_t st);  // a.masks: also the ReLU masks
int64_t mask_words_w16(int64_t m);
int launch_pack_w16t(const Params& P, float* packed, hipStream_t st);
// code_bias + the CN_FMT_F32_W16 / _T packs + a zeroed buffer (any of them null: skipped), for one or
// two models on the same codes, in one launch
struct PrepareModel {
  Params P;
  float* code_bias;
  float* code_act;   // (n_codes, 768) code-layer activations, or null
  float* packed;
  float* packed_t;
  float* zero;
  int64_t n_zero;
};
int launch_field_prepare_w16(const PrepareModel* models, int n_models, const float* z_s, const float* z_t,
                             int64_t n_codes, hipStream_t st);
int launch_field_w16_bwd(int mode, FieldArgs& a, hipStream_t st);
int launch_field_w16_bwd2(int mode, FieldArgs& a0, FieldArgs& a1, hipStream_t st);
// cn_field_backward_fused's argument checks, into a (mlp.hip).
int fused_backward_args(int fmt_t, const float* packed_t, const uint32_t* masks, const float* d_raw,
                        const float* pts, const float* ro, const float* rd, const float* z, int64_t n_rays,
                        int64_t n_samples, int64_t chunk_rows, const int64_t* code_index, int64_t n_codes,
                        const float* freqs_xyz, const float* freqs_dir, float* g_code, float* d_pts, float* d_ro,
                        float* d_rd, FieldArgs& a);
// The training backwards' no-geometry schedule (no d ro / d rd / d pts wanted) unless CN_BWD_NOGEO=0.
bool nogeo_enabled();

// 3xbf16 16x16x32 two-waves-per-SIMD variant (mlp_x3w.hip): inference forward only.
int64_t packed_floats_x3w();
int launch_pack_x3w(const Params& P, float* packed, hipStream_t st);
int launch_field_x3w(int mode, FieldArgs& a, hipStream_t st);

// Pre-encoded rows: the same 2P+2 values gathered from x (base = column offset).
template <int P, int T = 0>
__device__ __forceinline__ void gather_pairs(const float* xr, int base, int h, float* out) {
  if constexpr (T < 2 * P + 2) {
    constexpr int e0 = k_from_enc(T, 0, P), e1 = k_from_enc(T, 1, P);
    const float v0 = e0 >= 0 ? xr[base + (e0 < 0 ? 0 : e0)] : 0.0f;
    const float v1 = e1 >= 0 ? xr[base + (e1 < 0 ? 0 : e1)] : 0.0f;
    out[T] = h ? v1 : v0;
    gather_pairs<P, T + 1>(xr, base, h, out);
  }
}

}  // namespace mlp
}  // namespace cn
