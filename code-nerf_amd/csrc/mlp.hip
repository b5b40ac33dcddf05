// Code-conditioned MLP: CodeNeRFModel (view_synthesis/models/model.py:123-194)
// fused with the positional encoding and Q1 view-direction mapping of
// forward_pass (view_synthesis/nerf/__init__.py:94-134).
//
// Per sample the reference evaluates 9 Linear layers over concatenated inputs.
// Three of them (the code layers, model.py:174-177) and the code halves of
// layer_xyz2 / fc_out / fc_rgb depend only on the object's codes, so they are
// folded once per code row into bias vectors (cn_code_bias).  The remaining
// per-sample work -- 63->256, 256->256, 256->257, (256+27)->256, 256->256,
// 256->3 -- is 286,208 MAC = 572,416 FLOP per sample and runs on fp32 MFMA
// (v_mfma_f32_32x32x2_f32, exact f32 products, ~157 TFLOP/s peak on gfx950).
//
// Kernel shape: 256-thread workgroup = 4 waves, one wave per SIMD (the layer's
// 256-wide input and output tiles take ~300 VGPRs), 32 samples per wave, 128
// per workgroup.  Activations never leave registers: each layer's accumulator
// is the next layer's B operand (mlp_layout.h).  Weights (1.25 MiB packed,
// resident in every XCD's L2) stream through a double-buffered LDS ring in
// chunks of 16 k-steps; each chunk is 128-144 MFMAs per wave (8-9 K cycles),
// its successor is loaded into registers while it runs and written to LDS
// behind it.
#include "mlp_common.h"

namespace cn {
namespace mlp {

// ---------------------------------------------------------------- packing

__global__ void pack_kernel(Params P, float* __restrict__ packed) {
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < kPackedFloats;
       idx += gridDim.x * blockDim.x) {
    float v = 0.0f;
    if (idx >= kBiasXyz1) {
      const int j = idx - kBiasXyz1;
      v = j < 256 ? P.p[kBXyz1][j] : (j < 512 ? P.p[kBDir1][j - 256] : P.p[kBDir2][j - 512]);
    } else {
      constexpr int offs[kNumLayers + 1] = {layer_offset(0), layer_offset(1), layer_offset(2),
                                            layer_offset(3), layer_offset(4), layer_offset(5),
                                            layer_offset(6)};
      int l = 0;
      while (l + 1 < kNumLayers && idx >= offs[l + 1]) ++l;
      int rem = idx - offs[l];
      const int nbp = kBlocksPad[l];
      const int ob = rem % nbp;
      rem /= nbp;
      const int lane = rem % 64, t = rem / 64;
      const int i = lane & 31, h = lane >> 5;
      int row = -1, col = -1, in_dim = 0;
      const float* W = nullptr;
      switch (l) {
        case kXyz1: W = P.p[kWXyz1]; in_dim = kDimXyz; row = 32 * ob + i; col = k_from_enc(t, h, 15); break;
        case kXyz2: W = P.p[kWXyz2]; in_dim = kHidden + kCode; row = 32 * ob + i; col = k_from_acc(t, h); break;
        case kOut:
          W = P.p[kWOut]; in_dim = kHidden + kCode; col = k_from_acc(t, h);
          row = ob < 8 ? 1 + 32 * ob + i : ((ob == 8 && i == 0) ? 0 : -1);
          break;
        case kDir1:
          W = P.p[kWDir1]; in_dim = kCode + kDimDir; row = 32 * ob + i;
          if (t < 128) {
            col = k_from_acc(t, h);
          } else {
            const int e = k_from_enc(t - 128, h, 6);
            col = e < 0 ? -1 : kCode + e;
          }
          break;
        case kDir2: W = P.p[kWDir2]; in_dim = kHidden; row = 32 * ob + i; col = k_from_acc(t, h); break;
        default: W = P.p[kWRgb]; in_dim = kHidden + kCode; row = (ob == 0 && i < 3) ? i : -1; col = k_from_acc(t, h); break;
      }
      if (row >= 0 && col >= 0) v = W[row * in_dim + col];
    }
    packed[idx] = v;
  }
}

// ---------------------------------------------------------------- code bias
// (code_bias_block, mlp_common.h: one workgroup of kCbThreads per (code, slice))

__global__ __launch_bounds__(kCbThreads) void code_bias_kernel(Params P, const float* __restrict__ z_s,
                                                               const float* __restrict__ z_t,
                                                               float* __restrict__ out) {
  code_bias_block(P, z_s, z_t, out, blockIdx.x);
}

// ---------------------------------------------------------------- field kernel

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kTile = 32 * kWaves;          // samples per workgroup
constexpr int kChunkSteps = 16;
constexpr int kMaxChunkFloats = kChunkSteps * 64 * 12;  // fc_out chunks (nbp 12)

struct Chunk {
  int layer, t0, steps;
};

// The weight stream: every layer in 16-k-step chunks (layer_dir1 ends with
// its 14-step view-direction chunk).
constexpr int kNumChunks = 2 + 8 + 8 + 9 + 8 + 8;
__host__ __device__ constexpr Chunk chunk_at(int c) {
  return c < 2 ? Chunk{kXyz1, 16 * c, 16}
       : c < 10 ? Chunk{kXyz2, 16 * (c - 2), 16}
       : c < 18 ? Chunk{kOut, 16 * (c - 10), 16}
       : c < 27 ? Chunk{kDir1, 16 * (c - 18), c == 26 ? 14 : 16}
       : c < 35 ? Chunk{kDir2, 16 * (c - 27), 16}
                : Chunk{kRgb, 16 * (c - 35), 16};
}
__host__ __device__ constexpr int chunk_floats(int c) {
  return chunk_at(c).steps * 64 * kBlocksPad[chunk_at(c).layer];
}
__host__ __device__ constexpr int chunk_src(int c) {
  return layer_offset(chunk_at(c).layer) + chunk_at(c).t0 * 64 * kBlocksPad[chunk_at(c).layer];
}
// float4 loads per thread to stage a chunk
__host__ __device__ constexpr int chunk_loads(int c) { return (chunk_floats(c) / 4 + kThreads - 1) / kThreads; }
constexpr int kMaxLoads = (kMaxChunkFloats / 4) / kThreads;  // 12

struct State {
  float* save_row;   // this sample's row of plane 0 of FieldArgs::save (or null)
  int64_t plane;     // floats between save planes
  floatx16 act[8];   // layer input (B operands), 256 features x 32 samples
  floatx16 acc[9];   // layer output accumulators
  floatx16 denc;     // view-direction encoding (14 k-steps of layer_dir1)
  float4 stage[kMaxLoads];
  float sigma;
  int lane, h;
  int64_t cb_row;    // code-bias row (floats offset)
  float vd[3];       // unit view direction of this sample's Q1 ray
};

template <int C>
__device__ __forceinline__ void load_chunk(State& s, const float* __restrict__ packed) {
  constexpr int n4 = chunk_floats(C) / 4;
  const float4* src = reinterpret_cast<const float4*>(packed + chunk_src(C));
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < chunk_loads(C); ++i) {
    const int q = i * kThreads + tid;
    if (n4 % kThreads == 0 || q < n4) s.stage[i] = src[q];
  }
}

template <int C>
__device__ __forceinline__ void store_chunk(State& s, float* lds) {
  constexpr int n4 = chunk_floats(C) / 4;
  float4* dst = reinterpret_cast<float4*>(lds);
  const int tid = threadIdx.x;
#pragma unroll
  for (int i = 0; i < chunk_loads(C); ++i) {
    const int q = i * kThreads + tid;
    if (n4 % kThreads == 0 || q < n4) dst[q] = s.stage[i];
  }
}

// Bias-initialised accumulators for layer L (acc = b, then acc += W x).
template <int L>
__device__ __forceinline__ void init_acc(State& s, const FieldArgs& a) {
  const float* cb = a.code_bias + s.cb_row;
  const float* base = L == kXyz1 ? a.packed + kBiasXyz1
                    : L == kXyz2 ? cb + kCbXyz2
                    : L == kOut ? cb + kCbFeat
                    : L == kDir1 ? a.packed + kBiasDir1
                    : L == kDir2 ? a.packed + kBiasDir2
                                 : cb + kCbRgb;
  if constexpr (L == kRgb) {
    // block 0 rows 0..2 (lane half 0, registers 0..2)
    s.acc[0] = floatx16{0};
    if (s.h == 0) {
      s.acc[0][0] = base[0];
      s.acc[0][1] = base[1];
      s.acc[0][2] = base[2];
    }
  } else {
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 b = *reinterpret_cast<const float4*>(base + 32 * ob + 8 * q + 4 * s.h);
        s.acc[ob][4 * q + 0] = b.x;
        s.acc[ob][4 * q + 1] = b.y;
        s.acc[ob][4 * q + 2] = b.z;
        s.acc[ob][4 * q + 3] = b.w;
      }
    }
    if constexpr (L == kOut) {
      s.acc[8] = floatx16{0};
      if (s.h == 0) s.acc[8][0] = cb[kCbSigma];
    }
  }
}

// B operand of k-step t (global within layer L).
template <int L, int T>
__device__ __forceinline__ float b_operand(const State& s) {
  if constexpr (L == kXyz1) {
    return s.act[T >> 4][T & 15];
  } else if constexpr (L == kDir1 && T >= 128) {
    return s.denc[T - 128];
  } else {
    return s.act[T >> 4][T & 15];
  }
}

template <int C, int T>
__device__ __forceinline__ void mfma_step(State& s, const float* lds) {
  constexpr Chunk ch = chunk_at(C);
  constexpr int L = ch.layer;
  constexpr int nbp = kBlocksPad[L];
  constexpr int nb = kBlocks[L];
  const float* ap = lds + (T * 64 + s.lane) * nbp;
  float a[nbp];
  if constexpr (nbp % 4 == 0) {
#pragma unroll
    for (int j = 0; j < nbp / 4; ++j) {
      const float4 v = *reinterpret_cast<const float4*>(ap + 4 * j);
      a[4 * j] = v.x; a[4 * j + 1] = v.y; a[4 * j + 2] = v.z; a[4 * j + 3] = v.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < nbp; ++j) a[j] = ap[j];
  }
  const float b = b_operand<L, ch.t0 + T>(s);
#pragma unroll
  for (int ob = 0; ob < nb; ++ob) s.acc[ob] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[ob], b, s.acc[ob], 0, 0, 0);
}

template <int C, int T>
__device__ __forceinline__ void mfma_steps(State& s, const float* lds) {
  if constexpr (T < chunk_at(C).steps) {
    mfma_step<C, T>(s, lds);
    mfma_steps<C, T + 1>(s, lds);
  }
}

template <int N>
__device__ __forceinline__ void put_act(State& s, const float* v) {
#pragma unroll
  for (int t = 0; t < N; ++t) s.act[t >> 4][t & 15] = v[t];
}

// Training mode: the layer's post-activation outputs, row-major (m, 256) per layer.
template <int L>
__device__ __forceinline__ void save_layer(const State& s) {
  if constexpr (L != kRgb) {
    if (s.save_row) {
      float* dst = s.save_row + L * s.plane;
#pragma unroll
      for (int ob = 0; ob < 8; ++ob)
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<float4*>(dst + 32 * ob + 8 * q + 4 * s.h) =
              make_float4(s.act[ob][4 * q], s.act[ob][4 * q + 1], s.act[ob][4 * q + 2], s.act[ob][4 * q + 3]);
    }
  }
}

template <int L>
__device__ __forceinline__ void finish_layer(State& s) {
  if constexpr (L == kOut) {
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) s.act[ob] = s.acc[ob];  // feat: no activation
    s.sigma = s.acc[8][0];
  } else if constexpr (L != kRgb) {
#pragma unroll
    for (int ob = 0; ob < 8; ++ob)
#pragma unroll
      for (int r = 0; r < 16; ++r)  // ReLU as v_max_i32 on the bits (fmaxf: canonicalize + max)
        s.act[ob][r] = __int_as_float(max(__float_as_int(s.acc[ob][r]), 0));
  }
}

template <int MODE, int C>
__device__ __forceinline__ void run_chunks(State& s, const FieldArgs& a, float* lds0, float* lds1) {
  if constexpr (C < kNumChunks) {
    constexpr Chunk ch = chunk_at(C);
    float* cur = (C & 1) ? lds1 : lds0;
    float* nxt = (C & 1) ? lds0 : lds1;
    if constexpr (ch.t0 == 0) init_acc<ch.layer>(s, a);
    if constexpr (C + 1 < kNumChunks) load_chunk<C + 1>(s, a.packed);
    if constexpr (ch.layer == kDir1 && ch.t0 == 0 && MODE != kFromEncoded) {
      float v[14];
      encode_pairs<6, 4>(s.vd, a.fd, s.h, v);
#pragma unroll
      for (int t = 0; t < 14; ++t) s.denc[t] = v[t];
    }
    mfma_steps<C, 0>(s, cur);
    constexpr bool last_of_layer = (C + 1 == kNumChunks) || chunk_at(C + 1).layer != ch.layer;
    if constexpr (last_of_layer) {
      finish_layer<ch.layer>(s);
      save_layer<ch.layer>(s);
    }
    if constexpr (C + 1 < kNumChunks) {
      store_chunk<C + 1>(s, nxt);
      __syncthreads();
    }
    run_chunks<MODE, C + 1>(s, a, lds0, lds1);
  }
}

template <int MODE>
__global__ __launch_bounds__(kThreads, 1) void field_kernel(FieldArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[2][kMaxChunkFloats];
  State s;
  s.lane = threadIdx.x & 63;
  s.h = s.lane >> 5;
  const int wave = threadIdx.x >> 6;
  const int64_t row = (int64_t)blockIdx.x * kTile + wave * 32 + (s.lane & 31);
  const bool valid = row < a.m;
  const int64_t rc = valid ? row : a.m - 1;
  s.save_row = (a.save && valid) ? a.save + row * 256 : nullptr;
  s.plane = a.m * 256;

  // ---- per-sample inputs
  const SampleIn in = decode_sample<MODE>(a, rc);
  float enc[32];
  if constexpr (MODE == kFromEncoded) {
    const float* xr = a.x + rc * (kDimXyz + kDimDir);
    gather_pairs<15>(xr, 0, s.h, enc);
    float d[14];
    gather_pairs<6>(xr, kDimXyz, s.h, d);
#pragma unroll
    for (int t = 0; t < 14; ++t) s.denc[t] = d[t];
  } else {
    encode_pairs<15, 10>(in.x, a.fx, s.h, enc);
#pragma unroll
    for (int j = 0; j < 3; ++j) s.vd[j] = in.vd[j];
  }
  put_act<32>(s, enc);
  s.cb_row = code_row(a, in.code_of) * kCbStride;

  // ---- weight stream prologue: chunk 0 into buffer 0
  load_chunk<0>(s, a.packed);
  store_chunk<0>(s, lds[0]);
  __syncthreads();
  run_chunks<MODE, 0>(s, a, lds[0], lds[1]);

  // ---- raw = [rgb(3), sigma]: block 0 rows 0..2 of fc_rgb live in lane half 0
  if (valid && s.h == 0) {
    float4 o;
    o.x = s.acc[0][0];
    o.y = s.acc[0][1];
    o.z = s.acc[0][2];
    o.w = s.sigma;
    reinterpret_cast<float4*>(a.raw)[row] = o;
  }
}

}  // namespace mlp
}  // namespace cn

using namespace cn::mlp;

namespace {

int make_params(const float* const* params, Params* P) {
  if (!params) return CN_EINVAL;
  for (int i = 0; i < CN_NUM_PARAMS; ++i) {
    if (!params[i]) return CN_EINVAL;
    P->p[i] = params[i];
  }
  return CN_OK;
}

int launch_field(int fmt, int mode, FieldArgs& a, hipStream_t st) {
  if (fmt == CN_FMT_BF16X3) return launch_field_x3(mode, a, st);
  if (fmt == CN_FMT_F32_W16) return launch_field_w16(mode, a, st);
  if (fmt == CN_FMT_BF16X3_W16) return launch_field_x3w(mode, a, st);
  const unsigned grid = static_cast<unsigned>(cn::ceil_div(a.m, kTile));
  switch (mode) {
    case kFromPts: hipLaunchKernelGGL(field_kernel<kFromPts>, dim3(grid), dim3(kThreads), 0, st, a); break;
    case kFromRayZ: hipLaunchKernelGGL(field_kernel<kFromRayZ>, dim3(grid), dim3(kThreads), 0, st, a); break;
    default: hipLaunchKernelGGL(field_kernel<kFromEncoded>, dim3(grid), dim3(kThreads), 0, st, a); break;
  }
  return cn::launch_status();
}

bool valid_fmt(int fmt) {
  return fmt == CN_FMT_F32 || fmt == CN_FMT_BF16X3 || fmt == CN_FMT_F32_W16 || fmt == CN_FMT_BF16X3_W16;
}
bool valid_pack_fmt(int fmt) { return valid_fmt(fmt) || fmt == CN_FMT_BF16X3_T || fmt == CN_FMT_F32_W16_T; }

}  // namespace

static_assert(kPackedFloats == 327424, "packed layout changed: update docs");
static_assert(kCbStride == CN_CODE_BIAS_STRIDE, "code-bias stride mismatch");

extern "C" int64_t cn_mlp_packed_floats(int fmt) {
  if (!valid_pack_fmt(fmt)) return -1;
  if (fmt == CN_FMT_F32_W16 || fmt == CN_FMT_F32_W16_T) return packed_floats_w16();
  if (fmt == CN_FMT_BF16X3_W16) return packed_floats_x3w();
  return fmt == CN_FMT_F32 ? kPackedFloats : packed_floats_x3();
}

extern "C" int cn_mlp_pack(const float* const* params, int fmt, float* packed, cn_stream_t stream) {
  Params P;
  if (make_params(params, &P) != CN_OK || !packed || !valid_pack_fmt(fmt)) return CN_EINVAL;
  if (fmt == CN_FMT_BF16X3) return launch_pack_x3(P, packed, cn::as_stream(stream));
  if (fmt == CN_FMT_BF16X3_T) return launch_pack_x3t(P, packed, cn::as_stream(stream));
  if (fmt == CN_FMT_F32_W16) return launch_pack_w16(P, packed, cn::as_stream(stream));
  if (fmt == CN_FMT_F32_W16_T) return launch_pack_w16t(P, packed, cn::as_stream(stream));
  if (fmt == CN_FMT_BF16X3_W16) return launch_pack_x3w(P, packed, cn::as_stream(stream));
  hipLaunchKernelGGL(pack_kernel, dim3(cn::elementwise_grid(kPackedFloats, 256)), dim3(256), 0,
                     cn::as_stream(stream), P, packed);
  return cn::launch_status();
}

extern "C" int cn_code_bias(const float* const* params, const float* z_s, const float* z_t,
                            int64_t n_codes, float* code_bias, cn_stream_t stream) {
  Params P;
  if (make_params(params, &P) != CN_OK) return CN_EINVAL;
  CN_CHECK_ARG(z_s && z_t && code_bias && n_codes > 0 && n_codes * kCbSlices <= (1ll << 31) - 1);
  hipLaunchKernelGGL(code_bias_kernel, dim3(static_cast<unsigned>(n_codes * kCbSlices)), dim3(kCbThreads), 0,
                     cn::as_stream(stream), P, z_s, z_t, code_bias);
  return cn::launch_status();
}

extern "C" int cn_field_prepare(const float* const* params, const float* z_s, const float* z_t, int64_t n_codes,
                                float* code_bias, float* packed, float* packed_t, float* zero, int64_t n_zero,
                                cn_stream_t stream) {
  const cn_field_prep m = {params, code_bias, packed, packed_t, zero, n_zero, nullptr};
  return cn_field_prepare_models(&m, 1, z_s, z_t, n_codes, stream);
}

extern "C" int cn_field_prepare_models(const cn_field_prep* models, int n_models, const float* z_s, const float* z_t,
                                       int64_t n_codes, cn_stream_t stream) {
  CN_CHECK_ARG(models && n_models >= 1 && n_models <= 2);
  PrepareModel pm[2];
  for (int k = 0; k < n_models; ++k) {
    const cn_field_prep& m = models[k];
    if (make_params(m.params, &pm[k].P) != CN_OK) return CN_EINVAL;
    CN_CHECK_ARG(m.n_zero >= 0 && (m.n_zero == 0 || m.zero));
    CN_CHECK_ARG(!m.code_bias || (z_s && z_t && n_codes > 0 && n_codes * kCbSlices + 256 <= 0x7fffffff));
    CN_CHECK_ARG(!m.code_act || m.code_bias);
    pm[k].code_bias = m.code_bias;
    pm[k].code_act = m.code_act;
    pm[k].packed = m.packed;
    pm[k].packed_t = m.packed_t;
    pm[k].zero = m.zero;
    pm[k].n_zero = m.n_zero;
  }
  return launch_field_prepare_w16(pm, n_models, z_s, z_t, n_codes, cn::as_stream(stream));
}

extern "C" int cn_mlp_forward(const float* packed, int fmt, const float* code_bias,
                              const int64_t* code_index, int64_t n_codes, const float* x,
                              int64_t m, float* raw, cn_stream_t stream) {
  CN_CHECK_ARG(packed && code_bias && x && raw && m > 0 && n_codes > 0 && valid_fmt(fmt));
  CN_CHECK_ARG(code_index || n_codes == 1 || n_codes == m);
  CN_CHECK_ARG(cn::ceil_div(m, kTile) <= 0x7fffffff);
  FieldArgs a = {};
  a.packed = packed;
  a.code_bias = code_bias;
  a.code_index = code_index;
  a.n_codes = n_codes;
  a.x = x;
  a.m = m;
  a.raw = raw;
  CN_CHECK_ARG(cn::aligned16(raw));  // float4 rows (include/codenerf.h)
  return launch_field(fmt, kFromEncoded, a, cn::as_stream(stream));
}

extern "C" int cn_radiance_field(const float* packed, int fmt, const float* code_bias,
                                 const int64_t* code_index, int64_t n_codes, const float* pts,
                                 const float* ro, const float* rd, const float* z, int64_t n_rays,
                                 int64_t n_samples, int64_t chunk_rows, const float* freqs_xyz,
                                 const float* freqs_dir, float* raw, cn_stream_t stream) {
  CN_CHECK_ARG(packed && code_bias && rd && raw && freqs_xyz && freqs_dir && valid_fmt(fmt));
  CN_CHECK_ARG(n_rays > 0 && n_samples > 0 && chunk_rows > 0 && n_codes > 0);
  CN_CHECK_ARG(pts || (ro && z));
  CN_CHECK_ARG(code_index || n_codes == 1 || n_codes == n_rays);
  FieldArgs a = {};
  a.packed = packed;
  a.code_bias = code_bias;
  a.code_index = code_index;
  a.n_codes = n_codes;
  a.pts = pts;
  a.ro = ro;
  a.rd = rd;
  a.z = z;
  a.n_rays = n_rays;
  a.n_samples = n_samples;
  a.chunk_rows = chunk_rows;
  a.m = n_rays * n_samples;
  CN_CHECK_ARG(cn::ceil_div(a.m, kTile) <= 0x7fffffff);
  for (int i = 0; i < 10; ++i) a.fx[i] = freqs_xyz[i];
  for (int i = 0; i < 4; ++i) a.fd[i] = freqs_dir[i];
  a.raw = raw;
  CN_CHECK_ARG(cn::aligned16(raw));  // float4 rows (include/codenerf.h)
  return launch_field(fmt, pts ? kFromPts : kFromRayZ, a, cn::as_stream(stream));
}

extern "C" int cn_radiance_field_train(const float* packed, const float* code_bias, const int64_t* code_index,
                                       int64_t n_codes, const float* pts, const float* ro, const float* rd,
                                       const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                                       const float* freqs_xyz, const float* freqs_dir, float* raw, float* save,
                                       cn_stream_t stream) {
  CN_CHECK_ARG(packed && code_bias && rd && raw && save && freqs_xyz && freqs_dir);
  CN_CHECK_ARG(n_rays > 0 && n_samples > 0 && chunk_rows > 0 && n_codes > 0);
  CN_CHECK_ARG(pts || (ro && z));
  CN_CHECK_ARG(code_index || n_codes == 1 || n_codes == n_rays);
  FieldArgs a = {};
  a.packed = packed;
  a.code_bias = code_bias;
  a.code_index = code_index;
  a.n_codes = n_codes;
  a.pts = pts;
  a.ro = ro;
  a.rd = rd;
  a.z = z;
  a.n_rays = n_rays;
  a.n_samples = n_samples;
  a.chunk_rows = chunk_rows;
  a.m = n_rays * n_samples;
  CN_CHECK_ARG(cn::ceil_div(a.m, kTile) <= 0x7fffffff);
  for (int i = 0; i < 10; ++i) a.fx[i] = freqs_xyz[i];
  for (int i = 0; i < 4; ++i) a.fd[i] = freqs_dir[i];
  a.raw = raw;
  CN_CHECK_ARG(cn::aligned16(raw));  // float4 rows (include/codenerf.h)
  a.save = save;
  return launch_field(CN_FMT_F32, pts ? kFromPts : kFromRayZ, a, cn::as_stream(stream));
}

extern "C" int cn_mlp_forward_train(const float* packed, const float* code_bias, const int64_t* code_index,
                                    int64_t n_codes, const float* x, int64_t m, float* raw, float* save,
                                    cn_stream_t stream) {
  CN_CHECK_ARG(packed && code_bias && x && raw && save && m > 0 && n_codes > 0);
  CN_CHECK_ARG(code_index || n_codes == 1 || n_codes == m);
  CN_CHECK_ARG(cn::ceil_div(m, kTile) <= 0x7fffffff);
  FieldArgs a = {};
  a.packed = packed;
  a.code_bias = code_bias;
  a.code_index = code_index;
  a.n_codes = n_codes;
  a.x = x;
  a.m = m;
  a.raw = raw;
  CN_CHECK_ARG(cn::aligned16(raw));  // float4 rows (include/codenerf.h)
  a.save = save;
  return launch_field(CN_FMT_F32, kFromEncoded, a, cn::as_stream(stream));
}

extern "C" int64_t cn_field_mask_words(int64_t m) { return m > 0 ? mask_words_x3(m) : -1; }

extern "C" int64_t cn_field_mask_words_fmt(int fmt, int64_t m) {
  if (m <= 0) return -1;
  if (fmt == CN_FMT_BF16X3) return mask_words_x3(m);
  if (fmt == CN_FMT_F32_W16) return mask_words_w16(m);
  return -1;
}

extern "C" int cn_radiance_field_masks(const float* packed, const float* code_bias, const int64_t* code_index,
                                       int64_t n_codes, const float* pts, const float* ro, const float* rd,
                                       const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                                       const float* freqs_xyz, const float* freqs_dir, float* raw, uint32_t* masks,
                                       cn_stream_t stream) {
  return cn_radiance_field_masks_fmt(CN_FMT_BF16X3, packed, code_bias, code_index, n_codes, pts, ro, rd, z, n_rays,
                                     n_samples, chunk_rows, freqs_xyz, freqs_dir, raw, masks, stream);
}

extern "C" int cn_radiance_field_masks_fmt(int fmt, const float* packed, const float* code_bias,
                                           const int64_t* code_index, int64_t n_codes, const float* pts,
                                           const float* ro, const float* rd, const float* z, int64_t n_rays,
                                           int64_t n_samples, int64_t chunk_rows, const float* freqs_xyz,
                                           const float* freqs_dir, float* raw, uint32_t* masks, cn_stream_t stream) {
  CN_CHECK_ARG(fmt == CN_FMT_BF16X3 || fmt == CN_FMT_F32_W16);
  CN_CHECK_ARG(packed && code_bias && rd && raw && masks && freqs_xyz && freqs_dir);
  CN_CHECK_ARG(n_rays > 0 && n_samples > 0 && chunk_rows > 0 && n_codes > 0);
  CN_CHECK_ARG(pts || (ro && z));
  CN_CHECK_ARG(code_index || n_codes == 1 || n_codes == n_rays);
  FieldArgs a = {};
  a.packed = packed;
  a.code_bias = code_bias;
  a.code_index = code_index;
  a.n_codes = n_codes;
  a.pts = pts;
  a.ro = ro;
  a.rd = rd;
  a.z = z;
  a.n_rays = n_rays;
  a.n_samples = n_samples;
  a.chunk_rows = chunk_rows;
  a.m = n_rays * n_samples;
  CN_CHECK_ARG(cn::ceil_div(a.m, kTile) <= 0x7fffffff);
  for (int i = 0; i < 10; ++i) a.fx[i] = freqs_xyz[i];
  for (int i = 0; i < 4; ++i) a.fd[i] = freqs_dir[i];
  a.raw = raw;
  CN_CHECK_ARG(cn::aligned16(raw));  // float4 rows (include/codenerf.h)
  a.masks = masks;
  return fmt == CN_FMT_BF16X3 ? launch_field_x3(pts ? kFromPts : kFromRayZ, a, cn::as_stream(stream))
                              : launch_field_w16(pts ? kFromPts : kFromRayZ, a, cn::as_stream(stream));
}

extern "C" int cn_radiance_field_train_w16(const float* packed, const float* code_bias, const int64_t* code_index,
                                           int64_t n_codes, const float* pts, const float* ro, const float* rd,
                                           const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                                           const float* freqs_xyz, const float* freqs_dir, float* raw, float* save,
                                           uint32_t* masks, cn_stream_t stream) {
  return cn_radiance_field_train_fmt(CN_FMT_F32_W16, packed, code_bias, code_index, n_codes, pts, ro, rd, z, n_rays,
                                     n_samples, chunk_rows, freqs_xyz, freqs_dir, raw, save, masks, stream);
}

extern "C" int cn_radiance_field_train_fmt(int fmt, const float* packed, const float* code_bias,
                                           const int64_t* code_index, int64_t n_codes, const float* pts,
                                           const float* ro, const float* rd, const float* z, int64_t n_rays,
                                           int64_t n_samples, int64_t chunk_rows, const float* freqs_xyz,
                                           const float* freqs_dir, float* raw, float* save, uint32_t* masks,
                                           cn_stream_t stream) {
  CN_CHECK_ARG(fmt == CN_FMT_F32_W16 || fmt == CN_FMT_BF16X3);
  CN_CHECK_ARG(packed && code_bias && rd && raw && save && masks && freqs_xyz && freqs_dir);
  CN_CHECK_ARG(n_rays > 0 && n_samples > 0 && chunk_rows > 0 && n_codes > 0);
  CN_CHECK_ARG(pts || (ro && z));
  CN_CHECK_ARG(code_index || n_codes == 1 || n_codes == n_rays);
  FieldArgs a = {};
  a.packed = packed;
  a.code_bias = code_bias;
  a.code_index = code_index;
  a.n_codes = n_codes;
  a.pts = pts;
  a.ro = ro;
  a.rd = rd;
  a.z = z;
  a.n_rays = n_rays;
  a.n_samples = n_samples;
  a.chunk_rows = chunk_rows;
  a.m = n_rays * n_samples;
  CN_CHECK_ARG(cn::ceil_div(a.m, kTile) <= 0x7fffffff);
  for (int i = 0; i < 10; ++i) a.fx[i] = freqs_xyz[i];
  for (int i = 0; i < 4; ++i) a.fd[i] = freqs_dir[i];
  a.raw = raw;
  CN_CHECK_ARG(cn::aligned16(raw));  // float4 rows (include/codenerf.h)
  a.save = save;
  a.masks = masks;
  // fp32: the encoding plane follows the five activation planes (cn_field_train_saved_floats)
  if (fmt == CN_FMT_F32_W16) a.xenc = save + 5 * a.m * 256;
  return fmt == CN_FMT_BF16X3 ? launch_field_x3(pts ? kFromPts : kFromRayZ, a, cn::as_stream(stream))
                              : launch_field_w16(pts ? kFromPts : kFromRayZ, a, cn::as_stream(stream));
}

extern "C" int64_t cn_field_train_saved_floats(int fmt, int64_t m) {
  if (m <= 0 || !(fmt == CN_FMT_F32_W16 || fmt == CN_FMT_BF16X3)) return -1;
  // five (m, 256) activation planes; fp32: then the (m, 64) encoding plane; a 256-float scratch row
  return 5 * m * 256 + (fmt == CN_FMT_F32_W16 ? 64 * m : 0) + 256;
}

extern "C" int cn_field_backward_x3(const float* packed_t, const uint32_t* masks, const float* d_raw,
                                    const float* pts, const float* ro, const float* rd, const float* z,
                                    int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                                    const int64_t* code_index, int64_t n_codes, const float* freqs_xyz,
                                    const float* freqs_dir, float* g_code, float* d_pts, float* d_ro, float* d_rd,
                                    cn_stream_t stream) {
  return cn_field_backward_fused(CN_FMT_BF16X3_T, packed_t, masks, d_raw, pts, ro, rd, z, n_rays, n_samples,
                                 chunk_rows, code_index, n_codes, freqs_xyz, freqs_dir, g_code, d_pts, d_ro, d_rd,
                                 stream);
}

namespace cn {
namespace mlp {
// cn_field_backward_fused's checks and kernel arguments (shared with cn_field_backward_fused_ws).
int fused_backward_args(int fmt_t, const float* packed_t, const uint32_t* masks, const float* d_raw,
                        const float* pts, const float* ro, const float* rd, const float* z, int64_t n_rays,
                        int64_t n_samples, int64_t chunk_rows, const int64_t* code_index, int64_t n_codes,
                        const float* freqs_xyz, const float* freqs_dir, float* g_code, float* d_pts, float* d_ro,
                        float* d_rd, FieldArgs& a) {
  CN_CHECK_ARG(fmt_t == CN_FMT_BF16X3_T || fmt_t == CN_FMT_F32_W16_T);
  CN_CHECK_ARG(packed_t && masks && d_raw && rd && g_code && freqs_xyz && freqs_dir);
  CN_CHECK_ARG(n_rays > 0 && n_samples > 0 && chunk_rows > 0 && n_codes > 0);
  CN_CHECK_ARG(pts || (ro && z));
  CN_CHECK_ARG(!d_pts || pts);
  CN_CHECK_ARG(!d_ro || (ro && z && !pts));
  CN_CHECK_ARG(code_index || n_codes == 1 || n_codes == n_rays);
  // one code row per wave (32 samples x3, 16 samples w16): a single code, or every wave inside one ray
  const int wave_samples = fmt_t == CN_FMT_BF16X3_T ? 32 : 16;
  if (!(n_codes == 1 || n_samples % wave_samples == 0)) return CN_EUNSUPPORTED;
  a = FieldArgs{};
  a.packed = packed_t;
  a.code_index = code_index;
  a.n_codes = n_codes;
  a.pts = pts;
  a.ro = ro;
  a.rd = rd;
  a.z = z;
  a.n_rays = n_rays;
  a.n_samples = n_samples;
  a.chunk_rows = chunk_rows;
  a.m = n_rays * n_samples;
  CN_CHECK_ARG(cn::ceil_div(a.m, kTile) <= 0x7fffffff);
  for (int i = 0; i < 10; ++i) a.fx[i] = freqs_xyz[i];
  for (int i = 0; i < 4; ++i) a.fd[i] = freqs_dir[i];
  a.masks = const_cast<uint32_t*>(masks);
  a.d_raw = d_raw;
  CN_CHECK_ARG(cn::aligned16(d_raw));  // float4 rows (include/codenerf.h)
  a.g_code = g_code;
  a.d_pts = d_pts;
  a.d_ro = d_ro;
  a.d_rd = d_rd;
  return CN_OK;
}
}  // namespace mlp
}  // namespace cn

extern "C" int cn_field_backward_fused(int fmt_t, const float* packed_t, const uint32_t* masks, const float* d_raw,
                                       const float* pts, const float* ro, const float* rd, const float* z,
                                       int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                                       const int64_t* code_index, int64_t n_codes, const float* freqs_xyz,
                                       const float* freqs_dir, float* g_code, float* d_pts, float* d_ro,
                                       float* d_rd, cn_stream_t stream) {
  FieldArgs a;
  const int rc = fused_backward_args(fmt_t, packed_t, masks, d_raw, pts, ro, rd, z, n_rays, n_samples, chunk_rows,
                                     code_index, n_codes, freqs_xyz, freqs_dir, g_code, d_pts, d_ro, d_rd, a);
  if (rc != CN_OK) return rc;
  return fmt_t == CN_FMT_BF16X3_T ? launch_field_x3_bwd(pts ? kFromPts : kFromRayZ, a, cn::as_stream(stream))
                                  : launch_field_w16_bwd(pts ? kFromPts : kFromRayZ, a, cn::as_stream(stream));
}
