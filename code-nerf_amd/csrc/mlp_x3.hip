// 3xbf16-split field kernel: the same fused posenc + CodeNeRF MLP as mlp.hip,
// with every fp32 GEMM x.W computed as  Wh.Xh + Wh.Xl + Wl.Xh  on
// v_mfma_f32_32x32x16_bf16 (fp32 accumulate), where Wh = bf16(W),
// Wl = bf16(W - Wh) (packed once) and Xh/Xl the same split of the activations
// (done in registers at each layer's epilogue).  The dropped Wl.Xl term and the
// lo rounding leave ~2^-17 relative error per product -- far inside the 1e-4
// rendered-RGB tolerance -- at 3/16 of the fp32-MFMA cost: 1,776 MFMAs x 32
// cycles per 32-sample wave tile instead of 4,720 x 64.
//
// Register dataflow as in mlp.hip: a 32x32 fp32 accumulator block's registers
// 8s..8s+7 become k-step s (16 features) of the next layer's B operand after a
// hi/lo split (element j of lane half h = feature 16s + 8(j>>2) + 4h + (j&3) of
// the block, cdna_hip_programming.md section 3), so activations never leave
// registers.  Weight fragments (32 B per lane per output block per k-step: hi
// then lo) stream through a 2 x 72 KiB LDS ring in 22 chunks of <= 4 k-steps.
#include "mlp_common.h"

namespace cn {
namespace mlp {
namespace x3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kSteps[kNumLayers] = {4, 16, 16, 18, 16, 16};   // 16-wide k-steps
constexpr int kNb[kNumLayers] = {8, 8, 9, 8, 8, 1};

// Layout in 16-byte quads: layer l, k-step s, lane L, block ob, {hi, lo}.
__host__ __device__ constexpr int layer_quads(int l) { return kSteps[l] * 64 * kNb[l] * 2; }
__host__ __device__ constexpr int layer_off(int l) { return l == 0 ? 0 : layer_off(l - 1) + layer_quads(l - 1); }
constexpr int kQuads = layer_off(kNumLayers);
constexpr int kBiasXyz1 = kQuads * 4;   // floats
constexpr int kBiasDir1 = kBiasXyz1 + 256;
constexpr int kBiasDir2 = kBiasDir1 + 256;
constexpr int kPackedFloats = kBiasDir2 + 256;

// Input feature of lane half h, element j, k-step s of layer l (-1 = zero pad).
__host__ __device__ constexpr int in_col(int l, int s, int h, int j) {
  if (l == kXyz1) return k_from_enc(8 * s + j, h, 15);
  if (l == kDir1 && s >= 16) {
    const int t = 8 * (s - 16) + j;
    if (t >= 14) return -1;
    const int e = k_from_enc(t, h, 6);
    return e < 0 ? -1 : kCode + e;
  }
  return acc_row(s >> 1, 8 * (s & 1) + j, h);
}

__device__ __forceinline__ unsigned short bf16_bits(float x) {
  const __bf16 b = static_cast<__bf16>(x);
  return __builtin_bit_cast(unsigned short, b);
}

__global__ void pack_x3_kernel(Params P, float* __restrict__ packed) {
  unsigned short* q16 = reinterpret_cast<unsigned short*>(packed);
  const int n_elems = kQuads * 8;  // bf16 elements
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n_elems + 768;
       idx += gridDim.x * blockDim.x) {
    if (idx >= n_elems) {
      const int j = idx - n_elems;
      packed[kBiasXyz1 + j] =
          j < 256 ? P.p[kBXyz1][j] : (j < 512 ? P.p[kBDir1][j - 256] : P.p[kBDir2][j - 512]);
      continue;
    }
    const int quad = idx >> 3, j = idx & 7;
    constexpr int offs[kNumLayers + 1] = {layer_off(0), layer_off(1), layer_off(2), layer_off(3),
                                          layer_off(4), layer_off(5), layer_off(6)};
    int l = 0;
    while (l + 1 < kNumLayers && quad >= offs[l + 1]) ++l;
    int rem = quad - offs[l];
    const int part = rem & 1;  // 0 hi, 1 lo
    rem >>= 1;
    const int nb = kNb[l];
    const int ob = rem % nb;
    rem /= nb;
    const int lane = rem % 64, s = rem / 64;
    const int i = lane & 31, h = lane >> 5;
    const int col = in_col(l, s, h, j);
    int row = -1, in_dim = 0;
    const float* W = nullptr;
    switch (l) {
      case kXyz1: W = P.p[kWXyz1]; in_dim = kDimXyz; row = 32 * ob + i; break;
      case kXyz2: W = P.p[kWXyz2]; in_dim = kHidden + kCode; row = 32 * ob + i; break;
      case kOut: W = P.p[kWOut]; in_dim = kHidden + kCode;
        row = ob < 8 ? 1 + 32 * ob + i : ((ob == 8 && i == 0) ? 0 : -1); break;
      case kDir1: W = P.p[kWDir1]; in_dim = kCode + kDimDir; row = 32 * ob + i; break;
      case kDir2: W = P.p[kWDir2]; in_dim = kHidden; row = 32 * ob + i; break;
      default: W = P.p[kWRgb]; in_dim = kHidden + kCode; row = (ob == 0 && i < 3) ? i : -1; break;
    }
    const float w = (row >= 0 && col >= 0) ? W[row * in_dim + col] : 0.0f;
    const __bf16 hi = static_cast<__bf16>(w);
    const float lo = w - static_cast<float>(hi);
    q16[idx] = part == 0 ? bf16_bits(w) : bf16_bits(lo);
  }
}

// ---------------------------------------------------------------- kernel

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kTile = 32 * kWaves;
constexpr int kChunkSteps = 4;
constexpr int kMaxChunkQuads = kChunkSteps * 64 * 9 * 2;   // fc_out chunk: 72 KiB

struct Chunk {
  int layer, s0, steps;
};
constexpr int kNumChunks = 1 + 4 + 4 + 5 + 4 + 4;
__host__ __device__ constexpr Chunk chunk_at(int c) {
  return c < 1 ? Chunk{kXyz1, 0, 4}
       : c < 5 ? Chunk{kXyz2, 4 * (c - 1), 4}
       : c < 9 ? Chunk{kOut, 4 * (c - 5), 4}
       : c < 14 ? Chunk{kDir1, 4 * (c - 9), c == 13 ? 2 : 4}
       : c < 18 ? Chunk{kDir2, 4 * (c - 14), 4}
                : Chunk{kRgb, 4 * (c - 18), 4};
}
__host__ __device__ constexpr int chunk_quads(int c) { return chunk_at(c).steps * 64 * kNb[chunk_at(c).layer] * 2; }
__host__ __device__ constexpr int chunk_src(int c) {
  return layer_off(chunk_at(c).layer) + chunk_at(c).s0 * 64 * kNb[chunk_at(c).layer] * 2;
}
__host__ __device__ constexpr int chunk_loads(int c) { return (chunk_quads(c) + kThreads - 1) / kThreads; }
constexpr int kMaxLoads = (kMaxChunkQuads / kThreads + 1) / 2;  // 9 (half a chunk)

struct State {
  bf16x8 bh[16], bl[16];  // B operands (hi / lo) of the current layer's 16 k-steps
  bf16x8 dh[2], dl[2];    // view-direction encoding k-steps of layer_dir1
  floatx16 acc[9];
  float4 stage[kMaxLoads];
  float sigma;
  int lane, h;
  int64_t cb_row;
  float vd[3];
};

__device__ __forceinline__ void split8(const float* v, bf16x8& hi, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const __bf16 b = static_cast<__bf16>(v[j]);
    hi[j] = b;
    lo[j] = static_cast<__bf16>(v[j] - static_cast<float>(b));
  }
}

// The next chunk is staged through registers in two halves (one per half of
// the current chunk's k-steps) to keep the staging to 9 float4 per thread.
constexpr int kParts = 2;
template <int C, int PART>
__device__ __forceinline__ void load_chunk(State& s, const float* __restrict__ packed) {
  constexpr int n = chunk_quads(C);
  constexpr int nl = chunk_loads(C);
  constexpr int i0 = PART * ((nl + kParts - 1) / kParts);
  constexpr int i1 = (PART + 1) * ((nl + kParts - 1) / kParts) < nl ? (PART + 1) * ((nl + kParts - 1) / kParts) : nl;
  const float4* src = reinterpret_cast<const float4*>(packed) + chunk_src(C);
#pragma unroll
  for (int i = i0; i < i1; ++i) {
    const int q = i * kThreads + threadIdx.x;
    if (n % kThreads == 0 || q < n) s.stage[i - i0] = src[q];
  }
}

template <int C, int PART>
__device__ __forceinline__ void store_chunk(State& s, float4* lds) {
  constexpr int n = chunk_quads(C);
  constexpr int nl = chunk_loads(C);
  constexpr int i0 = PART * ((nl + kParts - 1) / kParts);
  constexpr int i1 = (PART + 1) * ((nl + kParts - 1) / kParts) < nl ? (PART + 1) * ((nl + kParts - 1) / kParts) : nl;
#pragma unroll
  for (int i = i0; i < i1; ++i) {
    const int q = i * kThreads + threadIdx.x;
    if (n % kThreads == 0 || q < n) lds[q] = s.stage[i - i0];
  }
}

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

template <int C, int T>
__device__ __forceinline__ void mfma_step(State& s, const float4* lds) {
  constexpr Chunk ch = chunk_at(C);
  constexpr int L = ch.layer;
  constexpr int nb = kNb[L];
  constexpr int ks = ch.s0 + T;  // k-step within the layer
  const bf16x8 bh = (L == kDir1 && ks >= 16) ? s.dh[ks - 16] : s.bh[ks < 16 ? ks : 0];
  const bf16x8 bl = (L == kDir1 && ks >= 16) ? s.dl[ks - 16] : s.bl[ks < 16 ? ks : 0];
  const float4* ap = lds + (T * 64 + s.lane) * nb * 2;
#pragma unroll
  for (int ob = 0; ob < nb; ++ob) {
    const float4 qh = ap[2 * ob], ql = ap[2 * ob + 1];
    const bf16x8 ah = __builtin_bit_cast(bf16x8, qh);
    const bf16x8 al = __builtin_bit_cast(bf16x8, ql);
    s.acc[ob] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, s.acc[ob], 0, 0, 0);
    s.acc[ob] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, s.acc[ob], 0, 0, 0);
    s.acc[ob] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, s.acc[ob], 0, 0, 0);
  }
}

template <int C, int T, int T1>
__device__ __forceinline__ void mfma_steps(State& s, const float4* lds) {
  if constexpr (T < T1) {
    mfma_step<C, T>(s, lds);
    mfma_steps<C, T + 1, T1>(s, lds);
  }
}

template <int L>
__device__ __forceinline__ void finish_layer(State& s) {
  if constexpr (L == kRgb) {
    return;
  } else {
    if constexpr (L == kOut) s.sigma = s.acc[8][0];
#pragma unroll
    for (int b = 0; b < 8; ++b) {
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        float v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = s.acc[b][8 * sp + j];
          v[j] = (L == kOut) ? x : fmaxf(x, 0.0f);  // feat = fc_out[1:] has no activation
        }
        split8(v, s.bh[2 * b + sp], s.bl[2 * b + sp]);
      }
    }
  }
}

template <int MODE, int C>
__device__ __forceinline__ void run_chunks(State& s, const FieldArgs& a, float4* lds0, float4* lds1) {
  if constexpr (C < kNumChunks) {
    constexpr Chunk ch = chunk_at(C);
    float4* cur = (C & 1) ? lds1 : lds0;
    float4* nxt = (C & 1) ? lds0 : lds1;
    if constexpr (ch.s0 == 0) init_acc<ch.layer>(s, a);
    if constexpr (C + 1 < kNumChunks) load_chunk<C + 1, 0>(s, a.packed);
    constexpr int half = (ch.steps + 1) / 2;
    mfma_steps<C, 0, half>(s, cur);
    if constexpr (C + 1 < kNumChunks) {
      store_chunk<C + 1, 0>(s, nxt);
      load_chunk<C + 1, 1>(s, a.packed);
    }
    mfma_steps<C, half, ch.steps>(s, cur);
    constexpr bool last_of_layer = (C + 1 == kNumChunks) || chunk_at(C + 1).layer != ch.layer;
    if constexpr (last_of_layer) finish_layer<ch.layer>(s);
    // view-direction encoding for layer_dir1, made while the fc_out accumulators are dead
    if constexpr (last_of_layer && ch.layer == kOut && MODE != kFromEncoded) {
      float v[16];
      encode_pairs<6, 4>(s.vd, a.fd, s.h, v);
      v[14] = 0.0f;
      v[15] = 0.0f;
      split8(v, s.dh[0], s.dl[0]);
      split8(v + 8, s.dh[1], s.dl[1]);
    }
    if constexpr (C + 1 < kNumChunks) {
      store_chunk<C + 1, 1>(s, nxt);
      __syncthreads();
    }
    run_chunks<MODE, C + 1>(s, a, lds0, lds1);
  }
}

template <int MODE>
__global__ __launch_bounds__(kThreads, 1) void field_x3_kernel(FieldArgs a) {
  __shared__ float4 lds[2][kMaxChunkQuads];
  State s;
  s.lane = threadIdx.x & 63;
  s.h = s.lane >> 5;
  const int wave = threadIdx.x >> 6;
  const int64_t row = (int64_t)blockIdx.x * kTile + wave * 32 + (s.lane & 31);
  const bool valid = row < a.m;
  const int64_t rc = valid ? row : a.m - 1;

  const SampleIn in = decode_sample<MODE>(a, rc);
  float enc[32];
  if constexpr (MODE == kFromEncoded) {
    const float* xr = a.x + rc * (kDimXyz + kDimDir);
    gather_pairs<15>(xr, 0, s.h, enc);
    float d[16];
    gather_pairs<6>(xr, kDimXyz, s.h, d);
    d[14] = 0.0f;
    d[15] = 0.0f;
    split8(d, s.dh[0], s.dl[0]);
    split8(d + 8, s.dh[1], s.dl[1]);
  } else {
    encode_pairs<15, 10>(in.x, a.fx, s.h, enc);
#pragma unroll
    for (int j = 0; j < 3; ++j) s.vd[j] = in.vd[j];
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) split8(enc + 8 * k, s.bh[k], s.bl[k]);
  s.cb_row = code_row(a, in.code_of) * kCbStride;

  load_chunk<0, 0>(s, a.packed);
  store_chunk<0, 0>(s, lds[0]);
  load_chunk<0, 1>(s, a.packed);
  store_chunk<0, 1>(s, lds[0]);
  __syncthreads();
  run_chunks<MODE, 0>(s, a, lds[0], lds[1]);

  if (valid && s.h == 0) {
    float4 o;
    o.x = s.acc[0][0];
    o.y = s.acc[0][1];
    o.z = s.acc[0][2];
    o.w = s.sigma;
    reinterpret_cast<float4*>(a.raw)[row] = o;
  }
}

}  // namespace x3

int64_t packed_floats_x3() { return x3::kPackedFloats; }

int launch_pack_x3(const Params& P, float* packed, hipStream_t st) {
  const int64_t n = (int64_t)x3::kQuads * 8 + 768;
  hipLaunchKernelGGL(x3::pack_x3_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0, st, P, packed);
  return cn::launch_status();
}

int launch_field_x3(int mode, FieldArgs& a, hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(cn::ceil_div(a.m, x3::kTile));
  switch (mode) {
    case kFromPts: hipLaunchKernelGGL(x3::field_x3_kernel<kFromPts>, dim3(grid), dim3(x3::kThreads), 0, st, a); break;
    case kFromRayZ: hipLaunchKernelGGL(x3::field_x3_kernel<kFromRayZ>, dim3(grid), dim3(x3::kThreads), 0, st, a); break;
    default: hipLaunchKernelGGL(x3::field_x3_kernel<kFromEncoded>, dim3(grid), dim3(x3::kThreads), 0, st, a); break;
  }
  return cn::launch_status();
}

}  // namespace mlp
}  // namespace cn
