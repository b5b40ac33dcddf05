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
//
// Weight stream: 44 chunks of <= 2 k-steps (<= 36 KiB) through a 4-slot LDS
// ring filled by LDS-DMA (global_load_lds, 1 KiB per wave-instruction, no
// VGPR staging).  Chunk c+3 is issued when chunk c starts, so three chunks
// (~4.6 K MFMA cycles) are in flight; one raw s_barrier per chunk, preceded by
// a counted `s_waitcnt vmcnt(N)` that retires only this wave's DMA for chunk c.
// No ordinary global load is live inside the stream (hipcc would wait
// vmcnt(0) for it, draining the ring): per-layer biases are read with scalar
// loads (see init_acc).

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kTile = 32 * kWaves;
constexpr int kChunkSteps = 2;
constexpr int kSlotQuads = kChunkSteps * 64 * 9 * 2;   // 36 KiB: an fc_out chunk
constexpr int kSlots = 4;
constexpr int kAhead = kSlots - 1;                      // chunks in flight
constexpr int kLdsFloats = kSlots * kSlotQuads * 4;    // 144 KiB ring

struct Chunk {
  int layer, s0, steps;
};
// chunk c -> (layer, first k-step, k-steps); layer_dir1 ends with its 2 view-direction k-steps
constexpr int kChunksPerLayer[kNumLayers] = {2, 8, 8, 9, 8, 8};
constexpr int kNumChunks = 2 + 8 + 8 + 9 + 8 + 8;
__host__ __device__ constexpr Chunk chunk_at(int c) {
  int l = 0;
  while (c >= kChunksPerLayer[l]) c -= kChunksPerLayer[l++];
  return Chunk{l, 2 * c, 2};
}
__host__ __device__ constexpr int chunk_quads(int c) { return chunk_at(c).steps * 64 * kNb[chunk_at(c).layer] * 2; }
__host__ __device__ constexpr int chunk_src(int c) {
  return layer_off(chunk_at(c).layer) + chunk_at(c).s0 * 64 * kNb[chunk_at(c).layer] * 2;
}
// wave-instructions (1 KiB = 64 quads each) per chunk and per wave
__host__ __device__ constexpr int chunk_dma(int c) { return chunk_quads(c) / 64; }
__host__ __device__ constexpr int wave_dma(int c, int w) {
  return c >= kNumChunks ? 0 : (chunk_dma(c) - w + kWaves - 1) / kWaves;
}

struct State {
  bf16x8 bh[16], bl[16];  // B operands (hi / lo) of the current layer's 16 k-steps
  bf16x8 dh[2], dl[2];    // view-direction encoding k-steps of layer_dir1
  floatx16 acc[9];
  float sigma;
  int lane, h, wave;
  int crow;               // this lane's code-bias row
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

typedef __attribute__((address_space(3))) void* lds_ptr_t;
typedef const __attribute__((address_space(1))) void* gbl_ptr_t;

// Issue this wave's share of chunk C's DMA into ring slot C % kSlots.
template <int C>
__device__ __forceinline__ void issue_chunk(const State& s, const float* __restrict__ packed, float* lds) {
  if constexpr (C < kNumChunks) {
    constexpr int n = chunk_dma(C);
    const float4* src = reinterpret_cast<const float4*>(packed) + chunk_src(C);
    float4* slot = reinterpret_cast<float4*>(lds) + (C % kSlots) * kSlotQuads;
#pragma unroll
    for (int i = 0; i < (n + kWaves - 1) / kWaves; ++i) {
      const int ins = i * kWaves + s.wave;  // wave-uniform
      if (n % kWaves == 0 || ins < n) {
        __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src + ins * 64 + s.lane), (lds_ptr_t)(slot + ins * 64), 16, 0, 0);
      }
    }
  }
}

// Wait until this wave's DMA for chunk C has landed (later chunks stay in flight).
// One asm statement: the counted wait, this wave's LDS reads retired, the barrier.
// Nothing (no LDS read of chunk C) can be scheduled across it.
template <int C, int W>
__device__ __forceinline__ void wait_chunk_w() {
  constexpr int pending = wave_dma(C + 1, W) + wave_dma(C + 2, W);
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(pending) : "memory");
}
template <int C>
__device__ __forceinline__ void wait_chunk(int wave) {
  // the per-wave DMA count differs only when a chunk's instruction count is not a
  // multiple of 4; branch on the (wave-uniform) wave index with constant counts
  switch (wave) {
    case 0: wait_chunk_w<C, 0>(); break;
    case 1: wait_chunk_w<C, 1>(); break;
    case 2: wait_chunk_w<C, 2>(); break;
    default: wait_chunk_w<C, 3>(); break;
  }
}

typedef const __attribute__((address_space(4))) float* const_fptr;

// acc[ob][r] = bias[acc_row(ob, r, h)] (or keep acc where !take), from a
// wave-uniform bias vector read with scalar loads.
template <int L>
__device__ __forceinline__ void bias_from_row(State& s, const float* ub, bool take) {
  const_fptr cp = (const_fptr)ub;
  if constexpr (L == kRgb) {
    const float b0 = cp[0], b1 = cp[1], b2 = cp[2];
    if (take && s.h == 0) {
      s.acc[0][0] = b0;
      s.acc[0][1] = b1;
      s.acc[0][2] = b2;
    }
  } else {
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float v0 = cp[acc_row(ob, r, 0)], v1 = cp[acc_row(ob, r, 1)];
        const float v = s.h ? v1 : v0;
        s.acc[ob][r] = take ? v : s.acc[ob][r];
      }
    }
    if constexpr (L == kOut) {
      const float sg = cp[kCbSigma - kCbFeat];
      if (take && s.h == 0) s.acc[8][0] = sg;
    }
  }
}

// Bias-initialised accumulators (acc = b, then acc += W x).  Every bias read is
// a scalar load (s_load through the constant cache: lgkmcnt, so the DMA ring's
// vmcnt accounting is untouched).  Per-code biases loop over the distinct code
// rows of the wave (one pass when all 32 samples share an object).
template <int L>
__device__ __forceinline__ void init_acc(State& s, const FieldArgs& a) {
  constexpr int cb_off = L == kXyz2 ? kCbXyz2 : L == kOut ? kCbFeat : L == kRgb ? kCbRgb : 0;
  constexpr bool from_code = (L == kXyz2 || L == kOut || L == kRgb);
  constexpr int const_off = L == kXyz1 ? kBiasXyz1 : L == kDir1 ? kBiasDir1 : kBiasDir2;
#pragma unroll
  for (int ob = 0; ob < (L == kOut ? 9 : (L == kRgb ? 1 : 8)); ++ob) s.acc[ob] = floatx16{0};
  if constexpr (!from_code) {
    bias_from_row<L>(s, a.packed + const_off, true);
  } else {
    unsigned long long todo = ~0ull;
    while (todo) {
      const int first = __builtin_ctzll(todo);
      const int row = __builtin_amdgcn_readfirstlane(__shfl(s.crow, first));
      const bool mine = (s.crow == row);
      bias_from_row<L>(s, a.code_bias + (int64_t)row * kCbStride + cb_off, mine);
      todo &= ~__ballot(mine);
    }
  }
}

template <int C, int T>
__device__ __forceinline__ bf16x8 b_hi(const State& s) {
  constexpr Chunk ch = chunk_at(C);
  constexpr int ks = ch.s0 + T;
  return (ch.layer == kDir1 && ks >= 16) ? s.dh[ks >= 16 ? ks - 16 : 0] : s.bh[ks < 16 ? ks : 0];
}
template <int C, int T>
__device__ __forceinline__ bf16x8 b_lo(const State& s) {
  constexpr Chunk ch = chunk_at(C);
  constexpr int ks = ch.s0 + T;
  return (ch.layer == kDir1 && ks >= 16) ? s.dl[ks >= 16 ? ks - 16 : 0] : s.bl[ks < 16 ? ks : 0];
}

// A chunk's MFMAs in units of (k-step, group of <= 3 output blocks): the A
// fragments (hi + lo, 8 VGPRs per block) of unit u+1 are read from LDS while
// unit u's 3 x |group| MFMAs run -- two 24-VGPR buffers in flight.
constexpr int kGroup = 3;
template <int C>
__host__ __device__ constexpr int groups() { return (kNb[chunk_at(C).layer] + kGroup - 1) / kGroup; }
template <int C>
__host__ __device__ constexpr int units() { return chunk_at(C).steps * groups<C>(); }

template <int C, int U>
__device__ __forceinline__ void load_unit(const State& s, const float* lds, bf16x8* ah, bf16x8* al) {
  if constexpr (U < units<C>()) {
    constexpr int nb = kNb[chunk_at(C).layer];
    constexpr int T = U / groups<C>(), g = U % groups<C>();
    const float4* ap = reinterpret_cast<const float4*>(lds) + (C % kSlots) * kSlotQuads + (T * 64 + s.lane) * nb * 2;
#pragma unroll
    for (int i = 0; i < kGroup; ++i) {
      constexpr int dummy = 0;
      (void)dummy;
      if (g * kGroup + i < nb) {
        ah[i] = __builtin_bit_cast(bf16x8, ap[2 * (g * kGroup + i)]);
        al[i] = __builtin_bit_cast(bf16x8, ap[2 * (g * kGroup + i) + 1]);
      }
    }
  }
}

template <int C, int U>
__device__ __forceinline__ void mfma_unit(State& s, const bf16x8* ah, const bf16x8* al) {
  constexpr int nb = kNb[chunk_at(C).layer];
  constexpr int T = U / groups<C>(), g = U % groups<C>();
  const bf16x8 bh = b_hi<C, T>(s), bl = b_lo<C, T>(s);
#pragma unroll
  for (int i = 0; i < kGroup; ++i) {
    if (g * kGroup + i < nb) {
      floatx16& acc = s.acc[g * kGroup + i];
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bh, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[i], bl, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al[i], bh, acc, 0, 0, 0);
    }
  }
}

template <int C, int U>
__device__ __forceinline__ void chunk_units(State& s, const float* lds, bf16x8* ah_cur, bf16x8* al_cur,
                                            bf16x8* ah_nxt, bf16x8* al_nxt) {
  if constexpr (U < units<C>()) {
    load_unit<C, U + 1>(s, lds, ah_nxt, al_nxt);
    __builtin_amdgcn_sched_barrier(0);
    mfma_unit<C, U>(s, ah_cur, al_cur);
    __builtin_amdgcn_sched_barrier(0);
    chunk_units<C, U + 1>(s, lds, ah_nxt, al_nxt, ah_cur, al_cur);
  }
}

template <int C>
__device__ __forceinline__ void chunk_mfma(State& s, const float* lds) {
  bf16x8 ah0[kGroup], al0[kGroup], ah1[kGroup], al1[kGroup];
  load_unit<C, 0>(s, lds, ah0, al0);
  chunk_units<C, 0>(s, lds, ah0, al0, ah1, al1);
}

template <int L>
__device__ __forceinline__ void finish_layer(State& s) {
  if constexpr (L != kRgb) {
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
__device__ __forceinline__ void run_chunks(State& s, const FieldArgs& a, float* lds) {
  if constexpr (C < kNumChunks) {
    constexpr Chunk ch = chunk_at(C);
    // chunk C landed for every wave, and every wave is done with chunk C-1
    wait_chunk<C>(s.wave);
    __builtin_amdgcn_sched_barrier(0);
    issue_chunk<C + kAhead>(s, a.packed, lds);   // into the slot chunk C-1 used
    if constexpr (ch.s0 == 0) init_acc<ch.layer>(s, a);
    chunk_mfma<C>(s, lds);
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
    run_chunks<MODE, C + 1>(s, a, lds);
  }
}

template <int MODE>
__global__ __launch_bounds__(kThreads, 1) void field_x3_kernel(FieldArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[kLdsFloats];  // the ONE LDS object
  State s;
  s.lane = threadIdx.x & 63;
  s.h = s.lane >> 5;
  s.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t row = (int64_t)blockIdx.x * kTile + s.wave * 32 + (s.lane & 31);
  const bool valid = row < a.m;
  const int64_t rc = valid ? row : a.m - 1;

  // ---- per-sample inputs (ordinary loads, all before the DMA stream starts)
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
  s.crow = static_cast<int>(code_row(a, in.code_of));

  // ---- weight stream: every input load has landed (an s_waitcnt the compiler
  // sees, so it tracks nothing stale into the DMA stream); prime the ring
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  issue_chunk<0>(s, a.packed, lds);
  issue_chunk<1>(s, a.packed, lds);
  issue_chunk<2>(s, a.packed, lds);
  run_chunks<MODE, 0>(s, a, lds);

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
