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
// registers.
//
// Weight stream.  Every chunk has ONE format -- 2 k-steps x 9 block slots x
// {hi, lo} x 64 lanes quads = 36 KiB, fragment-major so a wave's ds_read_b128 of
// one fragment is 1 KiB contiguous (bank-conflict free) -- and the chunks lie in stream order in the
// packed buffer, so chunk c is just `packed + c * 36 KiB`.  A 4-slot LDS ring is
// filled by LDS-DMA (global_load_lds, 1 KiB per wave-instruction, 9 per wave per
// chunk); chunk c+3 is issued when chunk c starts, and a constant
// `s_waitcnt vmcnt(18)` + s_barrier retires chunk c (two dummy chunks at the end
// keep the count constant).  No ordinary global load is live in the stream
// (biases are scalar loads), so the counted waits are exact.
//
// Code size.  The four 256-input layers (layer_xyz2, fc_out, layer_dir1's feature
// part, layer_dir2) run through ONE runtime loop whose body is a single unrolled
// 16-k-step layer: fully unrolling all six layers (~140 KiB of code) made the
// kernel instruction-fetch bound (ablation: removing every MFMA saved only 4 %).
// fc_out's 9th output block (sigma) is a uniform branch.
#include "mlp_common.h"

namespace cn {
namespace mlp {
namespace x3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));

constexpr int kSlotBlocks = 9;
constexpr int kQuadsPerStep = 64 * kSlotBlocks * 2;      // one k-step of a chunk
constexpr int kChunkQuads = 2 * kQuadsPerStep;            // 2304 quads = 36 KiB
constexpr int kDmaPerWave = kChunkQuads / 64 / 4;        // 9
// stream: L0 2 | L1 8 | L2 8 | L3 8 + 1 (view dir) | L4 8 | L5 1 | 2 dummies
constexpr int kChunkL1 = 2, kChunkL2 = 10, kChunkL3 = 18, kChunkDir = 26, kChunkL4 = 27, kChunkRgb = 35;
constexpr int kRealChunks = 36;
constexpr int kStreamChunks = kRealChunks + 2;
constexpr int kQuads = kStreamChunks * kChunkQuads;
constexpr int kBiasXyz1 = kQuads * 4;  // floats
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

// (chunk, step-in-chunk T, slot j) -> (layer, k-step, output block); -1 layer = zeros
__device__ void chunk_map(int c, int T, int j, int& l, int& ks, int& ob) {
  l = -1;
  ks = 0;
  ob = j;
  if (c < kChunkL1) { l = kXyz1; ks = 2 * c + T; }
  else if (c < kChunkL2) { l = kXyz2; ks = 2 * (c - kChunkL1) + T; }
  else if (c < kChunkL3) { l = kOut; ks = 2 * (c - kChunkL2) + T; }
  else if (c < kChunkDir) { l = kDir1; ks = 2 * (c - kChunkL3) + T; }
  else if (c == kChunkDir) { l = kDir1; ks = 16 + T; }
  else if (c < kChunkRgb) { l = kDir2; ks = 2 * (c - kChunkL4) + T; }
  else if (c == kChunkRgb) { l = kRgb; ks = 9 * T + j; ob = 0; if (ks >= 16) l = -1; }
  if (l >= 0 && l != kOut && ob >= 8) l = -1;
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
    const int quad = idx >> 3, e = idx & 7;
    const int c = quad / kChunkQuads;
    int r = quad % kChunkQuads;
    const int T = r / kQuadsPerStep;
    r %= kQuadsPerStep;
    const int frag = r / 64, lane = r % 64;  // fragment-major: 1 KiB per (slot, hi|lo)
    const int slot = frag >> 1, part = frag & 1;
    int l, ks, ob;
    chunk_map(c, T, slot, l, ks, ob);
    float w = 0.0f;
    if (l >= 0) {
      const int i = lane & 31, h = lane >> 5;
      const int col = in_col(l, ks, h, e);
      int row = -1, in_dim = 0;
      const float* W = nullptr;
      switch (l) {
        case kXyz1: W = P.p[kWXyz1]; in_dim = kDimXyz; row = 32 * ob + i; break;
        case kXyz2: W = P.p[kWXyz2]; in_dim = kHidden + kCode; row = 32 * ob + i; break;
        case kOut: W = P.p[kWOut]; in_dim = kHidden + kCode;
          row = ob < 8 ? 1 + 32 * ob + i : (i == 0 ? 0 : -1); break;
        case kDir1: W = P.p[kWDir1]; in_dim = kCode + kDimDir; row = 32 * ob + i; break;
        case kDir2: W = P.p[kWDir2]; in_dim = kHidden; row = 32 * ob + i; break;
        default: W = P.p[kWRgb]; in_dim = kHidden + kCode; row = i < 3 ? i : -1; break;
      }
      if (row >= 0 && col >= 0) w = W[row * in_dim + col];
    }
    const __bf16 hi = static_cast<__bf16>(w);
    const float lo = w - static_cast<float>(hi);
    q16[idx] = part == 0 ? bf16_bits(w) : bf16_bits(lo);
  }
}

// ---------------------------------------------------------------- kernel

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kTile = 32 * kWaves;
constexpr int kSlots = 4;
constexpr int kLdsQuads = kSlots * kChunkQuads;  // 144 KiB ring

struct State {
  bf16x8 bh[16], bl[16];  // B operands (hi / lo) of the current layer's 16 k-steps
  bf16x8 dh[2], dl[2];    // view-direction encoding k-steps of layer_dir1
  floatx16 acc[9];
  float sigma;
  int lane, h, wave;
  int crow;               // this lane's code-bias row
  bool uniform_code;      // all 32 samples of the wave use one code row
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
typedef const __attribute__((address_space(4))) float* const_fptr;

// Issue this wave's 9 DMA instructions of chunk c into ring slot c % 4.
__device__ __forceinline__ void issue_chunk(const State& s, const float* __restrict__ packed, float4* lds, int c) {
  const float4* src = reinterpret_cast<const float4*>(packed) + c * kChunkQuads + s.wave * 64 + s.lane;
  float4* slot = lds + (c & (kSlots - 1)) * kChunkQuads + s.wave * 64;
#pragma unroll
  for (int i = 0; i < kDmaPerWave; ++i) {
#ifndef CN_ABLATE_NO_DMA
    __builtin_amdgcn_global_load_lds((gbl_ptr_t)(src + i * 256), (lds_ptr_t)(slot + i * 256), 16, 0, 0);
#endif
  }
}

// Chunk c landed for every wave and every wave is done with chunk c-1 (its slot
// is refilled next): one asm statement, so no LDS read can be scheduled across it.
__device__ __forceinline__ void chunk_barrier() {
#ifdef CN_ABLATE_NO_DMA
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(2 * kDmaPerWave) : "memory");
#endif
}

// Biases.  acc starts as b (1 x 32 rows) via ONE MFMA per output block: A holds
// {bf16(b_i), bf16(b_i - hi)} at k = 0, 1 (lane half 0), B holds ones at k = 0, 1
// for every sample, so D = hi + lo in fp32.  The bias vectors sit in LDS after the
// ring (constants + each wave's code row, staged before the DMA stream) and are
// read by inline-asm ds_reads: hipcc cannot prove them disjoint from the in-flight
// DMA and would otherwise wait vmcnt(0), draining the ring.  A wave whose samples
// use several code rows takes per-lane vector loads instead (slow path, rare:
// S < 32 with per-ray codes).
constexpr int kBiasLds = 768 + kWaves * kCbStride;

__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return static_cast<unsigned>(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) void*)p));
}

// 8 floats at p + 32*ob (ob = 0..7), one LDS round trip, invisible to hipcc's waitcnt pass.
__device__ __forceinline__ void lds_read8_stride32(const float* p, float* v) {
  asm volatile(
      "ds_read_b32 %0, %8\n\tds_read_b32 %1, %8 offset:128\n\tds_read_b32 %2, %8 offset:256\n\t"
      "ds_read_b32 %3, %8 offset:384\n\tds_read_b32 %4, %8 offset:512\n\tds_read_b32 %5, %8 offset:640\n\t"
      "ds_read_b32 %6, %8 offset:768\n\tds_read_b32 %7, %8 offset:896\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(lds_addr(p))
      : "memory");
}

__device__ __forceinline__ float lds_read1(const float* p) {
  float v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}

__device__ __forceinline__ void bias_mfma(floatx16& acc, float v, bf16x8 one) {
  bf16x8 f = {};
  const __bf16 hi = static_cast<__bf16>(v);
  f[0] = hi;
  f[1] = static_cast<__bf16>(v - static_cast<float>(hi));
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f, one, floatx16{0}, 0, 0, 0);
}

__device__ __forceinline__ void init_acc(State& s, const FieldArgs& a, const float* blds, int layer) {
#ifdef CN_ABLATE_NO_BIAS
#pragma unroll
  for (int ob = 0; ob < 9; ++ob) s.acc[ob] = floatx16{0};
  return;
#endif
  const bool per_code = (layer == kXyz2 || layer == kOut || layer == kRgb);
  const int i = s.lane & 31;
  if (!per_code || s.uniform_code) {
    bf16x8 one = {};
    if (s.h == 0) {
      one[0] = static_cast<__bf16>(1.0f);
      one[1] = static_cast<__bf16>(1.0f);
    }
    const float* src = per_code ? blds + 768 + s.wave * kCbStride
                                : blds + (layer == kXyz1 ? 0 : (layer == kDir1 ? 256 : 512));
    if (layer == kRgb) {
      const float v = lds_read1(src + kCbRgb + (i < 3 ? i : 0));
      bias_mfma(s.acc[0], (s.h == 0 && i < 3) ? v : 0.0f, one);
      return;
    }
    const int off = per_code ? (layer == kXyz2 ? kCbXyz2 : kCbFeat) : 0;
    float v[8];
    lds_read8_stride32(src + off + i, v);
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) bias_mfma(s.acc[ob], s.h == 0 ? v[ob] : 0.0f, one);
    if (layer == kOut) {
      const float sg = lds_read1(src + kCbSigma);
      bias_mfma(s.acc[8], (s.h == 0 && i == 0) ? sg : 0.0f, one);
    }
    return;
  }
  // slow path: per-lane code rows
  const float* base = a.code_bias + (int64_t)s.crow * kCbStride;
#pragma unroll
  for (int ob = 0; ob < 9; ++ob) s.acc[ob] = floatx16{0};
  if (layer == kRgb) {
    if (s.h == 0) {
      s.acc[0][0] = base[kCbRgb];
      s.acc[0][1] = base[kCbRgb + 1];
      s.acc[0][2] = base[kCbRgb + 2];
    }
  } else {
    const float* b = base + (layer == kXyz2 ? kCbXyz2 : kCbFeat);
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 v = *reinterpret_cast<const float4*>(b + 32 * ob + 8 * q + 4 * s.h);
        s.acc[ob][4 * q + 0] = v.x;
        s.acc[ob][4 * q + 1] = v.y;
        s.acc[ob][4 * q + 2] = v.z;
        s.acc[ob][4 * q + 3] = v.w;
      }
    }
    if (layer == kOut && s.h == 0) s.acc[8][0] = base[kCbSigma];
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): nothing pending leaks past the branch
}

// A fragments of slot blocks [J0, J0+3) of k-step T of the chunk in `slot`.
template <int T, int J0>
__device__ __forceinline__ void load_a(const State& s, const float4* slot, bf16x8* ah, bf16x8* al) {
  const float4* ap = slot + T * kQuadsPerStep + s.lane;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    ah[i] = __builtin_bit_cast(bf16x8, ap[(2 * (J0 + i)) * 64]);
    al[i] = __builtin_bit_cast(bf16x8, ap[(2 * (J0 + i) + 1) * 64]);
  }
}

__device__ __forceinline__ void mfma3(floatx16& acc, bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl) {
#ifdef CN_ABLATE_NO_MFMA
  asm volatile("" ::"v"(ah), "v"(al), "v"(bh), "v"(bl));
#else
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
#endif
}

// One 2-k-step chunk against 8 (+ block 8 when with9) output blocks.  The A
// fragments of the next group of 3 blocks are read while the current group's
// MFMAs run (two 24-VGPR buffers).
__device__ __forceinline__ void chunk_mfma(State& s, const float4* slot, bf16x8 bh0, bf16x8 bl0, bf16x8 bh1,
                                           bf16x8 bl1, bool with9) {
  bf16x8 ah[3], al[3], nh[3], nl[3];
  load_a<0, 0>(s, slot, ah, al);
  load_a<0, 3>(s, slot, nh, nl);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 3; ++i) mfma3(s.acc[i], ah[i], al[i], bh0, bl0);
  __builtin_amdgcn_sched_barrier(0);
  load_a<0, 6>(s, slot, ah, al);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 3; ++i) mfma3(s.acc[3 + i], nh[i], nl[i], bh0, bl0);
  __builtin_amdgcn_sched_barrier(0);
  load_a<1, 0>(s, slot, nh, nl);
  __builtin_amdgcn_sched_barrier(0);
  mfma3(s.acc[6], ah[0], al[0], bh0, bl0);
  mfma3(s.acc[7], ah[1], al[1], bh0, bl0);
  if (with9) mfma3(s.acc[8], ah[2], al[2], bh0, bl0);
  __builtin_amdgcn_sched_barrier(0);
  load_a<1, 3>(s, slot, ah, al);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 3; ++i) mfma3(s.acc[i], nh[i], nl[i], bh1, bl1);
  __builtin_amdgcn_sched_barrier(0);
  load_a<1, 6>(s, slot, nh, nl);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int i = 0; i < 3; ++i) mfma3(s.acc[3 + i], ah[i], al[i], bh1, bl1);
  __builtin_amdgcn_sched_barrier(0);
  mfma3(s.acc[6], nh[0], nl[0], bh1, bl1);
  mfma3(s.acc[7], nh[1], nl[1], bh1, bl1);
  if (with9) mfma3(s.acc[8], nh[2], nl[2], bh1, bl1);
}

// Barrier, refill, MFMAs of chunk c with B operands of k-steps (k0, k0+1).
__device__ __forceinline__ void run_chunk(State& s, const FieldArgs& a, float4* lds, int& c, bf16x8 bh0,
                                          bf16x8 bl0, bf16x8 bh1, bf16x8 bl1, bool with9) {
  chunk_barrier();
  __builtin_amdgcn_sched_barrier(0);
  if (c + 3 < kStreamChunks) issue_chunk(s, a.packed, lds, c + 3);
  chunk_mfma(s, lds + (c & (kSlots - 1)) * kChunkQuads, bh0, bl0, bh1, bl1, with9);
  ++c;
}

// acc -> next layer's B operands: relu (not for fc_out's feat), hi/lo split.
__device__ __forceinline__ void finish_layer(State& s, bool relu) {
  const float lo = relu ? 0.0f : -__builtin_inff();
#pragma unroll
  for (int b = 0; b < 8; ++b) {
#pragma unroll
    for (int sp = 0; sp < 2; ++sp) {
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = s.acc[b][8 * sp + j];
        asm("v_max_f32 %0, %1, %2" : "=v"(v[j]) : "v"(x), "v"(lo));
      }
      split8(v, s.bh[2 * b + sp], s.bl[2 * b + sp]);
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(kThreads, 1) void field_x3_kernel(FieldArgs a) {
  // ONE LDS object (a second one makes hipcc wait vmcnt(0) before every ring read):
  // the DMA ring, then the bias vectors
  __shared__ __attribute__((aligned(16))) float4 lds[kLdsQuads + kBiasLds / 4];
  float* blds = reinterpret_cast<float*>(lds + kLdsQuads);
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
  const int crow0 = __builtin_amdgcn_readfirstlane(s.crow);
  // wave-uniform by construction; readfirstlane makes it an SGPR so the bias
  // fast/slow choice is a scalar branch (a VGPR bool would run both paths masked)
  s.uniform_code = __builtin_amdgcn_readfirstlane(__ballot(s.crow != crow0) == 0 ? 1 : 0) != 0;
  for (int j = threadIdx.x; j < 768; j += kThreads) blds[j] = a.packed[kBiasXyz1 + j];
  if (s.uniform_code) {
    const float* src = a.code_bias + (int64_t)crow0 * kCbStride;
    for (int j = s.lane; j < kCbStride; j += 64) blds[768 + s.wave * kCbStride + j] = src[j];
  }
  __syncthreads();

  // every input load has landed (an s_waitcnt the compiler sees, so nothing stale
  // is tracked into the DMA stream); prime the ring with chunks 0..2
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  issue_chunk(s, a.packed, lds, 0);
  issue_chunk(s, a.packed, lds, 1);
  issue_chunk(s, a.packed, lds, 2);
  int c = 0;

  // ---- layer_xyz1 (63 -> 256): 4 k-steps of encoding
  init_acc(s, a, blds, kXyz1);
  run_chunk(s, a, lds, c, s.bh[0], s.bl[0], s.bh[1], s.bl[1], false);
  run_chunk(s, a, lds, c, s.bh[2], s.bl[2], s.bh[3], s.bl[3], false);
  finish_layer(s, true);

  // ---- layer_xyz2, fc_out, layer_dir1 (feature part), layer_dir2: one loop body
  for (int layer = kXyz2; layer <= kDir2; ++layer) {
    init_acc(s, a, blds, layer);
    const bool with9 = (layer == kOut);
#pragma unroll
    for (int k = 0; k < 16; k += 2) run_chunk(s, a, lds, c, s.bh[k], s.bl[k], s.bh[k + 1], s.bl[k + 1], with9);
    if (layer == kDir1) run_chunk(s, a, lds, c, s.dh[0], s.dl[0], s.dh[1], s.dl[1], false);
    if (layer == kOut) {
      s.sigma = s.acc[8][0];
      if constexpr (MODE != kFromEncoded) {
        // view-direction encoding for layer_dir1 (fc_out's accumulators are dead)
        float v[16];
        encode_pairs<6, 4>(s.vd, a.fd, s.h, v);
        v[14] = 0.0f;
        v[15] = 0.0f;
        split8(v, s.dh[0], s.dl[0]);
        split8(v + 8, s.dh[1], s.dl[1]);
      }
    }
    finish_layer(s, layer != kOut);  // fc_out's feat has no activation
  }

  // ---- fc_rgb (256 -> 3): one chunk holding its 16 k-steps of block 0
  init_acc(s, a, blds, kRgb);
  chunk_barrier();
  {
    const float4* slot = lds + (c & (kSlots - 1)) * kChunkQuads;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const float4* ap = slot + (k / 9) * kQuadsPerStep + (2 * (k % 9)) * 64 + s.lane;
      mfma3(s.acc[0], __builtin_bit_cast(bf16x8, ap[0]), __builtin_bit_cast(bf16x8, ap[64]), s.bh[k], s.bl[k]);
    }
  }
  // drain the dummy chunks' DMA before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  if (valid && s.h == 0) {
    float4 o;
    o.x = s.acc[0][0];
    o.y = s.acc[0][1];
    o.z = s.acc[0][2];
    o.w = s.sigma;
    reinterpret_cast<float4*>(a.raw)[row] = o;
  }
}

static_assert(kChunkRgb + 1 == kRealChunks, "chunk schedule");
static_assert(kDmaPerWave * 64 * 4 == kChunkQuads, "chunk = 36 DMA wave-instructions");

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
