// 3xbf16 field kernel, w16 form: the fused posenc + CodeNeRF MLP (forward_pass,
// view_synthesis/nerf/__init__.py:94-134 + CodeNeRFModel.forward, models/model.py:160-194)
// with every fp32 GEMM computed as Wh.Xh + Wh.Xl + Wl.Xh (Wh = bf16(W), Wl = bf16(W - Wh),
// the same split of the activations, fp32 accumulate) on v_mfma_f32_16x16x32_bf16 at TWO
// waves per SIMD -- the fp32 w16 kernel's machinery (mlp_f32.hip) with bf16 hi/lo operands.
//
// Why this shape.  The 32x32x16 kernel (mlp_x3.hip) holds 32 samples x 256 features of
// accumulators plus their hi/lo B operands per wave (one wave per SIMD); measured (r02aj) its
// matrix pipe is busy 68 % of the time at the 2.00 GHz the chip holds under it: a lone wave
// must issue every LDS read, DMA piece, conversion and barrier itself.  A 16-sample wave holds
// 64 accumulator + 64 operand registers, so two waves share each SIMD and one's MFMAs cover
// the other's stalls (the fp32 w16 kernel runs its pipe 92.5 % busy this way); and the chip
// holds a higher clock on 16x16x32 than on 32x32x16 bf16 loops (MI355X guide, DVFS item 7).
//
// Register dataflow.  D = W x X^T, A = 16 rows of W (lane l: row l & 15, k = 8 (l >> 4) + e),
// B = the samples' inputs (lane l: sample l & 15, the same k), D = 16 features x 16 samples
// with feature 4 (l >> 4) + r in register r (the w16 accumulator layout).  k-step t of a
// 256-input layer feeds, in lane group g, element e, input feature
//     16 (2t + (e >> 2)) + 4 g + (e & 3)
// = registers 0..3 of accumulator blocks 2t and 2t+1: a layer's output is split into hi/lo
// bf16 once (8 values -> 2 bf16x8 per k-step) and is the next layer's B operand as it stands.
// The pack permutes every W to that order once.  Encodings: the w16 kernel's per-lane enc[16]
// (pairs p = 4i + g) is k-steps 0, 1 of layer_xyz1; the view-direction encoding denc[8] is the
// one k-step of the view-dir chunk.
//
// Weight stream.  Chunk = one 32-wide k-step x 16 output blocks x {hi, lo} fragments of
// 1 KiB (64 lanes x 16 B) = 32 KiB, fragment f = 2 ob + part at quads f*64 + lane (a wave's
// ds_read_b128 of one fragment is 1 KiB contiguous, conflict free).  36 chunks (xyz1 2 |
// xyz2 8 | fc_out 8 | dir1 8 | view-dir 1 | dir2 8 | rgb 1: fragments 2t + part of block 0
// over its 8 k-steps) = 1.15 MB, the same stream as the fp32 w16 kernel, through the same
// 4-slot LDS ring (LDS-DMA, 4 pieces per wave per chunk, one barrier in mid-chunk; cyclic
// across tiles).  A chunk is 8 groups of 2 output blocks: 4 A reads and 6 MFMAs per group,
// the next group's reads in flight during the current group's MFMAs.
//
// sigma (fc_out row 0) is an fp32 dot product of h2 with the fp32 weights (exact products),
// taken before h2 is split into its hi/lo operands.
//
// Measured (r02 x3w1-3, pmc_x3w; C2-sized launch of 1 M samples): 1.50 ms vs 1.37-1.41 ms for
// the 32x32x16 kernel -- the chip does hold a higher clock under it (2.19 vs 2.00 GHz) but the
// matrix pipe is busy only 54 % (waves parked at waitcnt / barrier 41 % of their cycles: a chunk
// is 1536 MFMA cycles per SIMD, 5.3x less than the fp32 w16 kernel's, so the per-chunk barrier
// and the A-fragment reads issued one group ahead are not covered); without the LDS-DMA stream
// it runs 1.22-1.26 ms (the 32x32x16 kernel 1.17).  Both forms therefore sit at the same
// ~25-27 GB/s per CU of weight stream.  Kept as the opt-in format "bf16x3_w16" (parity-tested
// like every field kernel); "bf16x3" stays on mlp_x3.hip.
#include <algorithm>

#include "mlp_common.h"

namespace cn {
namespace mlp {
namespace x3w {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kTile = 16 * kWaves;         // samples per workgroup tile
constexpr int kChunkQuads = 32 * 64;       // 32 fragments x 64 lanes x 16 B = 32 KiB
constexpr int kRing = 4;
constexpr int kPiecesPerWave = kChunkQuads / (64 * kWaves);   // 4 x 1 KiB per wave per chunk
constexpr int kCL2 = 2, kCL3 = 10, kCL4 = 18, kCDir = 26, kCL5 = 27, kCRgb = 35, kChunks = 36;
constexpr int kStreamFloats = kChunks * kChunkQuads * 4;
// constants after the stream (as the w16 pack): b_xyz1 | b_dir1 | b_dir2 | sigma weights
// [g][ob][r] = W_out[0][16 ob + 4 g + r]
constexpr int kCB1 = 0, kCBD1 = 256, kCBD2 = 512, kCSig = 768, kConsts = 1024;
constexpr int kPackedFloats = kStreamFloats + kConsts;
constexpr int kLdsQuads = kRing * kChunkQuads + (kConsts + kWaves * kCbStride) / 4;

static_assert(kChunks % kRing == 0, "cyclic stream: chunk c + 36 reuses chunk c's ring slot");
static_assert(kPiecesPerWave == 4, "4 DMA wave-instructions per chunk per wave");
static_assert(kLdsQuads * 16 <= 160 * 1024, "LDS budget");

// ---------------------------------------------------------------- feature maps

// Input feature of a 256-wide layer fed at k-step t by lane group g, element e.
__host__ __device__ constexpr int col_b(int t, int g, int e) { return 16 * (2 * t + (e >> 2)) + 4 * g + (e & 3); }

// xyz / view-direction encoding columns: the w16 kernel's maps (mlp_f32.hip), 4-wide k-step
// 8t + e of the w16 order = element e of 32-wide k-step t here.
__host__ __device__ constexpr int col_enc_xyz(int t, int g) {
  const int i = t & 7, p = 4 * i + g;
  if (p < 30) return (t < 8 ? 3 : 6) + 6 * (p / 3) + p % 3;
  return t < 8 ? (g == 2 ? 0 : 2) : (g == 2 ? 1 : -1);
}
__host__ __device__ constexpr int col_enc_dir(int s, int g) {
  if (s < 6) {
    const int p = 4 * (s % 3) + g;
    return (s < 3 ? 3 : 6) + 6 * (p / 3) + p % 3;
  }
  return (s == 6 && g < 3) ? g : -1;
}

__device__ __forceinline__ unsigned short bf16_bits(float x) {
  return __builtin_bit_cast(unsigned short, static_cast<__bf16>(x));
}

// ---------------------------------------------------------------- packing

__global__ void pack_x3w_kernel(Params P, float* __restrict__ packed) {
  unsigned short* q16 = reinterpret_cast<unsigned short*>(packed);
  constexpr int n_elems = kStreamFloats * 2;  // bf16 elements of the stream
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n_elems + kConsts; idx += gridDim.x * blockDim.x) {
    if (idx >= n_elems) {
      const int j = idx - n_elems;
      float v;
      if (j < 256) v = P.p[kBXyz1][j];
      else if (j < 512) v = P.p[kBDir1][j - 256];
      else if (j < 768) v = P.p[kBDir2][j - 512];
      else {
        const int t = j - kCSig, g = t >> 6, ob = (t >> 2) & 15, r = t & 3;
        v = P.p[kWOut][16 * ob + 4 * g + r];
      }
      packed[kStreamFloats + j] = v;
      continue;
    }
    const int quad = idx >> 3, e = idx & 7;
    const int c = quad / kChunkQuads, rem = quad % kChunkQuads;
    const int f = rem >> 6, lane = rem & 63;
    const int i = lane & 15, g = lane >> 4;
    int ob = f >> 1, part = f & 1, t = 0, row = -1, col = -1, in_dim = 0;
    const float* W = nullptr;
    if (c < kCL2) { W = P.p[kWXyz1]; in_dim = kDimXyz; row = 16 * ob + i; col = col_enc_xyz(8 * c + e, g); }
    else if (c < kCL3) { W = P.p[kWXyz2]; in_dim = kHidden + kCode; row = 16 * ob + i; col = col_b(c - kCL2, g, e); }
    else if (c < kCL4) { W = P.p[kWOut]; in_dim = kHidden + kCode; row = 1 + 16 * ob + i; col = col_b(c - kCL3, g, e); }
    else if (c < kCDir) { W = P.p[kWDir1]; in_dim = kCode + kDimDir; row = 16 * ob + i; col = col_b(c - kCL4, g, e); }
    else if (c == kCDir) {
      W = P.p[kWDir1]; in_dim = kCode + kDimDir; row = 16 * ob + i;
      const int d = e < 7 ? col_enc_dir(e, g) : -1;
      col = d < 0 ? -1 : kCode + d;
    } else if (c < kCRgb) { W = P.p[kWDir2]; in_dim = kHidden; row = 16 * ob + i; col = col_b(c - kCL5, g, e); }
    else {
      // fc_rgb: fragment f = 2 t + part of block 0 over k-steps t = 0..7; fragments 16..31 zero
      W = P.p[kWRgb]; in_dim = kHidden + kCode;
      t = f >> 1; part = f & 1;
      row = (f < 16 && i < 3) ? i : -1;
      col = col_b(t, g, e);
    }
    const float w = (row >= 0 && col >= 0) ? W[row * in_dim + col] : 0.0f;
    const float hi = static_cast<float>(static_cast<__bf16>(w));
    q16[idx] = part == 0 ? bf16_bits(w) : bf16_bits(w - hi);
  }
}

// ---------------------------------------------------------------- kernel state

struct State {
  floatx4 acc[16];   // layer output accumulators (feature 16 ob + 4 g + r)
  bf16x8 bh[8];      // layer input, hi bf16 of k-steps 0..7
  bf16x8 bl[8];      // ... and lo
  bf16x8 pre[4];     // the next chunk's group-0 A fragments
  float denc[8];     // view-direction encoding (the view-dir chunk's k-step)
  float sig;         // sigma partial (this lane group's 64 features of h2)
  int lane, g, wave;
  int crow;          // this lane's code-bias row
  bool uniform_code; // all 16 samples of the wave use one code row
  __amdgpu_buffer_rsrc_t wsrc;
  unsigned voff;
};

// 8 fp32 values -> hi / lo bf16x8 (v - float(hi) rounded to bf16).
__device__ __forceinline__ void split8(const float* v, bf16x8& hi, bf16x8& lo) {
  u32x4 h, l;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    f32x2 p = {v[2 * k], v[2 * k + 1]};
    const bf16x2 hb = __builtin_convertvector(p, bf16x2);
    const unsigned hu = __builtin_bit_cast(unsigned, hb);
    f32x2 back;
    back.x = __uint_as_float(hu << 16);
    back.y = __uint_as_float(hu & 0xffff0000u);
    const bf16x2 lb = __builtin_convertvector(p - back, bf16x2);
    h[k] = hu;
    l[k] = __builtin_bit_cast(unsigned, lb);
  }
  hi = __builtin_bit_cast(bf16x8, h);
  lo = __builtin_bit_cast(bf16x8, l);
}

// The previous layer's accumulators -> this layer's B operands (ReLU unless RELU is false).
template <bool RELU>
__device__ __forceinline__ void to_operands(State& s) {
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    float v[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v[r] = RELU ? fmaxf(s.acc[2 * t][r], 0.0f) : s.acc[2 * t][r];
      v[4 + r] = RELU ? fmaxf(s.acc[2 * t + 1][r], 0.0f) : s.acc[2 * t + 1][r];
    }
    split8(v, s.bh[t], s.bl[t]);
  }
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return static_cast<unsigned>(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) void*)p));
}

// sigma's h2 part: fc_out row 0 . relu(acc) in fp32 (exact products), before the split.  The
// weights are loop-invariant LDS reads: volatile asm keeps LLVM from hoisting all 64 of them
// out of the layer loop (64 registers live across every layer: spills).
__device__ __forceinline__ void sigma_h2(State& s, const float* clds) {
  float sg = 0.0f;
  const unsigned base = lds_addr(clds + kCSig + 64 * s.g);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    u32x4 w[4];
    asm volatile(
        "ds_read_b128 %0, %4 offset:%5\n\tds_read_b128 %1, %4 offset:%6\n\t"
        "ds_read_b128 %2, %4 offset:%7\n\tds_read_b128 %3, %4 offset:%8\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(w[0]), "=&v"(w[1]), "=&v"(w[2]), "=&v"(w[3])
        : "v"(base), "i"(64 * q), "i"(64 * q + 16), "i"(64 * q + 32), "i"(64 * q + 48)
        : "memory");
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) sg = fmaf(__uint_as_float(w[j][r]), fmaxf(s.acc[4 * q + j][r], 0.0f), sg);
  }
  s.sig = sg;
}

// One LDS-DMA piece: 1 KiB of chunk cn (piece p of 4 for this wave).
__device__ __forceinline__ void dma_piece(const State& s, float4* lds, int cn, int p) {
  const int src = cn < kChunks ? cn : cn - kChunks;
  const unsigned soff = __builtin_amdgcn_readfirstlane((unsigned)(src * kChunkQuads + p * 64 * kWaves) * 16u);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      s.wsrc, (lds_ptr_t)(lds + (cn & (kRing - 1)) * kChunkQuads + p * 64 * kWaves + s.wave * 64), 16, s.voff,
      soff, 0, 0);
}

__device__ __forceinline__ void dma_chunk(const State& s, float4* lds, int cn) {
#pragma unroll
  for (int p = 0; p < kPiecesPerWave; ++p) dma_piece(s, lds, cn, p);
}

// M_c: chunk c+1 landed for every wave (all but this wave's 4 youngest DMA pieces --
// chunk c+2's -- retired), every wave past chunk c-1, this wave's LDS reads returned.
__device__ __forceinline__ void chunk_barrier() {
  asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// A fragments {hi, lo} of blocks 2G, 2G+1 of the chunk at `slot` (float4 units, lane applied).
template <int G>
__device__ __forceinline__ void read_group(const float4* slot, bf16x8* a) {
#pragma unroll
  for (int q = 0; q < 4; ++q) a[q] = *reinterpret_cast<const bf16x8*>(slot + (4 * G + q) * 64);
}

// Two output blocks' three products, the blocks alternating so no MFMA waits on the one just
// before it (a dependent srcC costs wait states; the alternation leaves one MFMA between).
__device__ __forceinline__ void mfma3x2(floatx4& c0, floatx4& c1, const bf16x8* a, bf16x8 bh, bf16x8 bl) {
  c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bh, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], bh, c1, 0, 0, 0);
  c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bl, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], bl, c1, 0, 0, 0);
  c0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bh, c0, 0, 0, 0);
  c1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[3], bh, c1, 0, 0, 0);
}

// Scheduling of one group: the 4 A reads of the next group between the first MFMAs.
__device__ __forceinline__ void group_pattern() {
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
  }
  __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
}

// One 16-block chunk: acc[ob] += W_chunk[ob] x (bh, bl) for the chunk's k-step; the last group
// reads the next chunk's first fragments into s.pre.
__device__ __forceinline__ void chunk16(State& s, float4* lds, int c, bf16x8 bh, bf16x8 bl) {
  const float4* slot = lds + (c & (kRing - 1)) * kChunkQuads + s.lane;
  const float4* nslot = lds + ((c + 1) & (kRing - 1)) * kChunkQuads + s.lane;
  bf16x8 a0[4], a1[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) a0[q] = s.pre[q];
  __builtin_amdgcn_sched_barrier(0);
#define CN_GROUP(G, CUR, NXT)                                             \
  {                                                                       \
    if constexpr ((G) < 7) read_group<(G) + 1>(slot, NXT);                \
    else read_group<0>(nslot, s.pre);                                     \
    mfma3x2(s.acc[2 * (G)], s.acc[2 * (G) + 1], CUR, bh, bl);             \
    group_pattern();                                                      \
    __builtin_amdgcn_sched_barrier(0);                                    \
    if constexpr ((G) == 3) {                                             \
      chunk_barrier();                                                    \
      dma_chunk(s, lds, c + 3);                                           \
    }                                                                     \
  }
  CN_GROUP(0, a0, a1)
  CN_GROUP(1, a1, a0)
  CN_GROUP(2, a0, a1)
  CN_GROUP(3, a1, a0)
  CN_GROUP(4, a0, a1)
  CN_GROUP(5, a1, a0)
  CN_GROUP(6, a0, a1)
  CN_GROUP(7, a1, a0)
#undef CN_GROUP
}

// A 256-input layer: 8 chunks, B from s.bh / s.bl.
__device__ __forceinline__ void layer256(State& s, float4* lds, int& c) {
#pragma unroll
  for (int t = 0; t < 8; ++t) chunk16(s, lds, c + t, s.bh[t], s.bl[t]);
  c += 8;
}

// Bias-initialise the 16 accumulators from a 256-vector (row 16 ob + 4 g + r).
__device__ __forceinline__ void bias_from(State& s, const float* v) {
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) s.acc[ob] = *reinterpret_cast<const floatx4*>(v + 16 * ob + 4 * s.g);
}

__device__ __forceinline__ void bias_code(State& s, const FieldArgs& a, const float* crow_lds, int off) {
  if (s.uniform_code) {
    bias_from(s, crow_lds + off);
  } else {
    bias_from(s, a.code_bias + (int64_t)s.crow * kCbStride + off);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): nothing ordinary stays in flight in the stream
  }
}

template <int MODE>
__device__ __forceinline__ void field_tile(State& s, const FieldArgs& a, float4* lds, float* clds, float* crow_lds,
                                          int64_t tile, int& c) {
  const int64_t row = tile * kTile + s.wave * 16 + (s.lane & 15);
  const bool valid = row < a.m;
  const int64_t rc = valid ? row : a.m - 1;

  // ---- per-sample inputs, code row (ordinary loads: the in-flight DMA retires with them)
  const SampleIn in = decode_sample<MODE>(a, rc);
  s.crow = static_cast<int>(code_row(a, in.code_of));
  const int crow0 = __builtin_amdgcn_readfirstlane(s.crow);
  s.uniform_code = __builtin_amdgcn_readfirstlane(__ballot(s.crow != crow0) == 0 ? 1 : 0) != 0;
  float cbr[9];
  {
    const float* src = a.code_bias + (int64_t)crow0 * kCbStride;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int j = s.lane + 64 * k;
      cbr[k] = j < kCbStride ? src[j] : 0.0f;
    }
  }
  float enc[16];
  if constexpr (MODE == kFromEncoded) {
    const float* xr = a.x + rc * (kDimXyz + kDimDir);
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int col = col_enc_xyz(t, s.g);
      enc[t] = col >= 0 ? xr[col] : 0.0f;
    }
#pragma unroll
    for (int t = 0; t < 7; ++t) {
      const int col = col_enc_dir(t, s.g);
      s.denc[t] = col >= 0 ? xr[kDimXyz + col] : 0.0f;
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int j = s.lane + 64 * k;
    if (j < kCbStride) crow_lds[j] = cbr[k];
  }

  // ---- encodings: lane group g owns pairs p = 4 i + g
  if constexpr (MODE != kFromEncoded) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int p = 4 * i + s.g;
      const int pc = p < 30 ? p : 0;
      const float arg = __fmul_rn(pick3(in.x, pc % 3), a.fx[pc / 3]);
      float sn, cs;
      sincosf(arg, &sn, &cs);
      if (i == 7 && p >= 30) {  // groups 2, 3: raw inputs
        sn = s.g == 2 ? in.x[0] : in.x[2];
        cs = s.g == 2 ? in.x[1] : 0.0f;
      }
      enc[i] = sn;
      enc[8 + i] = cs;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int p = 4 * i + s.g;
      const float arg = __fmul_rn(pick3(in.vd, p % 3), a.fd[p / 3]);
      sincosf(arg, &s.denc[i], &s.denc[3 + i]);
    }
    s.denc[6] = s.g == 0 ? in.vd[0] : (s.g == 1 ? in.vd[1] : (s.g == 2 ? in.vd[2] : 0.0f));
  }
  s.denc[7] = 0.0f;

  // ---- layer_xyz1 (63 -> 256): 2 chunks of encoding k-steps
  bias_from(s, clds + kCB1);
  {
    bf16x8 h0, l0, h1, l1;
    split8(enc, h0, l0);
    split8(enc + 8, h1, l1);
    chunk16(s, lds, c + 0, h0, l0);
    chunk16(s, lds, c + 1, h1, l1);
  }
  c += 2;

  // ---- layer_xyz2, fc_out, layer_dir1 (+ view-dir chunk), layer_dir2 (one runtime loop: a
  // fully unrolled kernel is instruction-fetch bound and spills)
  for (int layer = kXyz2; layer <= kDir2; ++layer) {
    // the previous layer's outputs -> this layer's operands: ReLU, none after fc_out (feat)
    if (layer == kOut) sigma_h2(s, clds);
    if (layer == kDir1) to_operands<false>(s);
    else to_operands<true>(s);
    if (layer == kXyz2) bias_code(s, a, crow_lds, kCbXyz2);
    else if (layer == kOut) bias_code(s, a, crow_lds, kCbFeat);
    else bias_from(s, clds + (layer == kDir1 ? kCBD1 : kCBD2));
    __builtin_amdgcn_sched_barrier(0);
    layer256(s, lds, c);
    if (layer == kDir1) {
      bf16x8 dh, dl;
      split8(s.denc, dh, dl);
      chunk16(s, lds, c, dh, dl);
      c += 1;
    }
  }
  to_operands<true>(s);                         // v2

  // ---- fc_rgb (256 -> 3): block 0 over 8 k-steps, fragments 2t, 2t+1 of the rgb chunk
  {
    float b0 = 0.0f, b1 = 0.0f, b2 = 0.0f, bs = 0.0f;
    if (s.uniform_code) {
      b0 = crow_lds[kCbRgb];
      b1 = crow_lds[kCbRgb + 1];
      b2 = crow_lds[kCbRgb + 2];
      bs = crow_lds[kCbSigma];
    } else {
      const float* cb = a.code_bias + (int64_t)s.crow * kCbStride;
      b0 = cb[kCbRgb];
      b1 = cb[kCbRgb + 1];
      b2 = cb[kCbRgb + 2];
      bs = cb[kCbSigma];
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    // lane group 0 holds output rows 0..3 (registers 0..3) of block 0
    s.acc[0] = s.g == 0 ? floatx4{b0, b1, b2, 0.0f} : floatx4{0.0f, 0.0f, 0.0f, 0.0f};
    s.acc[1] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
    float sg = s.sig;
    sg += __shfl_xor(sg, 16);
    sg += __shfl_xor(sg, 32);
    s.sig = sg + bs;
  }
  {
    const float4* slot = lds + (c & (kRing - 1)) * kChunkQuads + s.lane;
    const float4* nslot = lds + ((c + 1) & (kRing - 1)) * kChunkQuads + s.lane;
    bf16x8 a0[4], a1[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) a0[q] = s.pre[q];
    // group G = k-steps 2G, 2G+1 (fragments 4G .. 4G+3), two accumulation chains
#define CN_RGB(G, CUR, NXT)                                                      \
  {                                                                              \
    if constexpr ((G) < 3) read_group<(G) + 1>(slot, NXT);                       \
    else read_group<0>(nslot, s.pre);                                            \
    s.acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(CUR[0], s.bh[2 * (G)], s.acc[0], 0, 0, 0);     \
    s.acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(CUR[2], s.bh[2 * (G) + 1], s.acc[1], 0, 0, 0); \
    s.acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(CUR[0], s.bl[2 * (G)], s.acc[0], 0, 0, 0);     \
    s.acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(CUR[2], s.bl[2 * (G) + 1], s.acc[1], 0, 0, 0); \
    s.acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(CUR[1], s.bh[2 * (G)], s.acc[0], 0, 0, 0);     \
    s.acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(CUR[3], s.bh[2 * (G) + 1], s.acc[1], 0, 0, 0); \
    group_pattern();                                                             \
    __builtin_amdgcn_sched_barrier(0);                                           \
    if constexpr ((G) == 1) {                                                    \
      chunk_barrier();                                                           \
      dma_chunk(s, lds, c + 3);                                                  \
    }                                                                            \
  }
    CN_RGB(0, a0, a1)
    CN_RGB(1, a1, a0)
    CN_RGB(2, a0, a1)
    CN_RGB(3, a1, a0)
#undef CN_RGB
    c += 1;
  }
  if (valid && s.g == 0) {
    const floatx4 r = s.acc[0] + s.acc[1];
    float4 o;
    o.x = r[0];
    o.y = r[1];
    o.z = r[2];
    o.w = s.sig;
    reinterpret_cast<float4*>(a.raw)[row] = o;
  }
}

template <int MODE>
__global__ __launch_bounds__(kThreads, 2) void field_x3w_kernel(FieldArgs a) {
  // ONE LDS object: the DMA ring, then the constants, then one code-bias row per wave
  __shared__ __attribute__((aligned(16))) float4 lds[kLdsQuads];
  float* clds = reinterpret_cast<float*>(lds + kRing * kChunkQuads);
  State s;
  s.lane = threadIdx.x & 63;
  s.g = s.lane >> 4;
  s.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  s.wsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.packed), 0, kPackedFloats * 4, 0x00020000);
  s.voff = static_cast<unsigned>(s.wave * 64 + s.lane) * 16u;
  s.sig = 0.0f;
  float* crow_lds = clds + kConsts + s.wave * kCbStride;

  for (int k = threadIdx.x; k < kConsts; k += kThreads) clds[k] = a.packed[kStreamFloats + k];
  // prime the ring with chunks 0..2, wait for chunk 0 everywhere, read its first fragments
  dma_chunk(s, lds, 0);
  dma_chunk(s, lds, 1);
  dma_chunk(s, lds, 2);
  asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  read_group<0>(lds + s.lane, s.pre);

  const int64_t n_tiles = (a.m + kTile - 1) / kTile;
  int c = 0;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    c = 0;
    field_tile<MODE>(s, a, lds, clds, crow_lds, tile, c);
  }
  // the last tile prefetched chunks 0..2 of a tile that does not exist: they must land
  // before the workgroup's LDS is released
  __builtin_amdgcn_s_waitcnt(0x0F70);
}

}  // namespace x3w

static int64_t cu_count_x3w() {
  static int n[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (n[dev] == 0) {
    int v = 0;
    n[dev] = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
  }
  return n[dev];
}

int64_t packed_floats_x3w() { return x3w::kPackedFloats; }

int launch_pack_x3w(const Params& P, float* packed, hipStream_t st) {
  hipLaunchKernelGGL(x3w::pack_x3w_kernel, dim3(cn::elementwise_grid(x3w::kStreamFloats * 2 + x3w::kConsts, 256)),
                     dim3(256), 0, st, P, packed);
  return cn::launch_status();
}

int launch_field_x3w(int mode, FieldArgs& a, hipStream_t st) {
  if (a.masks || a.save) return CN_EUNSUPPORTED;  // inference only: masks / planes come from mlp_x3.hip
  const unsigned grid = static_cast<unsigned>(std::min<int64_t>(cn::ceil_div(a.m, x3w::kTile), cu_count_x3w()));
  const dim3 b(x3w::kThreads);
  switch (mode) {
    case kFromPts: hipLaunchKernelGGL((x3w::field_x3w_kernel<kFromPts>), dim3(grid), b, 0, st, a); break;
    case kFromRayZ: hipLaunchKernelGGL((x3w::field_x3w_kernel<kFromRayZ>), dim3(grid), b, 0, st, a); break;
    default: hipLaunchKernelGGL((x3w::field_x3w_kernel<kFromEncoded>), dim3(grid), b, 0, st, a); break;
  }
  return cn::launch_status();
}

}  // namespace mlp
}  // namespace cn
