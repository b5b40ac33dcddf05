// 3xbf16-split field kernel: the same fused posenc + CodeNeRF MLP as mlp.hip,
// with every fp32 GEMM x.W computed as  Wh.Xh + Wh.Xl + Wl.Xh  on
// v_mfma_f32_32x32x16_bf16 (fp32 accumulate), where Wh = bf16(W),
// Wl = bf16(W - Wh) (packed once) and Xh/Xl the same split of the activations
// (done in registers).  The dropped Wl.Xl term and the lo rounding leave ~2^-17
// relative error per product -- far inside the 1e-4 rendered-RGB tolerance --
// at 3/16 of the fp32-MFMA cost.
//
// Register dataflow.  A 32x32 fp32 accumulator block's registers 0..7 / 8..15
// are the next layer's B operand for k-steps 2b / 2b+1 (element j of lane half h
// = feature 32b + (j&3) + 8(j>>2) + 4h of the block, mlp_layout.h), so
// activations never leave registers.  Each wave keeps one "slot" of 16 VGPRs
// per accumulator block.  At the end of a layer the accumulators are copied
// raw (fp32) into the slots, interleaved with the layer's last MFMAs; the next
// layer converts slot b+1 (activation + hi/lo bf16 split, ~10 VALU per pair)
// while its MFMAs on slot b run, so the epilogue hides in the MFMA issue gaps
// instead of standing between layers (one wave per SIMD: nothing else would
// cover it).
//
// sigma (fc_out row 0) is an fp32 dot product over layer_xyz2's outputs taken
// during that same conversion (2 FMAs per pair), so every weight chunk has the
// same 8-block shape.
//
// Weight stream.  Chunk = 2 k-steps x 8 blocks x {hi, lo} x 64 lanes quads =
// 32 KiB, fragment-major so a wave's ds_read_b128 of one fragment is 1 KiB
// contiguous (bank-conflict free); chunk c lies at packed + c * 32 KiB.  A 4-slot
// LDS ring is filled by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB per
// wave-instruction, 8 per wave per chunk, offsets in SGPRs).  Each chunk is
// split by ONE barrier M_c after its 4th MFMA group (of 8): M_c = chunk c+1
// landed for every wave (counted `s_waitcnt vmcnt(8)`) and every wave is done
// with chunk c-1.  Groups 0-3 of chunk c issue pieces 4-7 of chunk c+2, groups
// 4-7 pieces 0-3 of chunk c+3 (slot of chunk c-1), one piece per group so the
// DMA issue cost hides in MFMA gaps, and group 7 already reads chunk c+1's
// first A fragments -- the MFMA pipe never waits for a chunk boundary.  No
// ordinary global load is live in the stream, so the counted waits are exact.
//
// Persistent tiles.  The grid is one workgroup per CU; each loops over
// 128-sample tiles.  The stream is cyclic (36 chunks, a multiple of the 4 ring
// slots): the last three chunks of a tile prefetch the first three of the
// next, so the ring never drains or re-primes between tiles.
//
// Code size.  The four 256-input layers run through ONE runtime loop whose body
// is a single unrolled 16-k-step layer (a fully unrolled kernel is
// instruction-fetch bound).
#include <algorithm>
#include <type_traits>

#include "mlp_common.h"

namespace cn {
namespace mlp {
namespace x3 {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int kBlk = 8;                              // 32-row output blocks per k-step
constexpr int kQuadsPerStep = 64 * kBlk * 2;         // one k-step of a chunk (16 KiB)
constexpr int kChunkQuads = 2 * kQuadsPerStep;       // 2048 quads = 32 KiB
constexpr int kDmaPerWave = kChunkQuads / 64 / 4;    // 8
// stream: xyz1 2 | xyz2 8 | fc_out 8 | layer_dir1 view-dir k-steps 1 | layer_dir1 8 | layer_dir2 8 | fc_rgb 1
constexpr int kChunkL1 = 2, kChunkL2 = 10, kChunkDir = 18, kChunkL3 = 19, kChunkL4 = 27, kChunkRgb = 35;
constexpr int kChunks = 36;
constexpr int kQuads = kChunks * kChunkQuads;
constexpr int kBiasXyz1 = kQuads * 4;  // floats
constexpr int kSigmaOff = 768;         // after b_xyz1, b_dir1, b_dir2: fc_out row 0 over h2, [h][b][reg]
constexpr int kConsts = 1024;
constexpr int kPackedFloats = kBiasXyz1 + kConsts;

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

// (chunk, step-in-chunk T, slot j) -> (layer, k-step, output block)
__device__ void chunk_map(int c, int T, int j, int& l, int& ks, int& ob) {
  ob = j;
  if (c < kChunkL1) { l = kXyz1; ks = 2 * c + T; }
  else if (c < kChunkL2) { l = kXyz2; ks = 2 * (c - kChunkL1) + T; }
  else if (c < kChunkDir) { l = kOut; ks = 2 * (c - kChunkL2) + T; }
  else if (c == kChunkDir) { l = kDir1; ks = 16 + T; }
  else if (c < kChunkL4) { l = kDir1; ks = 2 * (c - kChunkL3) + T; }
  else if (c < kChunkRgb) { l = kDir2; ks = 2 * (c - kChunkL4) + T; }
  else { l = kRgb; ks = 8 * T + j; ob = 0; }
}

__global__ void pack_x3_kernel(Params P, float* __restrict__ packed) {
  unsigned short* q16 = reinterpret_cast<unsigned short*>(packed);
  const int n_elems = kQuads * 8;  // bf16 elements
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n_elems + kConsts;
       idx += gridDim.x * blockDim.x) {
    if (idx >= n_elems) {
      const int j = idx - n_elems;
      float v;
      if (j < 256) v = P.p[kBXyz1][j];
      else if (j < 512) v = P.p[kBDir1][j - 256];
      else if (j < 768) v = P.p[kBDir2][j - 512];
      else {
        const int t = j - kSigmaOff, h = t >> 7, b = (t >> 4) & 7, r = t & 15;
        v = P.p[kWOut][acc_row(b, r, h)];  // fc_out row 0 at input feature acc_row(b, r, h) of h2
      }
      packed[kBiasXyz1 + j] = v;
      continue;
    }
    const int quad = idx >> 3, e = idx & 7;
    const int c = quad / kChunkQuads;
    int r = quad % kChunkQuads;
    const int T = r / kQuadsPerStep;
    r %= kQuadsPerStep;
    const int frag = r / 64, lane = r % 64;  // fragment-major: 1 KiB per (block, hi|lo)
    const int slot = frag >> 1, part = frag & 1;
    int l, ks, ob;
    chunk_map(c, T, slot, l, ks, ob);
    const int i = lane & 31, h = lane >> 5;
    const int col = in_col(l, ks, h, e);
    int row = -1, in_dim = 0;
    const float* W = nullptr;
    switch (l) {
      case kXyz1: W = P.p[kWXyz1]; in_dim = kDimXyz; row = 32 * ob + i; break;
      case kXyz2: W = P.p[kWXyz2]; in_dim = kHidden + kCode; row = 32 * ob + i; break;
      case kOut: W = P.p[kWOut]; in_dim = kHidden + kCode; row = 1 + 32 * ob + i; break;
      case kDir1: W = P.p[kWDir1]; in_dim = kCode + kDimDir; row = 32 * ob + i; break;
      case kDir2: W = P.p[kWDir2]; in_dim = kHidden; row = 32 * ob + i; break;
      default: W = P.p[kWRgb]; in_dim = kHidden + kCode; row = i < 3 ? i : -1; break;
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
constexpr int kRing = 4;
constexpr int kLdsQuads = kRing * kChunkQuads;  // 128 KiB ring
// after the ring: the constant vectors (1024), then each wave's code row
constexpr int kBiasLds = kConsts + kWaves * kCbStride;

struct State {
  float sl[8][16];        // per accumulator block: raw fp32 copy, then {hi, lo} bf16 of k-steps 2b, 2b+1
  bf16x8 dh[2], dl[2];    // view-direction encoding k-steps of layer_dir1
  floatx16 acc[8];
  float sigma, sig;       // fc_out row 0; running partial of this lane half
  int lane, h, wave;
  int crow;               // this lane's code-bias row
  bool uniform_code;      // all 32 samples of the wave use one code row
  bf16x8 pre[4];          // next chunk's group-0 A fragments, read by the chunk before it
  unsigned mw[4];         // training forward: ReLU mask words being built for the current layer
  __amdgpu_buffer_rsrc_t wsrc;  // the packed stream as a buffer resource
  unsigned voff;          // this lane's byte offset inside a 1 KiB-per-wave piece row
  float* sv;              // training: this lane's row of the plane being written (+4h), or null
  float pend[2];          // training backward: the even piece's values, stored with the odd one
  int cbase;              // no-geometry backward: chunk counter at the tile's first chunk (DmaNoGeo)
};

typedef __attribute__((address_space(3))) void* lds_ptr_t;

__device__ __forceinline__ bf16x8 dw8(const float* f) {
  const u32x4 u = {__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3])};
  return __builtin_bit_cast(bf16x8, u);
}

template <int J>
__device__ __forceinline__ bf16x8 Bh(const State& s, int t) { return dw8(s.sl[J] + 8 * t); }
template <int J>
__device__ __forceinline__ bf16x8 Bl(const State& s, int t) { return dw8(s.sl[J] + 8 * t + 4); }
#define CN_SLOT_B(J) Bh<J>(s, 0), Bl<J>(s, 0), Bh<J>(s, 1), Bl<J>(s, 1)

__device__ __forceinline__ float vmax(float x, float lo) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(lo));
  return r;
}

// Values 2K, 2K+1 of a raw block -> activation, hi/lo bf16 into `out` (k-step
// K/4, dword K%4); sig += w . v (the sigma dot product, kept only in fc_out).
// mb (training forward): bits 2K, 2K+1 of the slot's 16-bit ReLU mask |= [v > 0]
// (v is post-activation, so >= +0: the mask bit is min(bits(v), 1)).
template <int K>
__device__ __forceinline__ void conv_piece(const float* raw, float* out, float lo_clamp, const float* w, float& sig,
                                           unsigned* mb = nullptr) {
  f32x2 v;
  v.x = vmax(raw[2 * K], lo_clamp);
  v.y = vmax(raw[2 * K + 1], lo_clamp);
  if (w) {
    sig = fmaf(w[2 * K], v.x, sig);
    sig = fmaf(w[2 * K + 1], v.y, sig);
  }
  if (mb) {
    *mb |= min(__float_as_uint(v.x), 1u) << (2 * K);
    *mb |= min(__float_as_uint(v.y), 1u) << (2 * K + 1);
  }
  const bf16x2 hb = __builtin_convertvector(v, bf16x2);
  const unsigned hu = __builtin_bit_cast(unsigned, hb);
  f32x2 back;
  back.x = __uint_as_float(hu << 16);
  back.y = __uint_as_float(hu & 0xffff0000u);
  const bf16x2 lb = __builtin_convertvector(v - back, bf16x2);
  unsigned hi_w = hu, lo_w = __builtin_bit_cast(unsigned, lb);
  // pin the piece here: without it LLVM sinks the arithmetic to the B operand's
  // first use (the next chunk), out of the MFMA gaps it is meant to fill
  asm volatile("" : "+v"(hi_w), "+v"(lo_w), "+v"(sig));
  constexpr int t = K / 4, d = K % 4;
  out[8 * t + d] = __uint_as_float(hi_w);
  out[8 * t + 4 + d] = __uint_as_float(lo_w);
}

template <int K = 0>
__device__ __forceinline__ void conv_all(const float* raw, float* out, float lo, const float* w, float& sig,
                                         unsigned* mb = nullptr) {
  if constexpr (K < 8) {
    conv_piece<K>(raw, out, lo, w, sig, mb);
    conv_all<K + 1>(raw, out, lo, w, sig, mb);
  }
}

// The 16 mask bits of slot J go to bits 16 (J & 1) .. of word J >> 1.
template <int J>
__device__ __forceinline__ void put_mask(unsigned* mw, unsigned mb) {
  mw[J >> 1] |= mb << (16 * (J & 1));
}

// Training forward: post-activation values 4q..4q+3 of raw slot J (features 32J + 8q + 4h ..
// + 3, one 16-B store into the plane row s.sv; lo = 0 for a ReLU, -inf for feat).
template <int J, int Q>
__device__ __forceinline__ void save_quad(const State& s, float lo) {
  float4 o;
  o.x = vmax(s.sl[J][4 * Q], lo);
  o.y = vmax(s.sl[J][4 * Q + 1], lo);
  o.z = vmax(s.sl[J][4 * Q + 2], lo);
  o.w = vmax(s.sl[J][4 * Q + 3], lo);
  *reinterpret_cast<float4*>(s.sv + 32 * J + 8 * Q) = o;
}

template <int J>
__device__ __forceinline__ void save_slot(const State& s, float lo) {
  save_quad<J, 0>(s, lo);
  save_quad<J, 1>(s, lo);
  save_quad<J, 2>(s, lo);
  save_quad<J, 3>(s, lo);
}

// One LDS-DMA piece: 1 KiB per wave (16 B per lane) of chunk `cn`, piece `i`
// (piece i of chunk cn covers quads [i*256, i*256+256) of the chunk; this wave
// moves quads i*256 + wave*64 + lane).
__device__ __forceinline__ void dma_piece(const State& s, float4* lds, int cn, int i) {
  const unsigned soff = __builtin_amdgcn_readfirstlane((unsigned)(cn * kChunkQuads + i * 256) * 16u);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(s.wsrc, (lds_ptr_t)(lds + (cn & (kRing - 1)) * kChunkQuads + i * 256 + s.wave * 64),
                                           16, s.voff, soff, 0, 0);
}

// The pieces running chunk c issues: groups 0-3 pieces 4-7 of chunk c+2, groups
// 4-7 pieces 0-3 of chunk c+3, wrapping into the next tile's first chunks
// (kChunks is a multiple of kRing, so the ring slot is unchanged by the wrap).
struct Dma {
  const State& s;
  float4* lds;
  int ca, cb;  // c+2, c+3 mod kChunks
  template <int G>
  __device__ __forceinline__ void piece() const {
    if constexpr (G < 4) dma_piece(s, lds, ca, 4 + G);
    else dma_piece(s, lds, cb, G - 4);
  }
};

__device__ __forceinline__ Dma dma_for(const State& s, float4* lds, int c) {
  const int ca = c + 2 < kChunks ? c + 2 : c + 2 - kChunks;
  const int cb = c + 3 < kChunks ? c + 3 : c + 3 - kChunks;
  return Dma{s, lds, ca, cb};
}
// The default chunk stream: the 36 chunks from c = 0 in every tile.
struct DmaFull {
  static __device__ __forceinline__ Dma make(const State& s, float4* lds, int c) { return dma_for(s, lds, c); }
};

// The no-geometry training backward's stream: 33 of the transposed pack's 36 chunks (not the
// view-direction chunk kNoGeoSkip, nor the two layer_xyz1^T chunks).  33 is not a multiple of the
// ring, so the chunk counter runs on across tiles: ring slot = counter & 3, packed chunk = the
// counter's position in the tile's stream (s.cbase: the counter at the tile's first chunk).
constexpr int kNoGeoSkip = 17, kNoGeoChunks = kChunks - 3;
__device__ __forceinline__ void dma_piece_ng(const State& s, float4* lds, int cn, int i) {
  int k = cn - s.cbase;
  if (k >= kNoGeoChunks) k -= kNoGeoChunks;
  const int src = k + (k >= kNoGeoSkip ? 1 : 0);
  const unsigned soff = __builtin_amdgcn_readfirstlane((unsigned)(src * kChunkQuads + i * 256) * 16u);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(s.wsrc, (lds_ptr_t)(lds + (cn & (kRing - 1)) * kChunkQuads + i * 256 + s.wave * 64),
                                           16, s.voff, soff, 0, 0);
}
struct DmaNoGeoPieces {
  const State& s;
  float4* lds;
  int ca, cb;  // c+2, c+3 (running counters)
  template <int G>
  __device__ __forceinline__ void piece() const {
    if constexpr (G < 4) dma_piece_ng(s, lds, ca, 4 + G);
    else dma_piece_ng(s, lds, cb, G - 4);
  }
};
struct DmaNoGeo {
  static __device__ __forceinline__ DmaNoGeoPieces make(const State& s, float4* lds, int c) {
    return DmaNoGeoPieces{s, lds, c + 2, c + 3};
  }
};

// M_c: chunk c+1 landed for every wave (all but this wave's OUT youngest DMA
// pieces retired), every wave is past chunk c-1, and every LDS read of this
// wave (incl. the asynchronous sigma-weight reads) has returned.  One asm
// statement, so no LDS read can be scheduled across it.
template <int OUT>
__device__ __forceinline__ void chunk_barrier() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"n"(OUT) : "memory");
  __builtin_amdgcn_sched_barrier(0);  // nothing (ring reads included) is scheduled above the wait
}
constexpr int kMidOut = 8;  // chunk c+2's pieces are younger than chunk c+1's at M_c

// Small LDS reads outside the ring (biases, sigma weights).  Inline asm: hipcc
// cannot prove them disjoint from the in-flight DMA and would otherwise wait
// vmcnt(0), draining the ring.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return static_cast<unsigned>(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) void*)p));
}

// 8 floats at p + 32*ob (ob = 0..7), one LDS round trip.
__device__ __forceinline__ void lds_read8_stride32(const float* p, float* v) {
  asm volatile(
      "ds_read_b32 %0, %8\n\tds_read_b32 %1, %8 offset:128\n\tds_read_b32 %2, %8 offset:256\n\t"
      "ds_read_b32 %3, %8 offset:384\n\tds_read_b32 %4, %8 offset:512\n\tds_read_b32 %5, %8 offset:640\n\t"
      "ds_read_b32 %6, %8 offset:768\n\tds_read_b32 %7, %8 offset:896\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(lds_addr(p))
      : "memory");
}

// 16 consecutive floats (64 B aligned), one LDS round trip.
__device__ __forceinline__ void lds_read16(const float* p, float* v) {
  u32x4 a, b, c, d;
  asm volatile(
      "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\t"
      "ds_read_b128 %3, %4 offset:48\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
      : "v"(lds_addr(p))
      : "memory");
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = __uint_as_float(a[i]);
    v[4 + i] = __uint_as_float(b[i]);
    v[8 + i] = __uint_as_float(c[i]);
    v[12 + i] = __uint_as_float(d[i]);
  }
}

// The same without a wait: the values are first used after the next chunk
// barrier, whose lgkmcnt(0) covers them (volatile asm keeps the order).
__device__ __forceinline__ void lds_read16_async(const float* p, float* v) {
  u32x4 a, b, c, d;
  asm volatile(
      "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:16\n\tds_read_b128 %2, %4 offset:32\n\t"
      "ds_read_b128 %3, %4 offset:48"
      : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
      : "v"(lds_addr(p))
      : "memory");
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[i] = __uint_as_float(a[i]);
    v[4 + i] = __uint_as_float(b[i]);
    v[8 + i] = __uint_as_float(c[i]);
    v[12 + i] = __uint_as_float(d[i]);
  }
}

__device__ __forceinline__ float lds_read1(const float* p) {
  float v;
  asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=&v"(v) : "v"(lds_addr(p)) : "memory");
  return v;
}

// Biases.  acc starts as b via ONE MFMA per output block: A holds {bf16(b_i),
// bf16(b_i - hi)} at k = 0, 1 (lane half 0), B holds ones at k = 0, 1, so D = hi
// + lo in fp32.
__device__ __forceinline__ floatx16 bias_mfma(float v, bf16x8 one) {
  bf16x8 f = {};
  const __bf16 hi = static_cast<__bf16>(v);
  f[0] = hi;
  f[1] = static_cast<__bf16>(v - static_cast<float>(hi));
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(f, one, floatx16{0}, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 ones_b(int h) {
  bf16x8 one = {};
  if (h == 0) {
    one[0] = static_cast<__bf16>(1.0f);
    one[1] = static_cast<__bf16>(1.0f);
  }
  return one;
}

// Bias vector of `layer` for this lane's 8 blocks (lane half 0 carries it).
__device__ __forceinline__ void bias_values(const State& s, const float* blds, int layer, float* v) {
  const bool per_code = (layer == kXyz2 || layer == kOut);
  const float* src = per_code ? blds + kConsts + s.wave * kCbStride + (layer == kXyz2 ? kCbXyz2 : kCbFeat)
                              : blds + (layer == kXyz1 ? 0 : (layer == kDir1 ? 256 : 512));
  lds_read8_stride32(src + (s.lane & 31), v);
}

// Slow path (a wave whose samples use several code rows): per-lane loads.
__device__ __forceinline__ void init_acc_per_lane(State& s, const FieldArgs& a, int layer) {
  const float* base = a.code_bias + (int64_t)s.crow * kCbStride;
  if (layer == kRgb) {
    s.acc[0] = floatx16{0};
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
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): nothing pending leaks out
}

__device__ __forceinline__ void mfma3(floatx16& acc, bf16x8 ah, bf16x8 al, bf16x8 bh, bf16x8 bl) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc, 0, 0, 0);
}

// A fragments {hi, lo} of blocks (2P, 2P+1) of k-step T of the chunk in `slot`.
template <int T, int P>
__device__ __forceinline__ void load_a(const State& s, const float4* slot, bf16x8* a) {
  const float4* ap = slot + T * kQuadsPerStep + s.lane;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    a[2 * i] = __builtin_bit_cast(bf16x8, ap[(2 * (2 * P + i)) * 64]);
    a[2 * i + 1] = __builtin_bit_cast(bf16x8, ap[(2 * (2 * P + i) + 1) * 64]);
  }
}

// Scheduling pattern of one group: 6 MFMAs, each followed by up to N VALU; the
// next group's 4 A reads go out with the first two MFMAs, the group's DMA piece
// with the third.
template <int N, bool READS = true>
__device__ __forceinline__ void group_pattern() {
#pragma unroll
  for (int m = 0; m < 6; ++m) {
    if (READS && m < 2) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    if (m == 2) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    if constexpr (N > 0) __builtin_amdgcn_sched_group_barrier(0x002, N, 0);
  }
}

struct NoFill {
  template <int G>
  __device__ __forceinline__ void step() {}
};

// Convert slot J (raw block of the previous layer) into packed B operands, one
// pair of values per group; sigma partial alongside.
template <int J, bool MASKS = false, bool SAVE = false>
struct ConvFill {
  State& s;
  float lo;
  float w[16];  // sigma weights of this slot
  float out[16];
  unsigned mb;
  template <int G>
  __device__ __forceinline__ void step() {
    if constexpr (SAVE && (G & 1)) save_quad<J, G / 2>(s, lo);  // before G == 7 overwrites the slot
    // w (read asynchronously at the chunk start) is usable only after M_c, so the
    // sigma products of pieces 0-3 are taken in steps 4-7 from the raw values
    if constexpr (G < 4) {
      conv_piece<G>(s.sl[J], out, lo, nullptr, s.sig, MASKS ? &mb : nullptr);
    } else {
      conv_piece<G>(s.sl[J], out, lo, w, s.sig, MASKS ? &mb : nullptr);
      constexpr int K = G - 4;
      const float v0 = vmax(s.sl[J][2 * K], lo), v1 = vmax(s.sl[J][2 * K + 1], lo);
      s.sig = fmaf(w[2 * K], v0, s.sig);
      s.sig = fmaf(w[2 * K + 1], v1, s.sig);
    }
    if constexpr (G == 7) {
#pragma unroll
      for (int i = 0; i < 16; ++i) s.sl[J][i] = out[i];
      if constexpr (MASKS) put_mask<J>(s.mw, mb);
    }
  }
};

__device__ __forceinline__ void copy_acc(State& s, int b) {
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    float x = s.acc[b][i];
    asm volatile("" : "+v"(x));  // materialise the copy here (see conv_piece)
    s.sl[b][i] = x;
  }
}

// Last chunk of a layer: once block pair P's final MFMAs (T = 1, group 4 + P) are
// issued, copy the pair's accumulators into their slots during the next group.
struct CopyFill {
  State& s;
  template <int G>
  __device__ __forceinline__ void step() {
    if constexpr (G >= 5) {
      copy_acc(s, 2 * (G - 5));
      copy_acc(s, 2 * (G - 5) + 1);
    }
  }
};

// One 2-k-step chunk against the 8 output blocks: 8 groups (T, block pair) of 6
// MFMAs; the A fragments of group g+1 are read during group g (group 7 reads
// the next chunk's group 0 into s.pre when PREF); fill.step<g>() is VALU work
// (independent of the chunk) placed in group g's MFMA issue gaps; group g also
// issues one DMA piece; M_c sits between groups 3 and 4.  SELF: group 0's
// fragments are read here (first chunk of a tile) instead of arriving in s.pre.
template <int NV, bool SELF, bool PREF, typename D = DmaFull, typename Fill>
__device__ __forceinline__ void chunk_mfma(State& s, float4* lds, int c, bf16x8 bh0, bf16x8 bl0, bf16x8 bh1,
                                           bf16x8 bl1, Fill& fill) {
  const float4* slot = lds + (c & (kRing - 1)) * kChunkQuads;
  const float4* nslot = lds + ((c + 1) & (kRing - 1)) * kChunkQuads;
  const auto dma = D::make(s, lds, c);
  bf16x8 a0[4], a1[4];
  if constexpr (SELF) {
    load_a<0, 0>(s, slot, a0);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) a0[i] = s.pre[i];
  }
  __builtin_amdgcn_sched_barrier(0);
#define CN_GROUP(G, CUR, NXT)                                                     \
  {                                                                              \
    constexpr int T = (G) / 4, P = (G) % 4;                                      \
    if constexpr ((G) < 7) load_a<((G) + 1) / 4, ((G) + 1) % 4>(s, slot, NXT);  \
    else if constexpr (PREF) load_a<0, 0>(s, nslot, s.pre);                      \
    const bf16x8 bh = T ? bh1 : bh0, bl = T ? bl1 : bl0;                         \
    mfma3(s.acc[2 * P], CUR[0], CUR[1], bh, bl);                                 \
    mfma3(s.acc[2 * P + 1], CUR[2], CUR[3], bh, bl);                             \
    dma.template piece<G>();                                                     \
    fill.template step<G>();                                                     \
    group_pattern<NV, ((G) < 7 || PREF)>();                                      \
    __builtin_amdgcn_sched_barrier(0);                                           \
    if constexpr ((G) == 3) chunk_barrier<kMidOut>();                            \
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

// Chunk c's MFMAs (with its DMA pieces and M_c inside).
template <int NV, bool SELF = false, typename D = DmaFull, typename Fill>
__device__ __forceinline__ void run_chunk(State& s, const FieldArgs& a, float4* lds, int& c, bf16x8 bh0, bf16x8 bl0,
                                          bf16x8 bh1, bf16x8 bl1, Fill& fill) {
  chunk_mfma<NV, SELF, true, D>(s, lds, c, bh0, bl0, bh1, bl1, fill);
  ++c;
}

// Chunk J of a 256-input layer: B from slot J, converting slot J+1 meanwhile
// (the last chunk copies the accumulators out instead).
template <int J, bool MASKS = false, bool SAVE = false>
__device__ __forceinline__ void layer_chunk(State& s, const FieldArgs& a, float4* lds, int& c, const float* blds,
                                            float lo) {
  if constexpr (J < 7) {
    ConvFill<J + 1, MASKS, SAVE> f{s, lo, {}, {}, 0u};
    lds_read16_async(blds + kSigmaOff + (s.h * 8 + J + 1) * 16, f.w);
    run_chunk<2>(s, a, lds, c, CN_SLOT_B(J), f);
  } else {
    CopyFill f{s};
    run_chunk<6>(s, a, lds, c, CN_SLOT_B(J), f);
    copy_acc(s, 6);
    copy_acc(s, 7);
  }
}

// Bias-initialise the accumulators of `layer` while converting slot 0.
template <bool MASKS = false, bool SAVE = false>
__device__ __forceinline__ void begin_layer(State& s, const FieldArgs& a, const float* blds, int layer, float lo) {
  if constexpr (SAVE) save_slot<0>(s, lo);
  float w[16];
  lds_read16(blds + kSigmaOff + (s.h * 8) * 16, w);
  float out[16];
  unsigned mb = 0;
  unsigned* mbp = MASKS ? &mb : nullptr;
  if (s.uniform_code || !(layer == kXyz2 || layer == kOut)) {
    float v[8];
    bias_values(s, blds, layer, v);
    const bf16x8 one = ones_b(s.h);
#define CN_BIAS(B)                                   \
  s.acc[B] = bias_mfma(s.h == 0 ? v[B] : 0.0f, one); \
  conv_piece<B>(s.sl[0], out, lo, w, s.sig, mbp);
    CN_BIAS(0) CN_BIAS(1) CN_BIAS(2) CN_BIAS(3) CN_BIAS(4) CN_BIAS(5) CN_BIAS(6) CN_BIAS(7)
#undef CN_BIAS
  } else {
    init_acc_per_lane(s, a, layer);
    conv_all(s.sl[0], out, lo, w, s.sig, mbp);
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) s.sl[0][i] = out[i];
  if constexpr (MASKS) put_mask<0>(s.mw, mb);
  __builtin_amdgcn_sched_barrier(0);
}

// Training forward: the 4 mask words of one converted layer (tile, wave, slot l
// of kMaskLayers) as one 16-B store per lane.
constexpr int kMaskLayers = 5;  // h1, h2, feat (unused), v1, v2
constexpr int kMaskWordsPerTile = kWaves * kMaskLayers * 64 * 4;
__device__ __forceinline__ void store_masks(State& s, const FieldArgs& a, int64_t tile, int l) {
  uint4 v;
  v.x = s.mw[0];
  v.y = s.mw[1];
  v.z = s.mw[2];
  v.w = s.mw[3];
  reinterpret_cast<uint4*>(a.masks)[((tile * kWaves + s.wave) * kMaskLayers + l) * 64 + s.lane] = v;
#pragma unroll
  for (int i = 0; i < 4; ++i) s.mw[i] = 0u;
}

// One 128-sample tile: inputs, encodings, the six layers (chunks 0..35 of the
// stream, which also prefetch chunks 0..2 for the next tile), the raw store.
template <int MODE, bool MASKS, bool SAVE>
__device__ __forceinline__ void field_tile(State& s, const FieldArgs& a, float4* lds, float* blds, int64_t tile) {
#pragma unroll
  for (int i = 0; i < 4; ++i) s.mw[i] = 0u;
  s.sig = 0.0f;
  s.sigma = 0.0f;
  const int64_t row = tile * kTile + s.wave * 32 + (s.lane & 31);
  const bool valid = row < a.m;
  const int64_t rc = valid ? row : a.m - 1;
  // training: padding lanes store into the scratch row after the planes (no branch per store)
  float* const scratch = SAVE ? a.save + 5 * a.m * 256 : nullptr;

  // ---- per-sample inputs and this wave's code row (ordinary loads; the DMA in
  // flight -- chunks 0..2 of this tile -- retires with them)
  const SampleIn in = decode_sample<MODE>(a, rc);
  s.crow = static_cast<int>(code_row(a, in.code_of));
  const int crow0 = __builtin_amdgcn_readfirstlane(s.crow);
  // wave-uniform by construction; readfirstlane makes it an SGPR so the bias
  // fast/slow choice is a scalar branch (a VGPR bool would run both paths masked)
  s.uniform_code = __builtin_amdgcn_readfirstlane(__ballot(s.crow != crow0) == 0 ? 1 : 0) != 0;
  float cbr[9];
  {
    const float* src = a.code_bias + (int64_t)crow0 * kCbStride;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int j = s.lane + 64 * k;
      cbr[k] = (s.uniform_code && j < kCbStride) ? src[j] : 0.0f;
    }
  }
  float enc[32];
  float dv[16];
  if constexpr (MODE == kFromEncoded) {
    const float* xr = a.x + rc * (kDimXyz + kDimDir);
    gather_pairs<15>(xr, 0, s.h, enc);
    gather_pairs<6>(xr, kDimXyz, s.h, dv);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): every ordinary load has landed
  int c = 0;

  // ---- encodings (VALU)
  if constexpr (MODE != kFromEncoded) {
    encode_pairs<15, 10>(in.x, a.fx, s.h, enc);
    encode_pairs<6, 4>(in.vd, a.fd, s.h, dv);
  }
  dv[14] = 0.0f;
  dv[15] = 0.0f;
  {
    float sg = 0.0f;
    const float lo = -__builtin_inff();
    conv_all(dv, s.sl[0], lo, nullptr, sg);
    conv_all(enc, s.sl[6], lo, nullptr, sg);
    conv_all(enc + 16, s.sl[7], lo, nullptr, sg);
  }
  s.dh[0] = Bh<0>(s, 0);
  s.dl[0] = Bl<0>(s, 0);
  s.dh[1] = Bh<0>(s, 1);
  s.dl[1] = Bl<0>(s, 1);
  // this wave's code row: read back only by this wave (LDS is in order per wave)
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int j = s.lane + 64 * k;
    if (j < kCbStride) blds[kConsts + s.wave * kCbStride + j] = cbr[k];
  }

  // ---- layer_xyz1 (63 -> 256): 4 k-steps of encoding in slots 6, 7
  {
    float v[8];
    bias_values(s, blds, kXyz1, v);
    const bf16x8 one = ones_b(s.h);
#pragma unroll
    for (int ob = 0; ob < 8; ++ob) s.acc[ob] = bias_mfma(s.h == 0 ? v[ob] : 0.0f, one);
    NoFill nf;
    run_chunk<0, true>(s, a, lds, c, CN_SLOT_B(6), nf);
    CopyFill cf{s};
    run_chunk<6>(s, a, lds, c, CN_SLOT_B(7), cf);
    copy_acc(s, 6);
    copy_acc(s, 7);
  }

  // ---- layer_xyz2, fc_out, layer_dir1, layer_dir2: one loop body
  for (int layer = kXyz2; layer <= kDir2; ++layer) {
    // activation of the layer that produced the slots: none after fc_out (feat)
    const float lo = layer == kDir1 ? -__builtin_inff() : 0.0f;
    s.sig = 0.0f;
    // training: the slots converted in this pass (h1, h2, feat, v1) go to plane layer - kXyz2
    if constexpr (SAVE) s.sv = (valid ? a.save + ((int64_t)(layer - kXyz2) * a.m + row) * 256 : scratch) + 4 * s.h;
    begin_layer<MASKS, SAVE>(s, a, blds, layer, lo);
    if (layer == kDir1) {
      NoFill nf;
      run_chunk<0>(s, a, lds, c, s.dh[0], s.dl[0], s.dh[1], s.dl[1], nf);
    }
    layer_chunk<0, MASKS, SAVE>(s, a, lds, c, blds, lo);
    layer_chunk<1, MASKS, SAVE>(s, a, lds, c, blds, lo);
    layer_chunk<2, MASKS, SAVE>(s, a, lds, c, blds, lo);
    layer_chunk<3, MASKS, SAVE>(s, a, lds, c, blds, lo);
    layer_chunk<4, MASKS, SAVE>(s, a, lds, c, blds, lo);
    layer_chunk<5, MASKS, SAVE>(s, a, lds, c, blds, lo);
    layer_chunk<6, MASKS, SAVE>(s, a, lds, c, blds, lo);
    layer_chunk<7, MASKS, SAVE>(s, a, lds, c, blds, lo);
    // the conversions of this pass were the previous layer's outputs: h1, h2, feat, v1
    if constexpr (MASKS) store_masks(s, a, tile, layer - kXyz2);
    // fc_out's pass converted layer_xyz2's outputs: its partials are sigma's h2 term
    if (layer == kOut) s.sigma = s.sig + __shfl_xor(s.sig, 32);
  }
  // sigma's code / bias term (cn_code_bias: b_out[0] + W_out[0, 256:] zs2)
  if (s.uniform_code) s.sigma += lds_read1(blds + kConsts + s.wave * kCbStride + kCbSigma);
  else s.sigma += a.code_bias[(int64_t)s.crow * kCbStride + kCbSigma];

  // ---- fc_rgb (256 -> 3): one chunk holding its 16 k-steps of block 0; it
  // prefetches chunk 2 of the next tile like any other chunk
  {
    if (s.uniform_code) {
      const int i = s.lane & 31;
      const float v = lds_read1(blds + kConsts + s.wave * kCbStride + kCbRgb + (i < 3 ? i : 0));
      s.acc[0] = bias_mfma((s.h == 0 && i < 3) ? v : 0.0f, ones_b(s.h));
    } else {
      init_acc_per_lane(s, a, kRgb);
    }
    if constexpr (SAVE) {
      s.sv = (valid ? a.save + ((int64_t)4 * a.m + row) * 256 : scratch) + 4 * s.h;  // v2
      save_slot<0>(s, 0.0f);
    }
    {
      float out[16];
      unsigned mb = 0;
      conv_all(s.sl[0], out, 0.0f, nullptr, s.sig, MASKS ? &mb : nullptr);
#pragma unroll
      for (int i = 0; i < 16; ++i) s.sl[0][i] = out[i];
      if constexpr (MASKS) put_mask<0>(s.mw, mb);
    }
    const Dma dma = dma_for(s, lds, c);
    const float4* slot = lds + (c & (kRing - 1)) * kChunkQuads + s.lane;
    // group 0's fragments arrived in s.pre (frags 0-3 of k-step 0 = CN_RGB(0)'s)
#define CN_RGB(B)                                                                                      \
  {                                                                                                    \
    const float4* ap = slot + ((B) / 4) * kQuadsPerStep + (2 * ((2 * (B)) % 8)) * 64;                  \
    const bf16x8 f0 = (B) == 0 ? s.pre[0] : __builtin_bit_cast(bf16x8, ap[0]);                         \
    const bf16x8 f1 = (B) == 0 ? s.pre[1] : __builtin_bit_cast(bf16x8, ap[64]);                        \
    const bf16x8 f2 = (B) == 0 ? s.pre[2] : __builtin_bit_cast(bf16x8, ap[128]);                       \
    const bf16x8 f3 = (B) == 0 ? s.pre[3] : __builtin_bit_cast(bf16x8, ap[192]);                       \
    mfma3(s.acc[0], f0, f1, Bh<B>(s, 0), Bl<B>(s, 0));                                                 \
    dma.template piece<B>();                                                                           \
    mfma3(s.acc[0], f2, f3, Bh<B>(s, 1), Bl<B>(s, 1));                                                 \
    if constexpr ((B) == 3) chunk_barrier<kMidOut>();                                                  \
  }
#define CN_RGB_CONV(B)                                                     \
  {                                                                        \
    if constexpr (SAVE) save_slot<B>(s, 0.0f);                             \
    float out[16];                                                         \
    unsigned mb = 0;                                                       \
    conv_all(s.sl[B], out, 0.0f, nullptr, s.sig, MASKS ? &mb : nullptr);   \
    _Pragma("unroll") for (int i = 0; i < 16; ++i) s.sl[B][i] = out[i];    \
    if constexpr (MASKS) put_mask<B>(s.mw, mb);                            \
  }
    CN_RGB(0) CN_RGB_CONV(1)
    CN_RGB(1) CN_RGB_CONV(2)
    CN_RGB(2) CN_RGB_CONV(3)
    CN_RGB(3) CN_RGB_CONV(4)
    CN_RGB(4) CN_RGB_CONV(5)
    CN_RGB(5) CN_RGB_CONV(6)
    CN_RGB(6) CN_RGB_CONV(7)
    CN_RGB(7)
#undef CN_RGB
#undef CN_RGB_CONV
  }

  if constexpr (MASKS) store_masks(s, a, tile, 4);  // v2
  if (valid && s.h == 0) {
    float4 o;
    o.x = s.acc[0][0];
    o.y = s.acc[0][1];
    o.z = s.acc[0][2];
    o.w = s.sigma;
    reinterpret_cast<float4*>(a.raw)[row] = o;
  }
}

template <int MODE, bool MASKS, bool SAVE = false>
__global__ __launch_bounds__(kThreads, 1) void field_x3_kernel(FieldArgs a) {
  // ONE LDS object (a second one makes hipcc wait vmcnt(0) before every ring read):
  // the DMA ring, then the constant vectors and code rows
  __shared__ __attribute__((aligned(16))) float4 lds[kLdsQuads + kBiasLds / 4];
  float* blds = reinterpret_cast<float*>(lds + kLdsQuads);
  State s;
  s.lane = threadIdx.x & 63;
  s.h = s.lane >> 5;
  s.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  s.wsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.packed), 0, kPackedFloats * 4, 0x00020000);
  s.voff = static_cast<unsigned>(s.wave * 64 + s.lane) * 16u;
  s.sv = nullptr;

  // constant vectors (biases, sigma weights) once per workgroup, then prime the ring
#pragma unroll
  for (int k = 0; k < kConsts / kThreads; ++k) blds[k * kThreads + threadIdx.x] = a.packed[kBiasXyz1 + k * kThreads + threadIdx.x];
  __syncthreads();
  // prime: chunks 0 and 1 and pieces 0-3 of chunk 2 (chunk 0's groups 0-3 issue the rest)
#pragma unroll
  for (int i = 0; i < kDmaPerWave; ++i) dma_piece(s, lds, 0, i);
#pragma unroll
  for (int i = 0; i < kDmaPerWave; ++i) dma_piece(s, lds, 1, i);
#pragma unroll
  for (int i = 0; i < kDmaPerWave / 2; ++i) dma_piece(s, lds, 2, i);

  const int64_t n_tiles = (a.m + kTile - 1) / kTile;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) field_tile<MODE, MASKS, SAVE>(s, a, lds, blds, tile);
  // the last tile prefetched chunks 0..2 of a tile that does not exist: they
  // must land before the workgroup's LDS is released
  __builtin_amdgcn_s_waitcnt(0x0F70);
}

static_assert(kChunkRgb + 1 == kChunks, "chunk schedule");
static_assert(kDmaPerWave * 64 * 4 == kChunkQuads, "chunk = 32 DMA wave-instructions");
static_assert(kDmaPerWave == 8, "one DMA piece per MFMA group (8 groups per chunk)");
static_assert(kChunks % kRing == 0, "cyclic stream: chunk c + 36 reuses chunk c's ring slot");


// ================================================================ fused backward
// The eval-step backward (frozen weights) of forward_pass + CodeNeRFModel.forward
// (nerf/__init__.py:94-134, model.py:160-194): from d raw (m, 4) to the per-code
// sums g_code and the ray gradients, in one persistent launch on the forward's
// machinery.  dX = dPre . W is computed as D = W^T . dPre^T: A = W^T streamed
// through the same ring (a transposed pack, again 36 chunks), B = dPre in the
// slots.  The ReLU masks come from the training forward (field_x3_kernel<.., true>:
// 128 bits per lane per layer).  Chunk schedule:
//   0      fc_rgb^T      d v2   = Wr^T d_rgb                          (k-step 0 real)
//   1-8    layer_dir2^T  d v1   = Wd2^T (m_v2 . d v2)
//   9-16   layer_dir1^T  d feat = Wd1[:, :256]^T (m_v1 . d v1)
//   17     layer_dir1^T  d dir  = Wd1[:, 256:]^T (m_v1 . d v1)        (1 block x 16 k-steps)
//   18-25  fc_out^T      d h2   = Wo[1:, :256]^T d feat + Wo[0, :256] d sigma (rank-1 init MFMA)
//   26-33  layer_xyz2^T  d h1   = Wx2[:, :256]^T (m_h2 . d h2)
//   34-35  layer_xyz1^T  d enc  = Wx1^T (m_h1 . d h1)                  (2 blocks x 16 k-steps)
// The output rows of the two encoding layers are ordered like the forward's
// encoding k-steps (k_from_enc), so each lane half back-propagates through the
// sin/cos pairs it owns with one sincosf per pair, as in the forward.
// g_code = sum over a code's samples of [m_h2 . d h2 | d feat | d sigma | d rgb]
// (cn_code_bias layout): 8-lane DPP sums + LDS float atomics into one row per
// wave, flushed to global atomics when the wave's code row changes.

constexpr int kTChunkD1 = 9, kTChunkDir = 17, kTChunkOut = 18, kTChunkX2 = 26, kTChunkX1 = 34;
constexpr int kTSigmaCol = 0, kTZeros = 256;  // transposed-pack constants: fc_out row 0 over h2, zeros
// LDS after the ring: constants, then one g_code row per wave.
constexpr int kGaccOff = kConsts;
constexpr int kBwdLdsFloats = kGaccOff + kWaves * kCbStride;

// Accumulator coordinates of A row rho of a block: register and lane half.
__host__ __device__ constexpr int reg_of_row(int rho) { return (rho & 3) + 4 * (rho >> 3); }
__host__ __device__ constexpr int half_of_row(int rho) { return (rho >> 2) & 1; }

__global__ void pack_x3t_kernel(Params P, float* __restrict__ packed) {
  unsigned short* q16 = reinterpret_cast<unsigned short*>(packed);
  const int n_elems = kQuads * 8;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < n_elems + kConsts; idx += gridDim.x * blockDim.x) {
    if (idx >= n_elems) {
      const int j = idx - n_elems;
      packed[kBiasXyz1 + j] = j < 256 ? P.p[kWOut][j] : 0.0f;  // fc_out row 0, h2 half
      continue;
    }
    const int quad = idx >> 3, e = idx & 7;
    const int c = quad / kChunkQuads;
    int r = quad % kChunkQuads;
    const int T = r / kQuadsPerStep;
    r %= kQuadsPerStep;
    const int frag = r / 64, lane = r % 64;
    const int slot = frag >> 1, part = frag & 1;
    const int i = lane & 31, h = lane >> 5;
    float w = 0.0f;
    if (c == 0) {  // fc_rgb^T: k = rgb channel e (lane half 0, k-step 0)
      if (T == 0 && h == 0 && e < 3) w = P.p[kWRgb][e * (kHidden + kCode) + 32 * slot + i];
    } else if (c < kTChunkDir) {
      const bool d2 = c < kTChunkD1;
      const int ks = 2 * (c - (d2 ? 1 : kTChunkD1)) + T;
      const int kf = acc_row(ks >> 1, 8 * (ks & 1) + e, h);
      w = d2 ? P.p[kWDir2][kf * kHidden + 32 * slot + i] : P.p[kWDir1][kf * (kCode + kDimDir) + 32 * slot + i];
    } else if (c == kTChunkDir) {
      const int ks = 8 * T + slot;
      const int kf = acc_row(ks >> 1, 8 * (ks & 1) + e, h);
      const int t = reg_of_row(i);
      const int col = t < 14 ? k_from_enc(t, half_of_row(i), 6) : -1;
      if (col >= 0) w = P.p[kWDir1][kf * (kCode + kDimDir) + kCode + col];
    } else if (c < kTChunkX1) {
      const bool out = c < kTChunkX2;
      const int ks = 2 * (c - (out ? kTChunkOut : kTChunkX2)) + T;
      const int kf = acc_row(ks >> 1, 8 * (ks & 1) + e, h);
      w = out ? P.p[kWOut][(1 + kf) * (kHidden + kCode) + 32 * slot + i]
              : P.p[kWXyz2][kf * (kHidden + kCode) + 32 * slot + i];
    } else {  // layer_xyz1^T: 2 blocks x 16 k-steps over 2 chunks
      const int q = c - kTChunkX1;
      const int ks = 8 * q + 4 * T + (slot >> 1), ob = slot & 1;
      const int kf = acc_row(ks >> 1, 8 * (ks & 1) + e, h);
      const int col = k_from_enc(16 * ob + reg_of_row(i), half_of_row(i), 15);
      if (col >= 0) w = P.p[kWXyz1][kf * kDimXyz + col];
    }
    const __bf16 hi = static_cast<__bf16>(w);
    const float lo = w - static_cast<float>(hi);
    q16[idx] = part == 0 ? bf16_bits(w) : bf16_bits(lo);
  }
}

// ---- backward pieces

// Masked value: raw if bit `bit` of word m is set, else +0.
__device__ __forceinline__ float masked(float raw, unsigned m, int bit) {
  return __uint_as_float(__float_as_uint(raw) &
                         static_cast<unsigned>(__builtin_amdgcn_sbfe(static_cast<int>(m), bit, 1)));
}

// Values 2K, 2K+1 of raw slot (mask word m, bits from `off`) -> hi/lo bf16 into
// `out` (conv_piece's layout); the masked values are returned for reductions.
template <int K>
__device__ __forceinline__ void convm_piece(const float* raw, float* out, unsigned m, int off, float& vx, float& vy) {
  f32x2 v;
  v.x = masked(raw[2 * K], m, off + 2 * K);
  v.y = masked(raw[2 * K + 1], m, off + 2 * K + 1);
  vx = v.x;
  vy = v.y;
  const bf16x2 hb = __builtin_convertvector(v, bf16x2);
  const unsigned hu = __builtin_bit_cast(unsigned, hb);
  f32x2 back;
  back.x = __uint_as_float(hu << 16);
  back.y = __uint_as_float(hu & 0xffff0000u);
  const bf16x2 lb = __builtin_convertvector(v - back, bf16x2);
  unsigned hi_w = hu, lo_w = __builtin_bit_cast(unsigned, lb);
  asm volatile("" : "+v"(hi_w), "+v"(lo_w));
  constexpr int t = K / 4, d = K % 4;
  out[8 * t + d] = __uint_as_float(hi_w);
  out[8 * t + 4 + d] = __uint_as_float(lo_w);
}

// Sum over each group of 8 lanes; lanes with (lane & 7) == 7 hold the sums.
__device__ __forceinline__ float sum8(float x) {
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0xB1, 0xF, 0xF, true));   // quad_perm 1,0,3,2
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x4E, 0xF, 0xF, true));   // quad_perm 2,3,0,1
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x114, 0xF, 0xF, true));  // row_shr:4
  return x;
}

// LDS float atomic at byte address base + IMM (no return) from the lanes of EXEC & {LO, HI}
// only: the sum holders (lanes 8k + 7) -- the LDS then processes 8 lanes per instruction
// instead of 64 -- without a branch (EXEC narrowed and restored inside the one asm
// statement, so the MFMA/VALU interleave around it keeps one basic block).
constexpr unsigned kHolders = 0x80808080u;
template <int IMM, unsigned LO = kHolders, unsigned HI = kHolders>
__device__ __forceinline__ void ds_add(unsigned base, float v) {
  const unsigned long long mask = (static_cast<unsigned long long>(HI) << 32) | LO;
  unsigned long long saved;
  // s_mov only (s_and_saveexec would clobber SCC behind the compiler's back); every call site runs
  // with all 64 lanes active
  asm volatile(
      "s_mov_b64 %0, exec\n\t"
      "s_mov_b64 exec, %3\n\t"
      "ds_add_f32 %1, %2 offset:%4\n\t"
      "s_mov_b64 exec, %0"
      : "=&s"(saved)
      : "v"(base), "v"(v), "s"(mask), "i"(IMM)
      : "memory");
}

// Row R of block J (lane half h) is feature acc_row(J, R, h); its g_code column sits at
// gbase + 4 * acc_row(J, R, 0) bytes (gbase carries the 4h and the layer's column offset).
template <int J, int R>
__device__ __forceinline__ void red_add(unsigned gbase, float v) {
  ds_add<4 * acc_row(J, R, 0)>(gbase, sum8(v));
}

// Training backward: masked values of pieces 2q, 2q+1 of slot J (features 32J + 8q + 4h ..
// + 3) as one 16-B store into the dPre plane row s.sv.
template <int J, int G>
__device__ __forceinline__ void save_piece(State& s, float vx, float vy) {
  if constexpr ((G & 1) == 0) {
    s.pend[0] = vx;
    s.pend[1] = vy;
  } else {
    *reinterpret_cast<float4*>(s.sv + 32 * J + 8 * (G / 2)) = make_float4(s.pend[0], s.pend[1], vx, vy);
  }
}

// Convert slot J of a backward pass (mask words mw; RED: also sum into the LDS row at gbase --
// g_code, or a bias gradient row; SAVE: store the masked values into the dPre plane).
template <int J, bool RED, bool SAVE = false>
struct ConvMaskFill {
  State& s;
  const unsigned* mw;
  unsigned gbase;
  float out[16];
  template <int G>
  __device__ __forceinline__ void step() {
    float vx, vy;
    convm_piece<G>(s.sl[J], out, mw[J >> 1], 16 * (J & 1), vx, vy);
    if constexpr (RED) {
      red_add<J, 2 * G>(gbase, vx);
      red_add<J, 2 * G + 1>(gbase, vy);
    }
    if constexpr (SAVE) save_piece<J, G>(s, vx, vy);
    if constexpr (G == 7) {
#pragma unroll
      for (int i = 0; i < 16; ++i) s.sl[J][i] = out[i];
    }
  }
};

template <int J, bool RED, bool SAVE = false>
__device__ __forceinline__ void conv_slot(State& s, const unsigned* mw, unsigned gbase) {
  ConvMaskFill<J, RED, SAVE> f{s, mw, gbase, {}};
  f.template step<0>();
  f.template step<1>();
  f.template step<2>();
  f.template step<3>();
  f.template step<4>();
  f.template step<5>();
  f.template step<6>();
  f.template step<7>();
}

// Init MFMA of a backward pass: acc[b] = A_b . [ds_h, ds_l, ds_h] with A_b row i =
// [wh, wh, wl] of blds[off + 32 b + i] -- fc_out^T's rank-1 sigma term, or zeros.
template <int NB>
__device__ __forceinline__ void bwd_init(State& s, const float* blds, int off, bf16x8 sig_b) {
  float v[8];
  lds_read8_stride32(blds + off + (s.lane & 31), v);
#pragma unroll
  for (int b = 0; b < NB; ++b) {
    bf16x8 f = {};
    if (s.h == 0) {
      const __bf16 hi = static_cast<__bf16>(v[b]);
      f[0] = hi;
      f[1] = hi;
      f[2] = static_cast<__bf16>(v[b] - static_cast<float>(hi));
    }
    s.acc[b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(f, sig_b, floatx16{0}, 0, 0, 0);
  }
}

// One backward pass over 8-block chunks: init, slot 0, chunks 0..6 converting
// slot J+1, chunk 7 copying the accumulators out (COPY) or leaving them
// (layer_dir1^T, whose d-dir chunk still reads the slots).
template <bool RED, bool COPY = true, bool SAVE = false, typename D = DmaFull>
__device__ __forceinline__ void bwd_pass(State& s, const FieldArgs& a, float4* lds, int& c, const float* blds,
                                         int init_off, bf16x8 sig_b, const unsigned* mw, unsigned gbase) {
  bwd_init<8>(s, blds, init_off, sig_b);
  conv_slot<0, RED, SAVE>(s, mw, gbase);
  __builtin_amdgcn_sched_barrier(0);
#define CN_BWD_CHUNK(J)                                              \
  {                                                                  \
    ConvMaskFill<(J) + 1, RED, SAVE> f{s, mw, gbase, {}};            \
    run_chunk<RED ? 4 : 2, false, D>(s, a, lds, c, CN_SLOT_B(J), f); \
  }
  CN_BWD_CHUNK(0)
  CN_BWD_CHUNK(1)
  CN_BWD_CHUNK(2)
  CN_BWD_CHUNK(3)
  CN_BWD_CHUNK(4)
  CN_BWD_CHUNK(5)
  CN_BWD_CHUNK(6)
#undef CN_BWD_CHUNK
  if constexpr (COPY) {
    CopyFill f{s};
    run_chunk<6, false, D>(s, a, lds, c, CN_SLOT_B(7), f);
    copy_acc(s, 6);
    copy_acc(s, 7);
  } else {
    NoFill f;
    run_chunk<0, false, D>(s, a, lds, c, CN_SLOT_B(7), f);
  }
}

// layer_dir1^T's d-dir chunk (1 block x 16 k-steps into acc2; step B reads slot B);
// d feat (acc[0..7], final) is copied into the slots one step behind the reads.
__device__ __forceinline__ void bwd_dir_chunk(State& s, float4* lds, int& c, floatx16& acc2) {
  const Dma dma = dma_for(s, lds, c);
  const float4* slot = lds + (c & (kRing - 1)) * kChunkQuads + s.lane;
  const float4* nslot = lds + ((c + 1) & (kRing - 1)) * kChunkQuads;
  acc2 = floatx16{0};
#define CN_DIR(B)                                                                                    \
  {                                                                                                  \
    const float4* ap = slot + ((B) / 4) * kQuadsPerStep + (2 * ((2 * (B)) % 8)) * 64;                \
    const bf16x8 f0 = (B) == 0 ? s.pre[0] : __builtin_bit_cast(bf16x8, ap[0]);                       \
    const bf16x8 f1 = (B) == 0 ? s.pre[1] : __builtin_bit_cast(bf16x8, ap[64]);                      \
    const bf16x8 f2 = (B) == 0 ? s.pre[2] : __builtin_bit_cast(bf16x8, ap[128]);                     \
    const bf16x8 f3 = (B) == 0 ? s.pre[3] : __builtin_bit_cast(bf16x8, ap[192]);                     \
    mfma3(acc2, f0, f1, Bh<B>(s, 0), Bl<B>(s, 0));                                                   \
    dma.template piece<B>();                                                                         \
    mfma3(acc2, f2, f3, Bh<B>(s, 1), Bl<B>(s, 1));                                                   \
    if constexpr ((B) > 0) copy_acc(s, (B) - 1);                                                     \
    if constexpr ((B) == 3) chunk_barrier<kMidOut>();                                                \
    if constexpr ((B) == 7) load_a<0, 0>(s, nslot, s.pre);                                           \
  }
  CN_DIR(0) CN_DIR(1) CN_DIR(2) CN_DIR(3) CN_DIR(4) CN_DIR(5) CN_DIR(6) CN_DIR(7)
#undef CN_DIR
  copy_acc(s, 7);
  ++c;
}

// Piece G of slot J of layer_xyz1^T's input (m_h1 . d h1); training: its dPre plane store.
template <int J, int G, bool TRAIN>
__device__ __forceinline__ void x1_piece(State& s, float* out, const unsigned* mw) {
  float vx, vy;
  convm_piece<G>(s.sl[J], out, mw[J >> 1], 16 * (J & 1), vx, vy);
  if constexpr (TRAIN) save_piece<J, G>(s, vx, vy);
}

// layer_xyz1^T chunk Q (k-steps 8Q..8Q+7, blocks 0 and 1): step B reads slot
// 4Q + B/2 and converts the next slot (4 pieces per step) with mask mw.
template <int Q, bool TRAIN = false>
__device__ __forceinline__ void bwd_xyz1_chunk(State& s, float4* lds, int& c, const unsigned* mw) {
  const Dma dma = dma_for(s, lds, c);
  const float4* slot = lds + (c & (kRing - 1)) * kChunkQuads + s.lane;
  const float4* nslot = lds + ((c + 1) & (kRing - 1)) * kChunkQuads;
  constexpr int kNext = 4 * Q + 1;  // first slot this chunk converts
  float out[4][16];
#define CN_X1(B)                                                                                        \
  {                                                                                                     \
    constexpr int SB = 4 * Q + (B) / 2, TT = (B) & 1;                                                   \
    const float4* ap = slot + ((B) / 4) * kQuadsPerStep + (4 * ((B) % 4)) * 64;                         \
    const bf16x8 f0 = (B) == 0 ? s.pre[0] : __builtin_bit_cast(bf16x8, ap[0]);                          \
    const bf16x8 f1 = (B) == 0 ? s.pre[1] : __builtin_bit_cast(bf16x8, ap[64]);                         \
    const bf16x8 f2 = (B) == 0 ? s.pre[2] : __builtin_bit_cast(bf16x8, ap[128]);                        \
    const bf16x8 f3 = (B) == 0 ? s.pre[3] : __builtin_bit_cast(bf16x8, ap[192]);                        \
    mfma3(s.acc[0], f0, f1, Bh<SB>(s, TT), Bl<SB>(s, TT));                                              \
    dma.template piece<B>();                                                                            \
    mfma3(s.acc[1], f2, f3, Bh<SB>(s, TT), Bl<SB>(s, TT));                                              \
    if constexpr (SB + 1 < 8) {                                                                         \
      constexpr int NS = SB + 1, P0 = 4 * TT;                                                           \
      x1_piece<NS, P0, TRAIN>(s, out[NS - kNext], mw);                                                  \
      x1_piece<NS, P0 + 1, TRAIN>(s, out[NS - kNext], mw);                                              \
      x1_piece<NS, P0 + 2, TRAIN>(s, out[NS - kNext], mw);                                              \
      x1_piece<NS, P0 + 3, TRAIN>(s, out[NS - kNext], mw);                                              \
      if constexpr (TT == 1) {                                                                          \
        _Pragma("unroll") for (int i = 0; i < 16; ++i) s.sl[NS][i] = out[NS - kNext][i];                \
      }                                                                                                 \
    }                                                                                                   \
    if constexpr ((B) == 3) chunk_barrier<kMidOut>();                                                   \
    if constexpr ((B) == 7 && Q == 0) load_a<0, 0>(s, nslot, s.pre);                                    \
  }
  CN_X1(0) CN_X1(1) CN_X1(2) CN_X1(3) CN_X1(4) CN_X1(5) CN_X1(6) CN_X1(7)
#undef CN_X1
  ++c;
}

// d input of one lane half from the encoding gradients g it holds (k_from_enc
// order: sines of its pairs, cosines, raw inputs): the forward's pairs, one
// sincosf each.
template <int P, int NF, int Q = 0>
__device__ __forceinline__ void posenc_bwd(const float* x, const float* f, int h, const float* g, float* dx) {
  if constexpr (Q < P) {
    constexpr int p0 = 2 * Q, p1 = 2 * Q + 1;
    constexpr int d0 = p0 % 3, d1 = p1 % 3, k0 = p0 / 3, k1 = p1 / 3;
    const bool live = k1 < NF || h == 0;
    const float fk = h ? f[k1 < NF ? k1 : 0] : f[k0];
    const float arg = __fmul_rn(h ? x[d1] : x[d0], fk);
    float sn, cs;
    sincosf(arg, &sn, &cs);
    const float v = live ? fk * (g[Q] * cs - g[P + Q] * sn) : 0.0f;
    dx[d0] += h ? 0.0f : v;
    dx[d1] += h ? v : 0.0f;
    posenc_bwd<P, NF, Q + 1>(x, f, h, g, dx);
  } else {
    // raw inputs: slot 2P = x0 (h 0) / x2 (h 1), slot 2P+1 = x1 (h 0)
    dx[0] += h ? 0.0f : g[2 * P];
    dx[2] += h ? g[2 * P] : 0.0f;
    dx[1] += h ? 0.0f : g[2 * P + 1];
  }
}

// Flush this wave's g_code row (LDS) into g_code[code] and zero it.  g_code null (a training chunk of
// one code row: its sums are the dPre planes' column sums, folded into the dW GEMMs in a fixed order):
// the row is only cleared.
__device__ __forceinline__ void flush_gcode(const State& s, const FieldArgs& a, float* blds, int code) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  float* row = blds + kGaccOff + s.wave * kCbStride;
#pragma unroll
  for (int k = 0; k < (kCbStride + 63) / 64; ++k) {
    const int j = s.lane + 64 * k;
    if (j < kCbStride) {
      float v;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(lds_addr(row + j)) : "memory");
      if (v != 0.0f && a.g_code) atomicAdd(a.g_code + (int64_t)code * kCbStride + j, v);
      asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(row + j)), "v"(0.0f) : "memory");
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// layer_xyz1's dPre plane (m_h1 . d h1, the raw d h1 in the slots) without its chunks (NOGEO).
template <int J = 0>
__device__ __forceinline__ void store_x1_plane(State& s, const unsigned* mw) {
  if constexpr (J < 8) {
#pragma unroll
    for (int g = 0; g < 8; g += 2) {
      const int off = 16 * (J & 1);
      const float4 v = make_float4(masked(s.sl[J][2 * g], mw[J >> 1], off + 2 * g),
                                   masked(s.sl[J][2 * g + 1], mw[J >> 1], off + 2 * g + 1),
                                   masked(s.sl[J][2 * g + 2], mw[J >> 1], off + 2 * g + 2),
                                   masked(s.sl[J][2 * g + 3], mw[J >> 1], off + 2 * g + 3));
      *reinterpret_cast<float4*>(s.sv + 32 * J + 8 * (g / 2)) = v;
    }
    store_x1_plane<J + 1>(s, mw);
  }
}

// NOGEO (the training backward with no d ro / d rd / d pts wanted -- train.py's rays are data,
// ray_sampler.py:53-82): the d-dir chunk, both layer_xyz1^T chunks and the encoding / ray epilogue
// only feed those outputs, so they are not streamed or run (33 chunks per tile, DmaNoGeo; layer_dir1^T
// copies its d feat out itself).  layer_xyz1's dPre plane is stored from the slots at the tile's end.
// crun: the running chunk counter.
template <int MODE, bool TRAIN, bool NOGEO = false, bool DET = false>
__device__ __forceinline__ void bwd_tile(State& s, const FieldArgs& a, float4* lds, float* blds, int64_t tile,
                                         int& cur_code, int& crun) {
  using D = typename std::conditional<NOGEO, DmaNoGeo, DmaFull>::type;
  const int64_t row = tile * kTile + s.wave * 32 + (s.lane & 31);
  const bool valid = row < a.m;
  const int64_t rc = valid ? row : a.m - 1;

  // ---- inputs: sample, d raw, masks (h1, h2, v1, v2), code row (wave-uniform: host-checked)
  const SampleIn in = decode_sample<MODE>(a, rc);
  const int crow0 = __builtin_amdgcn_readfirstlane(static_cast<int>(code_row(a, in.code_of)));
  float4 dr = reinterpret_cast<const float4*>(a.d_raw)[rc];
  const float zv = MODE == kFromRayZ ? a.z[rc] : 0.0f;
  unsigned mk[4][4];
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    const int ml = l < 2 ? l : l + 1;  // skip the feat slot
    const uint4 v =
        reinterpret_cast<const uint4*>(a.masks)[((tile * kWaves + s.wave) * kMaskLayers + ml) * 64 + s.lane];
    mk[l][0] = v.x;
    mk[l][1] = v.y;
    mk[l][2] = v.z;
    mk[l][3] = v.w;
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  if (!valid) dr = make_float4(0.f, 0.f, 0.f, 0.f);
  if (crow0 != cur_code) {
    if (cur_code >= 0) flush_gcode(s, a, blds, cur_code);
    cur_code = crow0;
  }
  int c = NOGEO ? crun : 0;
  s.cbase = c;
  const unsigned gl = lds_addr(blds + kGaccOff + s.wave * kCbStride) + 16u * s.h;  // + 4h floats
  const unsigned gbase = gl;  // the atomics run on the holder lanes only (ds_add)
  // training: the dPre plane rows (the bias gradients are folded into the dW GEMMs)
  // (padding lanes: the scratch row after the planes -- workspace the dW GEMMs overwrite later)
  auto plane = [&](int k) {
    return TRAIN ? (valid ? a.dpre + ((int64_t)k * a.m + row) * 256 : a.dpre + 5 * a.m * 256) + 4 * s.h : nullptr;
  };

  // g_code sigma / rgb: this wave's samples (lane half 1 repeats them)
  {
    const float sw = sum8(dr.w), sx = sum8(dr.x), sy = sum8(dr.y), sz = sum8(dr.z);
    // lane half 0's holders only (half 1 repeats the samples)
    ds_add<4 * kCbSigma, kHolders, 0u>(gl, sw);
    ds_add<4 * kCbRgb, kHolders, 0u>(gl, sx);
    ds_add<4 * (kCbRgb + 1), kHolders, 0u>(gl, sy);
    ds_add<4 * (kCbRgb + 2), kHolders, 0u>(gl, sz);
  }
  // B operands: d rgb at k-step 0 (lane half 0, k = channel) and the sigma init [dh, dl, dh]
  bf16x8 rh = {}, rl = {}, sig_b = {};
  if (s.h == 0) {
    const float d3[3] = {dr.x, dr.y, dr.z};
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      const __bf16 hi = static_cast<__bf16>(d3[e]);
      rh[e] = hi;
      rl[e] = static_cast<__bf16>(d3[e] - static_cast<float>(hi));
    }
    const __bf16 sh = static_cast<__bf16>(dr.w);
    sig_b[0] = sh;
    sig_b[1] = static_cast<__bf16>(dr.w - static_cast<float>(sh));
    sig_b[2] = sh;
  }
  const bf16x8 z8 = {};

  // ---- fc_rgb^T (chunk 0)
  {
    bwd_init<8>(s, blds, kTZeros, sig_b);
    CopyFill f{s};
    chunk_mfma<6, true, true, D>(s, lds, c, rh, rl, z8, z8, f);
    ++c;
    copy_acc(s, 6);
    copy_acc(s, 7);
  }
  // ---- layer_dir2^T (m_v2), layer_dir1^T (m_v1) + its d-dir chunk
  floatx16 acc2;
  s.sv = plane(0);
  bwd_pass<false, true, TRAIN, D>(s, a, lds, c, blds, kTZeros, sig_b, mk[3], gbase);
  s.sv = plane(1);
  bwd_pass<false, NOGEO, TRAIN, D>(s, a, lds, c, blds, kTZeros, sig_b, mk[2], gbase);
  if constexpr (!NOGEO) bwd_dir_chunk(s, lds, c, acc2);
  // ---- fc_out^T (d feat unmasked, sigma rank-1 init), layer_xyz2^T (m_h2): g_code sums
  const unsigned ones[4] = {~0u, ~0u, ~0u, ~0u};
  for (int l = 0; l < 2; ++l) {
    const unsigned* mw = l == 0 ? ones : mk[1];
    const unsigned gb = gbase + 4u * (l == 0 ? kCbFeat : kCbXyz2);
    s.sv = plane(2 + l);
    bwd_pass<true, true, TRAIN, D>(s, a, lds, c, blds, l == 0 ? kTSigmaCol : kTZeros, sig_b, mw, gb);
  }
  if constexpr (NOGEO) {
    s.sv = plane(4);
    store_x1_plane(s, mk[0]);
    crun = c;
    return;
  }
  // ---- layer_xyz1^T (m_h1) into acc[0..1]
  bwd_init<2>(s, blds, kTZeros, sig_b);
  s.sv = plane(4);
  {
    float out[16];
    x1_piece<0, 0, TRAIN>(s, out, mk[0]);
    x1_piece<0, 1, TRAIN>(s, out, mk[0]);
    x1_piece<0, 2, TRAIN>(s, out, mk[0]);
    x1_piece<0, 3, TRAIN>(s, out, mk[0]);
    x1_piece<0, 4, TRAIN>(s, out, mk[0]);
    x1_piece<0, 5, TRAIN>(s, out, mk[0]);
    x1_piece<0, 6, TRAIN>(s, out, mk[0]);
    x1_piece<0, 7, TRAIN>(s, out, mk[0]);
#pragma unroll
    for (int i = 0; i < 16; ++i) s.sl[0][i] = out[i];
  }
  __builtin_amdgcn_sched_barrier(0);
  bwd_xyz1_chunk<0, TRAIN>(s, lds, c, mk[0]);
  bwd_xyz1_chunk<1, TRAIN>(s, lds, c, mk[0]);

  // ---- encodings -> d pts, d view dir (each lane half its own pairs), then the rays
  float dx[3] = {0.f, 0.f, 0.f}, dv[3] = {0.f, 0.f, 0.f};
  {
    float g[32];
#pragma unroll
    for (int t = 0; t < 32; ++t) g[t] = s.acc[t >> 4][t & 15];
    posenc_bwd<15, 10>(in.x, a.fx, s.h, g, dx);
    float gd[14];
#pragma unroll
    for (int t = 0; t < 14; ++t) gd[t] = acc2[t];
    posenc_bwd<6, 4>(in.vd, a.fd, s.h, gd, dv);
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    dx[d] += __shfl_xor(dx[d], 32);
    dv[d] += __shfl_xor(dv[d], 32);
  }
  const int64_t S = a.n_samples;
  if constexpr (MODE == kFromRayZ) {
    // pts = ro + rd z (z detached): d ro += d pts, d rd += d pts z.  With S % 32 == 0 the
    // wave's 32 samples are one ray: sum over the lane half first, one atomic per value.
    float gro[3], grd[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      gro[d] = valid ? dx[d] : 0.0f;
      grd[d] = valid ? dx[d] * zv : 0.0f;
    }
    const bool one_ray = S % 32 == 0;
    if (one_ray) {
#pragma unroll
      for (int off = 16; off >= 1; off >>= 1)
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          gro[d] += __shfl_xor(gro[d], off);
          grd[d] += __shfl_xor(grd[d], off);
        }
    }
    if (valid && s.h == 0 && (!one_ray || (s.lane & 31) == 0)) {
      const int64_t ray = rc / S;
      if constexpr (DET) {
        // deterministic form (one ray per wave, host-checked): the wave's sums as its row of ray_part
        // (lane 0's rc is the wave's first sample, a multiple of 32)
        if (a.ray_part) {
          float* p = a.ray_part + (rc >> 5) * 6;
          for (int d = 0; d < 3; ++d) {
            p[d] = gro[d];
            p[3 + d] = grd[d];
          }
        }
      } else {
        if (a.d_ro)
          for (int d = 0; d < 3; ++d) atomicAdd(a.d_ro + 3 * ray + d, gro[d]);
        if (a.d_rd)
          for (int d = 0; d < 3; ++d) atomicAdd(a.d_rd + 3 * ray + d, grd[d]);
      }
    }
  }
  if (valid && s.h == 0) {
    const int64_t ray = rc / S, smp = rc - ray * S;
    if constexpr (MODE != kFromRayZ) {
      if (a.d_pts)
        for (int d = 0; d < 3; ++d) a.d_pts[3 * rc + d] = dx[d];
    }
    if (a.d_rd) {
      // Q1 view direction vd = rd[dray] / |rd[dray]|: d rd[dray] += (g - vd (vd . g)) / |rd[dray]|
      const int64_t base = (ray / a.chunk_rows) * a.chunk_rows;
      const int64_t rcnt = min(a.chunk_rows, a.n_rays - base);
      const int64_t dray = base + ((ray - base) * S + smp) % rcnt;
      const float d0 = a.rd[3 * dray], d1 = a.rd[3 * dray + 1], d2 = a.rd[3 * dray + 2];
      const float nrm = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
      const float dot = in.vd[0] * dv[0] + in.vd[1] * dv[1] + in.vd[2] * dv[2];
      if constexpr (DET) {
        for (int d = 0; d < 3; ++d) a.q1_part[3 * rc + d] = (dv[d] - in.vd[d] * dot) / nrm;
      } else {
        for (int d = 0; d < 3; ++d) atomicAdd(a.d_rd + 3 * dray + d, (dv[d] - in.vd[d] * dot) / nrm);
      }
    }
  }
}

template <int MODE, bool TRAIN = false, bool NOGEO = false, bool DET = false>
__global__ __launch_bounds__(kThreads, 1) void field_x3_bwd_kernel(FieldArgs a) {
  static_assert(!NOGEO || TRAIN, "the no-geometry schedule is the training backward's");
  __shared__ __attribute__((aligned(16))) float4 lds[kLdsQuads + kBwdLdsFloats / 4];
  float* blds = reinterpret_cast<float*>(lds + kLdsQuads);
  State s;
  s.lane = threadIdx.x & 63;
  s.h = s.lane >> 5;
  s.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  s.wsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.packed), 0, kPackedFloats * 4, 0x00020000);
  s.voff = static_cast<unsigned>(s.wave * 64 + s.lane) * 16u;
  s.sv = nullptr;
  s.cbase = 0;
#pragma unroll
  for (int k = 0; k < kConsts / kThreads; ++k)
    blds[k * kThreads + threadIdx.x] = a.packed[kBiasXyz1 + k * kThreads + threadIdx.x];
  for (int j = threadIdx.x; j < kBwdLdsFloats - kGaccOff; j += kThreads) blds[kGaccOff + j] = 0.0f;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kDmaPerWave; ++i) dma_piece(s, lds, 0, i);
#pragma unroll
  for (int i = 0; i < kDmaPerWave; ++i) dma_piece(s, lds, 1, i);
#pragma unroll
  for (int i = 0; i < kDmaPerWave / 2; ++i) dma_piece(s, lds, 2, i);
  int cur_code = -1;
  const int64_t n_tiles = (a.m + kTile - 1) / kTile;
  int crun = 0;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x)
    bwd_tile<MODE, TRAIN, NOGEO, DET>(s, a, lds, blds, tile, cur_code, crun);
  __builtin_amdgcn_s_waitcnt(0x0F70);
  if constexpr (DET) {
    // deterministic form (one code row, host-checked): this wave's g_code row into its gc_part row
    // (every wave writes its row, zeros included)
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const float* row = blds + kGaccOff + s.wave * kCbStride;
    float* out = a.gc_part + ((int64_t)blockIdx.x * kWaves + s.wave) * kCbStride;
#pragma unroll
    for (int k = 0; k < (kCbStride + 63) / 64; ++k) {
      const int j = s.lane + 64 * k;
      if (j < kCbStride) out[j] = row[j];
    }
  } else if (cur_code >= 0) {
    flush_gcode(s, a, blds, cur_code);
  }
}

static_assert(kTChunkX1 + 2 == kChunks, "backward chunk schedule");
static_assert(kTChunkDir == kNoGeoSkip && kTChunkDir + 1 == kTChunkOut, "no-geometry stream: skips the d-dir chunk");
static_assert(kBwdLdsFloats * 4 + kLdsQuads * 16 <= 160 * 1024, "LDS budget");

}  // namespace x3

int64_t packed_floats_x3() { return x3::kPackedFloats; }

int launch_pack_x3(const Params& P, float* packed, hipStream_t st) {
  const int64_t n = (int64_t)x3::kQuads * 8 + x3::kConsts;
  hipLaunchKernelGGL(x3::pack_x3_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0, st, P, packed);
  return cn::launch_status();
}

// Workgroups of the persistent grid: one per CU (the kernel holds a CU's LDS and
// every SIMD's registers), never more than there are tiles.
static int64_t cu_count() {
  static int n[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (n[dev] == 0) {
    int v = 0;
    n[dev] = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
  }
  return n[dev];
}

int launch_pack_x3t(const Params& P, float* packed, hipStream_t st) {
  const int64_t n = (int64_t)x3::kQuads * 8 + x3::kConsts;
  hipLaunchKernelGGL(x3::pack_x3t_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0, st, P, packed);
  return cn::launch_status();
}

int64_t mask_words_x3(int64_t m) { return cn::ceil_div(m, x3::kTile) * x3::kMaskWordsPerTile; }

int launch_field_x3_bwd(int mode, FieldArgs& a, hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(
      std::min<int64_t>(std::min<int64_t>(cn::ceil_div(a.m, x3::kTile), cu_count()), kMaxBwdBlocks));
  a.n_blocks = grid;
  if (a.dpre && !a.d_pts && !a.d_ro && !a.d_rd && nogeo_enabled()) {
    switch (mode) {
      case kFromPts: hipLaunchKernelGGL((x3::field_x3_bwd_kernel<kFromPts, true, true>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
      case kFromRayZ: hipLaunchKernelGGL((x3::field_x3_bwd_kernel<kFromRayZ, true, true>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
      default: return CN_EUNSUPPORTED;
    }
    return cn::launch_status();
  }
  if (a.dpre) {
    switch (mode) {
      case kFromPts: hipLaunchKernelGGL((x3::field_x3_bwd_kernel<kFromPts, true>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
      case kFromRayZ: hipLaunchKernelGGL((x3::field_x3_bwd_kernel<kFromRayZ, true>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
      default: return CN_EUNSUPPORTED;
    }
    return cn::launch_status();
  }
  if (a.gc_part) {   // the eval backward without float atomics (cn_field_backward_fused_ws)
    switch (mode) {
      case kFromPts: hipLaunchKernelGGL((x3::field_x3_bwd_kernel<kFromPts, false, false, true>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
      case kFromRayZ: hipLaunchKernelGGL((x3::field_x3_bwd_kernel<kFromRayZ, false, false, true>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
      default: return CN_EUNSUPPORTED;
    }
    return cn::launch_status();
  }
  switch (mode) {
    case kFromPts: hipLaunchKernelGGL(x3::field_x3_bwd_kernel<kFromPts>, dim3(grid), dim3(x3::kThreads), 0, st, a); break;
    case kFromRayZ: hipLaunchKernelGGL(x3::field_x3_bwd_kernel<kFromRayZ>, dim3(grid), dim3(x3::kThreads), 0, st, a); break;
    default: return CN_EUNSUPPORTED;
  }
  return cn::launch_status();
}

int launch_field_x3(int mode, FieldArgs& a, hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(std::min<int64_t>(cn::ceil_div(a.m, x3::kTile), cu_count()));
  if (a.masks && a.save) {
    switch (mode) {
      case kFromPts: hipLaunchKernelGGL((x3::field_x3_kernel<kFromPts, true, true>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
      case kFromRayZ: hipLaunchKernelGGL((x3::field_x3_kernel<kFromRayZ, true, true>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
      default: return CN_EUNSUPPORTED;
    }
    return cn::launch_status();
  }
  if (a.masks) {
    switch (mode) {
      case kFromPts: hipLaunchKernelGGL((x3::field_x3_kernel<kFromPts, true>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
      case kFromRayZ: hipLaunchKernelGGL((x3::field_x3_kernel<kFromRayZ, true>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
      default: return CN_EUNSUPPORTED;
    }
    return cn::launch_status();
  }
  switch (mode) {
    case kFromPts: hipLaunchKernelGGL((x3::field_x3_kernel<kFromPts, false>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
    case kFromRayZ: hipLaunchKernelGGL((x3::field_x3_kernel<kFromRayZ, false>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
    default: hipLaunchKernelGGL((x3::field_x3_kernel<kFromEncoded, false>), dim3(grid), dim3(x3::kThreads), 0, st, a); break;
  }
  return cn::launch_status();
}

}  // namespace mlp
}  // namespace cn
