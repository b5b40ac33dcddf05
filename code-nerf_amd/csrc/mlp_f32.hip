// fp32 field kernel, v2: the fused posenc + CodeNeRF MLP of mlp.hip (forward_pass,
// view_synthesis/nerf/__init__.py:94-134 + CodeNeRFModel.forward, models/model.py:160-194)
// on v_mfma_f32_16x16x4_f32 -- exact fp32 products and fp32 accumulation (an fmaf chain
// per MFMA), the reference's arithmetic -- at TWO waves per SIMD.
//
// Why 16x16x4 and not 32x32x2.  Both run at the fp32 peak (64 FLOP/clk/SIMD), but a
// 32-sample wave tile needs a 256-wide input AND a 256-wide output held in registers
// (~300 VGPRs: one wave per SIMD).  A lone wave leaves the matrix pipe idle at every
// barrier, LDS-read wait and layer epilogue.  A 16-sample tile holds the same two
// 256-vectors in 64 + 64 registers, so two waves share each SIMD and one's MFMAs cover
// the other's stalls.  Tile = 8 waves x 16 samples = 128 samples per workgroup.
//
// Register dataflow (as in mlp_layout.h, for the 16x16 shape).  D = W x X^T with
// A = 16 rows of W (lane l: row l & 15, k-step input g = l >> 4), B = the samples'
// inputs (lane l: sample l & 15, input g), D = 16 output features x 16 samples with
// feature 4(l >> 4) + r in register r.  So accumulator block ob, register r is the next
// layer's B operand for k-step 4ob + r: lane group g feeds input feature 16ob + 4g + r.
// The pack applies that permutation to every W once; activations never leave registers.
// The positional encodings are spread the same way: lane group g computes the sin/cos
// of pairs p = 4i + g (7-8 sincosf per lane for xyz, 3 for the view direction).
//
// Weight stream.  Chunk = 8 k-steps x 16 output blocks x 64 lanes = 32 KiB, laid out
// [k-step][block quad q][lane][block 4q..4q+3] so a lane's A values of one k-step are 4
// ds_read_b128 of a 1 KiB contiguous run (conflict free).  36 chunks per tile
// (xyz1 2 | xyz2 8 | fc_out 8 | dir1 8 + view-dir 1 | dir2 8 | rgb 1) stream through a
// 4-slot LDS ring by LDS-DMA (buffer_load_dwordx4 ... lds; 4 wave-instructions per wave
// per chunk).  One barrier M_c in the middle of chunk c: chunk c+1 has landed (counted
// vmcnt) and every wave is done with chunk c-1, whose slot then receives chunk c+3.  The
// first A fragments of chunk c+1 are read during chunk c's last k-step, so the matrix
// pipe never waits on a chunk boundary.  The stream is cyclic across tiles.
//
// sigma (fc_out row 0) is an fp32 dot product over layer_xyz2's outputs taken in the
// xyz2 epilogue (32 packed FMAs per lane + a 4-group butterfly); fc_rgb the same way for its
// 3 rows (96 packed FMAs per lane, weights from the rgb chunk's ring slot) -- as one 16-row
// MFMA block over 64 k-steps (r03, removed) 13 of its 16 rows were padding.
#include <algorithm>

#include "mlp_common.h"

namespace cn {
namespace mlp {
namespace w16 {

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef unsigned uint4v __attribute__((ext_vector_type(4)));
typedef unsigned uint2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kTile = 16 * kWaves;            // samples per workgroup tile
constexpr int kStepQuads = 16 * 64 / 4;       // one 16-block k-step: 256 float4 (4 KiB)
constexpr int kChunkSteps = 8;
constexpr int kChunkQuads = kChunkSteps * kStepQuads;   // 2048 float4 = 32 KiB
constexpr int kRing = 4;
constexpr int kPiecesPerWave = kChunkQuads / (64 * kWaves);   // 4 x 1 KiB per wave per chunk
// the stream: xyz1 2 | xyz2 8 | fc_out 8 | dir1 8 | dir1 view-dir 1 | dir2 8 | rgb 1
constexpr int kCL2 = 2, kCL3 = 10, kCL4 = 18, kCDir = 26, kCL5 = 27, kCRgb = 35, kChunks = 36;
constexpr int kStreamFloats = kChunks * kChunkQuads * 4;
constexpr int kRgbValu = 64 * 64;  // float offset of fc_rgb's VALU-form rows inside the rgb chunk
// constants after the stream: b_xyz1 | b_dir1 | b_dir2 | sigma weights (fc_out row 0 over
// h2, [g][ob][r] = W_out[0][16 ob + 4 g + r])
constexpr int kCB1 = 0, kCBD1 = 256, kCBD2 = 512, kCSig = 768, kConsts = 1024;
constexpr int kPackedFloats = kStreamFloats + kConsts;
// LDS constants: the packed ones, then the encoding frequencies (fx[10] | fd[4] | pad 2): a
// lane-varying index into the kernel arguments is a global load per use (or a register held
// across the tile loop), an LDS read is neither; the pad holds the largest |fx| and |fd|
constexpr int kCFreq = kConsts, kLdsConsts = kConsts + 16;
// LDS: the ring, the constants, one code-bias row per wave
constexpr int kLdsQuads = kRing * kChunkQuads + (kLdsConsts + kWaves * kCbStride) / 4;

static_assert(kChunks % kRing == 0, "cyclic stream: chunk c + 36 reuses chunk c's ring slot");
__host__ __device__ constexpr int col_enc_xyz(int t, int g);
constexpr bool xenc_map_ok(int cp = 0) {
  return cp == 64 || (xenc_col(cp) == col_enc_xyz(cp & 15, cp >> 4) && xenc_map_ok(cp + 1));
}
static_assert(kPiecesPerWave == 4, "4 DMA wave-instructions per chunk per wave");
static_assert(kLdsQuads * 16 <= 160 * 1024, "LDS budget");

// ---------------------------------------------------------------- feature maps

// Input feature (256-wide previous-layer output) fed at k-step t by lane group g.
__host__ __device__ constexpr int col_acc(int t, int g) { return 16 * (t >> 2) + 4 * g + (t & 3); }

// xyz encoding column (position_embed.py:44-53: x_d -> d, sin(f_k x_d) -> 3+6k+d,
// cos(f_k x_d) -> 6+6k+d) fed at k-step t (0..15) by lane group g: sines of pairs
// p = 4i + g at t = i, cosines at t = 8 + i; groups 2, 3 have 7 pairs and put the raw
// inputs in the free k-steps 7 / 15 (x0, x1 | x2, pad).
__host__ __device__ constexpr int col_enc_xyz(int t, int g) {
  const int i = t & 7, p = 4 * i + g;
  if (p < 30) return (t < 8 ? 3 : 6) + 6 * (p / 3) + p % 3;
  return t < 8 ? (g == 2 ? 0 : 2) : (g == 2 ? 1 : -1);
}

static_assert(xenc_map_ok(), "the encoding plane's column map is layer_xyz1's k-step feature map");

// View-direction encoding column (27 wide) at k-step s (0..6) of the view-dir chunk:
// sines of pairs p = 4i + g at s = i (i < 3), cosines at s = 3 + i, raw component g at s = 6.
__host__ __device__ constexpr int col_enc_dir(int s, int g) {
  if (s < 6) {
    const int p = 4 * (s % 3) + g;
    return (s < 3 ? 3 : 6) + 6 * (p / 3) + p % 3;
  }
  return (s == 6 && g < 3) ? g : -1;
}

// ---------------------------------------------------------------- packing

// Elements idx0, idx0 + stride, ... of the CN_FMT_F32_W16 pack (pack_w16_kernel; a role of
// field_prepare_kernel).
__device__ __forceinline__ void pack_w16_range(const Params& P, float* __restrict__ packed, int idx0, int stride) {
  for (int idx = idx0; idx < kPackedFloats; idx += stride) {
    float v = 0.0f;
    if (idx >= kStreamFloats) {
      const int j = idx - kStreamFloats;
      if (j < 256) v = P.p[kBXyz1][j];
      else if (j < 512) v = P.p[kBDir1][j - 256];
      else if (j < 768) v = P.p[kBDir2][j - 512];
      else {
        const int t = j - kCSig, g = t >> 6, ob = (t >> 2) & 15, r = t & 3;
        v = P.p[kWOut][16 * ob + 4 * g + r];  // fc_out row 0, input feature 16 ob + 4 g + r of h2
      }
    } else {
      const int c = idx / (kChunkQuads * 4), rem = idx % (kChunkQuads * 4);
      if (c == kCRgb) {
        // fc_rgb: 64 k-steps of block 0, [k-step quad][lane][k-step & 3] (the former MFMA form,
        // not read any more; the chunk keeps its size and place in the stream), then at kRgbValu
        // rows 0..2 over v2 for the VALU form,
        // [row][g][ob][r] = W_rgb[row][16 ob + 4 g + r]
        if (rem < 64 * 64) {
          const int lane = (rem % 256) / 4, t = 4 * (rem / 256) + rem % 4;
          const int i = lane & 15, g = lane >> 4;
          if (i < 3) v = P.p[kWRgb][i * (kHidden + kCode) + col_acc(t, g)];
        } else if (rem >= kRgbValu && rem < kRgbValu + 3 * 256) {
          const int t = rem - kRgbValu, i = t >> 8, g = (t >> 6) & 3, ob = (t >> 2) & 15, r = t & 3;
          v = P.p[kWRgb][i * (kHidden + kCode) + 16 * ob + 4 * g + r];
        }
      } else {
        const int s = rem / (kStepQuads * 4), q = (rem % (kStepQuads * 4)) / 256;
        const int lane = (rem % 256) / 4, ob = 4 * q + rem % 4;
        const int i = lane & 15, g = lane >> 4;
        int row = 16 * ob + i, col = -1, in_dim = 0;
        const float* W = nullptr;
        if (c < kCL2) { W = P.p[kWXyz1]; in_dim = kDimXyz; col = col_enc_xyz(8 * c + s, g); }
        else if (c < kCL3) { W = P.p[kWXyz2]; in_dim = kHidden + kCode; col = col_acc(8 * (c - kCL2) + s, g); }
        else if (c < kCL4) { W = P.p[kWOut]; in_dim = kHidden + kCode; row += 1; col = col_acc(8 * (c - kCL3) + s, g); }
        else if (c < kCDir) { W = P.p[kWDir1]; in_dim = kCode + kDimDir; col = col_acc(8 * (c - kCL4) + s, g); }
        else if (c == kCDir) {
          W = P.p[kWDir1]; in_dim = kCode + kDimDir;
          const int e = col_enc_dir(s, g);
          col = e < 0 ? -1 : kCode + e;
        } else { W = P.p[kWDir2]; in_dim = kHidden; col = col_acc(8 * (c - kCL5) + s, g); }
        if (col >= 0) v = W[row * in_dim + col];
      }
    }
    packed[idx] = v;
  }
}

__global__ void pack_w16_kernel(Params P, float* __restrict__ packed) {
  pack_w16_range(P, packed, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}

// ---------------------------------------------------------------- kernel state

struct State {
  floatx4 act[16];   // layer input: block ob register r = input feature 16 ob + 4 g + r
  floatx4 acc[16];   // layer output accumulators
  floatx4 pre[4];    // the next chunk's first A fragments (read during this chunk's last k-step)
  floatx4 acc2[4];   // backward: the narrow chunks' accumulators (2 blocks x 2 chains)
  float denc[8];     // view-direction encoding, k-steps of the view-dir chunk
  float sig;         // sigma partial (this lane group's 64 features)
  int lane, g, wave;
  int crow;          // this lane's code-bias row
  bool uniform_code; // all 16 samples of the wave use one code row
  __amdgpu_buffer_rsrc_t wsrc;
  unsigned voff;
  unsigned poff;     // this lane's byte offset in a (kTile, 256) fp32 plane block: row 16 wave + (lane & 15), col 4 g
  unsigned gbase;    // backward: this lane's byte offset in a 256-float sum row (rowsum64's features)
  int cbase;         // no-geometry backward: chunk counter at the tile's first chunk (stream_src)
};

// The kernel's LDS constants (after the ring): the packed ones and the encoding frequencies.
__device__ __forceinline__ void load_consts(const FieldArgs& a, float* clds) {
  for (int k = threadIdx.x; k < kConsts; k += kThreads) clds[k] = a.packed[kStreamFloats + k];
  if (threadIdx.x < 16) {
    const int t = threadIdx.x;
    float mx = 0.0f, md = 0.0f;  // the largest |frequency| of each encoding (fast_sincosf's range check)
#pragma unroll
    for (int k = 0; k < 10; ++k) mx = fmaxf(mx, fabsf(a.fx[k]));
#pragma unroll
    for (int k = 0; k < 4; ++k) md = fmaxf(md, fabsf(a.fd[k]));
    clds[kCFreq + t] = t < 10 ? a.fx[t] : (t < 14 ? a.fd[t - 10] : (t == 14 ? mx : md));
  }
}

// A buffer resource over rows [tile kTile, tile kTile + kTile) of plane `plane` of a (planes, m, 256)
// fp32 array (wave-uniform base; rows past m fall outside num_records, so their stores are dropped
// and their loads read 0 -- no per-lane 64-bit address arithmetic, no validity branch).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t plane_rsrc(const float* base, int plane, int64_t m, int64_t tile) {
  const int64_t r0 = tile * kTile;
  const int64_t rows = m - r0 < kTile ? m - r0 : kTile;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(base) + ((int64_t)plane * m + r0) * 256, 0,
                                           static_cast<int>(rows * 1024), 0x00020000);
}

// The tile's mask block: kMaskLayers x 64 uint2 per wave.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mask_rsrc(const unsigned* masks, int64_t tile);

// The 16 blocks' column offsets fold into the instructions' immediate field because the lane
// offset is "fresh" here (otherwise LICM hoists the 16 sums out of the tile loop into VGPRs, or,
// as soffsets, into 16 SGPRs that then spill into VGPR lanes).
__device__ __forceinline__ int fresh(int v);
// Plane stores are non-temporal (cpol 2): the 400 MB of planes per C3 chunk never fit the L2, and
// write-back stores evicted the weight stream (forward FETCH 58 -> 6 MB per launch, the backward
// that reads them 1.5 % faster; r03i).
constexpr int kPlaneCPol = 2;
template <int B0 = 0, int NB = 16>
__device__ __forceinline__ void store_plane(const State& s, __amdgpu_buffer_rsrc_t r, const floatx4* v) {
  const unsigned off = static_cast<unsigned>(fresh(static_cast<int>(s.poff)));
#pragma unroll
  for (int ob = B0; ob < B0 + NB; ++ob)
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, v[ob]), r, off + 64u * ob, 0, kPlaneCPol);
}


// The packed chunk the chunk counter cn streams.  The forward and the geometry backward run the
// whole 36-chunk stream from cn = 0 in every tile.  NG: the no-geometry training backward streams
// 33 of the transposed pack's chunks (not the view-direction chunk kNoGeoSkip, nor the two
// layer_xyz1^T chunks at the end); 33 is not a multiple of the ring, so its counter runs on across
// tiles (ring slot cn & 3) and s.cbase is the counter at the tile's first chunk.
constexpr int kNoGeoSkip = 17, kNoGeoChunks = kChunks - 3;
__device__ __forceinline__ int stream_src_ng(const State& s, int cn) {
  int k = cn - s.cbase;
  if (k >= kNoGeoChunks) k -= kNoGeoChunks;
  return k + (k >= kNoGeoSkip ? 1 : 0);
}

// One LDS-DMA piece: 1 KiB of chunk cn (piece p of 4 for this wave).
template <bool NG = false>
__device__ __forceinline__ void dma_piece(const State& s, float4* lds, int cn, int p) {
  const int src = NG ? stream_src_ng(s, cn) : (cn < kChunks ? cn : cn - kChunks);
  const unsigned soff = __builtin_amdgcn_readfirstlane((unsigned)(src * kChunkQuads + p * 64 * kWaves) * 16u);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(
      s.wsrc, (lds_ptr_t)(lds + (cn & (kRing - 1)) * kChunkQuads + p * 64 * kWaves + s.wave * 64), 16, s.voff,
      soff, 0, 0);
}

template <bool NG = false>
__device__ __forceinline__ void dma_chunk(const State& s, float4* lds, int cn) {
#pragma unroll
  for (int p = 0; p < kPiecesPerWave; ++p) dma_piece<NG>(s, lds, cn, p);
}

// M_c: chunk c+1 landed for every wave (all but this wave's 4 youngest DMA pieces --
// chunk c+2's -- retired), every wave past chunk c-1, this wave's LDS reads returned.
__device__ __forceinline__ void chunk_barrier() {
  asm volatile("s_waitcnt vmcnt(4)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// A fragments of k-step T (16 blocks) of the chunk at `slot` (float4 units, lane applied).
template <int T>
__device__ __forceinline__ void read_a(const float4* slot, floatx4* a) {
#pragma unroll
  for (int q = 0; q < 4; ++q) a[q] = *reinterpret_cast<const floatx4*>(slot + T * kStepQuads + q * 64);
}

__device__ __forceinline__ void mfma_step(State& s, const floatx4* a, float b) {
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      s.acc[4 * q + j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][j], b, s.acc[4 * q + j], 0, 0, 0);
}

// Scheduling of one k-step: the 4 A reads of the next k-step between the first MFMAs.
__device__ __forceinline__ void step_pattern() {
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
  }
  __builtin_amdgcn_sched_group_barrier(0x008, 12, 0);
}

// A k-step with VALU work of its own (LazyXyz): the A reads and 2-3 VALU instructions between
// consecutive MFMAs, the remainder after the last.
__device__ __forceinline__ void lazy_step_pattern() {
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
  }
#pragma unroll
  for (int m = 0; m < 12; ++m) {
    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);
  }
}

// Nothing to issue during a chunk.
struct NoPost {
  template <int CI, int T>
  __device__ __forceinline__ void step() const {}
  template <int CI>
  __device__ __forceinline__ void before_dma() const {}
};

// One 16-block chunk of NS k-steps; the B operand of k-step T is getb(T) (compile time).
// The last k-step reads the next chunk's first fragments into s.pre.  `post.step<CI, T>()` runs
// after k-step T's MFMAs (after the barrier and the DMA at T = 3) of the layer's chunk CI: the
// previous layer's plane / mask stores go there, spread over the layer (the layer input they save
// is this layer's B operand, live anyway).  Issued in bursts -- 16 per wave at the epilogue or
// after a barrier -- the stores of the CU's 8 waves queued in the vector-memory path with the
// weight stream's DMA and cost each wave ~250 cycles of issue stall and waitcnt per store (PMC,
// r03g: SQ_WAIT_INST_ANY +77 M and SQ_WAIT_ANY +55 M quad-cycles over the mask-only forward for
// 2.09 M stores); two per chunk they overlap the MFMAs.  They follow the chunk's DMA, so the next
// barrier's counted vmcnt still sees the ring's pieces in order.
template <int NS, int CI = 0, bool NG = false, typename GetB, typename Post = NoPost>
__device__ __forceinline__ void chunk16(State& s, float4* lds, int c, GetB getb, Post post = Post{}) {
  const float4* slot = lds + (c & (kRing - 1)) * kChunkQuads + s.lane;
  const float4* nslot = lds + ((c + 1) & (kRing - 1)) * kChunkQuads + s.lane;
  floatx4 a0[4], a1[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) a0[q] = s.pre[q];
  __builtin_amdgcn_sched_barrier(0);
#define CN_STEP(T, CUR, NXT)                                         \
  if constexpr ((T) < NS) {                                         \
    if constexpr ((T) + 1 < NS) read_a<(T) + 1>(slot, NXT);         \
    else read_a<0>(nslot, s.pre);                                   \
    mfma_step(s, CUR, getb.template at<(T)>());                     \
    getb.template prep<(T)>();                                      \
    if constexpr (GetB::kLazy) lazy_step_pattern();                 \
    else step_pattern();                                            \
    __builtin_amdgcn_sched_barrier(0);                              \
    if constexpr ((T) == 3) {                                       \
      chunk_barrier();                                              \
      post.template before_dma<CI>();                               \
      dma_chunk<NG>(s, lds, c + 3);                                 \
    }                                                               \
    post.template step<CI, (T)>();                                  \
  }
  CN_STEP(0, a0, a1)
  CN_STEP(1, a1, a0)
  CN_STEP(2, a0, a1)
  CN_STEP(3, a1, a0)
  CN_STEP(4, a0, a1)
  CN_STEP(5, a1, a0)
  CN_STEP(6, a0, a1)
  CN_STEP(7, a1, a0)
#undef CN_STEP
}

// B sources
template <int K0>
struct ActB {
  const State& s;
  template <int T>
  __device__ __forceinline__ float at() const {
    constexpr int t = K0 + T;
    return s.act[t >> 2][t & 3];
  }
  static constexpr bool kLazy = false;
  template <int T>
  __device__ __forceinline__ void prep() const {}
};
template <int K0>
struct ArrB {
  const float* v;
  template <int T>
  __device__ __forceinline__ float at() const { return v[K0 + T]; }
  static constexpr bool kLazy = false;
  template <int T>
  __device__ __forceinline__ void prep() const {}
};

// layer_xyz1's B operands computed where they are consumed: in its first chunk, k-step T's MFMAs
// use the sine of pair T (lane group g: pair p = 4 T + g) and, issued after them, the (sin, cos) of
// pair T + 1 is evaluated (fast_sincosf, branch-free), so its VALU fills the MFMAs' shadow instead
// of a tile prologue that both waves of every SIMD ran at once with the matrix pipe idle (~2.7 % of
// the inference forward's tile time, r03s).  The second chunk consumes the cosines and evaluates
// the three view-direction pairs and the raw direction component the view-dir chunk takes later.
struct LazyXyz {
  float (&enc)[16];
  float (&denc)[8];
  const float (&x)[3];
  const float (&vd)[3];
  const float (&fr)[11];  // this lane group's frequencies: pairs 0..7 (xyz), 0..2 (view direction)
  int g;
  bool second;            // the chunk of the cosines (k-steps 8..15)
  static constexpr bool kLazy = true;
  template <int T>
  __device__ __forceinline__ float at() const { return second ? enc[8 + T] : enc[T]; }
  // c ? a : b on the bits (lane-varying selects written as ternaries came out as EXEC-masked
  // branches here, which split the k-step's block and stopped the MFMA / VALU interleave)
  static __device__ __forceinline__ float bsel(bool c, float a, float b) {
    const int m = -static_cast<int>(c);
    return __int_as_float((__float_as_int(a) & m) | (__float_as_int(b) & ~m));
  }
  static __device__ __forceinline__ float sel3(const float (&v)[3], int c) {
    return bsel(c == 0, v[0], bsel(c == 1, v[1], v[2]));
  }
  // sin / cos of pair I of this lane group (I < 7, or groups 0, 1 at I = 7); groups 2, 3 take raw
  // inputs at I = 7 (col_enc_xyz).  p = 4 I + g: p % 3 = (I % 3 + g) mod 3, p / 3 = (11 p) >> 5
  // (exact for p < 32), no divisions.
  template <int I>
  __device__ __forceinline__ void pair() const {
    const int p = 4 * I + g;
    const int c0 = I % 3 + g;
    const int comp = c0 >= 3 ? c0 - 3 : c0;
    float sn, cs;
    fast_sincosf(__fmul_rn(sel3(x, comp), fr[I]), sn, cs);
    if constexpr (I == 7) {
      const bool raw = p >= 30;
      sn = bsel(raw, bsel(g == 2, x[0], x[2]), sn);
      cs = bsel(raw, bsel(g == 2, x[1], 0.0f), cs);
    }
    enc[I] = sn;
    enc[8 + I] = cs;
  }
  template <int T>
  __device__ __forceinline__ void prep() const {
    if (!second) {
      if constexpr (T + 1 < 8) pair<T + 1>();
    } else if constexpr (T < 3) {
      const int c0 = T + g;
      const int comp = c0 >= 3 ? c0 - 3 : c0;
      fast_sincosf(__fmul_rn(sel3(vd, comp), fr[8 + T]), denc[T], denc[3 + T]);
    } else if constexpr (T == 3) {
      denc[6] = bsel(g == 3, 0.0f, sel3(vd, g));
      denc[7] = 0.0f;
    }
  }
};

// A 256-input layer: 8 chunks, B from s.act.
template <bool NG = false, typename Post = NoPost>
__device__ __forceinline__ void layer256(State& s, float4* lds, int& c, Post post = Post{}) {
  chunk16<8, 0, NG>(s, lds, c + 0, ActB<0>{s}, post);
  chunk16<8, 1, NG>(s, lds, c + 1, ActB<8>{s}, post);
  chunk16<8, 2, NG>(s, lds, c + 2, ActB<16>{s}, post);
  chunk16<8, 3, NG>(s, lds, c + 3, ActB<24>{s}, post);
  chunk16<8, 4, NG>(s, lds, c + 4, ActB<32>{s}, post);
  chunk16<8, 5, NG>(s, lds, c + 5, ActB<40>{s}, post);
  chunk16<8, 6, NG>(s, lds, c + 6, ActB<48>{s}, post);
  chunk16<8, 7, NG>(s, lds, c + 7, ActB<56>{s}, post);
  c += 8;
}

// A per-lane value the compiler must treat as new here: the lane-derived addresses built from it
// are formed where they are used instead of being hoisted out of the tile loop (loop-invariant,
// so LICM would keep e.g. all 16 block addresses of a bias vector in VGPRs for the whole kernel).
__device__ __forceinline__ int fresh(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// Bias-initialise the 16 accumulators from a 256-vector (row 16 ob + 4 g + r): one address, the
// blocks at immediate offsets.
__device__ __forceinline__ void bias_from(State& s, const float* v) {
  const floatx4* p = reinterpret_cast<const floatx4*>(v) + fresh(s.g);
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) s.acc[ob] = p[4 * ob];
}

// The code-bias vector at `off` of this lane's code row: the wave's LDS copy, or (codes
// varying inside the wave) a per-lane global read.
__device__ __forceinline__ void bias_code(State& s, const FieldArgs& a, const float* crow_lds, int off) {
  if (s.uniform_code) {
    bias_from(s, crow_lds + off);
  } else {
    bias_from(s, a.code_bias + (int64_t)s.crow * kCbStride + off);
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): nothing ordinary stays in flight in the stream
  }
}

// ReLU masks for the fused backward: 4 layers (h1, h2, v1, v2) x 64 bits per lane (bit 4 ob + r
// of feature 16 ob + 4 g + r: pre-activation > 0), one 8-B store per lane per layer.
constexpr int kMaskLayers = 4;
constexpr int kMaskWordsPerTile = kWaves * kMaskLayers * 64 * 2;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t mask_rsrc(const unsigned* masks, int64_t tile) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned*>(masks) + tile * kMaskWordsPerTile, 0,
                                           kMaskWordsPerTile * 4, 0x00020000);
}
// Byte offset of (wave, layer ml) in a tile's mask block (soffset; the lane's 8 lane B in voffset).
__device__ __forceinline__ unsigned mask_soff(const State& s, int ml) {
  return static_cast<unsigned>(s.wave) * kMaskLayers * 512u + 512u * ml;
}

// act = relu(acc); MASKS: also store the layer's mask bits (slot ml of the tile's mask block): bit
// 4 ob + r of word ob >> 3 (ob & 7 there).  The words are built by shifting the accumulator left
// one bit per feature, highest first: a constant 1 << n per bit would be a VOP3 literal, which
// gfx9 encodings lack, so the compiler kept all 32 of them in VGPRs across the tile loop.
// The ReLU is a signed-integer max on the bits (v_max_i32; -0 and negatives -> +0): fmaxf on an
// MFMA result came out as two v_max_f32 per value (a canonicalize, then the max).
template <bool MASKS>
__device__ __forceinline__ uint2v relu_act(State& s) {
#pragma unroll
  for (int ob = 0; ob < 16; ++ob)
#pragma unroll
    for (int r = 0; r < 4; ++r) s.act[ob][r] = __int_as_float(max(__float_as_int(s.acc[ob][r]), 0));
  unsigned w[2] = {0u, 0u};
  if constexpr (MASKS) {
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int k = 31; k >= 0; --k) {
        const float v = s.acc[8 * h + (k >> 2)][k & 3];
        w[h] = (w[h] << 1) | (v > 0.0f ? 1u : 0u);
      }
  }
  return uint2v{w[0], w[1]};
}

// The stores a layer's input leaves behind (forward): its ReLU mask words (MASKS, slot ml; ml < 0:
// none) and, SAVE, its activation plane -- two blocks per chunk of the next layer, at k-step 4
// (chunk16's `post`), the mask words with the first of them.
template <bool MASKS, bool SAVE>
struct LayerStores {
  const State& s;
  const FieldArgs& a;
  int64_t tile;
  int ml, plane;
  uint2v w;
  template <int B0, int NB>
  __device__ __forceinline__ void blocks() const {
    if constexpr (MASKS) {
      if (B0 == 0 && ml >= 0)
        __builtin_amdgcn_raw_buffer_store_b64(w, mask_rsrc(a.masks, tile), 8u * s.lane, mask_soff(s, ml), 0);
    }
    if constexpr (SAVE) store_plane<B0, NB>(s, plane_rsrc(a.save, plane, a.m, tile), s.act);
  }
  template <int CI, int T>
  __device__ __forceinline__ void step() const {
    if constexpr (T == 4) blocks<2 * CI, 2>();
  }
  template <int CI>
  __device__ __forceinline__ void before_dma() const {}
};

// Training forward: the encodings layer_xyz1 multiplied (enc[16]: this lane group's k-step values),
// as the (m, 64) encoding plane -- row = sample, lane group g's 16 values at 16 g (xenc_col) -- which
// the backward's layer_xyz1 dW reads instead of regenerating them.  Four 16-B stores per lane,
// issued in layer_xyz1's second chunk right after its barrier and before its DMA: at the next
// barrier the counted vmcnt then leaves the ring's pieces in flight, not these.
struct XencStore {
  const State& s;
  const FieldArgs& a;
  int64_t tile;
  const float (&enc)[16];
  template <int CI, int T>
  __device__ __forceinline__ void step() const {}
  template <int CI>
  __device__ __forceinline__ void before_dma() const {
    const int64_t r0 = tile * kTile;
    const int64_t rows = a.m - r0 < kTile ? a.m - r0 : kTile;
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(a.xenc + r0 * 64, 0, static_cast<int>(rows * 256),
                                                                      0x00020000);
    const unsigned off = static_cast<unsigned>(fresh((s.wave * 16 + (s.lane & 15)) * 256 + 64 * s.g));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const floatx4 v{enc[4 * q], enc[4 * q + 1], enc[4 * q + 2], enc[4 * q + 3]};
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint4v, v), r, off + 16u * q, 0, kPlaneCPol);
    }
  }
};

// Training forward: the post-activation rows the weight gradients read (h1, h2, feat, v1, v2 as
// (5, m, 256) planes, feature 16 ob + 4 g + r: one 16-B store per block per lane).


template <int MODE, bool MASKS, bool SAVE = false>
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

  // ---- encodings (lane group g owns pairs p = 4 i + g) and layer_xyz1 (63 -> 256): 2 chunks of
  // encoding k-steps.  Lazily (LazyXyz) when every lane's arguments are in fast_sincosf's range,
  // else all evaluated up front with sincosf.
  bool lazy = false;
  if constexpr (MODE != kFromEncoded) {
    const float xa = fmaxf(fmaxf(fabsf(in.x[0]), fabsf(in.x[1])), fabsf(in.x[2])) * clds[kCFreq + 14];
    const float da = fmaxf(fmaxf(fabsf(in.vd[0]), fabsf(in.vd[1])), fabsf(in.vd[2])) * clds[kCFreq + 15];
    const bool ok = xa <= kFastSinBound && da <= kFastSinBound;  // false for NaN
    lazy = __builtin_amdgcn_readfirstlane(__ballot(!ok) == 0 ? 1 : 0) != 0;
  }
  if (lazy) {
    if constexpr (MODE != kFromEncoded) {
      // the frequencies of this lane group's pairs, read once here: an LDS read inside the k-steps
      // made each wait lgkmcnt(0) on the next k-step's A fragments too
      const int g = fresh(s.g);
      float fr[11];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int p = 4 * i + g;
        fr[i] = clds[kCFreq + ((p < 30 ? p : 0) * 11 >> 5)];  // (11 p) >> 5 = p / 3 for p < 32
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) fr[8 + i] = clds[kCFreq + 10 + ((4 * i + g) * 11 >> 5)];
      const LazyXyz l0{enc, s.denc, in.x, in.vd, fr, g, false};
      l0.pair<0>();
      bias_from(s, clds + kCB1);
      chunk16<8>(s, lds, c + 0, l0);
      if constexpr (SAVE)
        chunk16<8, 0>(s, lds, c + 1, LazyXyz{enc, s.denc, in.x, in.vd, fr, g, true}, XencStore{s, a, tile, enc});
      else
        chunk16<8>(s, lds, c + 1, LazyXyz{enc, s.denc, in.x, in.vd, fr, g, true});
    }
  } else {
    if constexpr (MODE != kFromEncoded) {
      const int g = fresh(s.g);  // the pair indices below are formed here, not held across tiles
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int p = 4 * i + g;
        const int pc = p < 30 ? p : 0;
        const float arg = __fmul_rn(pick3(in.x, pc % 3), clds[kCFreq + pc / 3]);
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
        const int p = 4 * i + g;
        const float arg = __fmul_rn(pick3(in.vd, p % 3), clds[kCFreq + 10 + p / 3]);
        sincosf(arg, &s.denc[i], &s.denc[3 + i]);
      }
      s.denc[6] = s.g == 0 ? in.vd[0] : (s.g == 1 ? in.vd[1] : (s.g == 2 ? in.vd[2] : 0.0f));
    }
    s.denc[7] = 0.0f;
    bias_from(s, clds + kCB1);
    chunk16<8>(s, lds, c + 0, ArrB<0>{enc});
    if constexpr (SAVE)
      chunk16<8, 0>(s, lds, c + 1, ArrB<8>{enc}, XencStore{s, a, tile, enc});
    else
      chunk16<8>(s, lds, c + 1, ArrB<8>{enc});
  }
  c += 2;

  // ---- layer_xyz2, fc_out, layer_dir1 (+ view-dir chunk), layer_dir2
  for (int layer = kXyz2; layer <= kDir2; ++layer) {
    // activation of the previous layer's outputs: ReLU, none after fc_out (feat); its mask words
    // and its plane (h1, h2, feat, v1) are stored at this layer's first chunk barrier
    uint2v mw = uint2v{0u, 0u};
    if (layer == kDir1) {
#pragma unroll
      for (int ob = 0; ob < 16; ++ob) s.act[ob] = s.acc[ob];
    } else {
      mw = relu_act<MASKS>(s);
    }
    const LayerStores<MASKS, SAVE> st{s, a, tile, layer == kXyz2 ? 0 : (layer == kOut ? 1 : (layer == kDir2 ? 2 : -1)),
                                     layer - kXyz2, mw};
    if (layer == kOut) {
      // sigma = fc_out row 0 . [h2, zs2] + b: the h2 part here, the code part from cn_code_bias
      // (two packed chains: 32 v_pk_fma_f32 instead of one 64-deep fmaf chain)
      typedef float float2v __attribute__((ext_vector_type(2)));
      // the weights in two batches of 8 LDS reads issued together (one wait per batch; read one at
      // a time, each FMA pair waited on its own read while both waves of the SIMD sat here)
      float2v s0{0.0f, 0.0f}, s1{0.0f, 0.0f};
      const floatx4* wsig = reinterpret_cast<const floatx4*>(clds + kCSig) + 16 * fresh(s.g);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        floatx4 w[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = wsig[8 * h + k];
        __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int ob = 8 * h + k;
          s0 = __builtin_elementwise_fma(float2v{w[k][0], w[k][1]}, float2v{s.act[ob][0], s.act[ob][1]}, s0);
          s1 = __builtin_elementwise_fma(float2v{w[k][2], w[k][3]}, float2v{s.act[ob][2], s.act[ob][3]}, s1);
        }
        __builtin_amdgcn_sched_group_barrier(0x002, 16, 0);
      }
      s.sig = (s0[0] + s0[1]) + (s1[0] + s1[1]);
    }
    if (layer == kXyz2) bias_code(s, a, crow_lds, kCbXyz2);
    else if (layer == kOut) bias_code(s, a, crow_lds, kCbFeat);
    else bias_from(s, clds + (layer == kDir1 ? kCBD1 : kCBD2));
    __builtin_amdgcn_sched_barrier(0);
    layer256(s, lds, c, st);
    if (layer == kDir1) {
      chunk16<7>(s, lds, c, ArrB<0>{s.denc});
      c += 1;
    }
  }

  // ---- fc_rgb (256 -> 3): one chunk, 64 k-steps of block 0 in 4 chains
  const LayerStores<MASKS, SAVE> st_v2{s, a, tile, 3, 4, relu_act<MASKS>(s)};  // v2: at the rgb chunk's barrier
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
    s.acc[1] = s.acc[2] = s.acc[3] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
    float sg = s.sig;
    sg += __shfl_xor(sg, 16);
    sg += __shfl_xor(sg, 32);
    s.sig = sg + bs;
  }
  // fc_rgb on the VALU: 3 of the 16 MFMA rows were real, so the chunk's 64 MFMAs per wave (4 k
  // pipe cycles per SIMD and tile) became 96 packed FMAs per lane over this lane group's 64 v2
  // features, weights read from the rgb chunk's slot (it has landed: the chunk is current), then
  // the 4-group butterfly as for sigma.  The chunk keeps its place in the stream, its barrier and
  // the next tile's DMA.
  {
    typedef float float2v __attribute__((ext_vector_type(2)));
    const floatx4* wr = reinterpret_cast<const floatx4*>(lds + (c & (kRing - 1)) * kChunkQuads) +
                        (kRgbValu / 4 + 16 * fresh(s.g));
    const float4* nslot = lds + ((c + 1) & (kRing - 1)) * kChunkQuads + s.lane;
    float2v p[3][2];
#pragma unroll
    for (int i = 0; i < 3; ++i) p[i][0] = p[i][1] = float2v{0.0f, 0.0f};
    auto blocks = [&](auto b0) {
      constexpr int B0 = decltype(b0)::value;
#pragma unroll
      for (int ob = B0; ob < B0 + 8; ++ob) {
        const float2v x0{s.act[ob][0], s.act[ob][1]}, x1{s.act[ob][2], s.act[ob][3]};
#pragma unroll
        for (int i = 0; i < 3; ++i) {
          const floatx4 w = wr[64 * i + ob];
          p[i][0] = __builtin_elementwise_fma(float2v{w[0], w[1]}, x0, p[i][0]);
          p[i][1] = __builtin_elementwise_fma(float2v{w[2], w[3]}, x1, p[i][1]);
        }
      }
    };
    blocks(std::integral_constant<int, 0>{});
    chunk_barrier();
    dma_chunk(s, lds, c + 3);
    st_v2.template blocks<0, 8>();
    blocks(std::integral_constant<int, 8>{});
    st_v2.template blocks<8, 8>();
    read_a<0>(nslot, s.pre);
    c += 1;
    float rgb[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      float v = (p[i][0][0] + p[i][0][1]) + (p[i][1][0] + p[i][1][1]);
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 32);
      rgb[i] = v;
    }
    if (valid && s.g == 0) {
      float4 o;
      o.x = rgb[0] + s.acc[0][0];  // the code-bias terms (lane group 0's acc[0], set above)
      o.y = rgb[1] + s.acc[0][1];
      o.z = rgb[2] + s.acc[0][2];
      o.w = s.sig;
      reinterpret_cast<float4*>(a.raw)[row] = o;
    }
  }
}


template <int MODE, bool MASKS, bool SAVE = false>
__global__ __launch_bounds__(kThreads, 2) void field_w16_kernel(FieldArgs a) {
  // ONE LDS object (a second one makes hipcc wait vmcnt(0) before ring reads): the DMA
  // ring, then the constants, then one code-bias row per wave
  __shared__ __attribute__((aligned(16))) float4 lds[kLdsQuads];
  float* clds = reinterpret_cast<float*>(lds + kRing * kChunkQuads);
  State s;
  s.lane = threadIdx.x & 63;
  s.g = s.lane >> 4;
  s.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  s.wsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.packed), 0, kPackedFloats * 4, 0x00020000);
  s.voff = static_cast<unsigned>(s.wave * 64 + s.lane) * 16u;
  s.poff = static_cast<unsigned>(s.wave * 16 + (s.lane & 15)) * 1024u + 16u * s.g;
  s.sig = 0.0f;
  float* crow_lds = clds + kLdsConsts + s.wave * kCbStride;

  load_consts(a, clds);
  // prime the ring with chunks 0..2, wait for chunk 0 everywhere, read its first fragments
  dma_chunk(s, lds, 0);
  dma_chunk(s, lds, 1);
  dma_chunk(s, lds, 2);
  asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  read_a<0>(lds + s.lane, s.pre);

  const int64_t n_tiles = (a.m + kTile - 1) / kTile;
  int c = 0;
  for (int64_t tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
    c = 0;
    field_tile<MODE, MASKS, SAVE>(s, a, lds, clds, crow_lds, tile, c);
  }
  // the last tile prefetched chunks 0..2 of a tile that does not exist: they must land
  // before the workgroup's LDS is released
  __builtin_amdgcn_s_waitcnt(0x0F70);
}


// ================================================================ fused backward
// The eval-step backward (frozen weights) of forward_pass + CodeNeRFModel.forward
// (nerf/__init__.py:94-134, model.py:160-194) in fp32 (exact products, the reference's
// arithmetic): from d raw (m, 4) to the per-code sums g_code and the ray gradients, in one
// persistent launch on the forward's machinery.  dX = dPre . W is D = W^T . dPre^T: A = W^T
// streamed through the same ring (the transposed pack CN_FMT_F32_W16_T, again 36 chunks),
// B = the masked gradients in registers (a layer's D layout is the next layer's B layout, as
// in the forward).  The ReLU masks come from the forward (field_w16_kernel<.., true>).
// Chunk schedule:
//   0      fc_rgb^T      d v2   = Wr[:, :256]^T d rgb                 (k-step 0 real)
//   1-8    layer_dir2^T  d v1   = Wd2^T (m_v2 . d v2)
//   9-16   layer_dir1^T  d feat = Wd1[:, :256]^T (m_v1 . d v1)
//   17     layer_dir1^T  d dir  = Wd1[:, 256:]^T (m_v1 . d v1)        (narrow: 2 blocks x 64 k-steps)
//   18-25  fc_out^T      d h2   = Wo[1:, :256]^T d feat + Wo[0, :256] d sigma (sigma term by VALU)
//   26-33  layer_xyz2^T  d h1   = Wx2[:, :256]^T (m_h2 . d h2)
//   34-35  layer_xyz1^T  d enc  = Wx1^T (m_h1 . d h1)                  (narrow: blocks 0-1, 2-3)
// A narrow chunk keeps the wide chunk's memory layout [k-step][q][lane][j] with q = (block
// b = q >> 1, half = q & 1) and k-step 8 T + 4 half + j, so it runs the same 8-step schedule.
// The narrow outputs are ordered like the forward's encoding k-steps (col_enc_xyz /
// col_enc_dir), so each lane group back-propagates through the sin/cos pairs it owns.
// g_code = per code row sum over its samples of [m_h2 . d h2 | d feat | d sigma | d rgb]
// (cn_code_bias layout): 16-lane DPP sums + LDS float atomics into one row per wave, flushed
// to global atomics when the wave's code row changes.

constexpr int kTRgb = 0, kTDir2 = 1, kTDir1 = 9, kTDDir = 17, kTOut = 18, kTXyz2 = 26, kTXyz1 = 34;
constexpr int kTSig = 0;  // transposed-pack constants: fc_out row 0 over h2, [g][ob][r]
// LDS after the ring: constants, one g_code row per wave
constexpr int kBGacc = kLdsConsts;
constexpr int kBwdLdsFloats = kBGacc + kWaves * kCbStride;
constexpr int kBwdLdsQuads = kRing * kChunkQuads + kBwdLdsFloats / 4;
static_assert(kBwdLdsQuads * 16 <= 160 * 1024, "LDS budget (backward)");
static_assert(kTXyz1 + 2 == kChunks, "backward chunk schedule");
static_assert(kTDDir == kNoGeoSkip && kTDDir + 1 == kTOut, "no-geometry stream: skips the view-dir chunk");

// Elements idx0, idx0 + stride, ... of the CN_FMT_F32_W16_T pack (pack_w16t_kernel; a role of
// field_prepare_kernel).
__device__ __forceinline__ void pack_w16t_range(const Params& P, float* __restrict__ packed, int idx0, int stride) {
  constexpr int kX2 = kHidden + kCode, kD1 = kCode + kDimDir;
  for (int idx = idx0; idx < kPackedFloats; idx += stride) {
    float v = 0.0f;
    if (idx >= kStreamFloats) {
      const int t = idx - kStreamFloats;
      if (t < 256) {
        const int g = t >> 6, ob = (t >> 2) & 15, r = t & 3;
        v = P.p[kWOut][16 * ob + 4 * g + r];  // fc_out row 0, h2 feature 16 ob + 4 g + r
      }
    } else {
      const int c = idx / (kChunkQuads * 4), rem = idx % (kChunkQuads * 4);
      const int st = rem / (kStepQuads * 4), q = (rem % (kStepQuads * 4)) / 256;
      const int lane = (rem % 256) / 4, j = rem % 4;
      const int i = lane & 15, g = lane >> 4;
      if (c == kTDDir || c >= kTXyz1) {
        const int b = q >> 1, t = 8 * st + 4 * (q & 1) + j;
        const int kin = col_acc(t, g);
        if (c == kTDDir) {
          const int e = col_enc_dir(4 * b + (i & 3), i >> 2);
          if (e >= 0) v = P.p[kWDir1][kin * kD1 + kCode + e];
        } else {
          const int bb = 2 * (c - kTXyz1) + b;
          const int col = col_enc_xyz(4 * bb + (i & 3), i >> 2);
          if (col >= 0) v = P.p[kWXyz1][kin * kDimXyz + col];
        }
      } else {
        const int row = 16 * (4 * q + j) + i;  // backward output = forward input feature
        if (c == kTRgb) {
          if (st == 0 && g < 3) v = P.p[kWRgb][g * kX2 + row];
        } else {
          // W^T[row][kin] = W[roff + kin][row] of the layer this chunk belongs to
          const float* W;
          int first, ld, roff = 0;
          if (c < kTDir1) {
            W = P.p[kWDir2], first = kTDir2, ld = kHidden;
          } else if (c < kTDDir) {
            W = P.p[kWDir1], first = kTDir1, ld = kD1;
          } else if (c < kTXyz2) {
            W = P.p[kWOut], first = kTOut, ld = kX2, roff = 1;
          } else {
            W = P.p[kWXyz2], first = kTXyz2, ld = kX2;
          }
          const int kin = col_acc(8 * (c - first) + st, g);
          v = W[(roff + kin) * ld + row];
        }
      }
    }
    packed[idx] = v;
  }
}

__global__ void pack_w16t_kernel(Params P, float* __restrict__ packed) {
  pack_w16t_range(P, packed, blockIdx.x * blockDim.x + threadIdx.x, gridDim.x * blockDim.x);
}

// What a training or eval step computes from the weights and codes before its field kernels, in ONE
// launch (cn_field_prepare): the per-code terms (code_bias_block, blocks [0, nb_cb)), the forward and
// backward packs (each over nb_pack blocks, grid-stride) and a zeroed buffer (the backward's g_code
// accumulator; blocks after the packs).  Four launches per model and chunk before (code_bias,
// pack_w16, pack_w16t, a torch fill); the roles write disjoint outputs from the same inputs.
struct Prepare {
  Params P;
  const float* z_s;
  const float* z_t;
  float* code_bias;
  float* code_act;   // code-layer activations (code_bias_block) or null
  float* packed;     // CN_FMT_F32_W16 or null
  float* packed_t;   // CN_FMT_F32_W16_T or null
  float* zero;
  int64_t n_zero;
  unsigned nb_cb, nb_pack, nb_zero;
};
constexpr int kPrepThreads = 512;
static_assert(kPrepThreads == kCbThreads, "code_bias_block's workgroup size");

// Up to two models' preparations in one launch (a render's coarse and fine fields share the codes):
// blocks first[1] .. belong to the second.
constexpr int kMaxPrepModels = 2;
struct PrepareSet {
  Prepare p[kMaxPrepModels];
  unsigned first[kMaxPrepModels];
};

__global__ __launch_bounds__(kPrepThreads) void field_prepare_kernel(PrepareSet set) {
  const int k = blockIdx.x >= set.first[1] ? 1 : 0;
  const Prepare& p = set.p[k];
  unsigned b = blockIdx.x - set.first[k];
  if (b < p.nb_cb) {
    code_bias_block(p.P, p.z_s, p.z_t, p.code_bias, b, p.code_act);
    return;
  }
  b -= p.nb_cb;
  if (p.packed) {
    if (b < p.nb_pack) {
      pack_w16_range(p.P, p.packed, b * kPrepThreads + threadIdx.x, p.nb_pack * kPrepThreads);
      return;
    }
    b -= p.nb_pack;
  }
  if (p.packed_t) {
    if (b < p.nb_pack) {
      pack_w16t_range(p.P, p.packed_t, b * kPrepThreads + threadIdx.x, p.nb_pack * kPrepThreads);
      return;
    }
    b -= p.nb_pack;
  }
  for (int64_t i = (int64_t)b * kPrepThreads + threadIdx.x; i < p.n_zero; i += (int64_t)p.nb_zero * kPrepThreads)
    p.zero[i] = 0.0f;
}

// Sum over each row of 16 lanes (the 16 samples of one lane group); lane 16 g + 15 holds it.
__device__ __forceinline__ float sum16(float x) {
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x111, 0xF, 0xF, true));  // row_shr:1
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x112, 0xF, 0xF, true));  // row_shr:2
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x114, 0xF, 0xF, true));  // row_shr:4
  x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x118, 0xF, 0xF, true));  // row_shr:8
  return x;
}

// One butterfly step of rowsum64 over N values: the lane keeps the half of x selected by `hi`
// (bit s of its row index) and adds the other half of lane i - 2^s (row rotation DPP).
template <int N, int ROR>
__device__ __forceinline__ void rowsum_step(const float* x, float* y, bool hi) {
#pragma unroll
  for (int k = 0; k < N / 2; ++k) {
    const float keep = hi ? x[k + N / 2] : x[k];
    const float send = hi ? x[k] : x[k + N / 2];
    y[k] = keep + __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(send), 0x120 + ROR, 0xF, 0xF, false));
  }
}

// Sums over the 16 samples of a lane group (the 16 lanes of a DPP row) of the 64 values v[ob][r]:
// a transpose-reduction in 4 row-rotation steps (60 DPP adds + 120 selects instead of 64 separate
// 16-lane reductions).  Lane i of the row ends with out[j] = the sum of k = 4 rev4(i) + j, i.e. of
// features 16 rev4(i) + 4 g + j (j = 0..3), rev4 = the 4-bit reversal of i: step s keeps the half
// chosen by bit s of i, and lane i - 2^s has the same lower bits and the other bit s.
__device__ __forceinline__ void rowsum64(const floatx4* v, float* out, int i) {
  float x0[64], x1[32], x2[16], x3[8];
#pragma unroll
  for (int k = 0; k < 64; ++k) x0[k] = v[k >> 2][k & 3];
  rowsum_step<64, 1>(x0, x1, (i & 1) != 0);
  rowsum_step<32, 2>(x1, x2, (i & 2) != 0);
  rowsum_step<16, 4>(x2, x3, (i & 4) != 0);
  rowsum_step<8, 8>(x3, out, (i & 8) != 0);
}

__device__ __forceinline__ int rev4(int i) { return ((i & 1) << 3) | ((i & 2) << 1) | ((i & 4) >> 1) | ((i & 8) >> 3); }

__device__ __forceinline__ unsigned lds_addr(const float* p) {
  return static_cast<unsigned>(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) float*)(p)));
}

// row[COL + 16 ob + 4 g + r] += sum over the wave's samples of v[ob][r] (all 64 features of this
// lane group; `row`: an LDS row, wave-uniform).  The 4 float atomics per lane are issued by inline
// asm: for a compiler-visible LDS write hipcc cannot rule out the in-flight LDS-DMA ring writes
// and puts an s_waitcnt vmcnt(0) before it, which drains the weight stream and the plane stores.
// The address is formed inside the asm from the lane's constant part (s.gbase) and the row's
// uniform offset, so no per-call address is hoisted out of the tile loop into a VGPR.  The asm is
// not counted in the compiler's lgkmcnt, so every reader of these rows waits lgkmcnt(0)
// explicitly (flush_gcode, the kernel's final flush).
template <int COL>
__device__ __forceinline__ void gcode_add64(const State& s, float* row, const floatx4* v) {
  float o[4];
  rowsum64(v, o, s.lane & 15);
  const unsigned roff = __builtin_amdgcn_readfirstlane(lds_addr(row));
  unsigned addr;
  asm volatile(
      "v_add_u32 %0, %1, %2\n\t"
      "ds_add_f32 %0, %3 offset:%7\n\t"
      "ds_add_f32 %0, %4 offset:%7+4\n\t"
      "ds_add_f32 %0, %5 offset:%7+8\n\t"
      "ds_add_f32 %0, %6 offset:%7+12"
      : "=&v"(addr)
      : "s"(roff), "v"(s.gbase), "v"(o[0]), "v"(o[1]), "v"(o[2]), "v"(o[3]), "i"(4 * COL)
      : "memory");
}

// act = acc where the mask bit is set, else +0 (torch's relu backward: grad * (pre > 0)).
__device__ __forceinline__ void mask_act(State& s, uint2 m) {
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) {
    const unsigned w = ob < 8 ? m.x : m.y;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const unsigned keep = static_cast<unsigned>(__builtin_amdgcn_sbfe(static_cast<int>(w), 4 * (ob & 7) + r, 1));
      s.act[ob][r] = __uint_as_float(__float_as_uint(s.acc[ob][r]) & keep);
    }
  }
}

__device__ __forceinline__ void zero_acc(State& s) {
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) s.acc[ob] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
}

// fc_rgb^T: only k-step 0 of chunk c is real; the chunk's barrier and DMA, then its 16 MFMAs.
// X1STORE (no-geometry training backward): s.act still holds the PREVIOUS tile's layer_xyz1 dPre
// (m_h1 . d h1, plane 4), which the geometry kernel stored beside its layer_xyz1^T chunks; here its
// 16 stores go out after the DMA, one beside each MFMA (rsrc x1 covers no rows before the first tile:
// the stores are dropped).
template <bool X1STORE = false>
__device__ __forceinline__ void chunk_k0(State& s, float4* lds, int c, float b, __amdgpu_buffer_rsrc_t x1) {
  const float4* nslot = lds + ((c + 1) & (kRing - 1)) * kChunkQuads + s.lane;
  floatx4 a0[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) a0[q] = s.pre[q];
  __builtin_amdgcn_sched_barrier(0);
  chunk_barrier();
  dma_chunk<X1STORE>(s, lds, c + 3);
  read_a<0>(nslot, s.pre);
  if constexpr (X1STORE) store_plane<0, 16>(s, x1, s.act);
  mfma_step(s, a0, b);
  if constexpr (X1STORE) {
#pragma unroll
    for (int m = 0; m < 16; ++m) {
      __builtin_amdgcn_sched_group_barrier(0x040, 1, 0);  // VMEM write
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
    }
  }
  __builtin_amdgcn_sched_barrier(0);
}

// A narrow step: blocks b = q >> 1 of k-steps 8 T + 4 (q & 1) + j, four independent chains.
template <int T>
__device__ __forceinline__ void mfma_narrow(State& s, const floatx4* a) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      s.acc2[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[q][j], s.act[2 * T + (q & 1)][j], s.acc2[q], 0, 0, 0);
}

// A narrow chunk (2 blocks x 64 k-steps, B from s.act) into s.acc2, on chunk16's schedule.
template <int CI = 0, typename Post = NoPost>
__device__ __forceinline__ void chunk_narrow(State& s, float4* lds, int c, Post post = Post{}) {
  const float4* slot = lds + (c & (kRing - 1)) * kChunkQuads + s.lane;
  const float4* nslot = lds + ((c + 1) & (kRing - 1)) * kChunkQuads + s.lane;
  floatx4 a0[4], a1[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) a0[q] = s.pre[q];
  __builtin_amdgcn_sched_barrier(0);
#define CN_NSTEP(T, CUR, NXT)                                        \
  {                                                                 \
    if constexpr ((T) + 1 < 8) read_a<(T) + 1>(slot, NXT);          \
    else read_a<0>(nslot, s.pre);                                   \
    mfma_narrow<(T)>(s, CUR);                                       \
    step_pattern();                                                 \
    __builtin_amdgcn_sched_barrier(0);                              \
    if constexpr ((T) == 3) {                                       \
      chunk_barrier();                                              \
      dma_chunk(s, lds, c + 3);                                     \
    }                                                               \
    post.template step<CI, (T)>();                                  \
  }
  CN_NSTEP(0, a0, a1)
  CN_NSTEP(1, a1, a0)
  CN_NSTEP(2, a0, a1)
  CN_NSTEP(3, a1, a0)
  CN_NSTEP(4, a0, a1)
  CN_NSTEP(5, a1, a0)
  CN_NSTEP(6, a0, a1)
  CN_NSTEP(7, a1, a0)
#undef CN_NSTEP
}

// Flush this wave's g_code row (LDS) into g_code[code] and zero it.
__device__ __forceinline__ void flush_gcode(const State& s, const FieldArgs& a, float* row, int code) {
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS atomics landed
#pragma unroll
  for (int k = 0; k < (kCbStride + 63) / 64; ++k) {
    const int j = s.lane + 64 * k;
    if (j < kCbStride) {
      const float v = row[j];
      if (v != 0.0f) atomicAdd(a.g_code + (int64_t)code * kCbStride + j, v);
      row[j] = 0.0f;
    }
  }
}

// Training backward: the masked input gradient of a layer (its dPre, what dW = dPre^T X reads) as
// plane `plane` of a.dpre: 0 layer_dir2, 1 layer_dir1, 2 fc_out rows 1.. (d feat), 3 layer_xyz2,
// 4 layer_xyz1.
template <bool TRAIN>
struct DpreStore {
  const State& s;
  const FieldArgs& a;
  int64_t tile;
  int plane;
  // two blocks per chunk of a 256-wide layer (see chunk16); in the xyz1 layer's two narrow chunks
  // (NARROW): eight per chunk, two per k-step 4..7
  bool narrow = false;
  template <int CI, int T>
  __device__ __forceinline__ void step() const {
    if constexpr (TRAIN) {
      if (narrow) {
        if constexpr (T >= 4) store_plane<8 * CI + 2 * (T - 4), 2>(s, plane_rsrc(a.dpre, plane, a.m, tile), s.act);
      } else if constexpr (T == 4) {
        store_plane<2 * CI, 2>(s, plane_rsrc(a.dpre, plane, a.m, tile), s.act);
      }
    }
  }
  template <int CI>
  __device__ __forceinline__ void before_dma() const {}
};

// The Q1 view-direction row of sample row rc (nerf/__init__.py:127-128; decode_sample's map).
__device__ __forceinline__ int64_t q1_dir_ray(const FieldArgs& a, int64_t rc) {
  const int64_t S = a.n_samples;
  const int64_t ray = rc / S, smp = rc - ray * S;
  const int64_t base = (ray / a.chunk_rows) * a.chunk_rows;
  const int64_t rcnt = min(a.chunk_rows, a.n_rays - base);
  return base + ((ray - base) * S + smp) % rcnt;
}

// The tile's ReLU mask words of layer l (slot l of the forward's mask block).
__device__ __forceinline__ uint2 load_mask(const State& s, const FieldArgs& a, int64_t tile, int l) {
  const uint2v w = __builtin_amdgcn_raw_buffer_load_b64(mask_rsrc(a.masks, tile), 8u * s.lane, mask_soff(s, l), 0);
  return make_uint2(w[0], w[1]);
}

// Live ranges, because this kernel sits at the 256-VGPR cap of two waves per SIMD (act, acc: 128;
// A fragments and the prefetch: 48): the mask words are loaded a layer pair ahead of their use
// (the compiler counts the weight stream's DMA pieces in between, so the wait it puts before the
// use does not drain the stream), the view-direction gradient is finished right after its narrow
// chunk (3 values to the end instead of 8 + the unit direction), and the code row is wave-uniform.
//
// NOGEO (the training backward with no d ro / d rd / d pts wanted -- train.py's rays are data,
// ray_sampler.py:53-82): the view-direction chunk, both layer_xyz1^T chunks and the encoding / ray
// epilogue only feed those outputs, so they are not streamed or run (33 chunks per tile instead of
// 36).  The one thing training needs from that schedule, layer_xyz1's dPre plane (m_h1 . d h1), is
// left in s.act at the tile's end and stored beside the next tile's fc_rgb^T MFMAs (chunk_k0), the
// last tile's after the tile loop.  crun: the running chunk counter (stream_src); prev: the tile
// whose plane 4 is pending (-1: none).
template <int MODE, bool TRAIN, bool NOGEO = false, bool DET = false>
__device__ __forceinline__ void bwd_tile(State& s, const FieldArgs& a, float4* lds, float* grow, int64_t tile,
                                        int& cur_code, int& crun, int64_t& prev) {
  const int64_t row = tile * kTile + s.wave * 16 + (s.lane & 15);
  const bool valid = row < a.m;
  const int64_t rc = valid ? row : a.m - 1;
  const float* clds = reinterpret_cast<const float*>(lds + kRing * kChunkQuads);

  // ---- inputs: sample, d raw, masks of v2 and v1, code row (wave-uniform: host-checked)
  const SampleIn in = decode_sample<MODE>(a, rc);
  const int crow = __builtin_amdgcn_readfirstlane(static_cast<int>(code_row(a, in.code_of)));
  float4 dr = reinterpret_cast<const float4*>(a.d_raw)[rc];
  const uint2 m_v2 = load_mask(s, a, tile, 3), m_v1 = load_mask(s, a, tile, 2);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
  if (!valid) dr = make_float4(0.f, 0.f, 0.f, 0.f);
  // a.g_code NULL: the caller forms g_code from the dPre planes (deterministic column sums folded
  // into the dW GEMMs; cn_field_backward_train_fmt with one code row) -- no code sums here
  const bool gc = a.g_code != nullptr;
  if (gc && crow != cur_code) {
    if (cur_code >= 0) flush_gcode(s, a, grow, cur_code);
    cur_code = crow;
  }
  // g_code sigma / rgb (lane group 0 carries the wave's 16 samples)
  if (gc) {
    const float t0 = sum16(dr.w), t1 = sum16(dr.x), t2 = sum16(dr.y), t3 = sum16(dr.z);
    if (s.lane == 15) {
      atomicAdd(grow + kCbSigma, t0);
      atomicAdd(grow + kCbRgb, t1);
      atomicAdd(grow + kCbRgb + 1, t2);
      atomicAdd(grow + kCbRgb + 2, t3);
    }
  }
  int c = NOGEO ? crun : 0;
  s.cbase = c;
  // ---- fc_rgb^T (chunk 0): B = d rgb channel g at k-step 0
  zero_acc(s);
  {
    const float b = s.g == 0 ? dr.x : (s.g == 1 ? dr.y : (s.g == 2 ? dr.z : 0.0f));
    if constexpr (NOGEO) {
      const __amdgpu_buffer_rsrc_t x1 =
          prev >= 0 ? plane_rsrc(a.dpre, 4, a.m, prev) : __builtin_amdgcn_make_buffer_rsrc(a.dpre, 0, 0, 0x00020000);
      chunk_k0<true>(s, lds, c, b, x1);
    } else {
      chunk_k0(s, lds, c, b, s.wsrc);  // (no stores: x1 unused)
    }
  }
  c += kTDir2;
  const float dsig = dr.w;
  // ---- layer_dir2^T (m_v2), layer_dir1^T (m_v1)
  // (each layer's masked input gradient -- the dW GEMMs' dPre plane -- is stored at the layer's first
  // chunk barrier: DpreStore as chunk16's `post`)
  mask_act(s, m_v2);
  zero_acc(s);
  __builtin_amdgcn_sched_barrier(0);
  layer256<NOGEO>(s, lds, c, DpreStore<TRAIN>{s, a, tile, 0});
  const uint2 m_h2 = load_mask(s, a, tile, 1), m_h1 = load_mask(s, a, tile, 0);
  mask_act(s, m_v1);
  zero_acc(s);
  __builtin_amdgcn_sched_barrier(0);
  layer256<NOGEO>(s, lds, c, DpreStore<TRAIN>{s, a, tile, 1});
  // ---- the view-direction rows of layer_dir1^T (narrow chunk, B = m_v1 . d v1 still in act)
  // d view dir -> the Q1 direction ray's d rd (its atomics at the end of the tile):
  // vd = rd[dray] / |rd[dray]|: d rd[dray] += (g - vd (vd . g)) / |rd[dray]|
  float grd_q1[3] = {0.f, 0.f, 0.f};
  if constexpr (!NOGEO) {
#pragma unroll
    for (int q = 0; q < 4; ++q) s.acc2[q] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
    chunk_narrow(s, lds, c);
    c += 1;
    float gdir[8];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      gdir[r] = s.acc2[0][r] + s.acc2[1][r];
      gdir[4 + r] = s.acc2[2][r] + s.acc2[3][r];
    }
    float dv[3] = {0.f, 0.f, 0.f};
    const int g = fresh(s.g);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int p = 4 * i + g, d = p % 3, k = p / 3;
      const float f = clds[kCFreq + 10 + k];
      float sn, cs;
      sincosf(__fmul_rn(pick3(in.vd, d), f), &sn, &cs);
      add3(dv, d, f * (gdir[i] * cs - gdir[3 + i] * sn));
    }
    add3(dv, g, gdir[6]);  // g == 3 adds nothing
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      dv[d] += __shfl_xor(dv[d], 16);
      dv[d] += __shfl_xor(dv[d], 32);
    }
    const float dot = in.vd[0] * dv[0] + in.vd[1] * dv[1] + in.vd[2] * dv[2];
#pragma unroll
    for (int d = 0; d < 3; ++d) grd_q1[d] = (dv[d] - in.vd[d] * dot) / in.nrm;
    if constexpr (DET) {
      // deterministic form: this sample's Q1 term as its q1_part row, here (not live to the tile's end)
      if (valid && s.g == 0 && a.d_rd)
        for (int d = 0; d < 3; ++d) a.q1_part[3 * rc + d] = grd_q1[d];
    }
  }
  // ---- fc_out^T: B = d feat (no activation), init = fc_out row 0 (h2 part) x d sigma
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) s.act[ob] = s.acc[ob];
  if (gc) gcode_add64<kCbFeat>(s, grow, s.act);
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) {
    const floatx4 w = *reinterpret_cast<const floatx4*>(clds + kTSig + 64 * fresh(s.g) + 4 * ob);
    s.acc[ob] = w * dsig;
  }
  __builtin_amdgcn_sched_barrier(0);
  layer256<NOGEO>(s, lds, c, DpreStore<TRAIN>{s, a, tile, 2});
  // ---- layer_xyz2^T (m_h2): its masked input gradient is the code term's too
  mask_act(s, m_h2);
  if (gc) gcode_add64<kCbXyz2>(s, grow, s.act);
  zero_acc(s);
  __builtin_amdgcn_sched_barrier(0);
  layer256<NOGEO>(s, lds, c, DpreStore<TRAIN>{s, a, tile, 3});
  // ---- layer_xyz1^T (m_h1): encoding k-steps 0-7, then 8-15
  mask_act(s, m_h1);
  if constexpr (NOGEO) {
    // its dPre plane goes out beside the next tile's fc_rgb^T (or after the tile loop)
    crun = c;
    prev = tile;
    return;
  }
  float genc[16];
#pragma unroll
  for (int half = 0; half < 2; ++half) {
#pragma unroll
    for (int q = 0; q < 4; ++q) s.acc2[q] = floatx4{0.0f, 0.0f, 0.0f, 0.0f};
    if (half == 0) chunk_narrow<0>(s, lds, c, DpreStore<TRAIN>{s, a, tile, 4, true});
    else chunk_narrow<1>(s, lds, c, DpreStore<TRAIN>{s, a, tile, 4, true});
    c += 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      genc[8 * half + r] = s.acc2[0][r] + s.acc2[1][r];
      genc[8 * half + 4 + r] = s.acc2[2][r] + s.acc2[3][r];
    }
  }

  // ---- encodings -> d pts: lane group g owns pairs p = 4 i + g (as the forward)
  float dx[3] = {0.f, 0.f, 0.f};
  const int g = fresh(s.g);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int p = 4 * i + g;
    if (p < 30) {
      const int d = p % 3, k = p / 3;
      float sn, cs;
      const float f = clds[kCFreq + k];
      sincosf(__fmul_rn(pick3(in.x, d), f), &sn, &cs);
      add3(dx, d, f * (genc[i] * cs - genc[8 + i] * sn));
    } else if (g == 2) {  // raw inputs x0 (k-step 7), x1 (k-step 15)
      dx[0] += genc[7];
      dx[1] += genc[15];
    } else {                // x2 (k-step 7)
      dx[2] += genc[7];
    }
  }
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    dx[d] += __shfl_xor(dx[d], 16);
    dx[d] += __shfl_xor(dx[d], 32);
  }
  const int64_t S = a.n_samples;
  if constexpr (MODE == kFromRayZ) {
    // pts = ro + rd z (z detached): d ro += d pts, d rd += d pts z.  With S % 16 == 0 the
    // wave's 16 samples are one ray: sum over them first, one atomic per value.
    const float zv = a.z[rc];
    float gro[3], grd[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      gro[d] = valid ? dx[d] : 0.0f;
      grd[d] = valid ? dx[d] * zv : 0.0f;
    }
    const bool one_ray = S % 16 == 0;
    if (one_ray) {
#pragma unroll
      for (int off = 8; off >= 1; off >>= 1)
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          gro[d] += __shfl_xor(gro[d], off);
          grd[d] += __shfl_xor(grd[d], off);
        }
    }
    if (valid && s.g == 0 && (!one_ray || s.lane == 0)) {
      const int64_t ray = rc / S;
      if constexpr (DET) {
        // deterministic form (one ray per wave, host-checked): the wave's sums as its row of ray_part
        // (lane 0's rc is the wave's first sample, a multiple of 16)
        if (a.ray_part) {
          float* p = a.ray_part + (rc >> 4) * 6;
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
  } else {
    if (valid && s.g == 0 && a.d_pts)
      for (int d = 0; d < 3; ++d) a.d_pts[3 * rc + d] = dx[d];
  }
  if constexpr (!DET) {
    if (valid && s.g == 0 && a.d_rd) {
      const int64_t dray = q1_dir_ray(a, rc);
      for (int d = 0; d < 3; ++d) atomicAdd(a.d_rd + 3 * dray + d, grd_q1[d]);
    }
  }
}

// One field's share of a backward launch: workgroup blk of nblk walks tiles blk, blk + nblk, ...
template <int MODE, bool TRAIN, bool NOGEO, bool DET>
__device__ __forceinline__ void bwd_body(const FieldArgs& a, float4* lds, const unsigned blk, const unsigned nblk) {
  float* blds = reinterpret_cast<float*>(lds + kRing * kChunkQuads);
  State s;
  s.lane = threadIdx.x & 63;
  s.g = s.lane >> 4;
  s.wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  s.wsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(a.packed), 0, kPackedFloats * 4, 0x00020000);
  s.voff = static_cast<unsigned>(s.wave * 64 + s.lane) * 16u;
  s.poff = static_cast<unsigned>(s.wave * 16 + (s.lane & 15)) * 1024u + 16u * s.g;
  s.gbase = static_cast<unsigned>(16 * rev4(s.lane & 15) + 4 * s.g) * 4u;
  s.cbase = 0;
  float* grow = blds + kBGacc + s.wave * kCbStride;
  load_consts(a, blds);
  for (int k = threadIdx.x; k < kBwdLdsFloats - kBGacc; k += kThreads) blds[kBGacc + k] = 0.0f;
  __syncthreads();
  dma_chunk(s, lds, 0);
  dma_chunk(s, lds, 1);
  dma_chunk(s, lds, 2);
  asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
  read_a<0>(lds + s.lane, s.pre);
  int cur_code = -1;
  const int64_t n_tiles = (a.m + kTile - 1) / kTile;
  int crun = 0;
  int64_t prev = -1;
  for (int64_t tile = blk; tile < n_tiles; tile += nblk) {
    bwd_tile<MODE, TRAIN, NOGEO, DET>(s, a, lds, grow, tile, cur_code, crun, prev);
  }
  if constexpr (NOGEO) {
    if (prev >= 0) store_plane<0, 16>(s, plane_rsrc(a.dpre, 4, a.m, prev), s.act);
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);
  if constexpr (DET) {
    // deterministic form (one code row, host-checked): this wave's g_code row into its gc_part row
    // (every wave writes its row, zeros included)
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's LDS atomics landed
    if (a.gc_rows) {
      // the workgroup's wave rows added in wave order into its one row (what ray_grad_reduce_kernel's row
      // blocks did from the per-wave rows: the same additions, without the (waves x 2 KiB) round trip)
      __syncthreads();
      const float* rows = blds + kBGacc;
      for (int j = threadIdx.x; j < kCbStride; j += kThreads) {
        float v = rows[j];
        for (int w = 1; w < kWaves; ++w) v += rows[w * kCbStride + j];
        a.gc_rows[(int64_t)blk * kCbStride + j] = v;
      }
    } else {
      float* out = a.gc_part + ((int64_t)blk * kWaves + s.wave) * kCbStride;
#pragma unroll
      for (int k = 0; k < (kCbStride + 63) / 64; ++k) {
        const int j = s.lane + 64 * k;
        if (j < kCbStride) out[j] = grow[j];
      }
    }
  } else if (cur_code >= 0) {
    flush_gcode(s, a, grow, cur_code);
  }
}

template <int MODE, bool TRAIN, bool NOGEO = false, bool DET = false>
__global__ __launch_bounds__(kThreads, 2) void field_w16_bwd_kernel(FieldArgs a) {
  static_assert(!NOGEO || TRAIN, "the no-geometry schedule is the training backward's");
  __shared__ __attribute__((aligned(16))) float4 lds[kBwdLdsQuads];
  bwd_body<MODE, TRAIN, NOGEO, DET>(a, lds, blockIdx.x, gridDim.x);
}

// A render's two fields (coarse, fine) in ONE launch: workgroups 0 .. first1 - 1 run field a0's tiles,
// the rest field a1's, each exactly as its own launch would (same workgroup count and tile walk, so the
// same sums in the same order).  One workgroup per CU is resident: field a1's workgroups start on the
// CUs field a0's leave, so the second field fills the first one's finish spread instead of waiting
// for its last workgroup and a new launch (point_sampler.py:115: the fine depths are detached, so the
// two backwards are independent).
template <int MODE, bool TRAIN, bool NOGEO = false, bool DET = false>
__global__ __launch_bounds__(kThreads, 2) void field_w16_bwd2_kernel(FieldArgs a0, FieldArgs a1, unsigned first1) {
  static_assert(!NOGEO || TRAIN, "the no-geometry schedule is the training backward's");
  __shared__ __attribute__((aligned(16))) float4 lds[kBwdLdsQuads];
  // two instances of the body, each reading its own kernel argument (a runtime select between the two
  // structs put the selected one in scratch: ~550 B per lane)
  if (blockIdx.x >= first1) bwd_body<MODE, TRAIN, NOGEO, DET>(a1, lds, blockIdx.x - first1, gridDim.x - first1);
  else bwd_body<MODE, TRAIN, NOGEO, DET>(a0, lds, blockIdx.x, first1);
}

}  // namespace w16

static int64_t cu_count_w16() {
  static int n[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (n[dev] == 0) {
    int v = 0;
    n[dev] = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
  }
  return n[dev];
}

int64_t packed_floats_w16() { return w16::kPackedFloats; }

int launch_pack_w16(const Params& P, float* packed, hipStream_t st) {
  hipLaunchKernelGGL(w16::pack_w16_kernel, dim3(cn::elementwise_grid(w16::kPackedFloats, 256)), dim3(256), 0, st, P,
                     packed);
  return cn::launch_status();
}

int launch_field_w16(int mode, FieldArgs& a, hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(std::min<int64_t>(cn::ceil_div(a.m, w16::kTile), cu_count_w16()));
  const dim3 b(w16::kThreads);
  if (a.masks && a.save) {
    if (mode == kFromPts) hipLaunchKernelGGL((w16::field_w16_kernel<kFromPts, true, true>), dim3(grid), b, 0, st, a);
    else if (mode == kFromRayZ) hipLaunchKernelGGL((w16::field_w16_kernel<kFromRayZ, true, true>), dim3(grid), b, 0, st, a);
    else return CN_EUNSUPPORTED;
    return cn::launch_status();
  }
  if (a.masks) {
    if (mode == kFromPts) hipLaunchKernelGGL((w16::field_w16_kernel<kFromPts, true>), dim3(grid), b, 0, st, a);
    else if (mode == kFromRayZ) hipLaunchKernelGGL((w16::field_w16_kernel<kFromRayZ, true>), dim3(grid), b, 0, st, a);
    else return CN_EUNSUPPORTED;
    return cn::launch_status();
  }
  switch (mode) {
    case kFromPts: hipLaunchKernelGGL((w16::field_w16_kernel<kFromPts, false>), dim3(grid), b, 0, st, a); break;
    case kFromRayZ: hipLaunchKernelGGL((w16::field_w16_kernel<kFromRayZ, false>), dim3(grid), b, 0, st, a); break;
    default: hipLaunchKernelGGL((w16::field_w16_kernel<kFromEncoded, false>), dim3(grid), b, 0, st, a); break;
  }
  return cn::launch_status();
}

int64_t mask_words_w16(int64_t m) { return cn::ceil_div(m, w16::kTile) * w16::kMaskWordsPerTile; }

int launch_field_prepare_w16(const PrepareModel* models, int n_models, const float* z_s, const float* z_t,
                             int64_t n_codes, hipStream_t st) {
  if (n_models < 1 || n_models > w16::kMaxPrepModels) return CN_EINVAL;
  w16::PrepareSet set = {};
  unsigned grid = 0;
  for (int k = 0; k < n_models; ++k) {
    const PrepareModel& m = models[k];
    w16::Prepare& p = set.p[k];
    p = w16::Prepare{m.P, z_s, z_t, m.code_bias, m.code_bias ? m.code_act : nullptr, m.packed, m.packed_t, m.zero,
                     m.n_zero, 0u, 0u, 0u};
    p.nb_cb = m.code_bias ? static_cast<unsigned>(n_codes * kCbSlices) : 0u;
    p.nb_pack = 64;  // 64 x 512 threads over each pack's 327,680 floats: 10 elements per thread
    p.nb_zero = m.n_zero > 0 ? static_cast<unsigned>(std::min<int64_t>(cn::ceil_div(m.n_zero, w16::kPrepThreads), 64))
                             : 0u;
    set.first[k] = grid;
    grid += p.nb_cb + (m.packed ? p.nb_pack : 0u) + (m.packed_t ? p.nb_pack : 0u) + p.nb_zero;
  }
  if (n_models == 1) set.first[1] = grid;   // no block reaches the second slot
  if (grid == 0) return CN_OK;
  hipLaunchKernelGGL(w16::field_prepare_kernel, dim3(grid), dim3(w16::kPrepThreads), 0, st, set);
  return cn::launch_status();
}

int launch_pack_w16t(const Params& P, float* packed, hipStream_t st) {
  hipLaunchKernelGGL(w16::pack_w16t_kernel, dim3(cn::elementwise_grid(w16::kPackedFloats, 256)), dim3(256), 0, st, P,
                     packed);
  return cn::launch_status();
}

// CN_BWD_NOGEO=0 keeps the geometry schedule in training too (A/B timing; the weight and code
// gradients are bitwise the same either way)
bool nogeo_enabled() {
  static const int on = [] {
    const char* e = getenv("CN_BWD_NOGEO");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return on != 0;
}

static unsigned bwd_grid_w16(const FieldArgs& a) {
  return static_cast<unsigned>(
      std::min<int64_t>(std::min<int64_t>(cn::ceil_div(a.m, w16::kTile), cu_count_w16()), kMaxBwdBlocks));
}

// Two fields' fused backwards in one launch (field_w16_bwd2_kernel): both must take the same kernel form
// (the same mode, training / no-geometry / deterministic choice), else CN_EUNSUPPORTED before any launch.
int launch_field_w16_bwd2(int mode, FieldArgs& a0, FieldArgs& a1, hipStream_t st) {
  auto form = [](const FieldArgs& a) {
    if (a.dpre) return (!a.d_pts && !a.d_ro && !a.d_rd && nogeo_enabled()) ? 2 : 1;
    return a.gc_part ? 3 : 0;
  };
  const int f = form(a0);
  if (form(a1) != f || mode != kFromRayZ) return CN_EUNSUPPORTED;
  const unsigned g0 = bwd_grid_w16(a0), g1 = bwd_grid_w16(a1);
  a0.n_blocks = g0;
  a1.n_blocks = g1;
  const dim3 grid(g0 + g1), b(w16::kThreads);
  switch (f) {
    case 2: hipLaunchKernelGGL((w16::field_w16_bwd2_kernel<kFromRayZ, true, true>), grid, b, 0, st, a0, a1, g0); break;
    case 1: hipLaunchKernelGGL((w16::field_w16_bwd2_kernel<kFromRayZ, true>), grid, b, 0, st, a0, a1, g0); break;
    case 3: hipLaunchKernelGGL((w16::field_w16_bwd2_kernel<kFromRayZ, false, false, true>), grid, b, 0, st, a0, a1, g0); break;
    default: hipLaunchKernelGGL((w16::field_w16_bwd2_kernel<kFromRayZ, false>), grid, b, 0, st, a0, a1, g0); break;
  }
  return cn::launch_status();
}

int launch_field_w16_bwd(int mode, FieldArgs& a, hipStream_t st) {
  const unsigned grid = static_cast<unsigned>(
      std::min<int64_t>(std::min<int64_t>(cn::ceil_div(a.m, w16::kTile), cu_count_w16()), kMaxBwdBlocks));
  a.n_blocks = grid;
  const dim3 b(w16::kThreads);
  // training with no geometry gradient wanted (train.py: the rays are data): the 33-chunk schedule
  if (a.dpre && !a.d_pts && !a.d_ro && !a.d_rd && nogeo_enabled()) {
    if (mode == kFromPts) hipLaunchKernelGGL((w16::field_w16_bwd_kernel<kFromPts, true, true>), dim3(grid), b, 0, st, a);
    else if (mode == kFromRayZ) hipLaunchKernelGGL((w16::field_w16_bwd_kernel<kFromRayZ, true, true>), dim3(grid), b, 0, st, a);
    else return CN_EUNSUPPORTED;
    return cn::launch_status();
  }
  if (a.dpre) {
    if (mode == kFromPts) hipLaunchKernelGGL((w16::field_w16_bwd_kernel<kFromPts, true>), dim3(grid), b, 0, st, a);
    else if (mode == kFromRayZ) hipLaunchKernelGGL((w16::field_w16_bwd_kernel<kFromRayZ, true>), dim3(grid), b, 0, st, a);
    else return CN_EUNSUPPORTED;
    return cn::launch_status();
  }
  if (a.gc_part) {   // the eval backward without float atomics (cn_field_backward_fused_ws)
    if (mode == kFromPts) hipLaunchKernelGGL((w16::field_w16_bwd_kernel<kFromPts, false, false, true>), dim3(grid), b, 0, st, a);
    else if (mode == kFromRayZ) hipLaunchKernelGGL((w16::field_w16_bwd_kernel<kFromRayZ, false, false, true>), dim3(grid), b, 0, st, a);
    else return CN_EUNSUPPORTED;
    return cn::launch_status();
  }
  if (mode == kFromPts) hipLaunchKernelGGL((w16::field_w16_bwd_kernel<kFromPts, false>), dim3(grid), b, 0, st, a);
  else if (mode == kFromRayZ) hipLaunchKernelGGL((w16::field_w16_bwd_kernel<kFromRayZ, false>), dim3(grid), b, 0, st, a);
  else return CN_EUNSUPPORTED;
  return cn::launch_status();
}

}  // namespace mlp
}  // namespace cn

