// Backward pass of the field: the gradients torch's
// autograd takes through forward_pass / CodeNeRFModel.forward
// (view_synthesis/nerf/__init__.py:94-134, models/model.py:160-194).
//
// Building blocks, all fp32 (exact-product MFMA, v_mfma_f32_32x32x2_f32):
//   gemm_nn  C[m][n]  = (A[m][:] . B[:][n]) * (mask[m][n] > 0)     dX = dPre . W  (+ ReLU mask)
//   gemm_tn  C[n][k] += sum_m A[m][n] B[m][k]   (split-M, atomics)   dW = dPre^T . X
//   col_sum  out[j]  += sum_m A[m][j]                                 db
//   seg_sum  out[code(m)][j] += A[m][j]                               per-object code-term gradients
// and the element-wise pieces: posenc backward, the Q1 view-direction scatter,
// pts = ro + rd z backward, and the code-layer backward.
#include <algorithm>

#include "cn_common.h"
#include "mlp_common.h"

namespace cn {
namespace grad {

typedef float floatx16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------- GEMMs

// gemm_nn: 256 x NT output tile per 256-thread block, 64 x NT per wave (2 x NT/32
// v_mfma_f32_32x32x2_f32 tiles; NT = 128 for the 256-wide layers halves the passes over A).  k runs in tiles of 16; inside
// a tile lane half h owns k = h*8 .. h*8+7, so MFMA step kk pairs k = kk and
// 8 + kk -- any pairing of k between the A and B operands gives the same sum,
// and this one makes each lane's A values 8 consecutive floats of its row (read
// straight from global memory, no LDS) and its B values 8 consecutive floats
// of B^T.  B^T (NT columns x K) is staged in LDS once per block.
constexpr int kMT = 256, kKT = 16;
constexpr int kMaxK = 288;  // B^T tile in LDS: 64 x 292 floats = 73 KiB

template <int NT>
__global__ __launch_bounds__(256) void gemm_nn_kernel(const float* __restrict__ A, int64_t lda,
                                                      const float* __restrict__ B, int64_t ldb,
                                                      float* __restrict__ C, int64_t ldc,
                                                      const float* __restrict__ mask, int64_t ldm,
                                                      int64_t M, int N, int K) {
  constexpr int NU = NT / 32;
  __shared__ __attribute__((aligned(16))) float Bt[NT][kMaxK + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * NT;
  const int kp = (K + kKT - 1) / kKT * kKT;
  // B^T: Bt[n][k] = B[k][n0 + n] (zero outside K x N)
  for (int e = tid; e < NT * kp; e += 256) {
    const int k = e / NT, n = e % NT;
    Bt[n][k] = (k < K && n0 + n < N) ? B[(int64_t)k * ldb + n0 + n] : 0.0f;
  }
  __syncthreads();
  const int64_t m0 = (int64_t)blockIdx.x * kMT + wave * 64;
  int64_t rows[2];
  bool rv[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    rows[t] = m0 + 32 * t + i;
    rv[t] = rows[t] < M;
    if (!rv[t]) rows[t] = M - 1;
  }
  floatx16 acc[2][NU] = {};
  // A of k-tile k0 + kKT is loaded while k-tile k0's MFMAs run (register double buffer)
  auto load_a = [&](int k0, float (&a)[2][8]) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float* ar = A + rows[t] * lda + k0 + h * 8;
#pragma unroll
      for (int q = 0; q < 8; ++q) a[t][q] = (k0 + h * 8 + q < K) ? ar[q] : 0.0f;
    }
  };
  float an[2][8];
  load_a(0, an);
  for (int k0 = 0; k0 < kp; k0 += kKT) {
    float a[2][8], b[NU][8];
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int q = 0; q < 8; ++q) a[t][q] = an[t][q];
    if (k0 + kKT < kp) load_a(k0 + kKT, an);
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const float4* bp = reinterpret_cast<const float4*>(&Bt[32 * u + i][k0 + h * 8]);
      const float4 x = bp[0], y = bp[1];
      b[u][0] = x.x; b[u][1] = x.y; b[u][2] = x.z; b[u][3] = x.w;
      b[u][4] = y.x; b[u][5] = y.y; b[u][6] = y.z; b[u][7] = y.w;
    }
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < NU; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[t][kk], b[u][kk], acc[t][u], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int col = n0 + 32 * u + i;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + 32 * t + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (m < M && col < N) {
          float v = acc[t][u][r];
          if (mask && !(mask[m * ldm + col] > 0.0f)) v = 0.0f;  // ReLU'(x) = [x > 0], torch's threshold_backward
          C[m * ldc + col] = v;
        }
      }
    }
}

// Flush of one 32 x 32 accumulator block (rows row0.., columns col0.. of C): float atomics
// into C, or -- the deterministic path -- plain stores into this workgroup's partial tile
// (N x K, row-major) of the workspace, summed in a fixed order by reduce_partials_kernel.
__device__ __forceinline__ void flush_block(const floatx16& acc, float* C, int64_t ldc, float* part, int N, int K,
                                            int row0, int col0, int i, int h) {
  const int col = col0 + i;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int row = row0 + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (row < N && col < K) {
      if (part) part[(int64_t)row * K + col] = acc[r];
      else atomicAdd(&C[(int64_t)row * ldc + col], acc[r]);
    }
  }
}

// C[n][k] += sum_p part[p][n][k] in a fixed order: the deterministic second pass of the split-M dW
// GEMMs.  The parts are split into G groups (4, or 16 for many parts: reduce_groups), each summed as
// four interleaved chains by one lane per element, the groups then combined in a pairwise tree.  Block
// b of a job covers reduce_block_elems(G, vec4) elements: a float per lane, or a float4 per lane
// (reduce_vec4: N K % 4 == 0 and a 16-B aligned workspace; 16-B loads, a quarter of the blocks).
// Either way element e's partials are added in the same order, so both forms give the same bits.
constexpr int kReduceBatch = 16;   // partials per quarter loaded together (C3's jobs: 12-16)

__host__ __device__ __forceinline__ bool reduce_vec4(const float* part, int64_t nk) {
  return nk % 4 == 0 && (reinterpret_cast<uintptr_t>(part) & 15) == 0;
}

__device__ __forceinline__ void reduce_add(float* __restrict__ C, int64_t ldc, int K, int64_t e, float v,
                                           float* __restrict__ C2 = nullptr) {
  C[(e / K) * ldc + e % K] += v;
  if (C2) C2[(e / K) * ldc + e % K] += v;
}

// One part group's chains: parts p0 .. p1 - 1 added in order into four interleaved chains (groups of
// four parts into s0..s3, the tail into s0), combined (s0 + s1) + (s2 + s3).  The loads go out
// kReduceBatch at a time (one memory latency per batch instead of one per group of four); the additions
// keep the loop's order, so the bits do not depend on the batching.
template <typename V, typename Load>
__device__ __forceinline__ V reduce_chains(int64_t p0, int64_t p1, V zero, Load load) {
  V s0 = zero, s1 = zero, s2 = zero, s3 = zero;
  const int64_t g4 = p0 + ((p1 - p0) & ~int64_t(3));   // end of the groups of four
  for (int64_t base = p0; base < p1; base += kReduceBatch) {
    V x[kReduceBatch];
#pragma unroll
    for (int u = 0; u < kReduceBatch; ++u) x[u] = base + u < p1 ? load(base + u) : zero;
    // static chain selection (a dynamically chosen reference would put the chains in scratch): part
    // base + u of a full group of four goes to chain u & 3, a tail part (p >= g4) to s0
#pragma unroll
    for (int u = 0; u < kReduceBatch; ++u) {
      const int64_t p = base + u;
      const bool full = p < g4, tail = !full && p < p1;
      if ((u & 3) == 0) {
        s0 = (full || tail) ? s0 + x[u] : s0;
      } else {
        V& c = (u & 3) == 1 ? s1 : (u & 3) == 2 ? s2 : s3;
        c = full ? c + x[u] : c;
        s0 = tail ? s0 + x[u] : s0;
      }
    }
  }
  return (s0 + s1) + (s2 + s3);
}

__device__ __forceinline__ float4& operator+=(float4& a, const float4& b) {
  a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
  return a;
}
__device__ __forceinline__ float4 operator+(float4 a, const float4& b) { return a += b; }

// The G part groups' sums combined in a fixed pairwise tree: (r0 + r1) + (r2 + r3) for G = 4; for
// G = 16 the same over the four quads.
template <int G, typename V>
__device__ __forceinline__ V reduce_tree(const V* r) {
  if constexpr (G == 4) {
    return (r[0] + r[1]) + (r[2] + r[3]);
  } else {
    static_assert(G == 16, "part groups: 4 or 16");
    return (((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]))) +
           (((r[8] + r[9]) + (r[10] + r[11])) + ((r[12] + r[13]) + (r[14] + r[15])));
  }
}

// Elements per reduce block: 256 threads = G part groups x 256 / G lanes, a float4 (reduce_vec4) or a
// float per lane.
__host__ __device__ constexpr int reduce_block_elems(int G, bool vec4) { return (256 / G) * (vec4 ? 4 : 1); }
// Part groups of a reduction over n_parts partials: 4 (each group's partials in one or two load
// batches up to 64 parts), 16 past that (layer_xyz1's 512 encoding partials: 32 per group instead of
// 128 in eight dependent batches -- that job held the whole reduce launch).
__host__ __device__ constexpr int reduce_groups(int64_t n_parts) { return n_parts > 4 * kReduceBatch ? 16 : 4; }

// C (and C2, when set: a second target of the same layout) += the fixed-order sum of the n_parts
// partial (N, K) tiles, elements of block b; G part groups (reduce_groups).
template <int G>
__device__ __forceinline__ void reduce_block(const float* __restrict__ part, int64_t n_parts, int N, int K,
                                             float* __restrict__ C, int64_t ldc, int64_t b, float4 (&red)[16][64],
                                             float* __restrict__ C2 = nullptr) {
  constexpr int L = 256 / G;   // lanes per part group
  const int q = threadIdx.x / L, t = threadIdx.x % L;
  const int64_t nk = (int64_t)N * K;
  const int64_t p0 = n_parts * q / G, p1 = n_parts * (q + 1) / G;
  if (reduce_vec4(part, nk)) {
    const int64_t e = b * reduce_block_elems(G, true) + 4 * t;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (e < nk) {
      const float4* pp = reinterpret_cast<const float4*>(part + e);
      const int64_t st = nk / 4;
      s = reduce_chains(p0, p1, s, [&](int64_t p) { return pp[p * st]; });
    }
    red[q][t] = s;
    __syncthreads();
    if (q == 0 && e < nk) {
      float4 r[G];
#pragma unroll
      for (int g = 0; g < G; ++g) r[g] = red[g][t];
      const float4 v = reduce_tree<G>(r);
      reduce_add(C, ldc, K, e, v.x, C2);
      reduce_add(C, ldc, K, e + 1, v.y, C2);
      reduce_add(C, ldc, K, e + 2, v.z, C2);
      reduce_add(C, ldc, K, e + 3, v.w, C2);
    }
    return;
  }
  const int64_t e = b * reduce_block_elems(G, false) + t;
  float s = 0.0f;
  if (e < nk) s = reduce_chains(p0, p1, 0.0f, [&](int64_t p) { return part[p * nk + e]; });
  red[q][t].x = s;
  __syncthreads();
  if (q == 0 && e < nk) {
    float r[G];
#pragma unroll
    for (int g = 0; g < G; ++g) r[g] = red[g][t].x;
    reduce_add(C, ldc, K, e, reduce_tree<G>(r), C2);
  }
}

__global__ __launch_bounds__(256) void reduce_partials_kernel(const float* __restrict__ part, int64_t n_parts,
                                                              int N, int K, float* __restrict__ C, int64_t ldc) {
  __shared__ float4 red[16][64];
  if (reduce_groups(n_parts) == 16) reduce_block<16>(part, n_parts, N, K, C, ldc, blockIdx.x, red);
  else reduce_block<4>(part, n_parts, N, K, C, ldc, blockIdx.x, red);
}

// Several reductions in one launch (a backward's dW GEMMs queue theirs and flush once).
struct ReduceJob {
  const float* part;
  float* C;
  int64_t n_parts, ldc, first_block;
  int N, K;
  float* C2;  // a second target (g_code's entries that are also bias gradients), or null
};
constexpr int kMaxReduceJobs = 32;   // a training backward queues <= 15 per field; two fields flush together
struct ReduceJobs {
  ReduceJob j[kMaxReduceJobs];
  int n;
};

__global__ __launch_bounds__(256) void reduce_jobs_kernel(ReduceJobs jobs) {
  __shared__ float4 red[16][64];
  int k = jobs.n - 1;
  while (k > 0 && (int64_t)blockIdx.x < jobs.j[k].first_block) --k;
  const ReduceJob& jb = jobs.j[k];
  const int64_t b = (int64_t)blockIdx.x - jb.first_block;
  if (reduce_groups(jb.n_parts) == 16) reduce_block<16>(jb.part, jb.n_parts, jb.N, jb.K, jb.C, jb.ldc, b, red, jb.C2);
  else reduce_block<4>(jb.part, jb.n_parts, jb.N, jb.K, jb.C, jb.ldc, b, red, jb.C2);
}

// gemm_tn: C[n][k] += sum_m A[m][n] B[m][k] (dW = dPre^T X).  No LDS: on
// v_mfma_f32_32x32x2_f32 lane l's A operand is A[m + (l >> 5)][n + (l & 31)] and its B
// operand B[m + (l >> 5)][k + (l & 31)], so each half-wave reads 32 consecutive floats of
// one row straight from global memory (L2).  Block = 4 waves over a 128 x 128 output
// tile, each wave 64 x 64 = 2 x 2 accumulators (4 independent MFMAs per row pair); M is
// split over blockIdx.z (rows_per_block rows each, sized so the grid fills the chip) and
// each block flushes its partial tile with one atomic per output.  Rows are consumed
// kTnPairs pairs at a time: all loads of a group are issued before its MFMAs.
constexpr int kTnTile = 128, kTnPairs = 8;

__global__ __launch_bounds__(256) void gemm_tn_kernel(const float* __restrict__ A, int64_t lda,
                                                      const float* __restrict__ B, int64_t ldb,
                                                      float* __restrict__ C, int64_t ldc, float* __restrict__ part,
                                                      int64_t M, int N, int K, int64_t rows_per_block) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.x * kTnTile + (wave >> 1) * 64;
  const int k0 = blockIdx.y * kTnTile + (wave & 1) * 64;
  if (n0 >= N || k0 >= K) return;  // wave-uniform
  const int64_t mb = (int64_t)blockIdx.z * rows_per_block;
  const int64_t me = min(M, mb + rows_per_block);
  // columns past N / K compute rows / columns of C that are never stored: clamp, no zeroing
  const int na0 = min(n0 + i, N - 1), na1 = min(n0 + 32 + i, N - 1);
  const int kb0 = min(k0 + i, K - 1), kb1 = min(k0 + 32 + i, K - 1);
  floatx16 acc00 = {0}, acc01 = {0}, acc10 = {0}, acc11 = {0};
  for (int64_t m = mb; m < me; m += 2 * kTnPairs) {
    float a0[kTnPairs], a1[kTnPairs], b0[kTnPairs], b1[kTnPairs];
#pragma unroll
    for (int p = 0; p < kTnPairs; ++p) {
      const int64_t r = m + 2 * p + h;
      const bool ok = r < me;
      const float* ar = A + (ok ? r : mb) * lda;
      const float* br = B + (ok ? r : mb) * ldb;
      a0[p] = ok ? ar[na0] : 0.0f;   // a zero A row adds nothing, whatever B holds
      a1[p] = ok ? ar[na1] : 0.0f;
      b0[p] = br[kb0];
      b1[p] = br[kb1];
    }
#pragma unroll
    for (int p = 0; p < kTnPairs; ++p) {
      acc00 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[p], b0[p], acc00, 0, 0, 0);
      acc01 = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[p], b1[p], acc01, 0, 0, 0);
      acc10 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[p], b0[p], acc10, 0, 0, 0);
      acc11 = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[p], b1[p], acc11, 0, 0, 0);
    }
  }
  float* pt = part ? part + (int64_t)blockIdx.z * N * K : nullptr;
  flush_block(acc00, C, ldc, pt, N, K, n0, k0, i, h);
  flush_block(acc01, C, ldc, pt, N, K, n0, k0 + 32, i, h);
  flush_block(acc10, C, ldc, pt, N, K, n0 + 32, k0, i, h);
  flush_block(acc11, C, ldc, pt, N, K, n0 + 32, k0 + 32, i, h);
}

// gemm_tn for the 256 x 256 weight gradients (layer_dir2 / layer_dir1 / fc_out / layer_xyz2),
// row-contiguous operands (lda = ldb = 256): one 512-thread workgroup per CU owns the WHOLE
// 256 x 256 tile over its slab of M rows, so every dPre / X value crosses HBM once.  The slab
// streams through a 4-stage LDS ring by LDS-DMA (buffer_load_dwordx4 ... lds, 1 KiB = one row per
// wave-instruction; a stage = 16 rows of A and of B = 32 KiB), three stages in flight, one
// counted-vmcnt barrier per stage -- the field kernels' scheme.  Wave w: rows 64 (w >> 1) .. of
// n, columns 128 (w & 1) .. of k = 2 x 4 accumulators of v_mfma_f32_32x32x2_f32 (128 registers),
// two waves per SIMD; per row pair it reads its 6 operands with ds_read_b32 (a half-wave reads
// 128 contiguous bytes of one row: conflict free).  Rows past M load as zeros (buffer bounds).
// The slab's partial tile is flushed with one float atomic per element, or stored to the
// workspace for the deterministic reduction.  X3: the same stream with 3xbf16 MFMAs (x3_stage).
constexpr int kTwRows = 16;                    // rows of A and of B per stage
constexpr int kTwStage = 2 * kTwRows * 256 + 64;  // floats per stage: A rows, B rows, SIG: 16 d raw rows
constexpr int kTwRing = 4;

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// 3xbf16 form of one stage (X3: the bf16x3 training step): the stage's 16 rows are ONE k-step of
// v_mfma_f32_32x32x16_bf16 (lane l = 32h + i: rows 8h .. 8h + 7 of feature i of a block).  Each
// lane reads its 8 rows per block with ds_read_b32 (a half-wave reads 128 contiguous bytes of a
// row: conflict free), splits them x = hi + lo and issues Ah.Bh + Ah.Bl + Al.Bh per output block
// (24 MFMAs per wave and stage).  At 3 bf16 MFMAs per 32x32x16 product the kernel is HBM-bound.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split_pair(float x, float y, unsigned& hi, unsigned& lo) {
  const f32x2 v = {x, y};
  const unsigned hu = __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2));
  const f32x2 back = {__uint_as_float(hu << 16), __uint_as_float(hu & 0xffff0000u)};
  hi = hu;
  lo = __builtin_bit_cast(unsigned, __builtin_convertvector(v - back, bf16x2));
}

__device__ __forceinline__ void split8(const float* v, u32x4& hi, u32x4& lo) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    unsigned h, l;
    split_pair(v[2 * q], v[2 * q + 1], h, l);
    hi[q] = h;
    lo[q] = l;
  }
}

__device__ __forceinline__ floatx16 mfma3(floatx16 acc, u32x4 ah, u32x4 al, u32x4 bh, u32x4 bl) {
  const bf16x8 a_h = __builtin_bit_cast(bf16x8, ah), a_l = __builtin_bit_cast(bf16x8, al);
  const bf16x8 b_h = __builtin_bit_cast(bf16x8, bh), b_l = __builtin_bit_cast(bf16x8, bl);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, b_h, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_h, b_l, acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a_l, b_h, acc, 0, 0, 0);
  return acc;
}

static_assert(kTwRows == 16, "x3_stage: one stage = one 16-deep k-step");
__device__ __forceinline__ float sum8v(const float* v) {
  return ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
}

// bsum[t]: running column sums of A's block t over this lane's rows (the bias gradient dPre^T 1).
// SIG (fc_out: its sigma row d sigma^T h2 rides on the h2 stream): sacc[u] += sum over this lane's
// rows of d sigma x B (the stage's d raw rows sit after the B rows).
template <bool SIG>
__device__ __forceinline__ void x3_stage(const float* slot, int i, int h, int n0, int k0, floatx16 (&acc)[2][4],
                                         float (&bsum)[2], float (&sacc)[4], bool sig_wave) {
  const float* sa = slot + 8 * h * 256 + i;
  const float* sb = sa + kTwRows * 256;
  u32x4 ah[2], al[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = sa[j * 256 + n0 + 32 * t];
    bsum[t] += sum8v(v);
    split8(v, ah[t], al[t]);
  }
  float ds[8];
  if constexpr (SIG) {
    const float* sr = slot + 2 * kTwRows * 256 + 8 * h * 4 + 3;
#pragma unroll
    for (int j = 0; j < 8; ++j) ds[j] = sr[4 * j];
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = sb[j * 256 + k0 + 32 * u];
    if constexpr (SIG) {
      if (sig_wave) {
#pragma unroll
        for (int j = 0; j < 8; ++j) sacc[u] = fmaf(ds[j], v[j], sacc[u]);
      }
    }
    u32x4 bh, bl;
    split8(v, bh, bl);
#pragma unroll
    for (int t = 0; t < 2; ++t) acc[t][u] = mfma3(acc[t][u], ah[t], al[t], bh, bl);
  }
}

// DIRS (layer_dir1 only): its 27 view-encoding columns folded into the [feat] pass.  The view
// direction of sample row k of a chunk of rcnt rays is ray k mod rcnt's (Q1, decode_sample), so the
// 16 rows j rcnt + d0 .. + 15 of one sample index j share the directions d0 .. d0 + 15 of every j.
// A stage ("unit") is such a row block, units are ordered (direction group g of 16, j) and each
// workgroup streams a contiguous run of units; it sums its dPre rows per direction (column sums per
// stage row) and stores them per (workgroup, group) run into gsum slot (workgroup + g), 16 x 256
// floats.  dir_enc_dw_kernel then forms dW[:, 256:283] = sum_d dsum[d]^T enc(d) and the bias from
// them -- the encodings are evaluated once per direction instead of once per sample, and the
// (M, 256) dPre plane is streamed once instead of twice (by gemm_tn_enc_kernel as well).
struct DirFold {
  unsigned n_rays, n_samples, chunk_rows;  // rays, samples per ray, Q1 chunk (multiples of 16)
  unsigned units_per_block, total_units;   // 16-row units: total = n_rays / 16 * n_samples
  float* gsum;                             // (workgroups + n_rays / 16) slots of 16 x 256
};


template <bool X3, bool SIG, bool DIRS>
__device__ __forceinline__ void tn256_body(float* ring, const float* __restrict__ A, const float* __restrict__ B,
                                           float* __restrict__ C, int64_t ldc, float* __restrict__ part,
                                           float* __restrict__ bias_part, const float* __restrict__ draw,
                                           float* __restrict__ sig_part, int64_t M, int64_t rows_per_block,
                                           const DirFold& dir, const unsigned blk, const unsigned nblk) {
  static_assert(!(DIRS && (X3 || SIG)), "the direction fold is the fp32 layer_dir1 pass");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int i = lane & 31, h = lane >> 5;
  const int n0 = (wave >> 1) * 64, k0 = (wave & 1) * 128;
  // DIRS: the whole plane as one resource (host: M * 1 KiB + 1 KiB < 4 GiB), units u0 .. u1 - 1
  constexpr bool kIlv = false;
  const int64_t mb = (DIRS || kIlv) ? 0 : (int64_t)blk * rows_per_block;
  const int64_t rows = (DIRS || kIlv) ? M : min(rows_per_block, M - mb);
  const unsigned u0 = DIRS ? blk * dir.units_per_block : 0u;
  const unsigned u1 = DIRS ? min(u0 + dir.units_per_block, dir.total_units) : 0u;
  const unsigned bytes = static_cast<unsigned>(rows * 256 * 4);
  const __amdgpu_buffer_rsrc_t ra =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(A + mb * 256), 0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rb =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(B + mb * 256), 0, bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(SIG ? draw + mb * 4 : A), 0, static_cast<unsigned>(SIG ? rows * 16 : 0), 0x00020000);
  const int n_stages = DIRS ? static_cast<int>(u1 - u0)
                      : kIlv ? static_cast<int>((rows_per_block + kTwRows - 1) / kTwRows)
                             : static_cast<int>((rows + kTwRows - 1) / kTwRows);
  // stage st: wave w moves rows w + 8 j of A and of B (j < kTwRows / 8), one 16-B-per-lane
  // wave-instruction per 1 KiB row: kTwRows / 4 wave-instructions per stage; SIG: every wave also
  // moves the stage's 16 d raw rows (256 B, the same bytes: the per-wave vmcnt stays uniform)
  // DIRS: the DMA's unit cursor (dma() runs for st = 0, 1, 2, ... in order): sample index dj of
  // direction group dg, whose chunk's first row and ray count are dbase * S / drcnt
  unsigned dj = 0, dg = 0, dbase = 0, drcnt = 0;
  if constexpr (DIRS) {
    dg = u0 / dir.n_samples;
    dj = u0 - dg * dir.n_samples;
    dbase = (16 * dg / dir.chunk_rows) * dir.chunk_rows;
    drcnt = min(dir.chunk_rows, dir.n_rays - dbase);
  }
  auto dma = [&](int st) {
    float* slot = ring + (st & (kTwRing - 1)) * kTwStage;
    // DIRS: the unit's first row; units past the run's end (prefetch) read as zeros
    unsigned row0 = static_cast<unsigned>(st * kTwRows);
    if constexpr (kIlv) row0 = static_cast<unsigned>((st * nblk + blk) * kTwRows);
    if constexpr (DIRS) {
      row0 = u0 + static_cast<unsigned>(st) < dir.total_units ? dbase * dir.n_samples + dj * drcnt + (16 * dg - dbase)
                                                               : static_cast<unsigned>(M);
      if (++dj == dir.n_samples) {
        dj = 0;
        ++dg;
        if (16 * dg >= dbase + drcnt) {  // the next Q1 chunk
          dbase += drcnt;
          drcnt = min(dir.chunk_rows, dir.n_rays - dbase);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kTwRows / 8; ++j) {
      const int r = wave + 8 * j;
      const unsigned soff = __builtin_amdgcn_readfirstlane((row0 + static_cast<unsigned>(r)) * 1024u);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(slot + r * 256), 16, lane * 16u, soff, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (lds_ptr_t)(slot + (kTwRows + r) * 256), 16, lane * 16u, soff, 0, 0);
    }
    if constexpr (SIG) {
      const unsigned soff = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(st * kTwRows * 16));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_ptr_t)(slot + 2 * kTwRows * 256), 4, lane * 4u, soff, 0, 0);
    }
  };
  const bool sig_wave = (wave >> 1) == 0;  // waves 0, 1: columns 0..127, 128..255 of the sigma row
  float sacc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  floatx16 acc[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[t][u] = floatx16{0};
  float bsum[2] = {0.0f, 0.0f};
  // DIRS: per-direction column sums of the current unit run, rows 2 p + h of columns n0 + 32 t + i
  // (both waves of a pair sum both column blocks -- a select by wave would become an indexed
  // private array, which the compiler moves to LDS -- and wave 2 q + t stores block t); flushed:
  // the previous stage stored them
  float dsum[DIRS ? 8 : 1][2] = {};
  const int tw = wave & 1;
  bool flushed = false;
  dma(0);
  dma(1);
  dma(2);
  // operands of row pair p + 1 are read while pair p's MFMAs run -- across stages too: the last pair
  // of stage st reads stage st+1's first, so the barrier is followed by MFMAs, not by LDS latency
  float a[2][2], b[2][4];
  float dsg[2] = {0.0f, 0.0f};  // SIG: the pair's d sigma (d raw column 3), read with its operands
  for (int st = 0; st < n_stages; ++st) {
    // stages st AND st+1 landed (all but this wave's kTwRows / 4 youngest pieces: stage st+2's) and
    // every wave is done with stage st-1, whose slot then receives stage st+3 (issued after this
    // stage's first row pair, beside its MFMAs); after a DIRS flush its 8 stores are the youngest 8
    // vector-memory ops as well.  Waiting for st+1 here (it was issued two stages ago) is what lets
    // the last row pair prefetch from it.
    static_assert(kTwRows / 4 == 4, "the vmcnt below counts stage st+2");
    // lgkmcnt(0) as the compiler's own wait (it does not read the asm's): the next stage's first
    // operands, read during the last pair, have landed, so nothing is owed at the loop header and the
    // first MFMAs start at once
    __builtin_amdgcn_s_waitcnt(0xC07F);
    if constexpr (SIG) asm volatile("s_waitcnt vmcnt(5)\n\ts_barrier" ::: "memory");
    else if (DIRS && flushed) asm volatile("s_waitcnt vmcnt(12)\n\ts_barrier" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (X3) {
      dma(st + 3);
      x3_stage<SIG>(ring + (st & (kTwRing - 1)) * kTwStage, i, h, n0, k0, acc, bsum, sacc, sig_wave);
      continue;
    }
    const float* sa = ring + (st & (kTwRing - 1)) * kTwStage + h * 256 + i;
    const float* sb = sa + kTwRows * 256;
    const float* sa1 = ring + ((st + 1) & (kTwRing - 1)) * kTwStage + h * 256 + i;  // stage st+1
    const float* sb1 = sa1 + kTwRows * 256;
    if (st == 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t) a[0][t] = sa[n0 + 32 * t];
#pragma unroll
      for (int u = 0; u < 4; ++u) b[0][u] = sb[k0 + 32 * u];
      if constexpr (SIG) dsg[0] = sb[kTwRows * 256 - (h * 256 + i) + h * 4 + 3];
    }
#pragma unroll
    for (int p = 0; p < kTwRows / 2; ++p) {
      const int c = p & 1, nx = c ^ 1;
      if (p + 1 < kTwRows / 2) {
#pragma unroll
        for (int t = 0; t < 2; ++t) a[nx][t] = sa[(p + 1) * 512 + n0 + 32 * t];
#pragma unroll
        for (int u = 0; u < 4; ++u) b[nx][u] = sb[(p + 1) * 512 + k0 + 32 * u];
        if constexpr (SIG) dsg[nx] = sb[kTwRows * 256 - (h * 256 + i) + (2 * (p + 1) + h) * 4 + 3];
      } else {
        // stage st+1's first pair (past the last stage: slot st+1 holds zeros or a stale stage; unused)
#pragma unroll
        for (int t = 0; t < 2; ++t) a[nx][t] = sa1[n0 + 32 * t];
#pragma unroll
        for (int u = 0; u < 4; ++u) b[nx][u] = sb1[k0 + 32 * u];
        if constexpr (SIG) dsg[nx] = sb1[kTwRows * 256 - (h * 256 + i) + h * 4 + 3];
      }
      // keep the next pair's reads above this pair's MFMAs: left to itself the scheduler sinks them
      // below, and every pair then opens with an exposed LDS round trip (lgkmcnt(0) before its MFMAs)
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        // the bias gradient's column sum (DIRS: per direction) rides on the A stream (VALU beside MFMA)
        if constexpr (DIRS) dsum[p][t] += a[c][t];
        else bsum[t] += a[c][t];
#pragma unroll
        for (int u = 0; u < 4; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c][t], b[c][u], acc[t][u], 0, 0, 0);
      }
      if constexpr (SIG) {
        // every wave (no branch in the MFMA stream); only the sig waves' sums are stored
#pragma unroll
        for (int u = 0; u < 4; ++u) sacc[u] = fmaf(dsg[c], b[c][u], sacc[u]);
      }
      if (p == 0) {
        __builtin_amdgcn_sched_barrier(0);
        dma(st + 3);  // beside the first pair's MFMAs
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (DIRS) {
      // the run of direction group g ends with this stage: its sums go to slot (workgroup + g)
      const unsigned u = u0 + static_cast<unsigned>(st);
      flushed = st + 1 == n_stages || (u + 1) % dir.n_samples == 0;
      if (flushed) {
        float* gs = dir.gsum + (int64_t)(blk + u / dir.n_samples) * 4096 + h * 256 + n0 + 32 * tw + i;
#pragma unroll
        for (int p = 0; p < 8; ++p) {
          gs[p * 512] = tw ? dsum[p][1] : dsum[p][0];
          dsum[p][0] = 0.0f;
          dsum[p][1] = 0.0f;
        }
      }
    }
  }
  // the prefetched stages past the slab must land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float* pt = part ? part + (int64_t)blk * 65536 : nullptr;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 4; ++u) flush_block(acc[t][u], C, ldc, pt, 256, 256, n0 + 32 * t, k0 + 32 * u, i, h);
  // bias_part: this slab's column sums of A, in row order per lane (the waves of column half 0
  // cover all 256 columns)
  if (bias_part && (wave & 1) == 0) {
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const float b = bsum[t] + __shfl_xor(bsum[t], 32);
      if (h == 0) bias_part[(int64_t)blk * 256 + n0 + 32 * t + i] = b;
    }
  }
  if (SIG && sig_wave) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float v = sacc[u] + __shfl_xor(sacc[u], 32);
      if (h == 0) sig_part[(int64_t)blk * 256 + k0 + 32 * u + i] = v;
    }
  }
}
// One dW GEMM per launch (gemm_tn's whole-tile plan).
template <bool X3, bool SIG, bool DIRS = false>
__global__ __launch_bounds__(512, 2) void gemm_tn256_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                            float* __restrict__ C, int64_t ldc, float* __restrict__ part,
                                                            float* __restrict__ bias_part, const float* __restrict__ draw,
                                                            float* __restrict__ sig_part, int64_t M,
                                                            int64_t rows_per_block, DirFold dir = {}) {
  __shared__ __attribute__((aligned(16))) float ring[kTwRing * kTwStage];
  tn256_body<X3, SIG, DIRS>(ring, A, B, C, ldc, part, bias_part, draw, sig_part, M, rows_per_block, dir, blockIdx.x,
                            gridDim.x);
}

// Several whole-tile dW GEMMs in ONE launch (a training backward's four 256 x 256 layers): job k
// owns workgroups first_block .. first_block + n_blocks - 1 and splits its M rows over them.  Fewer
// workgroups per GEMM means fewer partial tiles (each 256 KiB, written at the end and read back by
// the deterministic reduction) and one launch's prologue and tail instead of four; the jobs' block
// counts are weighted by their per-row cost so they end together.
struct TnJob {
  const float* A;
  const float* B;
  float* part;       // n_blocks partial tiles (256 x 256; RGB: 3 x 256)
  float* bias_part;  // optional: n_blocks x 256 column sums of A (RGB: the d raw column sums, 4 per block)
  const float* draw; // SIG, RGB: the (M, 4) d raw rows
  float* sig_part;   // SIG: n_blocks x 256
  int64_t M, rows_per_block;
  int kind;          // 0 plain, 1 SIG (fc_out's sigma row), 2 DIRS (layer_dir1's view-encoding fold), 3 RGB,
                     // 4 XENC (layer_xyz1's dW from the encoding plane, gemm_tn_xenc_kernel's row pass)
  int first_block, n_blocks;
  DirFold dir;
};
constexpr int kMaxTnJobs = 12;   // a field's five (six with the XENC role), or a render's two fields' (tn_batch_launch2)
struct TnJobs {
  TnJob j[kMaxTnJobs];
  int n;
};

// RGB (kind 3): fc_rgb's dW, C += d rgb^T v2 (3 x 256), and the column sums of the d raw rows
// (g_code's rgb / sigma entries with one code row) -- gemm_tn_skinny_kernel<3, true>'s work as a
// role of the whole-tile launch.  It is a bandwidth pass (1 KiB of v2 per row, 24 FMAs per row per
// 256 threads), so it runs on a few workgroups beside the MFMA-bound GEMMs instead of taking the
// whole chip for its own ~80 us: a deep LDS-DMA ring (kRgbRing stages of 16 v2 rows + their 16 d
// raw rows, all but one in flight, ~100 KiB per CU) keeps one CU's loads streaming.  Thread t sums
// column t & 255 over rows 8 (t >> 8) .. + 7 of every stage; the two halves and the per-row d raw
// sums (threads 0, 256) are added in a fixed order at the end: deterministic.
constexpr int kRgbRing = 7;
constexpr int kRgbStage = kTwRows * 256 + kTwRows * 4;
static_assert(kRgbRing * kRgbStage <= kTwRing * kTwStage, "the RGB ring lives in the whole-tile ring's LDS");

__device__ __forceinline__ void rgb_body(float* ring, const float* __restrict__ draw, const float* __restrict__ v2,
                                         float* __restrict__ part, float* __restrict__ cpart, int64_t M,
                                         int64_t rows_per_block, const unsigned blk, const unsigned nblk) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t mb = (int64_t)blk * rows_per_block;
  const int64_t rows = min(rows_per_block, M - mb);
  const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(v2 + mb * 256), 0,
                                                                      static_cast<unsigned>(rows * 1024), 0x00020000);
  const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(draw + mb * 4), 0,
                                                                      static_cast<unsigned>(rows * 16), 0x00020000);
  const int n_stages = static_cast<int>((rows + kTwRows - 1) / kTwRows);
  // stage st: wave w moves v2 rows w, w + 8 (1 KiB each) and -- every wave, the same 256 bytes, so the
  // per-wave vmcnt stays uniform -- the stage's 16 d raw rows; rows past the slab read as zeros
  auto dma = [&](int st) {
    float* slot = ring + (st % kRgbRing) * kRgbStage;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = wave + 8 * j;
      const unsigned soff = __builtin_amdgcn_readfirstlane(static_cast<unsigned>((st * kTwRows + r) * 1024));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rv, (lds_ptr_t)(slot + r * 256), 16, lane * 16u, soff, 0, 0);
    }
    const unsigned soff = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(st * kTwRows * 16));
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rr, (lds_ptr_t)(slot + kTwRows * 256), 4, lane * 4u, soff, 0, 0);
  };
  const int c = tid & 255, hh = tid >> 8;
  float a0 = 0.0f, a1 = 0.0f, a2 = 0.0f;
  float cs[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
  for (int st = 0; st < kRgbRing - 1; ++st) dma(st);
  for (int st = 0; st < n_stages; ++st) {
    // stage st landed (all but this wave's pieces of stages st+1 .. st+kRgbRing-2: 3 each) and every
    // wave is past stage st-1, whose slot then receives stage st+kRgbRing-1
    static_assert(3 * (kRgbRing - 2) == 15, "the vmcnt below");
    asm volatile("s_waitcnt vmcnt(15)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    dma(st + kRgbRing - 1);
    const float* slot = ring + (st % kRgbRing) * kRgbStage;
    const float* sv = slot + 8 * hh * 256 + c;
    const float4* sd = reinterpret_cast<const float4*>(slot + kTwRows * 256) + 8 * hh;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = sv[j * 256];
      const float4 d = sd[j];
      a0 = fmaf(d.x, v, a0);
      a1 = fmaf(d.y, v, a1);
      a2 = fmaf(d.z, v, a2);
      if (c == 0) {
        cs[0] += d.x;
        cs[1] += d.y;
        cs[2] += d.z;
        cs[3] += d.w;
      }
    }
  }
  // the prefetched stages past the slab land, then the halves meet in the (free) ring
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (hh == 1) {
    ring[c] = a0;
    ring[256 + c] = a1;
    ring[512 + c] = a2;
    if (c == 0)
      for (int n = 0; n < 4; ++n) ring[768 + n] = cs[n];
  }
  __syncthreads();
  if (hh == 0) {
    float* pt = part + (int64_t)blk * 3 * 256;
    pt[c] = a0 + ring[c];
    pt[256 + c] = a1 + ring[256 + c];
    pt[512 + c] = a2 + ring[512 + c];
    if (c == 0) {
      for (int n = 0; n < 3; ++n) cpart[(int64_t)blk * 3 + n] = cs[n] + ring[768 + n];
      cpart[3 * (int64_t)nblk + blk] = cs[3] + ring[771];
    }
  }
}



// gemm_tn for a skinny dPre (N = NA <= 4 columns, e.g. d rgb / d sigma of d raw) against a
// 256-wide X: a streaming pass over X (float4 per lane, 4 rows per 256-thread step) with the
// 4 x NA partial sums in registers, folded through LDS and flushed with NA x 256 atomics per
// workgroup (or stored as the workgroup's partial row block: the deterministic path).
// Bandwidth-bound: X crosses HBM once.
// CS (A = the (M, 4) d raw rows, NA = 3): also the column sums of all 4 columns of A -- g_code's
// rgb and sigma entries when the code gradient is folded (one code row) -- in row order per row
// group, the 4 groups added in order: cpart[b * 3 + n] (n < 3) and cpart[3 nb + b] (sigma).
template <int NA, bool CS = false>
__global__ __launch_bounds__(256) void gemm_tn_skinny_kernel(const float* __restrict__ A, int64_t lda,
                                                             const float* __restrict__ B, float* __restrict__ C,
                                                             int64_t ldc, float* __restrict__ part, int64_t M,
                                                             int64_t rows_per_block, float* __restrict__ cpart = nullptr) {
  __shared__ float red[4][NA][256];
  __shared__ float cred[4][4];
  const int t = threadIdx.x, rg = t >> 6, c4 = t & 63;
  const int64_t mb = (int64_t)blockIdx.x * rows_per_block;
  const int64_t me = min(M, mb + rows_per_block);
  float acc[NA][4] = {};
  float cs[4] = {0.f, 0.f, 0.f, 0.f};
  for (int64_t m = mb + rg; m < me; m += 4) {
    const float4 x = reinterpret_cast<const float4*>(B + m * 256)[c4];
#pragma unroll
    for (int n = 0; n < NA; ++n) {
      const float av = A[m * lda + n];
      acc[n][0] = fmaf(av, x.x, acc[n][0]);
      acc[n][1] = fmaf(av, x.y, acc[n][1]);
      acc[n][2] = fmaf(av, x.z, acc[n][2]);
      acc[n][3] = fmaf(av, x.w, acc[n][3]);
    }
    if constexpr (CS) {
      const float4 a4 = reinterpret_cast<const float4*>(A)[m];
      cs[0] += a4.x;
      cs[1] += a4.y;
      cs[2] += a4.z;
      cs[3] += a4.w;
    }
  }
  if constexpr (CS) {
    if (c4 == 0)
#pragma unroll
      for (int n = 0; n < 4; ++n) cred[rg][n] = cs[n];
  }
#pragma unroll
  for (int n = 0; n < NA; ++n)
#pragma unroll
    for (int j = 0; j < 4; ++j) red[rg][n][4 * c4 + j] = acc[n][j];
  __syncthreads();
#pragma unroll
  for (int n = 0; n < NA; ++n) {
    const float v = (red[0][n][t] + red[1][n][t]) + (red[2][n][t] + red[3][n][t]);
    if (part) part[((int64_t)blockIdx.x * NA + n) * 256 + t] = v;
    else atomicAdd(&C[n * ldc + t], v);
  }
  if constexpr (CS) {
    if (t < 4) {
      const float v = (cred[0][t] + cred[1][t]) + (cred[2][t] + cred[3][t]);
      if (t < 3) cpart[(int64_t)blockIdx.x * 3 + t] = v;
      else cpart[3 * (int64_t)gridDim.x + blockIdx.x] = v;
    }
  }
}

// ---------------------------------------------------------------- 3xbf16 GEMMs
// The same two products on v_mfma_f32_32x32x16_bf16 with each fp32 operand split
// x = hi + lo (hi = bf16(x), lo = bf16(x - hi)) and Ah.Bh + Ah.Bl + Al.Bh accumulated in
// fp32 (the dropped Al.Bl and the lo rounding leave ~2^-17 relative error per product,
// the field kernel's scheme).  On 32x32x16 lane l = 32h + i holds A[row i][k = 8h + j]
// and B[k = 8h + j][col i], j = 0..7: exactly the 8 consecutive k values the fp32
// kernels' lanes already load, so one bf16 MFMA triple replaces 8 fp32 MFMAs.

// XCD-aware block order: workgroups are dispatched to the 8 XCDs round-robin, so
// block b runs on XCD b % 8.  Renumber so each XCD takes a contiguous range of the
// logical tile order: the tiles that share input rows (the column blocks of one row
// tile, the output tiles of one M split) then run back to back on ONE XCD and the
// shared rows come from its L2 instead of HBM once per tile.
__device__ __forceinline__ unsigned xcd_order(unsigned b, unsigned total) {
  if (total % 8 != 0) return b;
  return (b % 8) * (total / 8) + b / 8;
}

// gemm_nn_x3: block = kNnWaves (4) waves x 32 rows = 128 rows, each wave all 32 NU columns of its
// column group (NU <= 8 accumulators, so A is read from HBM exactly once for N <= 256).
// k runs in 32-deep pairs of MFMA k-tiles.  Any permutation of k inside a pair is valid if
// A and B use the same one, so lane half h takes k = 16h .. 16h + 15 of the pair (k-tile s
// of the pair: 16h + 8s + j): each lane reads one full 64-byte run of its row per pair
// (a whole 128-byte line per row across the two halves) instead of scattered 32-byte
// pieces.  B^T streams through LDS one pair (two 16-deep slabs) at a time, double-buffered
// and fragment-major (slab, column block u, hi|lo, lane: one fragment read is 1 KiB
// contiguous).  During pair p each thread loads its B entries and the wave its A run of
// pair p + 1, runs p's MFMAs, then splits and stores pair p + 1.  One barrier per pair.
// VEC: lda % 4 == 0 and A 16-byte aligned (four dwordx4 per row per pair).
constexpr int kNnWaves = 4, kNnRows = 32 * kNnWaves, kNnThreads = 64 * kNnWaves;

template <int NU, bool VEC>
__global__ __launch_bounds__(kNnThreads, 2) void gemm_nn_x3_kernel(const float* __restrict__ A, int64_t lda,
                                                         const float* __restrict__ B, int64_t ldb,
                                                         float* __restrict__ C, int64_t ldc,
                                                         const float* __restrict__ mask, int64_t ldm,
                                                         int64_t M, int N, int K) {
  __shared__ u32x4 Bs[2][2][NU * 2 * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 31, h = lane >> 5;
  const int n0 = blockIdx.y * 256;
  const int nkp = (K + 31) / 32;
  const int64_t m0 = (int64_t)blockIdx.x * kNnRows + wave * 32;
  const int64_t row = min(m0 + i, M - 1);
  const float* arow = A + row * lda + h * 16;
  // this thread's B entries of a slab: column blocks u = tid / 64 + kNnWaves e (< NU), lane tid % 64
  constexpr int kSE = (NU + kNnWaves - 1) / kNnWaves;
  const int sl = tid & 63;
  const int sk = 16 * (sl >> 5);
  auto load_b = [&](int p, float (&bv)[kSE][2][8]) {
#pragma unroll
    for (int e = 0; e < kSE; ++e) {
      const int su = (tid >> 6) + kNnWaves * e;
      const int sn = n0 + 32 * su + (sl & 31);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int k = 32 * p + sk + 8 * t + j;
          bv[e][t][j] = (su < NU && k < K && sn < N) ? B[(int64_t)k * ldb + sn] : 0.0f;
        }
    }
  };
  auto store_b = [&](int buf, const float (&bv)[kSE][2][8]) {
#pragma unroll
    for (int e = 0; e < kSE; ++e) {
      const int su = (tid >> 6) + kNnWaves * e;
      if (su < NU) {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          u32x4 hi, lo;
          split8(bv[e][t], hi, lo);
          Bs[buf][t][(su * 2) * 64 + sl] = hi;
          Bs[buf][t][(su * 2 + 1) * 64 + sl] = lo;
        }
      }
    }
  };
  auto load_a = [&](int p, float (&a)[16]) {
    const int kb = 32 * p + h * 16;
    if (VEC && kb + 16 <= K) {
      const float4* ap = reinterpret_cast<const float4*>(arow + 32 * p);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float4 x = ap[q];
        a[4 * q] = x.x; a[4 * q + 1] = x.y; a[4 * q + 2] = x.z; a[4 * q + 3] = x.w;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 16; ++q) a[q] = (kb + q < K) ? arow[32 * p + q] : 0.0f;
    }
  };
  floatx16 acc[NU];
#pragma unroll
  for (int u = 0; u < NU; ++u) acc[u] = floatx16{0};
  float an[16], bn[kSE][2][8];
  load_b(0, bn);
  load_a(0, an);
  store_b(0, bn);
  __syncthreads();
  for (int p = 0; p < nkp; ++p) {
    const int buf = p & 1;
    u32x4 ah[2], al[2];
    split8(an, ah[0], al[0]);
    split8(an + 8, ah[1], al[1]);
    const bool more = p + 1 < nkp;
    if (more) {
      load_b(p + 1, bn);
      load_a(p + 1, an);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const u32x4 bh = Bs[buf][t][(u * 2) * 64 + lane];
        const u32x4 bl = Bs[buf][t][(u * 2 + 1) * 64 + lane];
        acc[u] = mfma3(acc[u], ah[t], al[t], bh, bl);
      }
    if (more) store_b(buf ^ 1, bn);
    __syncthreads();
  }
  // Epilogue.  Full tiles (the common case) take the mask in batches of 16 loads with no
  // per-element branch, so a batch is one memory round trip; ragged tiles are guarded.
  if (m0 + 32 <= M && n0 + 32 * NU <= N) {
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      const int col = n0 + 32 * u + i;
      float mk[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        mk[r] = mask ? mask[m * ldm + col] : 1.0f;
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int64_t m = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
        C[m * ldc + col] = mk[r] > 0.0f ? acc[u][r] : 0.0f;
      }
    }
    return;
  }
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int col = n0 + 32 * u + i;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t m = m0 + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m < M && col < N) {
        float x = acc[u][r];
        if (mask && !(mask[m * ldm + col] > 0.0f)) x = 0.0f;
        C[m * ldc + col] = x;
      }
    }
  }
}

// gemm_tn_x3: C[n][k] += sum_m A[m][n] B[m][k].  Wave = 64 x 64 output (2 x 2
// accumulators), block = 128 x 128; lane (i, h) reads A[m + 8h + j][n + i] and
// B[m + 8h + j][k + i] for j = 0..7 (each half-wave row read is 128 contiguous bytes).
// 1D grid over (M split, output tile), XCD-ordered so the tiles of one split share L2.
constexpr int kTnRowsX3 = 16, kTnGroupsX3 = 2;

__global__ __launch_bounds__(256) void gemm_tn_x3_kernel(const float* __restrict__ A, int64_t lda,
                                                         const float* __restrict__ B, int64_t ldb,
                                                         float* __restrict__ C, int64_t ldc, float* __restrict__ part,
                                                         int64_t M, int N, int K, int64_t rows_per_block, int tiles_n,
                                                         int tiles) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int i = lane & 31, h = lane >> 5;
  const unsigned v = xcd_order(blockIdx.x, gridDim.x);
  const int tile = v % tiles;
  const int64_t split = v / tiles;
  const int n0 = (tile % tiles_n) * kTnTile + (wave >> 1) * 64;
  const int k0 = (tile / tiles_n) * kTnTile + (wave & 1) * 64;
  if (n0 >= N || k0 >= K) return;  // wave-uniform
  const int64_t mb = split * rows_per_block;
  const int64_t me = min(M, mb + rows_per_block);
  const int na0 = min(n0 + i, N - 1), na1 = min(n0 + 32 + i, N - 1);
  const int kb0 = min(k0 + i, K - 1), kb1 = min(k0 + 32 + i, K - 1);
  floatx16 acc00 = {0}, acc01 = {0}, acc10 = {0}, acc11 = {0};
  // kTnGroupsX3 16-row groups per iteration: all their loads are issued before any MFMA
  for (int64_t m = mb; m < me; m += kTnRowsX3 * kTnGroupsX3) {
    float a0[kTnGroupsX3][8], a1[kTnGroupsX3][8], b0[kTnGroupsX3][8], b1[kTnGroupsX3][8];
#pragma unroll
    for (int g = 0; g < kTnGroupsX3; ++g)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t r = m + kTnRowsX3 * g + 8 * h + j;
        const bool ok = r < me;
        const float* ar = A + (ok ? r : mb) * lda;
        const float* br = B + (ok ? r : mb) * ldb;
        a0[g][j] = ok ? ar[na0] : 0.0f;  // a zero A row adds nothing, whatever B holds
        a1[g][j] = ok ? ar[na1] : 0.0f;
        b0[g][j] = br[kb0];
        b1[g][j] = br[kb1];
      }
#pragma unroll
    for (int g = 0; g < kTnGroupsX3; ++g) {
      u32x4 a0h, a0l, a1h, a1l, b0h, b0l, b1h, b1l;
      split8(a0[g], a0h, a0l);
      split8(a1[g], a1h, a1l);
      split8(b0[g], b0h, b0l);
      split8(b1[g], b1h, b1l);
      acc00 = mfma3(acc00, a0h, a0l, b0h, b0l);
      acc01 = mfma3(acc01, a0h, a0l, b1h, b1l);
      acc10 = mfma3(acc10, a1h, a1l, b0h, b0l);
      acc11 = mfma3(acc11, a1h, a1l, b1h, b1l);
    }
  }
  float* pt = part ? part + split * N * K : nullptr;
  flush_block(acc00, C, ldc, pt, N, K, n0, k0, i, h);
  flush_block(acc01, C, ldc, pt, N, K, n0, k0 + 32, i, h);
  flush_block(acc10, C, ldc, pt, N, K, n0 + 32, k0, i, h);
  flush_block(acc11, C, ldc, pt, N, K, n0 + 32, k0 + 32, i, h);
}

// gemm_tn against the positional encodings, generated in the kernel: C[n][c] += sum_m A[m][n]
// enc(m)[c] with enc = the 63 xyz features of the sample point (ENC 0: layer_xyz1's dW) or the 27
// of its Q1 view direction (ENC 1: layer_dir1's view-direction columns), in
// PositionalEmbedder.embed order and with encode_inputs_kernel's exact arithmetic -- so the
// (M, 90) x_enc plane is never written or read.  Stage = 16 A rows, moved into a 3-slot LDS ring
// by LDS-DMA two stages ahead (one counted vmcnt + barrier per stage; until r02 they were
// register-staged one stage ahead and the kernel ran at ~2-2.7 TB/s, latency-bound); threads
// 0..15 decode the samples' geometry three stages ahead and 32 threads per sample evaluate its
// encoding (one sincosf per sin/cos pair) one stage ahead into a double-buffered table.
// Wave w owns output rows 32 w .. 32 w + 31 and all KB = 2 (xyz) / 1 (dir) column blocks;
// X3: one 32x32x16 bf16 k-step per stage (3 products), else 8 fp32 32x32x2 row pairs.
constexpr int kEncRows = 16;
constexpr int kEncRing = 3;  // A stages in LDS: the one being read, two landing

// 8 floats at p + k * S bytes (k = 0..7) of the LDS-DMA ring, one round trip.  Inline asm: hipcc
// cannot tell these reads from the ring slots the in-flight LDS-DMA pieces fill and would wait
// vmcnt(0) before them, draining the prefetch; the counted vmcnt + barrier at the top of the
// stage already guarantee the slot read here has landed.
template <int S>
__device__ __forceinline__ void ring_read8(const float* p, float* v) {
  const unsigned addr = static_cast<unsigned>(reinterpret_cast<uintptr_t>((const __attribute__((address_space(3))) void*)p));
  asm volatile(
      "ds_read_b32 %0, %8\n\tds_read_b32 %1, %8 offset:%9\n\tds_read_b32 %2, %8 offset:%10\n\t"
      "ds_read_b32 %3, %8 offset:%11\n\tds_read_b32 %4, %8 offset:%12\n\tds_read_b32 %5, %8 offset:%13\n\t"
      "ds_read_b32 %6, %8 offset:%14\n\tds_read_b32 %7, %8 offset:%15\n\ts_waitcnt lgkmcnt(0)"
      : "=&v"(v[0]), "=&v"(v[1]), "=&v"(v[2]), "=&v"(v[3]), "=&v"(v[4]), "=&v"(v[5]), "=&v"(v[6]), "=&v"(v[7])
      : "v"(addr), "i"(S), "i"(2 * S), "i"(3 * S), "i"(4 * S), "i"(5 * S), "i"(6 * S), "i"(7 * S)
      : "memory");
}

// The second half of the DIRS fold (gemm_tn256_kernel): workgroup w of this kernel takes direction
// groups kDirGroups w .. + kDirGroups - 1; per group it adds the gsum slots of the tn256 workgroups
// whose unit runs cover it (in workgroup order), evaluates the 16 directions' encodings with
// gemm_tn_enc_kernel's arithmetic (PositionalEmbedder order: raw 0..2, then per frequency sin 3,
// cos 3) and accumulates thread n's row of dW: part[w][n][k] = sum_d dsum[d][n] enc(d)[k], k < 27;
// the bias (enc 1) into bias_part[w][n].  Fixed order throughout: deterministic.
constexpr int kDirGroups = 1;
// Workgroup blk of that launch; threads 0..255 work (a 512-thread caller's upper half only takes
// part in the barriers: the role rides in gemm_tn_enc_kernel's launch).
__device__ __forceinline__ void dir_enc_dw_block(const mlp::FieldArgs& a, const DirFold& dir, float* __restrict__ part,
                                                 float* __restrict__ bias_part, unsigned blk) {
  __shared__ float encl[16][28];
  const int n = threadIdx.x;
  const bool act = n < 256;
  const unsigned S = dir.n_samples, U = dir.units_per_block, n_groups = dir.n_rays / 16;
  float acc[28];
#pragma unroll
  for (int k = 0; k < 28; ++k) acc[k] = 0.0f;
  for (int q = 0; q < kDirGroups; ++q) {
    const unsigned g = blk * kDirGroups + q;
    if (g >= n_groups) break;
    float ds[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) ds[r] = 0.0f;
    const unsigned b0 = g * S / U, b1 = ((g + 1) * S - 1) / U;
    if (act) {
      for (unsigned b = b0; b <= b1; ++b) {
        const float* gs = dir.gsum + (int64_t)(b + g) * 4096 + n;
#pragma unroll
        for (int r = 0; r < 16; ++r) ds[r] += gs[r * 256];
      }
    }
    __syncthreads();  // the previous group's encodings are read
    if (n < 16 * 12) {
      const int r = n / 12, p = n - 12 * (n / 12), comp = p % 3, c0 = 3 + 6 * (p / 3) + comp;
      float vd[3];
      mlp::view_dir(a, 16 * (int64_t)g + r, vd);
      float s, c;
      mlp::enc_sincosf(__fmul_rn(mlp::pick3(vd, comp), a.fd[p / 3]), s, c);
      encl[r][c0] = s;
      encl[r][c0 + 3] = c;
    } else if (n < 16 * 13) {
      const int r = n - 16 * 12;
      float vd[3];
      mlp::view_dir(a, 16 * (int64_t)g + r, vd);
      encl[r][0] = vd[0];
      encl[r][1] = vd[1];
      encl[r][2] = vd[2];
      encl[r][27] = 1.0f;
    }
    __syncthreads();
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int k = 0; k < 28; ++k) acc[k] = fmaf(ds[r], encl[r][k], acc[k]);
  }
  if (!act) return;
  float* pt = part + (int64_t)blk * 256 * 27 + n * 27;
#pragma unroll
  for (int k = 0; k < 27; ++k) pt[k] = acc[k];
  bias_part[(int64_t)blk * 256 + n] = acc[27];
}

// The DIRS fold's second half as a role of this launch (gemm_tn_enc_kernel's first n workgroups run
// dir_enc_dw_block instead of a separate 256-workgroup launch): both only need the batched dW launch's
// outputs (gsum / dPre planes), and their partials go to the same deferred reduction.
struct DirRole {
  DirFold dir;
  float* part;
  float* bias_part;
  unsigned n;  // workgroups of the role (0: none)
};

template <bool X3, int ENC, int MODE>
__global__ __launch_bounds__(512, 1) void gemm_tn_enc_kernel(const float* __restrict__ A, mlp::FieldArgs a,
                                                             float* __restrict__ C, int64_t ldc,
                                                             float* __restrict__ part, float* __restrict__ bias_part,
                                                             int64_t rows_per_block, DirRole dr) {
  if (blockIdx.x < dr.n) {
    dir_enc_dw_block(a, dr.dir, dr.part, dr.bias_part, blockIdx.x);
    return;
  }
  const unsigned blk = blockIdx.x - dr.n;
  constexpr int K = ENC == 0 ? 63 : 27, KB = ENC == 0 ? 2 : 1, EW = 32 * KB;
  // row strides (floats) of the A ring and the encoding table: the two rows a wave's half-waves
  // read together (fp32: rows 2 p and 2 p + 1; x3: rows j and 8 + j) sit 32 banks apart -- with
  // 256 / 64-float rows they hit the same banks (a 2-way conflict on every read)
  constexpr int RS = X3 ? 260 : 288;
  constexpr int ES = X3 ? EW + 4 : (EW % 64 == 0 ? EW + 32 : EW);
  __shared__ __attribute__((aligned(16))) float ring[kEncRing][kEncRows * RS];  // A stages, by LDS-DMA
  __shared__ __attribute__((aligned(16))) float senc[2][kEncRows * ES];
  __shared__ __attribute__((aligned(16))) float4 xs[3][kEncRows];  // decoded geometry, 3 stages
  __shared__ int xfast[3];  // ENC 0, fp32: the stage's 16 points all inside fast_sincosf's bound (below)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 31, h = lane >> 5;
  const int64_t M = a.m;
  const int64_t mb = (int64_t)blk * rows_per_block;
  const int64_t rows = min(rows_per_block, M - mb);
  const int n_stages = static_cast<int>((rows + kEncRows - 1) / kEncRows);
  // the slab's A rows as a buffer resource: rows past it (the last stage's tail, the stages the
  // loop prefetches past the end) read as zeros
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(A + mb * 256), 0, static_cast<unsigned>(rows * 256 * 4), 0x00020000);
  // roles: encoding sample es (16 per stage), slot j = tid & 31 of its table row: slot j < NP owns
  // the (sin, cos) pair p = j of PositionalEmbedder's layout (columns 3 + 6 (p / 3) + p % 3 and
  // that + 3: ONE sincosf), the next slots two of the extra columns each (raw inputs 0..2, zero
  // padding K..EW-1); threads 0..15 decode the geometry of stage st + 3 (one sample each: the Q1
  // map's integer divisions run once per sample)
  constexpr int NP = ENC == 0 ? 30 : 12;                 // 3 components x L frequencies
  constexpr int NX = (3 + (EW - K) + 1) / 2;             // slots of extra columns
  static_assert(NP + NX <= 32, "one table row per 32 threads");
  const int es = tid >> 5, j = tid & 31;
  // the slot's columns, resolved once: the frequency table is a kernel argument, and reading it
  // per stage (a per-lane index: a global load) would make every stage wait for the LDS-DMA
  // pieces in flight
  int kind = 0, c0 = 0, c1 = 0, comp = 0;  // kind 0 idle, 1 sin/cos pair, 2 extra columns
  float freq = 0.0f;
  if (j < NP) {
    kind = 1;
    comp = j % 3;
    c0 = 3 + 6 * (j / 3) + comp;
    c1 = c0 + 3;
    freq = ENC == 0 ? a.fx[j / 3] : a.fd[j / 3];
  } else if (j < NP + NX) {
    kind = 2;
    comp = 2 * (j - NP);  // logical extra columns comp, comp + 1: q < 3 raw input q, else column K + q - 3
    c0 = comp < 3 ? comp : K + comp - 3;
    c1 = comp + 1 < 3 ? comp + 1 : K + comp - 2;
  }
  float ev[2] = {0.0f, 0.0f};
  // stage st's 16 A rows: wave w moves rows w, w + 8 (1 KiB each, one 16-B-per-lane wave-instruction)
  auto dma = [&](int st) {
    float* slot = ring[st % kEncRing];
#pragma unroll
    for (int j = 0; j < kEncRows / 8; ++j) {
      const int r = wave + 8 * j;
      const unsigned soff = __builtin_amdgcn_readfirstlane(static_cast<unsigned>((st * kEncRows + r) * 1024));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(slot + r * RS), 16, lane * 16u, soff, 0, 0);
    }
  };
  // decode(st) only ISSUES the loads of stage st's geometry (threads 0..15 of wave 0): the point's
  // depth / origin / direction (ENC 0) or the Q1 direction ray's rd (ENC 1); put_x(st), one stage
  // later -- after the next barrier's counted vmcnt has seen them land -- forms the point (decode_
  // sample's arithmetic: ro + rd z) or the unit direction and puts it in the table.  Formed in
  // decode itself, the arithmetic made wave 0 wait vmcnt(0) for its loads AND the ring's in-flight
  // pieces every stage, and every other wave then waited at the barrier (r03q ISA).
  float g0 = 0.0f, g1[3] = {0.f, 0.f, 0.f}, g2[3] = {0.f, 0.f, 0.f};
  bool gvalid = false;  // rows past the slab: a zero table row (their A rows are zero too)
  const bool idx32 = M < (int64_t(1) << 31) && a.n_rays < (int64_t(1) << 31);
  auto decode = [&](int st) {
    const int64_t r = (int64_t)st * kEncRows + tid;
    gvalid = tid < kEncRows && r < rows;
    if (gvalid) {
      const int64_t rc = mb + r;
      const int64_t S = a.n_samples;
      const int64_t ray = idx32 ? static_cast<int64_t>(static_cast<unsigned>(rc) / static_cast<unsigned>(S)) : rc / S;
      if constexpr (ENC == 0) {
        if constexpr (MODE == mlp::kFromPts) {
#pragma unroll
          for (int c = 0; c < 3; ++c) g1[c] = a.pts[3 * rc + c];
        } else {
          g0 = a.z[rc];
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            g1[c] = a.ro[3 * ray + c];
            g2[c] = a.rd[3 * ray + c];
          }
        }
      } else {
        // Q1 (nerf/__init__.py:127-128): row k = r S + s of a chunk of rcnt rays takes ray k mod rcnt's
        const int64_t smp = rc - ray * S;
        const int64_t base = (ray / a.chunk_rows) * a.chunk_rows;
        const int64_t rcnt = min(a.chunk_rows, a.n_rays - base);
        const int64_t dray = base + ((ray - base) * S + smp) % rcnt;
#pragma unroll
        for (int c = 0; c < 3; ++c) g2[c] = a.rd[3 * dray + c];
      }
    }
  };
  // The encodings the forward multiplied (ENC 0, fp32): field_w16_kernel evaluates a 16-sample wave's
  // (sin, cos) pairs with fast_sincosf when every sample's max |x| * max |f_xyz| is inside kFastSinBound
  // (and its view direction's too: |vd| <= 1, so that holds whenever max |f_dir| is), else every pair of
  // the wave with ocml's sincosf.  The forward's waves are 16-row groups aligned to 16 rows, and so is
  // every stage here (rows_per_block is a multiple of kEncRows): the stage takes the same choice.  The
  // 3xbf16 forward always calls sincosf (enc_pair), and so does X3 here.  (A wave whose view direction is
  // NaN -- a zero-length ray -- took sincosf in the forward; its outputs are NaN either way.)
  float fast_freq_max = 0.0f, dir_freq_max = 0.0f;   // load_consts' mx / md
#pragma unroll
  for (int k = 0; k < 10; ++k) fast_freq_max = fmaxf(fast_freq_max, fabsf(a.fx[k]));
#pragma unroll
  for (int k = 0; k < 4; ++k) dir_freq_max = fmaxf(dir_freq_max, fabsf(a.fd[k]));
  // |vd_d| <= 1 up to the rounding of the normalisation (a few ulp): the margin keeps this true only
  // where the forward's per-sample test cannot fail (every embedder's max |f_dir| is far below it)
  const bool dir_fast = dir_freq_max * 1.0001f <= mlp::kFastSinBound;
  auto put_x = [&](int st) {
    if (tid < kEncRows) {
      float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!gvalid) {
      } else if constexpr (ENC == 0 && MODE == mlp::kFromPts) {
        v = make_float4(g1[0], g1[1], g1[2], 0.0f);
      } else if constexpr (ENC == 0) {
        v = make_float4(mul_add_rn(g2[0], g0, g1[0]), mul_add_rn(g2[1], g0, g1[1]), mul_add_rn(g2[2], g0, g1[2]), 0.0f);
      } else {  // view_dir's normalisation, the reference's op order
        const float nrm = __fsqrt_rn(__fadd_rn(__fadd_rn(__fmul_rn(g2[0], g2[0]), __fmul_rn(g2[1], g2[1])),
                                               __fmul_rn(g2[2], g2[2])));
        v = make_float4(__fdiv_rn(g2[0], nrm), __fdiv_rn(g2[1], nrm), __fdiv_rn(g2[2], nrm), 0.0f);
      }
      xs[st % 3][tid] = v;
      if constexpr (ENC == 0 && !X3) {
        // the forward's test: max |x_d| * max |f| <= kFastSinBound (false for NaN); rows past the
        // slab are zeros and pass
        const float xa = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fabsf(v.z)) * fast_freq_max;
        const bool ok = xa <= mlp::kFastSinBound;
        const unsigned long long bad = __ballot(!ok);  // lanes 0..15 of wave 0: the stage's rows
        if (tid == 0) xfast[st % 3] = (bad & 0xFFFFull) == 0 && dir_fast;
      }
    }
  };
  auto enc_of = [&](int st) {  // rows past M: their A rows are zero, so any value is harmless
    const float4 x4 = xs[st % 3][es];
    const float x[4] = {x4.x, x4.y, x4.z, 0.0f};
    if (kind == 1) {
      const float arg = __fmul_rn(x[comp], freq);
      if constexpr (X3) {
        sincosf(arg, &ev[0], &ev[1]);                 // the 3xbf16 forward's (enc_pair)
      } else if constexpr (ENC == 0) {
        if (xfast[st % 3]) mlp::fast_sincosf(arg, ev[0], ev[1]);   // the forward's choice for this wave
        else sincosf(arg, &ev[0], &ev[1]);
      } else {
        // view columns: fast inside the bound, per lane -- the forward's whenever its wave's points
        // were inside theirs (every sample of the runnable configs: |x| <= 2^14 / 2^9 = 32)
        mlp::enc_sincosf(arg, ev[0], ev[1]);
      }
    } else if (kind == 2) {
      ev[0] = comp < 3 ? x[comp] : 0.0f;
      ev[1] = comp + 1 < 3 ? x[comp + 1] : 0.0f;
    }
  };
  auto store_enc = [&](int buf) {
    if (kind != 0) {
      senc[buf][es * ES + c0] = ev[0];
      senc[buf][es * ES + c1] = ev[1];
    }
  };
  floatx16 acc[KB];
#pragma unroll
  for (int u = 0; u < KB; ++u) acc[u] = floatx16{0};
  float bsum = 0.0f;  // column sums of A (feature 32 wave + i) over this lane's rows
  decode(0);
  put_x(0);
  decode(1);
  put_x(1);
  decode(2);
  put_x(2);
  dma(0);
  dma(1);
  __syncthreads();
  enc_of(0);
  store_enc(0);
  for (int st = 0; st < n_stages; ++st) {
    // stage st landed for every wave (all but this wave's 2 youngest vector-memory ops -- stage
    // st+1's pieces; the geometry loads of decode(st+2), issued before them, are done too), every
    // wave is past stage st-1 (its ring slot is free, its senc / xs buffers were read)
    static_assert(kEncRows / 8 == 2, "the vmcnt below counts one stage of pieces");
    // (lgkmcnt(0): this wave's table writes of the previous stage are done before the barrier)
    asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (st > 0) put_x(st + 2);
    decode(st + 3);
    dma(st + 2);  // always (past the slab: zeros), so every wave's vmcnt above stays exact
    const bool more = st + 1 < n_stages;
    if (more) enc_of(st + 1);
    const float* sa = ring[st % kEncRing];
    const float* se = senc[st & 1];
    if constexpr (X3) {
      float v[8];
      ring_read8<RS * 4>(sa + (8 * h) * RS + 32 * wave + i, v);   // rows 8 h + j
      bsum += sum8v(v);
      u32x4 ah, al;
      split8(v, ah, al);
#pragma unroll
      for (int u = 0; u < KB; ++u) {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = se[(8 * h + j) * ES + 32 * u + i];
        u32x4 bh, bl;
        split8(v, bh, bl);
        acc[u] = mfma3(acc[u], ah, al, bh, bl);
      }
    } else {
      // the stage's A values and its encoding operands, each read in one round trip before the
      // MFMAs (read per row pair, the B operands exposed an LDS wait before every MFMA pair)
      float xa[8], xb[KB][8];
      ring_read8<2 * RS * 4>(sa + h * RS + 32 * wave + i, xa);          // rows 2 p + h
#pragma unroll
      for (int u = 0; u < KB; ++u) ring_read8<2 * ES * 4>(se + h * ES + 32 * u + i, xb[u]);
#pragma unroll
      for (int p = 0; p < kEncRows / 2; ++p) {
        const float x = xa[p];
        bsum += x;
#pragma unroll
        for (int u = 0; u < KB; ++u) acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, xb[u][p], acc[u], 0, 0, 0);
      }
    }
    if (more) store_enc((st + 1) & 1);
  }
  // the stages prefetched past the slab must land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  float* pt = part ? part + (int64_t)blk * 256 * K : nullptr;
#pragma unroll
  for (int u = 0; u < KB; ++u) flush_block(acc[u], C, ldc, pt, 256, K, 32 * wave, 32 * u, i, h);
  if (bias_part) {
    const float b = bsum + __shfl_xor(bsum, 32);
    if (h == 0) bias_part[(int64_t)blk * 256 + 32 * wave + i] = b;
  }
}

// layer_xyz1's dW from the encodings the fp32 training forward multiplied (its (M, 64) encoding plane,
// cn_radiance_field_train_fmt): C[n][xenc_col(c')] = sum_m A[m][n] X[m][c'], and the bias column
// sums of A.  Both operands move by LDS-DMA into 3-slot rings, two 16-row stages ahead: A's rows
// as 1 KiB dwordx4 pieces, X's 256-B rows as dword pieces (each wave two of each per stage), so the
// loop is one counted vmcnt + barrier, the ring reads and the MFMAs -- no geometry decode and no
// sin / cos per stage (gemm_tn_enc_kernel's VALU, which in this loop adds to the matrix time), and
// the encodings are exactly the forward's (lazy fast_sincosf or ocml sincosf, per wave).
// Wave w: output rows 32 w .. + 31, both 32-column blocks (c' 0..63); fp32 32x32x2.
constexpr int kXRS = 288, kXES = 96;   // LDS row strides (floats): 32 banks between a pair's rows
constexpr int kXencLds = kEncRing * kEncRows * (kXRS + kXES);   // floats of LDS the row pass takes
// Workgroup blk's rows of layer_xyz1's dW from the encoding plane; ring_a / ring_x: its LDS rings
// (kEncRing slots of kEncRows rows, strides kXRS / kXES floats).
__device__ __forceinline__ void xenc_rows(float* ring_a, float* ring_x, const float* __restrict__ A,
                                          const float* __restrict__ X, int64_t M, float* __restrict__ part,
                                          float* __restrict__ bias_part, int64_t rows_per_block, const unsigned blk) {
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int i = lane & 31, h = lane >> 5;
  const int64_t mb = (int64_t)blk * rows_per_block;
  const int64_t rows = min(rows_per_block, M - mb);
  const int n_stages = static_cast<int>((rows + kEncRows - 1) / kEncRows);
  // the slab's rows as buffer resources: rows past it (the tail, the stages prefetched past the end)
  // read as zeros
  const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(A + mb * 256), 0, static_cast<unsigned>(rows * 256 * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t rx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(X + mb * 64), 0, static_cast<unsigned>(rows * 64 * 4), 0x00020000);
  // stage st: wave w moves A rows w, w + 8 and X rows w, w + 8 (4 vector-memory ops per wave)
  auto dma = [&](int st) {
    float* slot = ring_a + (st % kEncRing) * (kEncRows * kXRS);
    float* xslot = ring_x + (st % kEncRing) * (kEncRows * kXES);
#pragma unroll
    for (int j = 0; j < kEncRows / 8; ++j) {
      const int r = wave + 8 * j;
      const unsigned soff = __builtin_amdgcn_readfirstlane(static_cast<unsigned>((st * kEncRows + r) * 1024));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (lds_ptr_t)(slot + r * kXRS), 16, lane * 16u, soff, 0, 0);
      const unsigned xoff = __builtin_amdgcn_readfirstlane(static_cast<unsigned>((st * kEncRows + r) * 256));
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx, (lds_ptr_t)(xslot + r * kXES), 4, lane * 4u, xoff, 0, 0);
    }
  };
  floatx16 acc[2] = {floatx16{0}, floatx16{0}};
  float bsum = 0.0f;  // column sums of A (feature 32 wave + i) over this lane's rows
  dma(0);
  dma(1);
  for (int st = 0; st < n_stages; ++st) {
    // stage st landed for every wave (all but this wave's 4 youngest vector-memory ops -- stage
    // st+1's -- retired), every wave is past stage st-1 (its ring slots are free)
    static_assert(kEncRows / 8 == 2, "the vmcnt below counts one stage of pieces");
    asm volatile("s_waitcnt vmcnt(4) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    dma(st + 2);  // always (past the slab: zeros), so every wave's vmcnt above stays exact
    const float* sa = ring_a + (st % kEncRing) * (kEncRows * kXRS);
    const float* sx = ring_x + (st % kEncRing) * (kEncRows * kXES);
    float xa[8], xb[2][8];
    ring_read8<2 * kXRS * 4>(sa + h * kXRS + 32 * wave + i, xa);   // rows 2 p + h
#pragma unroll
    for (int u = 0; u < 2; ++u) ring_read8<2 * kXES * 4>(sx + h * kXES + 32 * u + i, xb[u]);
#pragma unroll
    for (int p = 0; p < kEncRows / 2; ++p) {
      const float x = xa[p];
      bsum += x;
#pragma unroll
      for (int u = 0; u < 2; ++u) acc[u] = __builtin_amdgcn_mfma_f32_32x32x2f32(x, xb[u][p], acc[u], 0, 0, 0);
    }
  }
  // the stages prefetched past the slab must land before the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // the partial tile in PositionalEmbedder column order (part: (256, 63) per workgroup)
  float* pt = part + (int64_t)blk * 256 * 63;
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int col = mlp::xenc_col(32 * u + i);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * wave + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (col >= 0) pt[(int64_t)row * 63 + col] = acc[u][r];
    }
  }
  if (bias_part) {
    const float b = bsum + __shfl_xor(bsum, 32);
    if (h == 0) bias_part[(int64_t)blk * 256 + 32 * wave + i] = b;
  }
}

__device__ __forceinline__ void xenc_body(const float* __restrict__ A, const float* __restrict__ X, int64_t M,
                                          float* __restrict__ part, float* __restrict__ bias_part,
                                          int64_t rows_per_block, const mlp::FieldArgs& a, const DirRole& dr,
                                          const unsigned bid) {
  if (bid < dr.n) {
    dir_enc_dw_block(a, dr.dir, dr.part, dr.bias_part, bid);
    return;
  }
  __shared__ __attribute__((aligned(16))) float lds[kXencLds];
  xenc_rows(lds, lds + kEncRing * kEncRows * kXRS, A, X, M, part, bias_part, rows_per_block, bid - dr.n);
}

__global__ __launch_bounds__(512, 1) void gemm_tn_xenc_kernel(const float* __restrict__ A, const float* __restrict__ X,
                                                              int64_t M, float* __restrict__ part,
                                                              float* __restrict__ bias_part, int64_t rows_per_block,
                                                              mlp::FieldArgs a, DirRole dr) {
  xenc_body(A, X, M, part, bias_part, rows_per_block, a, dr, blockIdx.x);
}

// One field's layer_xyz1 dW pass (gemm_tn_xenc_kernel's arguments).
struct XencJob {
  const float* A;
  const float* X;
  int64_t M;
  float* part;
  float* bias_part;
  int64_t rows_per_block;
  mlp::FieldArgs a;
  DirRole dr;
};

// A render's two fields' layer_xyz1 dW passes in one launch: workgroups 0 .. first1 - 1 are field j0's
// launch (its DIRS role blocks, then its row blocks), the rest field j1's -- each the same blocks with the
// same rows as its own launch (bitwise the same partials).  Two instances of the body, each reading its
// own kernel argument (no runtime select between the structs).
__global__ __launch_bounds__(512, 1) void gemm_tn_xenc2_kernel(XencJob j0, XencJob j1, unsigned first1) {
  if (blockIdx.x >= first1)
    xenc_body(j1.A, j1.X, j1.M, j1.part, j1.bias_part, j1.rows_per_block, j1.a, j1.dr, blockIdx.x - first1);
  else
    xenc_body(j0.A, j0.X, j0.M, j0.part, j0.bias_part, j0.rows_per_block, j0.a, j0.dr, blockIdx.x);
}

// (the batched dW launch: defined after the roles it runs)
static_assert(kXencLds <= kTwRing * kTwStage, "the XENC role's rings live in the whole-tile ring's LDS");
template <bool X3>
__global__ __launch_bounds__(512, 2) void gemm_tn256_jobs_kernel(TnJobs jobs) {
  __shared__ __attribute__((aligned(16))) float ring[kTwRing * kTwStage];
  int k = jobs.n - 1;
  while (k > 0 && static_cast<int>(blockIdx.x) < jobs.j[k].first_block) --k;
  const TnJob& j = jobs.j[k];
  const unsigned blk = blockIdx.x - static_cast<unsigned>(j.first_block), nblk = static_cast<unsigned>(j.n_blocks);
  if (j.kind == 1) {
    tn256_body<X3, true, false>(ring, j.A, j.B, nullptr, 0, j.part, j.bias_part, j.draw, j.sig_part, j.M,
                                j.rows_per_block, j.dir, blk, nblk);
  } else if (!X3 && j.kind == 2) {
    tn256_body<false, false, true>(ring, j.A, j.B, nullptr, 0, j.part, j.bias_part, nullptr, nullptr, j.M,
                                   j.rows_per_block, j.dir, blk, nblk);
  } else if (!X3 && j.kind == 3) {
    rgb_body(ring, j.draw, j.B, j.part, j.bias_part, j.M, j.rows_per_block, blk, nblk);
  } else if (!X3 && j.kind == 4) {
    xenc_rows(ring, ring + kEncRing * kEncRows * kXRS, j.A, j.B, j.M, j.part, j.bias_part, j.rows_per_block, blk);
  } else {
    tn256_body<X3, false, false>(ring, j.A, j.B, nullptr, 0, j.part, j.bias_part, nullptr, nullptr, j.M,
                                 j.rows_per_block, j.dir, blk, nblk);
  }
}

__global__ __launch_bounds__(256) void dir_enc_dw_kernel(mlp::FieldArgs a, DirFold dir, float* __restrict__ part,
                                                         float* __restrict__ bias_part) {
  dir_enc_dw_block(a, dir, part, bias_part, blockIdx.x);
}

// Deterministic column sums (bias gradients dPre^T 1) where no dW kernel folds them in:
// part[b][n] = sum of A[m][n] over block b's rows, in row order.
__global__ __launch_bounds__(256) void colsum_kernel(const float* __restrict__ A, int64_t lda, int64_t M, int N,
                                                     float* __restrict__ part, int64_t rows_per_block) {
  const int j = threadIdx.x;
  if (j >= N) return;
  const int64_t mb = (int64_t)blockIdx.x * rows_per_block, me = min(M, mb + rows_per_block);
  float s = 0.0f;
  for (int64_t m = mb; m < me; ++m) s += A[m * lda + j];
  part[(int64_t)blockIdx.x * N + j] = s;
}

// out[code(m)][j] += A[m][j] for j < N; code(m) = code_index ? code_index[m / S]
// : (n_codes == 1 ? 0 : m / S).  Block = 4 waves over kSegRows consecutive rows
// and 64 columns: lane j of a wave owns column c0 + j (each row read is one
// coalesced 256-B segment), walks its quarter of the rows and flushes when the
// code changes (rows of one ray are contiguous, so the code is wave-uniform).
// Runs of one code are reduced across the 4 waves in LDS first, so the common
// single-code case costs one atomic per column per block.
constexpr int kSegRows = 1024;

__device__ __forceinline__ int64_t seg_code(int64_t m, int64_t S, const int64_t* code_index, int64_t n_codes) {
  const int64_t ray = m / S;
  return code_index ? code_index[ray] : (n_codes == 1 ? 0 : ray);
}

__global__ __launch_bounds__(256) void seg_sum_kernel(const float* __restrict__ A, int64_t lda, int64_t M,
                                                      int N, int64_t S, const int64_t* __restrict__ code_index,
                                                      int64_t n_codes, float* __restrict__ out,
                                                      int64_t out_ld) {
  __shared__ float part[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int c = blockIdx.y * 64 + lane;
  const int64_t mb = (int64_t)blockIdx.x * kSegRows, me = min(M, mb + kSegRows);
  // one code over the whole block: fast path with a cross-wave LDS reduction
  const int64_t code0 = seg_code(mb, S, code_index, n_codes);
  int diff = 0;
  if (code_index) {
    for (int64_t r = mb / S + threadIdx.x; r <= (me - 1) / S; r += blockDim.x) diff |= code_index[r] != code0;
  } else {
    diff = n_codes != 1 && (mb / S) != ((me - 1) / S);
  }
  const bool one = !__syncthreads_or(diff);
  constexpr int kQ = kSegRows / 4;
  const int64_t qb = mb + (int64_t)wave * kQ, qe = min(me, qb + kQ);
  if (one) {
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (c < N) {
      int64_t m = qb;
      for (; m + 4 <= qe; m += 4) {
        s0 += A[m * lda + c];
        s1 += A[(m + 1) * lda + c];
        s2 += A[(m + 2) * lda + c];
        s3 += A[(m + 3) * lda + c];
      }
      for (; m < qe; ++m) s0 += A[m * lda + c];
    }
    part[wave][lane] = (s0 + s1) + (s2 + s3);
    __syncthreads();
    if (wave == 0 && c < N) {
      const float t = (part[0][lane] + part[1][lane]) + (part[2][lane] + part[3][lane]);
      atomicAdd(&out[code0 * out_ld + c], t);
    }
    return;
  }
  if (c >= N || qb >= qe) return;
  float sum = 0.0f;
  int64_t cur = seg_code(qb, S, code_index, n_codes);
  for (int64_t m = qb; m < qe; ++m) {
    const int64_t code = seg_code(m, S, code_index, n_codes);
    if (code != cur) {
      atomicAdd(&out[cur * out_ld + c], sum);
      cur = code;
      sum = 0.0f;
    }
    sum += A[m * lda + c];
  }
  atomicAdd(&out[cur * out_ld + c], sum);
}

// ---------------------------------------------------------------- element-wise pieces

// PositionalEmbedder.embed backward: d x[m][d] from d enc[m][(inc + 2k + {0,1}) * D + d].
struct Freqs {
  float f[32];
};

__host__ inline Freqs make_freqs(const float* host, int n) {
  Freqs r = {};
  for (int i = 0; i < n; ++i) r.f[i] = host[i];
  return r;
}

__global__ void posenc_backward_kernel(const float* __restrict__ x, int64_t ldx, const float* __restrict__ denc,
                                       int64_t ldenc, int64_t M, int D, Freqs fr, int nf, int inc,
                                       float* __restrict__ dx, int64_t lddx) {
  const int64_t n = M * D;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = q / D;
    const int d = static_cast<int>(q - m * D);
    const float v = x[m * ldx + d];
    const float* g = denc + m * ldenc;
    float acc = inc ? g[d] : 0.0f;
    for (int k = 0; k < nf; ++k) {
      const float f_k = fr.f[k];
      float sn, cs;
      sincosf(__fmul_rn(v, f_k), &sn, &cs);
      acc += f_k * (g[(inc + 2 * k) * D + d] * cs - g[(inc + 2 * k + 1) * D + d] * sn);
    }
    dx[m * lddx + d] = acc;
  }
}

// forward_pass's view directions (nerf/__init__.py:125-128): vd = rd[dray] / |rd[dray]| with the Q1
// ray map; d rd[dray] += (g - vd (vd . g)) / |rd[dray]|.
__global__ void viewdir_backward_kernel(const float* __restrict__ rd, const float* __restrict__ dvd, int64_t lddvd,
                                        int64_t n_rays, int64_t S, int64_t chunk_rows, float* __restrict__ d_rd) {
  const int64_t M = n_rays * S;
  for (int64_t m = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; m < M; m += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ray = m / S, smp = m - ray * S;
    const int64_t base = (ray / chunk_rows) * chunk_rows;
    const int64_t rcnt = min(chunk_rows, n_rays - base);
    const int64_t dray = base + ((ray - base) * S + smp) % rcnt;
    const float d0 = rd[3 * dray], d1 = rd[3 * dray + 1], d2 = rd[3 * dray + 2];
    const float nrm = sqrtf(d0 * d0 + d1 * d1 + d2 * d2);
    const float v0 = d0 / nrm, v1 = d1 / nrm, v2 = d2 / nrm;
    const float g0 = dvd[m * lddvd], g1 = dvd[m * lddvd + 1], g2 = dvd[m * lddvd + 2];
    const float dot = v0 * g0 + v1 * g1 + v2 * g2;
    atomicAdd(&d_rd[3 * dray], (g0 - v0 * dot) / nrm);
    atomicAdd(&d_rd[3 * dray + 1], (g1 - v1 * dot) / nrm);
    atomicAdd(&d_rd[3 * dray + 2], (g2 - v2 * dot) / nrm);
  }
}

// pts = ro + rd * z (point_sampler.py:70, :118): d ro[r] += sum_s d pts, d rd[r] += sum_s d pts * z.
__global__ void ray_points_backward_kernel(const float* __restrict__ dpts, int64_t ldp, const float* __restrict__ z,
                                           int64_t n_rays, int64_t S, float* __restrict__ d_ro,
                                           float* __restrict__ d_rd) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < n_rays; r += (int64_t)gridDim.x * blockDim.x) {
    float o0 = 0.f, o1 = 0.f, o2 = 0.f, e0 = 0.f, e1 = 0.f, e2 = 0.f;
    for (int64_t s = 0; s < S; ++s) {
      const int64_t m = r * S + s;
      const float zz = z[m];
      const float g0 = dpts[m * ldp], g1 = dpts[m * ldp + 1], g2 = dpts[m * ldp + 2];
      o0 += g0; o1 += g1; o2 += g2;
      e0 += g0 * zz; e1 += g1 * zz; e2 += g2 * zz;
    }
    if (d_ro) {
      d_ro[3 * r] += o0; d_ro[3 * r + 1] += o1; d_ro[3 * r + 2] += o2;
    }
    if (d_rd) {
      d_rd[3 * r] += e0; d_rd[3 * r + 1] += e1; d_rd[3 * r + 2] += e2;
    }
  }
}

// Q1 view-direction + point encoding of forward_pass, row-major (M, 90) = [xyz 63 | dir 27]
// (the input the reference hands CodeNeRFModel.forward, nerf/__init__.py:116-132).
__global__ void encode_inputs_kernel(mlp::FieldArgs a, float* __restrict__ out) {
  const int64_t M = a.m;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < M * 90; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = q / 90;
    const int c = static_cast<int>(q - m * 90);
    const mlp::SampleIn in = a.pts ? mlp::decode_sample<mlp::kFromPts>(a, m) : mlp::decode_sample<mlp::kFromRayZ>(a, m);
    const bool dir = c >= 63;
    const int cc = dir ? c - 63 : c;
    const float* v = dir ? in.vd : in.x;
    float o;
    if (cc < 3) {
      o = v[cc];
    } else {
      const int b = (cc - 3) / 3, comp = (cc - 3) % 3;
      const float arg = __fmul_rn(v[comp], dir ? a.fd[b >> 1] : a.fx[b >> 1]);
      o = (b & 1) ? cosf(arg) : sinf(arg);
    }
    out[q] = o;
  }
}

// dst[m][0:ncols] = src[m][0:ncols] (strided), e.g. d raw[:, 3] -> fc_out's sigma row.
__global__ void copy_cols_kernel(const float* __restrict__ src, int64_t lds_, float* __restrict__ dst, int64_t ldd,
                                 int64_t M, int ncols) {
  const int64_t n = M * ncols;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = q / ncols;
    const int c = static_cast<int>(q - m * ncols);
    dst[m * ldd + c] = src[m * lds_ + c];
  }
}

// ---------------------------------------------------------------- code layers (model.py:174-177)
// Per code row: recompute zs1 / zs2 / zt1, pull the summed code-term gradients g
// (520-wide, cn_code_bias layout) back through the code halves of layer_xyz2 /
// fc_out / fc_rgb and the three code layers.  dW / db accumulate with atomics.  Rows
// whose g is all zero (codes no sample used) only write their zero code gradient.
constexpr int kCodeRowSplits = 16;
constexpr int kCodeThreads = 1024;  // 16 waves: every reduction below is split 4 ways

__global__ __launch_bounds__(kCodeThreads) void code_backward_kernel(mlp::Params P, const float* __restrict__ z_s,
                                                                     const float* __restrict__ z_t,
                                                                     const float* __restrict__ g,
                                                                     float* __restrict__ dz_s, float* __restrict__ dz_t,
                                                                     mlp::Params G) {
  using namespace mlp;
  __shared__ float zs[256], zt[256], s1[256], s2[256], t1[256], ds1[256], ds2[256], dt1[256], go[257];
  __shared__ float gx2[256], grgb[3];
  __shared__ float red[3][4][256];
  const int c = blockIdx.x, tid = threadIdx.x, j = tid & 255, q = tid >> 8;
  const float* gr = g + (int64_t)c * kCbStride;
  // a code no sample used this step (most rows of a training table) has g = 0: zero code
  // gradients, no parameter contribution
  const bool nz = q == 0 && (gr[kCbXyz2 + j] != 0.0f || gr[kCbFeat + j] != 0.0f || (j < 8 && gr[kCbSigma + j] != 0.0f));
  const bool lead = blockIdx.y == 0;  // writes dz and the bias / single-row terms
  if (!__syncthreads_or(nz)) {
    if (q == 0 && lead && dz_s) dz_s[(int64_t)c * 256 + j] = 0.0f;
    if (q == 0 && lead && dz_t) dz_t[(int64_t)c * 256 + j] = 0.0f;
    return;
  }
  if (q == 0) {
    zs[j] = z_s[(int64_t)c * 256 + j];
    zt[j] = z_t[(int64_t)c * 256 + j];
    go[1 + j] = gr[kCbFeat + j];
    gx2[j] = gr[kCbXyz2 + j];
    if (j == 0) go[0] = gr[kCbSigma];
    if (j < 3) grgb[j] = gr[kCbRgb + j];
  }
  __syncthreads();
  {
    // the three code layers (model.py:174-177) recomputed: wave w owns outputs 16 w .. 16 w + 15,
    // one row at a time with its 64 lanes over k (coalesced 1 KiB rows) and a butterfly sum
    const int lane = tid & 63, w = tid >> 6;
    // four rows at a time: their 48 loads are in flight together (a row at a time was 16 serial
    // memory latencies per wave); each row's sums in the same order as before
    for (int ob = 16 * w; ob < 16 * w + 16; ob += 4) {
      float a1[4], a2[4], a3[4];
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int o = ob + x;
        a1[x] = a2[x] = a3[x] = 0.f;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int k = lane + 64 * u;
          a1[x] = fmaf(P.p[kWSc1][o * 256 + k], zs[k], a1[x]);
          a2[x] = fmaf(P.p[kWSc2][o * 256 + k], zs[k], a2[x]);
          a3[x] = fmaf(P.p[kWTc1][o * 256 + k], zt[k], a3[x]);
        }
      }
#pragma unroll
      for (int x = 0; x < 4; ++x) {
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
          a1[x] += __shfl_xor(a1[x], off);
          a2[x] += __shfl_xor(a2[x], off);
          a3[x] += __shfl_xor(a3[x], off);
        }
        if (lane == 0) {
          const int o = ob + x;
          s1[o] = fmaxf(a1[x] + P.p[kBSc1][o], 0.f);
          s2[o] = fmaxf(a2[x] + P.p[kBSc2][o], 0.f);
          t1[o] = fmaxf(a3[x] + P.p[kBTc1][o], 0.f);
        }
      }
    }
  }
  // d zs1 = W_xyz2[:, 256:]^T g_x2, d zs2 = W_out[:, 256:]^T g_o, d zt1 = W_rgb[:, 256:]^T g_rgb:
  // quarter q of the n range per thread, the quarters summed in order
  {
    float a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll 16
    for (int n = 64 * q; n < 64 * q + 64; ++n) {
      a1 = fmaf(P.p[kWXyz2][n * 512 + 256 + j], gx2[n], a1);
      a2 = fmaf(P.p[kWOut][n * 512 + 256 + j], go[n], a2);
    }
    if (q == 3) a2 = fmaf(P.p[kWOut][256 * 512 + 256 + j], go[256], a2);
    if (q == 0)
      for (int n = 0; n < 3; ++n) a3 = fmaf(P.p[kWRgb][n * 512 + 256 + j], grgb[n], a3);
    red[0][q][j] = a1;
    red[1][q][j] = a2;
    red[2][q][j] = a3;
  }
  __syncthreads();
  if (q == 0) {
    const float a1 = (red[0][0][j] + red[0][1][j]) + (red[0][2][j] + red[0][3][j]);
    const float a2 = (red[1][0][j] + red[1][1][j]) + (red[1][2][j] + red[1][3][j]);
    ds1[j] = s1[j] > 0.f ? a1 : 0.f;
    ds2[j] = s2[j] > 0.f ? a2 : 0.f;
    dt1[j] = t1[j] > 0.f ? red[2][0][j] : 0.f;
  }
  __syncthreads();
  if (lead && (dz_s || dz_t)) {
    float a = 0.f, b = 0.f;
#pragma unroll 16
    for (int n = 64 * q; n < 64 * q + 64; ++n) {
      a = fmaf(P.p[kWSc1][n * 256 + j], ds1[n], a);
      a = fmaf(P.p[kWSc2][n * 256 + j], ds2[n], a);
      b = fmaf(P.p[kWTc1][n * 256 + j], dt1[n], b);
    }
    red[0][q][j] = a;
    red[1][q][j] = b;
  }
  __syncthreads();
  if (lead && q == 0) {
    if (dz_s) dz_s[(int64_t)c * 256 + j] = (red[0][0][j] + red[0][1][j]) + (red[0][2][j] + red[0][3][j]);
    if (dz_t) dz_t[(int64_t)c * 256 + j] = (red[1][0][j] + red[1][1][j]) + (red[1][2][j] + red[1][3][j]);
  }
  if (!G.p[kWSc1]) return;
  // weight gradients of the code layers and the code halves: outer products over this block's
  // rows (blockIdx.y of kCodeRowSplits; the per-code vectors above are recomputed by each, so the
  // atomics spread over the chip), thread (q, j) on rows r0 + q + 4 t, column j
  const float zsj = zs[j], ztj = zt[j], s1j = s1[j], s2j = s2[j], t1j = t1[j];
  const int r0 = blockIdx.y * (256 / kCodeRowSplits);
  for (int r = r0 + q; r < r0 + 256 / kCodeRowSplits; r += 4) {
    atomicAdd(&const_cast<float*>(G.p[kWSc1])[r * 256 + j], ds1[r] * zsj);
    atomicAdd(&const_cast<float*>(G.p[kWSc2])[r * 256 + j], ds2[r] * zsj);
    atomicAdd(&const_cast<float*>(G.p[kWTc1])[r * 256 + j], dt1[r] * ztj);
    atomicAdd(&const_cast<float*>(G.p[kWXyz2])[r * 512 + 256 + j], gx2[r] * s1j);
    atomicAdd(&const_cast<float*>(G.p[kWOut])[(1 + r) * 512 + 256 + j], go[1 + r] * s2j);
  }
  if (!lead || q != 0) return;
  atomicAdd(&const_cast<float*>(G.p[kBSc1])[j], ds1[j]);
  atomicAdd(&const_cast<float*>(G.p[kBSc2])[j], ds2[j]);
  atomicAdd(&const_cast<float*>(G.p[kBTc1])[j], dt1[j]);
  atomicAdd(&const_cast<float*>(G.p[kWOut])[256 + j], go[0] * s2j);                // fc_out row 0 (sigma)
  for (int r = 0; r < 3; ++r) atomicAdd(&const_cast<float*>(G.p[kWRgb])[r * 512 + 256 + j], grgb[r] * t1j);
}

// The same backward in two launches (cn_code_bias_backward_ws).  code_backward_kernel recomputes
// the three code layers and the three 256-long reductions in each of its 16 workgroups per code
// (about 2 MiB of L2 reads per workgroup: ~55 us for one code).  Here workgroup y of
// code_layers_dz_kernel forms outputs R y .. R y + R - 1 (R = kCodeRows) of s1 / s2 / t1 and of
// ds1 / ds2 / dt1 into the workspace (per code: s1 s2 t1 ds1 ds2 dt1, 6 x 256 floats), and workgroup
// y of code_outer_kernel forms dz_s / dz_t for columns R y .. and the outer products of rows R y ..
// Every sum keeps code_backward_kernel's order: bitwise the same results.  64 workgroups per code
// (4 rows each): the per-workgroup chains are latency-bound, so more and shorter ones.
constexpr int kCodeSlices = 64;                  // workgroups per code
constexpr int kCodeRows = 256 / kCodeSlices;     // outputs / outer-product rows per workgroup
static_assert(256 % kCodeSlices == 0 && kCodeRows <= 16, "phase-2 thread map: 16 columns per (quarter, vector)");

// Whether any sample used code row gr (all its code-term gradients zero otherwise), as
// code_backward_kernel tests it; every thread of the block gets the answer.
__device__ __forceinline__ bool code_row_used(const float* __restrict__ gr, int tid) {
  using namespace mlp;
  const bool nz = tid < 256 && (gr[kCbXyz2 + tid] != 0.0f || gr[kCbFeat + tid] != 0.0f ||
                                (tid < 8 && gr[kCbSigma + tid] != 0.0f));
  return __syncthreads_or(nz);
}

__global__ __launch_bounds__(256) void code_layers_dz_kernel(mlp::Params P, const float* __restrict__ z_s,
                                                             const float* __restrict__ z_t,
                                                             const float* __restrict__ g, float* __restrict__ ws) {
  using namespace mlp;
  constexpr int kPerWave = (kCodeRows + 3) / 4;  // outputs per wave (waves past kCodeRows idle)
  __shared__ float zs[256], zt[256], gx2[256], go[257], grgb[3], sv[3][kCodeRows];
  __shared__ float red[3][4][16];
  const int c = blockIdx.x, y = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const float* gr = g + (int64_t)c * kCbStride;
  if (!code_row_used(gr, tid)) return;  // code_outer_kernel writes its zero dz
  zs[tid] = z_s[(int64_t)c * 256 + tid];
  zt[tid] = z_t[(int64_t)c * 256 + tid];
  gx2[tid] = gr[kCbXyz2 + tid];
  go[1 + tid] = gr[kCbFeat + tid];
  if (tid == 0) go[0] = gr[kCbSigma];
  if (tid < 3) grgb[tid] = gr[kCbRgb + tid];
  __syncthreads();
  float* wc = ws + (int64_t)c * 6 * 256;
  {
    // outputs o = R y + kPerWave w + x: lanes over k (k = lane + 64 u), butterfly sum
    float a1[kPerWave], a2[kPerWave], a3[kPerWave];
#pragma unroll
    for (int x = 0; x < kPerWave; ++x) {
      const int i = kPerWave * w + x, o = kCodeRows * y + (i < kCodeRows ? i : 0);
      a1[x] = a2[x] = a3[x] = 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int k = lane + 64 * u;
        a1[x] = fmaf(P.p[kWSc1][o * 256 + k], zs[k], a1[x]);
        a2[x] = fmaf(P.p[kWSc2][o * 256 + k], zs[k], a2[x]);
        a3[x] = fmaf(P.p[kWTc1][o * 256 + k], zt[k], a3[x]);
      }
    }
#pragma unroll
    for (int x = 0; x < kPerWave; ++x) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        a1[x] += __shfl_xor(a1[x], off);
        a2[x] += __shfl_xor(a2[x], off);
        a3[x] += __shfl_xor(a3[x], off);
      }
      const int i = kPerWave * w + x;
      if (lane == 0 && i < kCodeRows) {
        const int o = kCodeRows * y + i;
        sv[0][i] = fmaxf(a1[x] + P.p[kBSc1][o], 0.f);
        sv[1][i] = fmaxf(a2[x] + P.p[kBSc2][o], 0.f);
        sv[2][i] = fmaxf(a3[x] + P.p[kBTc1][o], 0.f);
      }
    }
  }
  // ds1 / ds2 / dt1 for j = R y + jj: thread (quarter q, vector v, jj), the quarter's 64 n in order
  {
    const int q = tid >> 6, v = (tid >> 4) & 3, jj = tid & 15, j = kCodeRows * y + jj;
    float a = 0.f;
    if (jj < kCodeRows) {
      if (v == 0) {
#pragma unroll 16
        for (int n = 64 * q; n < 64 * q + 64; ++n) a = fmaf(P.p[kWXyz2][n * 512 + 256 + j], gx2[n], a);
      } else if (v == 1) {
#pragma unroll 16
        for (int n = 64 * q; n < 64 * q + 64; ++n) a = fmaf(P.p[kWOut][n * 512 + 256 + j], go[n], a);
        if (q == 3) a = fmaf(P.p[kWOut][256 * 512 + 256 + j], go[256], a);
      } else if (v == 2 && q == 0) {
        for (int n = 0; n < 3; ++n) a = fmaf(P.p[kWRgb][n * 512 + 256 + j], grgb[n], a);
      }
      if (v < 3) red[v][q][jj] = a;
    }
  }
  __syncthreads();
  if (tid < 48 && (tid & 15) < kCodeRows) {
    const int v = tid >> 4, jj = tid & 15, j = kCodeRows * y + jj;
    const float sum = v == 2 ? red[2][0][jj] : (red[v][0][jj] + red[v][1][jj]) + (red[v][2][jj] + red[v][3][jj]);
    wc[v * 256 + j] = sv[v][jj];
    wc[(3 + v) * 256 + j] = sv[v][jj] > 0.f ? sum : 0.f;
  }
}

// G[i] += v (returnless float atomic: one code -> one writer per element, the plain sum's bits)
__device__ __forceinline__ void grad_add(const float* p, int64_t i, float v) {
  atomicAdd(const_cast<float*>(p) + i, v);
}

// accumulate: dz_s / dz_t += the code gradients (the shape / texture tables' gradient rows), else =.
__global__ __launch_bounds__(256) void code_outer_kernel(mlp::Params P, const float* __restrict__ z_s,
                                                         const float* __restrict__ z_t, const float* __restrict__ g,
                                                         const float* __restrict__ ws, float* __restrict__ dz_s,
                                                         float* __restrict__ dz_t, mlp::Params G, int accumulate) {
  using namespace mlp;
  __shared__ float s1[256], s2[256], t1[256], ds1[256], ds2[256], dt1[256], go[257], gx2[256], grgb[3];
  __shared__ float red[2][4][16];
  const int c = blockIdx.x, y = blockIdx.y, tid = threadIdx.x;
  const int r0 = kCodeRows * y;
  const float* gr = g + (int64_t)c * kCbStride;
  if (!code_row_used(gr, tid)) {
    if (!accumulate && tid < kCodeRows && dz_s) dz_s[(int64_t)c * 256 + r0 + tid] = 0.0f;
    if (!accumulate && tid < kCodeRows && dz_t) dz_t[(int64_t)c * 256 + r0 + tid] = 0.0f;
    return;
  }
  const float* wc = ws + (int64_t)c * 6 * 256;
  s1[tid] = wc[tid];
  s2[tid] = wc[256 + tid];
  t1[tid] = wc[512 + tid];
  ds1[tid] = wc[768 + tid];
  ds2[tid] = wc[1024 + tid];
  dt1[tid] = wc[1280 + tid];
  gx2[tid] = gr[kCbXyz2 + tid];
  go[1 + tid] = gr[kCbFeat + tid];
  if (tid == 0) go[0] = gr[kCbSigma];
  if (tid < 3) grgb[tid] = gr[kCbRgb + tid];
  __syncthreads();
  if (dz_s || dz_t) {
    // columns j = R y + jj: thread (quarter q, vector v, jj), code_backward_kernel's chains
    const int q = tid >> 6, v = (tid >> 4) & 3, jj = tid & 15, j = r0 + jj;
    float a = 0.f;
    if (jj < kCodeRows) {
      if (v == 0) {
#pragma unroll 16
        for (int n = 64 * q; n < 64 * q + 64; ++n) {
          a = fmaf(P.p[kWSc1][n * 256 + j], ds1[n], a);
          a = fmaf(P.p[kWSc2][n * 256 + j], ds2[n], a);
        }
      } else if (v == 1) {
#pragma unroll 16
        for (int n = 64 * q; n < 64 * q + 64; ++n) a = fmaf(P.p[kWTc1][n * 256 + j], dt1[n], a);
      }
      if (v < 2) red[v][q][jj] = a;
    }
    __syncthreads();
    if (tid < 32 && (tid & 15) < kCodeRows) {
      const int vv = tid >> 4, k = tid & 15;
      const float sum = (red[vv][0][k] + red[vv][1][k]) + (red[vv][2][k] + red[vv][3][k]);
      float* dz = vv == 0 ? dz_s : dz_t;
      if (dz) {
        float* d = dz + (int64_t)c * 256 + r0 + k;
        *d = accumulate ? *d + sum : sum;
      }
    }
  }
  if (!G.p[kWSc1]) return;
  // rows r0 .. r0 + R - 1 of the outer products, column j = tid; the bias / single-row terms of
  // columns r0 ..
  const int j = tid;
  const float zsj = z_s[(int64_t)c * 256 + j], ztj = z_t[(int64_t)c * 256 + j];
  const float s1j = s1[j], s2j = s2[j];
#pragma unroll
  for (int r = r0; r < r0 + kCodeRows; ++r) {
    grad_add(G.p[kWSc1], r * 256 + j, ds1[r] * zsj);
    grad_add(G.p[kWSc2], r * 256 + j, ds2[r] * zsj);
    grad_add(G.p[kWTc1], r * 256 + j, dt1[r] * ztj);
    grad_add(G.p[kWXyz2], r * 512 + 256 + j, gx2[r] * s1j);
    grad_add(G.p[kWOut], (1 + r) * 512 + 256 + j, go[1 + r] * s2j);
  }
  if (tid < kCodeRows) {
    const int jb = r0 + tid;
    grad_add(G.p[kBSc1], jb, ds1[jb]);
    grad_add(G.p[kBSc2], jb, ds2[jb]);
    grad_add(G.p[kBTc1], jb, dt1[jb]);
    grad_add(G.p[kWOut], 256 + jb, go[0] * s2[jb]);  // fc_out row 0 (sigma)
    for (int r = 0; r < 3; ++r) grad_add(G.p[kWRgb], r * 512 + 256 + jb, grgb[r] * t1[jb]);
  }
}

// The code backward on the forward's own code-layer activations (act: s1 | s2 | t1 per code, written by
// the preparation launch, cn_field_prepare_models), in two kernels whose second may serve both fields of
// a render at once:
//   code_ds_outer_kernel: workgroup y forms ds1 / ds2 / dt1 for rows R y .. (masked by act > 0) into the
//     workspace and the outer products / bias terms of those rows -- no code layer is recomputed;
//   code_dz_kernel: dz_s / dz_t for columns R y .. from every row's ds, for one or two (model, g_code,
//     workspace) jobs added in job order.
// Each 256-long dot is split over the 16 lanes of a DPP row (16 n each, all loads in flight) and summed
// by a 16-lane butterfly: one memory round trip per chain instead of four.

// Sum over the 16 lanes of this lane's row group (every lane of the group gets it); fixed order.
__device__ __forceinline__ float sum16_bfly(float x) {
#pragma unroll
  for (int off = 8; off > 0; off >>= 1) x += __shfl_xor(x, off, 16);
  return x;
}

__device__ __forceinline__ void code_ds_outer_body(const mlp::Params& P, const float* __restrict__ z_s,
                                                   const float* __restrict__ z_t, const float* __restrict__ g,
                                                   const float* __restrict__ act, float* __restrict__ ws,
                                                   const mlp::Params& G, const int c, const int y) {
  using namespace mlp;
  static_assert(kCodeRows == 4, "thread map: 8 row groups of 16 lanes = 2 vectors x 4 rows");
  __shared__ float gx2[256], go[257], grgb[3], ds[3][kCodeRows];
  const int tid = threadIdx.x;
  const int r0 = kCodeRows * y;
  const float* gr = g + (int64_t)c * kCbStride;
  if (!code_row_used(gr, tid)) return;  // code_dz_kernel skips the code too
  gx2[tid] = gr[kCbXyz2 + tid];
  go[1 + tid] = gr[kCbFeat + tid];
  if (tid == 0) go[0] = gr[kCbSigma];
  if (tid < 3) grgb[tid] = gr[kCbRgb + tid];
  __syncthreads();
  const float* a = act + (int64_t)c * 3 * 256;
  if (tid < 128) {
    // group o = tid / 16: vector v = o / 4 (0: layer_xyz2's code half . gx2, 1: fc_out's . go), row i = o % 4;
    // lane p of the group: n = 16 p .. 16 p + 15 (fc_out's row 256 term last, in lane 15)
    const int o = tid >> 4, v = o >> 2, i = o & 3, pl = tid & 15, j = r0 + i;
    const float* W = P.p[v == 0 ? kWXyz2 : kWOut] + 256 + j;
    const float* gv = v == 0 ? gx2 : go;
    float wv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) wv[u] = W[(16 * pl + u) * 512];
    float acc = 0.f;
#pragma unroll
    for (int u = 0; u < 16; ++u) acc = fmaf(wv[u], gv[16 * pl + u], acc);
    if (v == 1 && pl == 15) acc = fmaf(P.p[kWOut][256 * 512 + 256 + j], go[256], acc);
    const float sum = sum16_bfly(acc);
    if (pl == 0) {
      const float d = a[v * 256 + j] > 0.f ? sum : 0.f;
      ds[v][i] = d;
      ws[(int64_t)c * 6 * 256 + (3 + v) * 256 + j] = d;
    }
  } else if (tid < 128 + kCodeRows) {
    const int i = tid - 128, j = r0 + i;
    float acc = 0.f;
    for (int n = 0; n < 3; ++n) acc = fmaf(P.p[kWRgb][n * 512 + 256 + j], grgb[n], acc);
    const float d = a[512 + j] > 0.f ? acc : 0.f;
    ds[2][i] = d;
    ws[(int64_t)c * 6 * 256 + 5 * 256 + j] = d;
  }
  __syncthreads();
  if (!G.p[kWSc1]) return;
  const int j = tid;
  const float zsj = z_s[(int64_t)c * 256 + j], ztj = z_t[(int64_t)c * 256 + j];
  const float s1j = a[j], s2j = a[256 + j];
#pragma unroll
  for (int i = 0; i < kCodeRows; ++i) {
    const int r = r0 + i;
    grad_add(G.p[kWSc1], r * 256 + j, ds[0][i] * zsj);
    grad_add(G.p[kWSc2], r * 256 + j, ds[1][i] * zsj);
    grad_add(G.p[kWTc1], r * 256 + j, ds[2][i] * ztj);
    grad_add(G.p[kWXyz2], r * 512 + 256 + j, gx2[r] * s1j);
    grad_add(G.p[kWOut], (1 + r) * 512 + 256 + j, go[1 + r] * s2j);
  }
  if (tid < kCodeRows) {
    const int jb = r0 + tid;
    grad_add(G.p[kBSc1], jb, ds[0][tid]);
    grad_add(G.p[kBSc2], jb, ds[1][tid]);
    grad_add(G.p[kBTc1], jb, ds[2][tid]);
    grad_add(G.p[kWOut], 256 + jb, go[0] * a[256 + jb]);  // fc_out row 0 (sigma)
    for (int r = 0; r < 3; ++r) grad_add(G.p[kWRgb], r * 512 + 256 + jb, grgb[r] * a[512 + jb]);
  }
}

__global__ __launch_bounds__(256) void code_ds_outer_kernel(mlp::Params P, const float* __restrict__ z_s,
                                                            const float* __restrict__ z_t, const float* __restrict__ g,
                                                            const float* __restrict__ act, float* __restrict__ ws,
                                                            mlp::Params G) {
  code_ds_outer_body(P, z_s, z_t, g, act, ws, G, blockIdx.x, blockIdx.y);
}

// One field's part of code_ds_outer2_kernel (cn_code_bias_backward_act's arguments).
struct CodeDsJob {
  mlp::Params P, G;
  const float* g;
  const float* act;
  float* ws;
};

// A render's two fields' code backward first halves in one launch (slices y < kCodeSlices: field j0's);
// each field writes only its own gradients and workspace, as its own launch would.
__global__ __launch_bounds__(256) void code_ds_outer2_kernel(CodeDsJob j0, CodeDsJob j1, const float* __restrict__ z_s,
                                                             const float* __restrict__ z_t) {
  if (static_cast<int>(blockIdx.y) >= kCodeSlices)
    code_ds_outer_body(j1.P, z_s, z_t, j1.g, j1.act, j1.ws, j1.G, blockIdx.x, blockIdx.y - kCodeSlices);
  else
    code_ds_outer_body(j0.P, z_s, z_t, j0.g, j0.act, j0.ws, j0.G, blockIdx.x, blockIdx.y);
}

struct DzJob {
  mlp::Params P;
  const float* g;
  const float* ws;
};
constexpr int kMaxDzJobs = 2;
struct DzJobs {
  DzJob j[kMaxDzJobs];
  int n;
};

// accumulate: dz += each job's code gradient (in job order), else dz = their sum (0 for a code no job
// used).  Group o = tid / 16 of the block: job o / 8, vector (o / 4) % 2 (dz_s: W_sc1^T ds1 + W_sc2^T
// ds2; dz_t: W_tc1^T dt1), column r0 + o % 4; its lane p takes n = 16 p .. 16 p + 15.
__global__ __launch_bounds__(256) void code_dz_kernel(DzJobs jobs, float* __restrict__ dz_s, float* __restrict__ dz_t,
                                                      int accumulate) {
  using namespace mlp;
  static_assert(kCodeRows == 4 && kMaxDzJobs == 2, "thread map: 2 jobs x 2 vectors x 4 columns x 16 lanes");
  __shared__ float dsv[kMaxDzJobs][3][256];
  __shared__ float part[kMaxDzJobs][2][kCodeRows];
  const int c = blockIdx.x, y = blockIdx.y, tid = threadIdx.x;
  const int r0 = kCodeRows * y;
  bool used[kMaxDzJobs] = {false, false};
  for (int jb = 0; jb < jobs.n; ++jb) {
    used[jb] = code_row_used(jobs.j[jb].g + (int64_t)c * kCbStride, tid);
    if (used[jb]) {
      const float* wc = jobs.j[jb].ws + (int64_t)c * 6 * 256;
      dsv[jb][0][tid] = wc[768 + tid];
      dsv[jb][1][tid] = wc[1024 + tid];
      dsv[jb][2][tid] = wc[1280 + tid];
    }
  }
  __syncthreads();
  {
    const int o = tid >> 4, jb = o >> 3, vv = (o >> 2) & 1, k = o & 3, pl = tid & 15, j = r0 + k;
    if (jb < jobs.n && used[jb]) {     // uniform over the 16-lane group
      const Params& Pj = jobs.j[jb].P;
      float acc = 0.f;
      if (vv == 0) {
        float w1[16], w2[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          w1[u] = Pj.p[kWSc1][(16 * pl + u) * 256 + j];
          w2[u] = Pj.p[kWSc2][(16 * pl + u) * 256 + j];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          acc = fmaf(w1[u], dsv[jb][0][16 * pl + u], acc);
          acc = fmaf(w2[u], dsv[jb][1][16 * pl + u], acc);
        }
      } else {
        float w1[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) w1[u] = Pj.p[kWTc1][(16 * pl + u) * 256 + j];
#pragma unroll
        for (int u = 0; u < 16; ++u) acc = fmaf(w1[u], dsv[jb][2][16 * pl + u], acc);
      }
      const float sum = sum16_bfly(acc);
      if (pl == 0) part[jb][vv][k] = sum;
    }
  }
  __syncthreads();
  if (tid < 2 * kCodeRows) {
    const int vv = tid / kCodeRows, k = tid % kCodeRows;
    float* dz = vv == 0 ? dz_s : dz_t;
    if (dz) {
      float* d = dz + (int64_t)c * 256 + r0 + k;
      bool has = accumulate != 0;
      float cur = has ? *d : 0.f;
      for (int jb = 0; jb < jobs.n; ++jb) {
        if (!used[jb]) continue;
        cur = has ? cur + part[jb][vv][k] : part[jb][vv][k];
        has = true;
      }
      *d = cur;
    }
  }
}

// The bias gradients that are column sums of g_code (the per-code sums of the code-bias terms):
// layer_xyz2 (cols 0..255), fc_out rows 1..256 (256..511) and row 0 (512), fc_rgb (513..515).
__global__ void gcode_bias_kernel(const float* __restrict__ g_code, int64_t n_codes, float* __restrict__ b_xyz2,
                                  float* __restrict__ b_out, float* __restrict__ b_rgb) {
  using namespace mlp;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= kCbRgb + 3) return;
  float acc = 0.0f;
  for (int64_t c = 0; c < n_codes; ++c) acc += g_code[c * kCbStride + j];
  if (j < kCbFeat) b_xyz2[j] += acc;
  else if (j < kCbSigma) b_out[1 + j - kCbFeat] += acc;
  else if (j == kCbSigma) b_out[0] += acc;
  else b_rgb[j - kCbRgb] += acc;
}

// The deterministic fused eval backward's ray gradients (cn_field_backward_fused_ws): one wave per
// ray r adds, in a fixed order (each lane its strided share, then a butterfly), the ray's wave rows of
// ray_part (d ro, d rd of its points: S / ws rows) and the Q1 view-direction terms of q1_part (the S
// samples k of r's chunk with k mod rcnt = r - base, nerf/__init__.py:127-128), then
// d ro[r] += points' d ro and d rd[r] += points' d rd + Q1 d rd.
// Blocks past the rays' (gc_blocks of them) add each backward workgroup's wave rows of gc_part in wave
// order into gc_rows (one row per workgroup), which reduce_partials_kernel then sums in block order.
// One ray's sums of one field's deterministic eval backward: v[0..2] its points' d ro, v[3..5] their d rd,
// v[6..8] its Q1 view-direction d rd (lane-strided over the wave, then a fixed butterfly).
__device__ __forceinline__ void ray_sums(const float* __restrict__ ray_part, const float* __restrict__ q1_part,
                                         int64_t n_rays, int64_t S, int64_t chunk_rows, int wave_samples, int64_t r,
                                         int lane, float (&v)[9]) {
#pragma unroll
  for (int i = 0; i < 9; ++i) v[i] = 0.0f;
  if (ray_part) {
    const int64_t nb = S / wave_samples;
    for (int64_t b = lane; b < nb; b += 64) {
      const float* p = ray_part + (r * nb + b) * 6;
#pragma unroll
      for (int i = 0; i < 6; ++i) v[i] += p[i];
    }
  }
  if (q1_part) {
    const int64_t base = (r / chunk_rows) * chunk_rows;
    const int64_t rcnt = min(chunk_rows, n_rays - base);
    const int64_t k0 = base * S + (r - base);
    for (int64_t j = lane; j < S; j += 64) {
      const float* q = q1_part + 3 * (k0 + j * rcnt);
#pragma unroll
      for (int i = 0; i < 3; ++i) v[6 + i] += q[i];
    }
  }
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1)
#pragma unroll
    for (int i = 0; i < 9; ++i) v[i] += __shfl_xor(v[i], off);
}

// Blocks past the rays': workgroup b's wave rows of gc_part added in wave order into gc_rows[b].
__device__ __forceinline__ void gc_rows_block(const float* __restrict__ gc_part, int gc_waves, float* __restrict__ gc_rows,
                                              int64_t b) {
  const float* rows = gc_part + b * gc_waves * mlp::kCbStride;
  for (int j = threadIdx.x; j < mlp::kCbStride; j += 256) {
    float v = rows[j];
    for (int w = 1; w < gc_waves; ++w) v += rows[(int64_t)w * mlp::kCbStride + j];
    gc_rows[b * mlp::kCbStride + j] = v;
  }
}

// The g_code rows' fixed-order sum (reduce_partials_kernel's reduce_block over the workgroups' rows) as
// blocks of the ray launch, when the backward already wrote one row per workgroup (fp32: gc_rows).
struct GcFinal {
  const float* rows;
  int64_t n_rows;
  float* g_code;
  int64_t blocks;
};

__device__ __forceinline__ void gc_final_block(const GcFinal& f, int64_t b, float4 (&red)[16][64]) {
  if (reduce_groups(f.n_rows) == 16) reduce_block<16>(f.rows, f.n_rows, 1, mlp::kCbStride, f.g_code, mlp::kCbStride, b, red);
  else reduce_block<4>(f.rows, f.n_rows, 1, mlp::kCbStride, f.g_code, mlp::kCbStride, b, red);
}

__global__ __launch_bounds__(256) void ray_grad_reduce_kernel(const float* __restrict__ ray_part,
                                                              const float* __restrict__ q1_part, int64_t n_rays,
                                                              int64_t S, int64_t chunk_rows, int wave_samples,
                                                              float* __restrict__ d_ro, float* __restrict__ d_rd,
                                                              const float* __restrict__ gc_part, int gc_waves,
                                                              float* __restrict__ gc_rows, int64_t gc_blocks,
                                                              GcFinal fin) {
  __shared__ float4 red[16][64];
  const int64_t ray_blocks = (n_rays + 3) / 4;
  if ((int64_t)blockIdx.x >= ray_blocks + gc_blocks) {
    gc_final_block(fin, (int64_t)blockIdx.x - ray_blocks - gc_blocks, red);
    return;
  }
  if ((int64_t)blockIdx.x >= ray_blocks) {
    gc_rows_block(gc_part, gc_waves, gc_rows, (int64_t)blockIdx.x - ray_blocks);
    return;
  }
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n_rays) return;  // wave-uniform
  float v[9];
  ray_sums(ray_part, q1_part, n_rays, S, chunk_rows, wave_samples, r, lane, v);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (d_ro) d_ro[3 * r + i] += v[i];
      if (d_rd) d_rd[3 * r + i] += v[3 + i] + v[6 + i];
    }
  }
}

// One field's part of ray_grad_reduce2_kernel.
struct RayRed {
  const float* ray_part;
  const float* q1_part;
  int64_t S, chunk_rows;
  GcFinal fin;        // the field's g_code: its workgroups' rows (written by the backward) summed here
  int wave_samples;
};

// ray_grad_reduce_kernel for a render's two fields on the same rays and the same d ro / d rd (the eval
// step's ray sink): per ray, d ro += field 0's, then += field 1's; d rd += field 0's, += between (the rays'
// gradient that reached them between the two field backwards -- the coarse volume render's), += field 1's:
// the additions of the two per-field launches with the volume render's in between, in their order.  Then
// both fields' g_code sums (their workgroups' rows, written by the backward).
__global__ __launch_bounds__(256) void ray_grad_reduce2_kernel(RayRed f0, RayRed f1, int64_t n_rays,
                                                               const float* __restrict__ between,
                                                               float* __restrict__ d_ro, float* __restrict__ d_rd) {
  __shared__ float4 red[16][64];
  const int64_t ray_blocks = (n_rays + 3) / 4;
  const int64_t b = (int64_t)blockIdx.x - ray_blocks;
  if (b >= f0.fin.blocks) {
    gc_final_block(f1.fin, b - f0.fin.blocks, red);
    return;
  }
  if (b >= 0) {
    gc_final_block(f0.fin, b, red);
    return;
  }
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= n_rays) return;  // wave-uniform
  float v0[9], v1[9];
  ray_sums(f0.ray_part, f0.q1_part, n_rays, f0.S, f0.chunk_rows, f0.wave_samples, r, lane, v0);
  ray_sums(f1.ray_part, f1.q1_part, n_rays, f1.S, f1.chunk_rows, f1.wave_samples, r, lane, v1);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if (d_ro) {
        float o = d_ro[3 * r + i];
        o += v0[i];
        o += v1[i];
        d_ro[3 * r + i] = o;
      }
      if (d_rd) {
        float d = d_rd[3 * r + i];
        d += v0[3 + i] + v0[6 + i];
        if (between) d += between[3 * r + i];
        d += v1[3 + i] + v1[6 + i];
        d_rd[3 * r + i] = d;
      }
    }
  }
}

// dst += src over n floats (the fallback of the paired eval backward's in-between ray gradient).
__global__ void add_into_kernel(float* __restrict__ dst, const float* __restrict__ src, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] += src[i];
}

}  // namespace grad
}  // namespace cn

// ================================================================ C ABI
using namespace cn;

// Row stride (floats) of the (M, 257) pre-activation gradient buffers of the field backward:
// padded to a multiple of 4 so every row starts 16-byte aligned (dwordx4 A loads).
constexpr int64_t kLdP = 260;

namespace {

int gemm_nn(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, const float* mask,
            int64_t ldm, int64_t M, int N, int K, hipStream_t st, bool x3 = false) {
  if (K > grad::kMaxK) return CN_EINVAL;
  if (x3) {
    const int nu = static_cast<int>(std::min<int64_t>(8, ceil_div(N, 32)));
    const bool vec = lda % 4 == 0 && (reinterpret_cast<uintptr_t>(A) & 15) == 0;
    dim3 grid(static_cast<unsigned>(ceil_div(M, grad::kNnRows)), static_cast<unsigned>(ceil_div(N, 256)));
#define CN_NN_X3(NU_)                                                                                          \
  case NU_:                                                                                                     \
    if (vec)                                                                                                    \
      hipLaunchKernelGGL((grad::gemm_nn_x3_kernel<NU_, true>), grid, dim3(grad::kNnThreads), 0, st, A, lda, B, ldb, C, ldc,  \
                         mask, ldm, M, N, K);                                                                   \
    else                                                                                                        \
      hipLaunchKernelGGL((grad::gemm_nn_x3_kernel<NU_, false>), grid, dim3(grad::kNnThreads), 0, st, A, lda, B, ldb, C, ldc, \
                         mask, ldm, M, N, K);                                                                   \
    break;
    switch (nu) {
      CN_NN_X3(1) CN_NN_X3(2) CN_NN_X3(3) CN_NN_X3(4) CN_NN_X3(5) CN_NN_X3(6) CN_NN_X3(7) CN_NN_X3(8)
      default: return CN_EINVAL;
    }
#undef CN_NN_X3
    return launch_status();
  }
  // 64 columns per block (2 blocks per CU); 128 (one 146 KiB block per CU, 1 wave per SIMD)
  // measured 12 % slower over the training step's layers
  dim3 grid(static_cast<unsigned>(ceil_div(M, grad::kMT)), static_cast<unsigned>(ceil_div(N, 64)));
  hipLaunchKernelGGL(grad::gemm_nn_kernel<64>, grid, dim3(256), 0, st, A, lda, B, ldb, C, ldc, mask, ldm, M, N, K);
  return launch_status();
}

// Launch plan of one dW GEMM C += A^T B: the kernel, its rows per workgroup / split and the
// number of partial N x K tiles it writes on the deterministic path.
enum TnKind { kTnGeneric, kTnGenericX3, kTnSkinny, kTn256, kTn256X3 };
struct TnPlan {
  TnKind kind;
  int64_t rows, parts;
};

TnPlan tn_plan(const float* A, int64_t lda, const float* B, int64_t ldb, int64_t M, int N, int K, bool x3) {
  const bool b16 = (reinterpret_cast<uintptr_t>(B) & 15) == 0;
  (void)A;
  if (N <= 4 && K == 256 && ldb == 256 && b16 && M >= 64 * 1024) {
    // fp32 FMAs in both precisions (bandwidth-bound either way); ~1024 workgroups
    const int64_t rows = ceil_div(ceil_div(M, 1024), 4) * 4;
    return {kTnSkinny, rows, ceil_div(M, rows)};
  }
  if (N == 256 && K == 256 && lda == 256 && ldb == 256 && M >= 64 * 1024) {
    // whole-tile kernels: one workgroup per CU over M / 256 rows each (a multiple of the stage)
    const int64_t rows = ceil_div(ceil_div(M, 256), grad::kTwRows) * grad::kTwRows;
    return {x3 ? kTn256X3 : kTn256, rows, ceil_div(M, rows)};
  }
  // about 1024 blocks (4 per CU) over the M split, at least 256 rows each, a multiple of the
  // row group so only the last block has a ragged tail
  const int64_t tiles = ceil_div(N, grad::kTnTile) * ceil_div(K, grad::kTnTile);
  const int64_t grp = x3 ? grad::kTnRowsX3 * grad::kTnGroupsX3 : 2 * grad::kTnPairs;
  const int64_t splits = std::max<int64_t>(1, 1024 / tiles);
  int64_t rows = std::max<int64_t>(256, ceil_div(M, splits));
  rows = ceil_div(rows, grp) * grp;
  return {x3 ? kTnGenericX3 : kTnGeneric, rows, ceil_div(M, rows)};
}

// ws (optional, tn_plan(..).parts * N * K floats): the deterministic two-pass reduction instead
// of float atomics.
// Deferred fixed-order reductions: with a Reducer, each dW kernel of a backward writes its partial
// tiles into its own slice of the workspace (bump allocation from `cursor`) and queues the sum;
// flush() runs every queued sum in ONE launch.  Without one, each sum runs right away.
struct Reducer {
  hipStream_t st;
  float* cursor;
  grad::ReduceJobs jobs;
  int64_t blocks;
  float* take(int64_t n) {
    float* p = cursor;
    cursor += ceil_div(n, 64) * 64;
    return p;
  }
  int flush() {
    if (jobs.n == 0) return CN_OK;
    hipLaunchKernelGGL(grad::reduce_jobs_kernel, dim3(static_cast<unsigned>(blocks)), dim3(256), 0, st, jobs);
    jobs.n = 0;
    blocks = 0;
    return launch_status();
  }
};

int reduce(Reducer* rd, const float* part, int64_t parts, int N, int K, float* C, int64_t ldc, hipStream_t st,
           float* C2 = nullptr) {
  if (C2 && !rd) return CN_EINVAL;  // a second target: the queued form only
  const int64_t nk = (int64_t)N * K;
  const int64_t nblk = ceil_div(nk, grad::reduce_block_elems(grad::reduce_groups(parts), grad::reduce_vec4(part, nk)));
  if (!rd) {
    hipLaunchKernelGGL(grad::reduce_partials_kernel, dim3(static_cast<unsigned>(nblk)), dim3(256), 0, st, part, parts,
                       N, K, C, ldc);
    return launch_status();
  }
  if (rd->jobs.n == grad::kMaxReduceJobs) {
    const int rc = rd->flush();
    if (rc != CN_OK) return rc;
  }
  rd->jobs.j[rd->jobs.n++] = grad::ReduceJob{part, C, parts, ldc, rd->blocks, N, K, C2};
  rd->blocks += nblk;
  return CN_OK;
}

// Column sums of A (N <= 256) added to bias in a fixed order (bias_ws: ceil(M / rows) * N floats,
// rows = max(256, M / 256)).
int64_t colsum_rows(int64_t M) { return std::max<int64_t>(256, ceil_div(M, 256)); }

int colsum(const float* A, int64_t lda, int64_t M, int N, float* bias, float* bias_ws, hipStream_t st,
           Reducer* rd = nullptr) {
  const int64_t rows = colsum_rows(M);
  const unsigned nb = static_cast<unsigned>(ceil_div(M, rows));
  if (rd) bias_ws = rd->take((int64_t)nb * N);
  hipLaunchKernelGGL(grad::colsum_kernel, dim3(nb), dim3(256), 0, st, A, lda, M, N, bias_ws, rows);
  const int rc = launch_status();
  if (rc != CN_OK) return rc;
  return reduce(rd, bias_ws, nb, 1, N, bias, N, st);
}

// bias (optional, with bias_ws >= 1024 * N floats): also bias += A^T 1 (deterministic; folded into
// the 3xbf16 whole-tile kernel, a separate column-sum pass otherwise).
// rd: the deterministic path with deferred sums (ws / bias_ws are then taken from the reducer).
// sig / sig_out (optional, with rd; B 256 wide): also sig_out[0..255] += sum_m sig[4 m] B[m][:] -- fc_out's
// sigma row; sig is column 3 of the (M, 4) d raw rows, which the whole-tile kernels stream whole
// (draw = sig - 3) beside B -- a skinny pass otherwise.
int gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M, int N, int K,
            hipStream_t st, bool x3 = false, float* ws = nullptr, float* bias = nullptr, float* bias_ws = nullptr,
            Reducer* rd = nullptr, const float* sig = nullptr, float* sig_out = nullptr) {
  const TnPlan pl = tn_plan(A, lda, B, ldb, M, N, K, x3);
  const bool fold_bias = bias && (pl.kind == kTn256X3 || pl.kind == kTn256);
  const bool fold_sig = sig && rd && (pl.kind == kTn256 || pl.kind == kTn256X3);
  const unsigned nb = static_cast<unsigned>(ceil_div(M, pl.rows));
  float* sig_ws = nullptr;
  if (rd) {
    ws = rd->take(pl.parts * N * K);
    if (fold_bias) bias_ws = rd->take((int64_t)nb * N);
    if (fold_sig) sig_ws = rd->take((int64_t)nb * 256);
  }
  switch (pl.kind) {
    case kTnSkinny:
      switch (N) {
        case 1: hipLaunchKernelGGL(grad::gemm_tn_skinny_kernel<1>, dim3(nb), dim3(256), 0, st, A, lda, B, C, ldc, ws, M, pl.rows); break;
        case 2: hipLaunchKernelGGL(grad::gemm_tn_skinny_kernel<2>, dim3(nb), dim3(256), 0, st, A, lda, B, C, ldc, ws, M, pl.rows); break;
        case 3: hipLaunchKernelGGL(grad::gemm_tn_skinny_kernel<3>, dim3(nb), dim3(256), 0, st, A, lda, B, C, ldc, ws, M, pl.rows); break;
        default: hipLaunchKernelGGL(grad::gemm_tn_skinny_kernel<4>, dim3(nb), dim3(256), 0, st, A, lda, B, C, ldc, ws, M, pl.rows); break;
      }
      break;
    case kTn256:
      if (fold_sig)
        hipLaunchKernelGGL((grad::gemm_tn256_kernel<false, true>), dim3(nb), dim3(512), 0, st, A, B, C, ldc, ws,
                           fold_bias ? bias_ws : nullptr, sig - 3, sig_ws, M, pl.rows);
      else
        hipLaunchKernelGGL((grad::gemm_tn256_kernel<false, false>), dim3(nb), dim3(512), 0, st, A, B, C, ldc, ws,
                           fold_bias ? bias_ws : nullptr, nullptr, nullptr, M, pl.rows);
      break;
    case kTn256X3:
      if (fold_sig)
        hipLaunchKernelGGL((grad::gemm_tn256_kernel<true, true>), dim3(nb), dim3(512), 0, st, A, B, C, ldc, ws,
                           fold_bias ? bias_ws : nullptr, sig - 3, sig_ws, M, pl.rows);
      else
        hipLaunchKernelGGL((grad::gemm_tn256_kernel<true, false>), dim3(nb), dim3(512), 0, st, A, B, C, ldc, ws,
                           fold_bias ? bias_ws : nullptr, nullptr, nullptr, M, pl.rows);
      break;
    case kTnGenericX3: {
      const int64_t tiles = ceil_div(N, grad::kTnTile) * ceil_div(K, grad::kTnTile);
      hipLaunchKernelGGL(grad::gemm_tn_x3_kernel, dim3(static_cast<unsigned>(nb * tiles)), dim3(256), 0, st, A, lda, B,
                         ldb, C, ldc, ws, M, N, K, pl.rows, static_cast<int>(ceil_div(N, grad::kTnTile)),
                         static_cast<int>(tiles));
      break;
    }
    default: {
      dim3 grid(static_cast<unsigned>(ceil_div(N, grad::kTnTile)), static_cast<unsigned>(ceil_div(K, grad::kTnTile)), nb);
      hipLaunchKernelGGL(grad::gemm_tn_kernel, grid, dim3(256), 0, st, A, lda, B, ldb, C, ldc, ws, M, N, K, pl.rows);
      break;
    }
  }
  int rc = launch_status();
  if (rc != CN_OK) return rc;
  if (ws) {
    rc = reduce(rd, ws, pl.parts, N, K, C, ldc, st);
    if (rc != CN_OK) return rc;
  }
  if (sig) {
    rc = fold_sig ? reduce(rd, sig_ws, nb, 1, 256, sig_out, 256, st)
                  : gemm_tn(sig, 4, B, ldb, sig_out, 256, M, 1, 256, st, x3, nullptr, nullptr, nullptr, rd);
    if (rc != CN_OK) return rc;
  }
  if (bias) {
    if (!fold_bias) return colsum(A, lda, M, N, bias, bias_ws, st, rd);
    return reduce(rd, bias_ws, nb, 1, N, bias, N, st);
  }
  return CN_OK;
}

// Upper bound of the partial-tile workspace (floats) of gemm_tn(.., ws) for an M x N x K
// product in either precision, whatever the operand strides / alignment.
int64_t tn_ws_floats(int64_t M, int N, int K) {
  static const float* const kAligned = reinterpret_cast<const float*>(256);
  int64_t best = 0;
  for (int x3 = 0; x3 < 2; ++x3) {
    for (int contig = 0; contig < 2; ++contig) {
      const int64_t lda = contig ? N : N + 1, ldb = contig ? K : K + 1;
      best = std::max(best, tn_plan(kAligned, lda, kAligned, ldb, M, N, K, x3 != 0).parts * N * K);
    }
  }
  return best;
}

// dW of an encoding layer (ENC 0: layer_xyz1 from dPre(xyz1), ENC 1: layer_dir1's view columns
// from dPre(dir1)) with the encodings generated in the kernel; ws: the deterministic path
// (enc_ws_parts(M) * 256 * K floats).
// about one round of two workgroups per CU: each workgroup's prologue (three geometry stages, two
// DMA stages) and partial tile are paid half as often as with 1024 (r03k: 144.8 -> 135.3 us per
// layer_xyz1 launch of 393 Ki rows)
constexpr int64_t kEncBlocks = 512;
int64_t enc_rows(int64_t M) {
  return std::max<int64_t>(grad::kEncRows, ceil_div(ceil_div(M, kEncBlocks), grad::kEncRows) * grad::kEncRows);
}
int64_t enc_parts(int64_t M) { return ceil_div(M, enc_rows(M)); }

int gemm_tn_enc(int enc, const float* A, const mlp::FieldArgs& a, float* C, int64_t ldc, hipStream_t st, bool x3,
                float* ws, float* bias = nullptr, float* bias_ws = nullptr, Reducer* rd = nullptr,
                grad::DirRole dr = {}) {
  const int64_t rows = enc_rows(a.m);
  const unsigned nb = static_cast<unsigned>(ceil_div(a.m, rows));
  const int K = enc == 0 ? 63 : 27;
  if (rd) {
    ws = rd->take((int64_t)nb * 256 * K);
    if (bias) bias_ws = rd->take((int64_t)nb * 256);
  }
#define CN_ENC(X3_, E_, M_) \
  hipLaunchKernelGGL((grad::gemm_tn_enc_kernel<X3_, E_, M_>), dim3(nb + dr.n), dim3(512), 0, st, A, a, C, ldc, ws, \
                     bias ? bias_ws : nullptr, rows, dr)
  const bool pts = a.pts != nullptr;
  if (x3) {
    if (enc == 0) { if (pts) CN_ENC(true, 0, mlp::kFromPts); else CN_ENC(true, 0, mlp::kFromRayZ); }
    else { if (pts) CN_ENC(true, 1, mlp::kFromPts); else CN_ENC(true, 1, mlp::kFromRayZ); }
  } else {
    if (enc == 0) { if (pts) CN_ENC(false, 0, mlp::kFromPts); else CN_ENC(false, 0, mlp::kFromRayZ); }
    else { if (pts) CN_ENC(false, 1, mlp::kFromPts); else CN_ENC(false, 1, mlp::kFromRayZ); }
  }
#undef CN_ENC
  int rc = launch_status();
  if (rc != CN_OK) return rc;
  if (ws) {
    rc = reduce(rd, ws, nb, 256, K, C, ldc, st);
    if (rc != CN_OK) return rc;
  }
  if (bias) return reduce(rd, bias_ws, nb, 1, 256, bias, 256, st);
  return CN_OK;
}

// layer_xyz1's dW (+ bias) from the fp32 training forward's encoding plane (gemm_tn_xenc_kernel), with the
// DIRS fold's per-direction role riding in the same launch (dr); partials through the reducer.
int gemm_tn_xenc(const float* A, const float* X, const mlp::FieldArgs& a, float* C, int64_t ldc, hipStream_t st,
                 float* bias, Reducer* rd, grad::DirRole dr) {
  const int64_t rows = enc_rows(a.m);
  const unsigned nb = static_cast<unsigned>(ceil_div(a.m, rows));
  float* ws = rd->take((int64_t)nb * 256 * 63);
  float* bws = bias ? rd->take((int64_t)nb * 256) : nullptr;
  hipLaunchKernelGGL(grad::gemm_tn_xenc_kernel, dim3(nb + dr.n), dim3(512), 0, st, A, X, a.m, ws, bws, rows, a, dr);
  int rc = launch_status();
  if (rc != CN_OK) return rc;
  rc = reduce(rd, ws, nb, 256, 63, C, ldc, st);
  if (rc != CN_OK) return rc;
  return bias ? reduce(rd, bws, nb, 1, 256, bias, 256, st) : CN_OK;
}

int seg_sum(const float* A, int64_t lda, int64_t M, int N, int64_t S, const int64_t* code_index, int64_t n_codes,
            float* out, int64_t out_ld, hipStream_t st) {
  dim3 grid(static_cast<unsigned>(ceil_div(M, grad::kSegRows)), static_cast<unsigned>(ceil_div(N, 64)));
  hipLaunchKernelGGL(grad::seg_sum_kernel, grid, dim3(256), 0, st,
                     A, lda, M, N, S, code_index, n_codes, out, out_ld);
  return launch_status();
}

#define CN_TRY(x)              \
  do {                         \
    const int rc_ = (x);       \
    if (rc_ != CN_OK) return rc_; \
  } while (0)

}  // namespace

extern "C" int cn_gemm_nn(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                          const float* mask, int64_t ldm, int64_t M, int64_t N, int64_t K, cn_stream_t stream) {
  CN_CHECK_ARG(A && B && C && M > 0 && N > 0 && K > 0 && N <= 65536 && K <= 288);
  CN_CHECK_ARG(lda >= K && ldb >= N && ldc >= N && (!mask || ldm >= N));
  return gemm_nn(A, lda, B, ldb, C, ldc, mask, ldm, M, (int)N, (int)K, as_stream(stream));
}

extern "C" int cn_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M,
                          int64_t N, int64_t K, cn_stream_t stream) {
  CN_CHECK_ARG(A && B && C && M > 0 && N > 0 && K > 0 && N <= 65536 && K <= 65536);
  CN_CHECK_ARG(lda >= N && ldb >= K && ldc >= K);
  return gemm_tn(A, lda, B, ldb, C, ldc, M, (int)N, (int)K, as_stream(stream));
}

extern "C" int64_t cn_gemm_tn_workspace_floats(int64_t M, int64_t N, int64_t K) {
  if (M <= 0 || N <= 0 || K <= 0 || N > 65536 || K > 65536) return -1;
  return tn_ws_floats(M, (int)N, (int)K);
}

extern "C" int cn_gemm_tn_ws(int fmt, const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                             int64_t M, int64_t N, int64_t K, float* workspace, cn_stream_t stream) {
  CN_CHECK_ARG(fmt == CN_FMT_F32 || fmt == CN_FMT_BF16X3);
  CN_CHECK_ARG(A && B && C && workspace && M > 0 && N > 0 && K > 0 && N <= 65536 && K <= 65536);
  CN_CHECK_ARG(lda >= N && ldb >= K && ldc >= K);
  return gemm_tn(A, lda, B, ldb, C, ldc, M, (int)N, (int)K, as_stream(stream), fmt == CN_FMT_BF16X3, workspace);
}

extern "C" int cn_gemm_nn_x3(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                             const float* mask, int64_t ldm, int64_t M, int64_t N, int64_t K, cn_stream_t stream) {
  CN_CHECK_ARG(A && B && C && M > 0 && N > 0 && K > 0 && N <= 65536 && K <= 288);
  CN_CHECK_ARG(lda >= K && ldb >= N && ldc >= N && (!mask || ldm >= N));
  return gemm_nn(A, lda, B, ldb, C, ldc, mask, ldm, M, (int)N, (int)K, as_stream(stream), true);
}

extern "C" int cn_gemm_tn_x3(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                             int64_t M, int64_t N, int64_t K, cn_stream_t stream) {
  CN_CHECK_ARG(A && B && C && M > 0 && N > 0 && K > 0 && N <= 65536 && K <= 65536);
  CN_CHECK_ARG(lda >= N && ldb >= K && ldc >= K);
  return gemm_tn(A, lda, B, ldb, C, ldc, M, (int)N, (int)K, as_stream(stream), true);
}

extern "C" int cn_encode_inputs(const float* pts, const float* ro, const float* rd, const float* z, int64_t n_rays,
                                int64_t n_samples, int64_t chunk_rows, const float* freqs_xyz, const float* freqs_dir,
                                float* x, cn_stream_t stream) {
  CN_CHECK_ARG(rd && x && freqs_xyz && freqs_dir && (pts || (ro && z)));
  CN_CHECK_ARG(n_rays > 0 && n_samples > 0 && chunk_rows > 0);
  mlp::FieldArgs a = {};
  a.pts = pts;
  a.ro = ro;
  a.rd = rd;
  a.z = z;
  a.n_rays = n_rays;
  a.n_samples = n_samples;
  a.chunk_rows = chunk_rows;
  a.m = n_rays * n_samples;
  for (int i = 0; i < 10; ++i) a.fx[i] = freqs_xyz[i];
  for (int i = 0; i < 4; ++i) a.fd[i] = freqs_dir[i];
  hipLaunchKernelGGL(grad::encode_inputs_kernel, dim3(elementwise_grid(a.m * 90, 256)), dim3(256), 0,
                     as_stream(stream), a, x);
  return launch_status();
}

// Field backward: see include/codenerf.h.
extern "C" int cn_field_backward(const float* const* params, const float* saved, const float* x_enc,
                                 const float* d_raw, const float* pts, const float* ro, const float* rd,
                                 const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                                 const int64_t* code_index, int64_t n_codes, const float* freqs_xyz,
                                 const float* freqs_dir, float* workspace, float* const* grads, float* g_code,
                                 float* d_pts, float* d_ro, float* d_rd, cn_stream_t stream) {
  return cn_field_backward_fmt(CN_FMT_F32, params, saved, x_enc, d_raw, pts, ro, rd, z, n_rays, n_samples,
                               chunk_rows, code_index, n_codes, freqs_xyz, freqs_dir, workspace, grads, g_code,
                               d_pts, d_ro, d_rd, stream);
}

extern "C" int cn_field_backward_fmt(int fmt, const float* const* params, const float* saved, const float* x_enc,
                                     const float* d_raw, const float* pts, const float* ro, const float* rd,
                                     const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                                     const int64_t* code_index, int64_t n_codes, const float* freqs_xyz,
                                     const float* freqs_dir, float* workspace, float* const* grads, float* g_code,
                                     float* d_pts, float* d_ro, float* d_rd, cn_stream_t stream) {
  using namespace mlp;
  CN_CHECK_ARG(fmt == CN_FMT_F32 || fmt == CN_FMT_BF16X3);
  const bool x3 = fmt == CN_FMT_BF16X3;
  CN_CHECK_ARG(params && saved && x_enc && d_raw && workspace);
  CN_CHECK_ARG(n_rays > 0 && n_samples > 0 && chunk_rows > 0 && n_codes > 0);
  if (d_pts || d_ro || d_rd) CN_CHECK_ARG(rd && freqs_xyz && freqs_dir && (pts || (ro && z)));
  CN_CHECK_ARG(!d_pts || pts);
  CN_CHECK_ARG(!d_ro || (ro && z && !pts));
  for (int i = 0; i < CN_NUM_PARAMS; ++i) CN_CHECK_ARG(params[i]);
  hipStream_t st = as_stream(stream);
  const int64_t M = n_rays * n_samples;
  const float* h1 = saved;
  const float* h2 = saved + M * 256;
  const float* feat = saved + 2 * M * 256;
  const float* v1 = saved + 3 * M * 256;
  const float* v2 = saved + 4 * M * 256;
  float* dpa = workspace;              // (M, 257) in rows of kLdP
  float* dpb = workspace + M * kLdP;    // (M, 257) in rows of kLdP
  float* denc = workspace + 2 * M * kLdP;  // (M, 90)
  float* dxp = workspace + 2 * M * kLdP + M * 90;  // (M, 6): d pts | d viewdir
  const bool wg = grads && grads[0];
  auto G = [&](int i) { return grads ? grads[i] : nullptr; };

  // fc_rgb: rgb = W_rgb [v2 | zt1] + b
  CN_TRY(gemm_nn(d_raw, 4, params[kWRgb], 512, dpa, kLdP, v2, 256, M, 256, 3, st, x3));  // d pre(layer_dir2)
  if (wg) {
    CN_TRY(gemm_tn(d_raw, 4, v2, 256, G(kWRgb), 512, M, 3, 256, st, x3));
    CN_TRY(seg_sum(d_raw, 4, M, 3, M, nullptr, 1, G(kBRgb), 1, st));
  }
  if (g_code) CN_TRY(seg_sum(d_raw, 4, M, 3, n_samples, code_index, n_codes, g_code + kCbRgb, kCbStride, st));
  // layer_dir2: v2 = relu(W v1 + b)
  CN_TRY(gemm_nn(dpa, kLdP, params[kWDir2], 256, dpb, kLdP, v1, 256, M, 256, 256, st, x3));  // d pre(layer_dir1)
  if (wg) {
    CN_TRY(gemm_tn(dpa, kLdP, v1, 256, G(kWDir2), 256, M, 256, 256, st, x3));
    CN_TRY(seg_sum(dpa, kLdP, M, 256, M, nullptr, 1, G(kBDir2), 1, st));
  }
  // layer_dir1: v1 = relu(W [feat | dir] + b) -> d feat into dpa[:, 1:], d dir into denc[:, 63:]
  CN_TRY(gemm_nn(dpb, kLdP, params[kWDir1], 283, dpa + 1, kLdP, nullptr, 0, M, 256, 256, st, x3));
  CN_TRY(gemm_nn(dpb, kLdP, params[kWDir1] + 256, 283, denc + 63, 90, nullptr, 0, M, 27, 256, st, x3));
  if (wg) {
    CN_TRY(gemm_tn(dpb, kLdP, feat, 256, G(kWDir1), 283, M, 256, 256, st, x3));
    CN_TRY(gemm_tn(dpb, kLdP, x_enc + 63, 90, G(kWDir1) + 256, 283, M, 256, 27, st, x3));
    CN_TRY(seg_sum(dpb, kLdP, M, 256, M, nullptr, 1, G(kBDir1), 1, st));
  }
  // fc_out: [sigma | feat] = W [h2 | zs2] + b (no activation)
  hipLaunchKernelGGL(grad::copy_cols_kernel, dim3(elementwise_grid(M, 256)), dim3(256), 0, st, d_raw + 3, 4, dpa, kLdP, M, 1);
  CN_TRY(launch_status());
  CN_TRY(gemm_nn(dpa, kLdP, params[kWOut], 512, dpb, kLdP, h2, 256, M, 256, 257, st, x3));  // d pre(layer_xyz2)
  if (wg) {
    CN_TRY(gemm_tn(dpa, kLdP, h2, 256, G(kWOut), 512, M, 257, 256, st, x3));
    CN_TRY(seg_sum(dpa, kLdP, M, 257, M, nullptr, 1, G(kBOut), 1, st));
  }
  if (g_code) {
    CN_TRY(seg_sum(dpa, kLdP, M, 1, n_samples, code_index, n_codes, g_code + kCbSigma, kCbStride, st));
    CN_TRY(seg_sum(dpa + 1, kLdP, M, 256, n_samples, code_index, n_codes, g_code + kCbFeat, kCbStride, st));
  }
  // layer_xyz2: h2 = relu(W [h1 | zs1] + b)
  CN_TRY(gemm_nn(dpb, kLdP, params[kWXyz2], 512, dpa, kLdP, h1, 256, M, 256, 256, st, x3));  // d pre(layer_xyz1)
  if (wg) {
    CN_TRY(gemm_tn(dpb, kLdP, h1, 256, G(kWXyz2), 512, M, 256, 256, st, x3));
    CN_TRY(seg_sum(dpb, kLdP, M, 256, M, nullptr, 1, G(kBXyz2), 1, st));
  }
  if (g_code) CN_TRY(seg_sum(dpb, kLdP, M, 256, n_samples, code_index, n_codes, g_code + kCbXyz2, kCbStride, st));
  // layer_xyz1: h1 = relu(W xyz63 + b)
  CN_TRY(gemm_nn(dpa, kLdP, params[kWXyz1], 63, denc, 90, nullptr, 0, M, 63, 256, st, x3));
  if (wg) {
    CN_TRY(gemm_tn(dpa, kLdP, x_enc, 90, G(kWXyz1), 63, M, 256, 63, st, x3));
    CN_TRY(seg_sum(dpa, kLdP, M, 256, M, nullptr, 1, G(kBXyz1), 1, st));
  }
  // encodings -> points / view directions
  if (d_pts || d_ro || d_rd) {
    hipLaunchKernelGGL(grad::posenc_backward_kernel, dim3(elementwise_grid(M * 3, 256)), dim3(256), 0, st, x_enc, 90,
                       denc, 90, M, 3, grad::make_freqs(freqs_xyz, 10), 10, 1, dxp, 6);
    CN_TRY(launch_status());
    hipLaunchKernelGGL(grad::posenc_backward_kernel, dim3(elementwise_grid(M * 3, 256)), dim3(256), 0, st, x_enc + 63,
                       90, denc + 63, 90, M, 3, grad::make_freqs(freqs_dir, 4), 4, 1, dxp + 3, 6);
    CN_TRY(launch_status());
    if (d_rd) {
      hipLaunchKernelGGL(grad::viewdir_backward_kernel, dim3(elementwise_grid(M, 256)), dim3(256), 0, st, rd, dxp + 3, 6,
                         n_rays, n_samples, chunk_rows, d_rd);
      CN_TRY(launch_status());
    }
    if (pts) {
      if (d_pts) {
        hipLaunchKernelGGL(grad::copy_cols_kernel, dim3(elementwise_grid(M * 3, 256)), dim3(256), 0, st, dxp, 6, d_pts, 3,
                           M, 3);
        CN_TRY(launch_status());
      }
    } else if (d_ro || d_rd) {
      hipLaunchKernelGGL(grad::ray_points_backward_kernel, dim3(elementwise_grid(n_rays, 256)), dim3(256), 0, st, dxp, 6, z,
                         n_rays, n_samples, d_ro, d_rd);
      CN_TRY(launch_status());
    }
  }
  return CN_OK;
}

extern "C" int64_t cn_field_backward_workspace_floats(int64_t m) { return m * (2 * kLdP + 90 + 6); }

// Offset (floats) of the (M, 90) dL/dx block inside that workspace (MLPForward's d x).
extern "C" int64_t cn_field_backward_dx_offset(int64_t m) { return m > 0 ? 2 * kLdP * m : -1; }

extern "C" int cn_code_bias_backward(const float* const* params, const float* z_s, const float* z_t, int64_t n_codes,
                                     const float* g_code, float* dz_s, float* dz_t, float* const* grads,
                                     cn_stream_t stream) {
  using namespace mlp;
  CN_CHECK_ARG(params && z_s && z_t && g_code && n_codes > 0 && n_codes < (1ll << 31));
  Params P, G = {};
  for (int i = 0; i < CN_NUM_PARAMS; ++i) {
    CN_CHECK_ARG(params[i]);
    P.p[i] = params[i];
    G.p[i] = grads ? grads[i] : nullptr;
  }
  hipLaunchKernelGGL(grad::code_backward_kernel, dim3(static_cast<unsigned>(n_codes), grads ? grad::kCodeRowSplits : 1),
                     dim3(grad::kCodeThreads), 0, as_stream(stream), P, z_s, z_t, g_code, dz_s, dz_t, G);
  return launch_status();
}


extern "C" int cn_code_bias_backward_act(const float* const* params, const float* z_s, const float* z_t,
                                         int64_t n_codes, const float* code_act, const float* g_code,
                                         float* const* grads, float* workspace, cn_stream_t stream) {
  using namespace mlp;
  CN_CHECK_ARG(params && z_s && z_t && code_act && g_code && workspace && n_codes > 0 && n_codes < (1ll << 31));
  Params P, G = {};
  for (int i = 0; i < CN_NUM_PARAMS; ++i) {
    CN_CHECK_ARG(params[i]);
    P.p[i] = params[i];
    G.p[i] = grads ? grads[i] : nullptr;
  }
  hipLaunchKernelGGL(grad::code_ds_outer_kernel, dim3(static_cast<unsigned>(n_codes), grad::kCodeSlices), dim3(256), 0,
                     as_stream(stream), P, z_s, z_t, g_code, code_act, workspace, G);
  return launch_status();
}

extern "C" int cn_code_dz(const cn_code_dz_job* jobs, int n_jobs, int64_t n_codes, float* dz_s, float* dz_t,
                          int accumulate, cn_stream_t stream) {
  using namespace mlp;
  CN_CHECK_ARG(jobs && n_jobs >= 1 && n_jobs <= grad::kMaxDzJobs && n_codes > 0 && n_codes < (1ll << 31));
  CN_CHECK_ARG(accumulate == 0 || accumulate == 1);
  grad::DzJobs dj = {};
  dj.n = n_jobs;
  for (int k = 0; k < n_jobs; ++k) {
    CN_CHECK_ARG(jobs[k].params && jobs[k].g_code && jobs[k].workspace);
    for (int i = 0; i < CN_NUM_PARAMS; ++i) {
      CN_CHECK_ARG(jobs[k].params[i]);
      dj.j[k].P.p[i] = jobs[k].params[i];
    }
    dj.j[k].g = jobs[k].g_code;
    dj.j[k].ws = jobs[k].workspace;
  }
  if (!dz_s && !dz_t) return CN_OK;
  hipLaunchKernelGGL(grad::code_dz_kernel, dim3(static_cast<unsigned>(n_codes), grad::kCodeSlices), dim3(256), 0,
                     as_stream(stream), dj, dz_s, dz_t, accumulate);
  return launch_status();
}

extern "C" int64_t cn_code_bias_backward_workspace_floats(int64_t n_codes) {
  return n_codes > 0 ? n_codes * 6 * 256 : -1;
}

extern "C" int cn_code_bias_backward_ws(const float* const* params, const float* z_s, const float* z_t,
                                        int64_t n_codes, const float* g_code, float* dz_s, float* dz_t,
                                        float* const* grads, float* workspace, int accumulate_dz,
                                        cn_stream_t stream) {
  using namespace mlp;
  CN_CHECK_ARG(params && z_s && z_t && g_code && workspace && n_codes > 0 && n_codes < (1ll << 31));
  CN_CHECK_ARG(accumulate_dz == 0 || accumulate_dz == 1);
  Params P, G = {};
  for (int i = 0; i < CN_NUM_PARAMS; ++i) {
    CN_CHECK_ARG(params[i]);
    P.p[i] = params[i];
    G.p[i] = grads ? grads[i] : nullptr;
  }
  hipStream_t st = as_stream(stream);
  const dim3 grid(static_cast<unsigned>(n_codes), grad::kCodeSlices);
  hipLaunchKernelGGL(grad::code_layers_dz_kernel, grid, dim3(256), 0, st, P, z_s, z_t, g_code, workspace);
  CN_TRY(launch_status());
  hipLaunchKernelGGL(grad::code_outer_kernel, grid, dim3(256), 0, st, P, z_s, z_t, g_code, workspace, dz_s, dz_t, G,
                     accumulate_dz);
  return launch_status();
}

extern "C" int cn_posenc_backward(const float* x, int64_t m, int64_t d, const float* freqs, int64_t num_freq,
                                  int include_input, const float* g_enc, float* dx, cn_stream_t stream) {
  CN_CHECK_ARG(x && g_enc && dx && m > 0 && d > 0 && num_freq >= 0 && num_freq <= 32 && (num_freq == 0 || freqs));
  const int inc = include_input ? 1 : 0;
  const int64_t ld = d * (inc + 2 * num_freq);
  CN_CHECK_ARG(ld > 0);
  hipLaunchKernelGGL(grad::posenc_backward_kernel, dim3(elementwise_grid(m * d, 256)), dim3(256), 0, as_stream(stream),
                     x, d, g_enc, ld, m, static_cast<int>(d), grad::make_freqs(freqs, static_cast<int>(num_freq)),
                     static_cast<int>(num_freq), inc, dx, d);
  return launch_status();
}

extern "C" int cn_ray_points_backward(const float* g_pts, const float* z, int64_t n_rays, int64_t n_samples,
                                      float* d_ro, float* d_rd, cn_stream_t stream) {
  CN_CHECK_ARG(g_pts && z && n_rays > 0 && n_samples > 0 && (d_ro || d_rd));
  hipLaunchKernelGGL(grad::ray_points_backward_kernel, dim3(elementwise_grid(n_rays, 256)), dim3(256), 0,
                     as_stream(stream), g_pts, 3, z, n_rays, n_samples, d_ro, d_rd);
  return launch_status();
}

// ---------------------------------------------------------------- fused fp32 training backward
// dX chain, g_code and the ray gradients in ONE fused fp32 launch (field_w16_bwd_kernel<.., true>,
// which also writes each layer's masked input gradient dPre), then the weight and bias
// gradients as split-M fp32 MFMA GEMMs dW = dPre^T X over those planes and the forward's saved
// activations (cn_radiance_field_train_w16).
// dPre planes, then the dW GEMMs' partial tiles (deterministic reduction, reused by each GEMM in
// stream order).
// Every dW GEMM of one backward keeps its partial tiles until the single deferred reduction:
// the sum of their slices (+ five column-sum partial blocks -- three biases, g_code's feat and xyz2
// rows -- the small d raw column sums and the 64-float alignment of each take).
// The DIRS fold's own slices (dir1_dw_folded, n_samples >= 32): gsum slots for <= 256 workgroups +
// m / 512 direction groups, and the encoding / bias partials of those groups.
static int64_t dirs_ws_floats(int64_t m) {
  const int64_t groups = ceil_div(m, 512);
  return (256 + groups) * 4096 + ceil_div(groups, grad::kDirGroups) * 256 * 28 + 4 * 64;
}

static int64_t train_dw_ws_floats(int64_t m) {
  return 4 * tn_ws_floats(m, 256, 256) + tn_ws_floats(m, 3, 256) + tn_ws_floats(m, 1, 256) +
         std::max(tn_ws_floats(m, 256, 27), enc_parts(m) * 256 * 27) +
         std::max(tn_ws_floats(m, 256, 63), enc_parts(m) * 256 * 63) + 5 * 1024 * 256 + 4 * 256 * 4 + 24 * 64 +
         dirs_ws_floats(m);
}

// layer_dir1's dW (C: [feat | 27 view-encoding columns], ldc 283) and bias in one pass over its dPre
// plane (the DIRS fold: gemm_tn256_kernel<false, false, true> + dir_enc_dw_kernel).  Needs the
// whole-tile plan, whole direction groups (n_rays and the Q1 chunk multiples of 16) and at most
// `budget` floats of reducer workspace; CN_EUNSUPPORTED otherwise, before anything is launched
// (the caller then runs the [feat] GEMM and gemm_tn_enc separately).
static int dir1_dw_folded(const float* dpre, const float* feat, float* C, float* bias, const mlp::FieldArgs& a,
                          hipStream_t st, Reducer* rd, int64_t budget) {
  const int64_t M = a.m;
  const TnPlan pl = tn_plan(dpre, 256, feat, 256, M, 256, 256, false);
  const int64_t rc = std::min(a.chunk_rows, a.n_rays);
  if (pl.kind != kTn256 || a.n_rays % 16 || rc % 16 || a.n_samples < 32 || M * 1024 + 64 * 1024 >= (int64_t(1) << 32))
    return CN_EUNSUPPORTED;
  const int64_t total = M / 16, per = ceil_div(total, 256), nb = ceil_div(total, per), groups = a.n_rays / 16;
  const int64_t nd = ceil_div(groups, grad::kDirGroups);
  const int64_t need = (nb + groups) * 4096 + nb * 65536 + nd * 256 * 28 + 4 * 64;
  if (nb > pl.parts || need > budget) return CN_EUNSUPPORTED;
  grad::DirFold d{static_cast<unsigned>(a.n_rays), static_cast<unsigned>(a.n_samples),
                  static_cast<unsigned>(rc), static_cast<unsigned>(per),
                  static_cast<unsigned>(total), rd->take((nb + groups) * 4096)};
  float* ws = rd->take(nb * 65536);
  hipLaunchKernelGGL((grad::gemm_tn256_kernel<false, false, true>), dim3(static_cast<unsigned>(nb)), dim3(512), 0, st,
                     dpre, feat, C, 283, ws, nullptr, nullptr, nullptr, M, 0, d);
  CN_TRY(launch_status());
  float* ep = rd->take(nd * 256 * 27);
  float* bp = rd->take(nd * 256);
  hipLaunchKernelGGL(grad::dir_enc_dw_kernel, dim3(static_cast<unsigned>(nd)), dim3(256), 0, st, a, d, ep, bp);
  CN_TRY(launch_status());
  CN_TRY(reduce(rd, ws, nb, 256, 256, C, 283, st));
  CN_TRY(reduce(rd, ep, nd, 256, 27, C + 256, 283, st));
  return reduce(rd, bp, nd, 1, 256, bias, 256, st);
}

// The whole-tile dW GEMMs of one training backward, queued and launched as ONE
// gemm_tn256_jobs_kernel (TnJobs).  add() records a GEMM C += A^T B (+ its bias column sums, the
// sigma row, the DIRS view-encoding fold); launch() splits the grid over the jobs in proportion to
// their rows times their per-row cost, takes each job's partial tiles from the reducer and queues
// the fixed-order sums (same partial order within a job: deterministic).  The costs belong to the
// layer slot, not to the job's kind, so a job's split -- and its summation order -- does not depend
// on whether another slot takes the DIRS fold.  CN_TN_JOBS=0 in the environment launches the GEMMs
// one by one (A/B); CN_TN_COST="c0,c1,c2,c3,c4" overrides the slot costs.
struct TnBatch {
  struct Pending {
    const float* A;
    const float* B;
    int64_t M;
    int kind;
    float* C;
    int64_t ldc;
    float* bias;      // += column sums of A (kinds 0, 1)
    const float* sig; // kind 1: d sigma (column 3 of the (M, 4) d raw rows)
    float* sig_out;
    mlp::FieldArgs a; // kind 2: the geometry (view directions) of the rows
    float cost;       // per-row cost of the slot (relative)
    float* bias2;     // a second target of the bias sums (g_code entries that are bias gradients), or null
    float* sig2;      // the same for sig_out
  };
  Pending p[grad::kMaxTnJobs];
  int n = 0;
};

// CN_XENC_PLANE=0: layer_xyz1's dW regenerates the encodings (gemm_tn_enc_kernel) instead of reading the
// forward's encoding plane (A/B)
static bool xenc_plane_enabled() {
  static const int on = [] {
    const char* e = getenv("CN_XENC_PLANE");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return on != 0;
}

// layer_xyz1's dW (the fp32 encoding-plane pass) as a job of the batched dW launch instead of its own
// launch (the DIRS fold's per-direction pass then runs alone after it, on the launch's direction sums):
// the batched launch grows by ~220 us per C3 chunk -- the pass is MFMA work (a quarter of a 256 x 256
// GEMM's per row), not a stream that hides beside the GEMMs -- against ~237 us for its own launch and
// fewer partial tiles to reduce (r06f: C3 39.14 / 39.19 -> 39.17 / 38.96 ms, 3080 13.77 / 13.80 ->
// 13.63 / 13.60 ms at slot cost 0.3; 0.25 starves it: 42.7 ms; 0.4 takes CUs from the GEMMs).
// CN_XENC_ROLE=0: its own launch (A/B).
static bool xenc_role_enabled() {
  static const int on = [] {
    const char* e = getenv("CN_XENC_ROLE");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return on != 0;
}

// CN_DIR_IN_ENC=0: the DIRS fold's dir_enc_dw pass as its own launch again (A/B; bitwise the same)
static bool dir_in_enc_enabled() {
  static const int on = [] {
    const char* e = getenv("CN_DIR_IN_ENC");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return on != 0;
}

// CN_FIELD_PAIR=0: a render's two fields' backward and dW launches one field after the other (A/B;
// bitwise the same gradients)
static bool pair_enabled() {
  static const int on = [] {
    const char* e = getenv("CN_FIELD_PAIR");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return on != 0;
}

static bool tn_jobs_enabled() {
  static const int on = [] {
    const char* e = getenv("CN_TN_JOBS");
    return (e && e[0] == '0') ? 0 : 1;
  }();
  return on != 0;
}

// The training backward's slot costs: layer_dir2, layer_dir1 (DIRS where it applies), fc_out
// (SIG), layer_xyz2 -- r03 per-launch times 375.5, 387.6, 394.7, 375.5 us -- and the RGB pass: an
// RGB workgroup streams ~40 GB/s of v2 beside the GEMMs (r03l: 6 of them, cost 0.1, held the
// launch 1.70 ms; 4 (0.07) 2.5 ms; 8-9 (0.14) balanced; r03n: 0.15 / 0.18 / 0.24 gave 41.5 / 41.7 /
// 41.7 ms per C3 iteration), 1 KiB per row, ~0.12 of a whole-tile row.  Kept a little above that:
// a late RGB workgroup holds up the whole launch, a spare one costs 1/256 of it.
static const float* tn_slot_cost() {
  static float w[6] = {1.0f, 1.03f, 1.05f, 1.0f, 0.16f, 0.3f};
  static const bool init = [] {
    const char* e = getenv("CN_TN_COST");
    if (e) sscanf(e, "%f,%f,%f,%f,%f,%f", &w[0], &w[1], &w[2], &w[3], &w[4], &w[5]);
    return true;
  }();
  (void)init;
  return w;
}

// DIRS fold applicability (dir1_dw_folded's conditions, without the workspace budget).
static bool dirs_foldable(const mlp::FieldArgs& a) {
  const int64_t rc = std::min(a.chunk_rows, a.n_rays);
  return a.n_rays % 16 == 0 && rc % 16 == 0 && a.n_samples >= 32 && a.m * 1024 + 64 * 1024 < (int64_t(1) << 32) &&
         a.m >= 64 * 1024;
}

// The batched launch's jobs for one TnBatch: the grid split over the jobs in proportion to their rows
// times their per-row cost (kGrid workgroups), each job's partial tiles taken from the reducer.  -> the
// workgroups the jobs use.
static int tn_batch_plan(TnBatch& b, Reducer* rd, grad::TnJobs& jobs) {
  double total = 0.0;
  for (int k = 0; k < b.n; ++k) total += b.p[k].cost * static_cast<double>(b.p[k].M);
  constexpr int kGrid = 256;  // one workgroup per CU (the ring fills the LDS)
  jobs = {};
  jobs.n = b.n;
  int first = 0;
  for (int k = 0; k < b.n; ++k) {
    const TnBatch::Pending& q = b.p[k];
    int want = static_cast<int>(kGrid * q.cost * static_cast<double>(q.M) / total + 0.5);
    want = std::max(1, std::min(want, kGrid - first - (b.n - 1 - k)));
    if (k == b.n - 1) want = std::max(1, kGrid - first);
    grad::TnJob& j = jobs.j[k];
    j.A = q.A;
    j.B = q.B;
    j.M = q.M;
    j.kind = q.kind;
    j.first_block = first;
    if (q.kind == 2) {
      const int64_t rc = std::min(q.a.chunk_rows, q.a.n_rays);
      const int64_t total_u = q.M / 16, per = ceil_div(total_u, want), nb = ceil_div(total_u, per);
      const int64_t groups = q.a.n_rays / 16;
      j.n_blocks = static_cast<int>(nb);
      j.rows_per_block = 0;
      j.dir = grad::DirFold{static_cast<unsigned>(q.a.n_rays), static_cast<unsigned>(q.a.n_samples),
                            static_cast<unsigned>(rc), static_cast<unsigned>(per), static_cast<unsigned>(total_u),
                            rd->take((nb + groups) * 4096)};
    } else {
      const int64_t rows = ceil_div(ceil_div(q.M, want), grad::kTwRows) * grad::kTwRows;
      j.n_blocks = static_cast<int>(ceil_div(q.M, rows));
      j.rows_per_block = rows;
    }
    if (q.kind == 4) {  // XENC: 256 x 63 partials (PositionalEmbedder column order), bias column sums
      j.part = rd->take((int64_t)j.n_blocks * 256 * 63);
      j.bias_part = q.bias ? rd->take((int64_t)j.n_blocks * 256) : nullptr;
      j.draw = nullptr;
      j.sig_part = nullptr;
      first += j.n_blocks;
      continue;
    }
    if (q.kind == 3) {  // RGB: 3 x 256 partials, 4 d raw column sums per block
      j.part = rd->take((int64_t)j.n_blocks * 3 * 256);
      j.bias_part = rd->take((int64_t)j.n_blocks * 4);
      j.draw = q.sig;
      j.sig_part = nullptr;
      first += j.n_blocks;
      continue;
    }
    j.part = rd->take((int64_t)j.n_blocks * 65536);
    j.bias_part = (q.bias && q.kind != 2) ? rd->take((int64_t)j.n_blocks * 256) : nullptr;  // DIRS: dir_enc_dw's
    j.draw = q.kind == 1 ? q.sig - 3 : nullptr;
    j.sig_part = q.kind == 1 ? rd->take((int64_t)j.n_blocks * 256) : nullptr;
    first += j.n_blocks;
  }
  return first;
}

static int tn_jobs_launch(const grad::TnJobs& jobs, int grid, bool x3, hipStream_t st) {
  if (x3) hipLaunchKernelGGL(grad::gemm_tn256_jobs_kernel<true>, dim3(static_cast<unsigned>(grid)), dim3(512), 0, st, jobs);
  else hipLaunchKernelGGL(grad::gemm_tn256_jobs_kernel<false>, dim3(static_cast<unsigned>(grid)), dim3(512), 0, st, jobs);
  return launch_status();
}

// After the launch: the fixed-order sums of every job's partials queued on the reducer (the DIRS job's
// dir_enc_dw pass launched here, or -- dir_out set -- returned as a role for the next gemm_tn_enc /
// gemm_tn_xenc launch; its partials' reductions are queued here either way).
static int tn_batch_post(TnBatch& b, const grad::TnJobs& jobs, hipStream_t st, Reducer* rd, grad::DirRole* dir_out) {
  for (int k = 0; k < b.n; ++k) {
    const TnBatch::Pending& q = b.p[k];
    const grad::TnJob& j = jobs.j[k];
    if (q.kind == 2) {
      const int64_t groups = q.a.n_rays / 16, nd = ceil_div(groups, grad::kDirGroups);
      float* ep = rd->take(nd * 256 * 27);
      float* bp = rd->take(nd * 256);
      if (dir_out) {
        *dir_out = grad::DirRole{j.dir, ep, bp, static_cast<unsigned>(nd)};
      } else {
        hipLaunchKernelGGL(grad::dir_enc_dw_kernel, dim3(static_cast<unsigned>(nd)), dim3(256), 0, st, q.a, j.dir, ep,
                           bp);
        CN_TRY(launch_status());
      }
      CN_TRY(reduce(rd, j.part, j.n_blocks, 256, 256, q.C, q.ldc, st));
      CN_TRY(reduce(rd, ep, nd, 256, 27, q.C + 256, q.ldc, st));
      CN_TRY(reduce(rd, bp, nd, 1, 256, q.bias, 256, st));
      continue;
    }
    if (q.kind == 4) {
      CN_TRY(reduce(rd, j.part, j.n_blocks, 256, 63, q.C, q.ldc, st));
      if (q.bias) CN_TRY(reduce(rd, j.bias_part, j.n_blocks, 1, 256, q.bias, 256, st));
      continue;
    }
    if (q.kind == 3) {
      CN_TRY(reduce(rd, j.part, j.n_blocks, 3, 256, q.C, q.ldc, st));
      CN_TRY(reduce(rd, j.bias_part, j.n_blocks, 1, 3, q.bias, 3, st, q.bias2));
      CN_TRY(reduce(rd, j.bias_part + 3 * (int64_t)j.n_blocks, j.n_blocks, 1, 1, q.sig_out, 1, st, q.sig2));
      continue;
    }
    CN_TRY(reduce(rd, j.part, j.n_blocks, 256, 256, q.C, q.ldc, st));
    if (q.kind == 1) CN_TRY(reduce(rd, j.sig_part, j.n_blocks, 1, 256, q.sig_out, 256, st));
    if (q.bias) CN_TRY(reduce(rd, j.bias_part, j.n_blocks, 1, 256, q.bias, 256, st, q.bias2));
  }
  b.n = 0;
  return CN_OK;
}

static int tn_batch_launch(TnBatch& b, bool x3, hipStream_t st, Reducer* rd, grad::DirRole* dir_out = nullptr) {
  if (b.n == 0) return CN_OK;
  grad::TnJobs jobs;
  const int grid = tn_batch_plan(b, rd, jobs);
  CN_TRY(tn_jobs_launch(jobs, grid, x3, st));
  return tn_batch_post(b, jobs, st, rd, dir_out);
}

// Two fields' batches (a render's coarse and fine backward) as ONE launch: each field's jobs keep the
// split of their own launch (the same workgroup counts and rows, so the same partial tiles), field 1's
// workgroups after field 0's -- they start on the CUs field 0's leave, filling its finish spread.
static int tn_batch_launch2(TnBatch& b0, Reducer* r0, grad::DirRole* d0, TnBatch& b1, Reducer* r1,
                            grad::DirRole* d1, bool x3, hipStream_t st) {
  if (b0.n == 0 || b1.n == 0 || b0.n + b1.n > grad::kMaxTnJobs) {
    CN_TRY(tn_batch_launch(b0, x3, st, r0, d0));
    return tn_batch_launch(b1, x3, st, r1, d1);
  }
  grad::TnJobs j0, j1, both = {};
  const int g0 = tn_batch_plan(b0, r0, j0);
  const int g1 = tn_batch_plan(b1, r1, j1);
  both.n = j0.n + j1.n;
  for (int k = 0; k < j0.n; ++k) both.j[k] = j0.j[k];
  for (int k = 0; k < j1.n; ++k) {
    both.j[j0.n + k] = j1.j[k];
    both.j[j0.n + k].first_block += g0;
  }
  CN_TRY(tn_jobs_launch(both, g0 + g1, x3, st));
  CN_TRY(tn_batch_post(b0, j0, st, r0, d0));
  return tn_batch_post(b1, j1, st, r1, d1);
}

// Two reducers' queued sums in one launch (each sum is computed exactly as in its own flush).
static int flush2(Reducer& a, Reducer& b) {
  if (a.jobs.n + b.jobs.n > grad::kMaxReduceJobs) {
    CN_TRY(a.flush());
    return b.flush();
  }
  for (int k = 0; k < b.jobs.n; ++k) {
    a.jobs.j[a.jobs.n] = b.jobs.j[k];
    a.jobs.j[a.jobs.n++].first_block += a.blocks;
  }
  a.blocks += b.blocks;
  b.jobs.n = 0;
  b.blocks = 0;
  return a.flush();
}

// fc_rgb's dW (C += d rgb^T v2, d_raw's columns 0..2) and, in the same pass, the d raw column sums
// g_rgb[0..2] += sum d rgb, g_sig[0] += sum d sigma (g_code's rgb / sigma entries with one code row).
static int rgb_dw_draw_sums(const float* d_raw, const float* v2, float* C, int64_t ldc, int64_t M, float* g_rgb,
                            float* g_sig, hipStream_t st, Reducer* rd) {
  const TnPlan pl = tn_plan(d_raw, 4, v2, 256, M, 3, 256, false);
  if (pl.kind != kTnSkinny) {
    CN_TRY(gemm_tn(d_raw, 4, v2, 256, C, ldc, M, 3, 256, st, false, nullptr, g_rgb, nullptr, rd));
    return colsum(d_raw + 3, 4, M, 1, g_sig, nullptr, st, rd);
  }
  const unsigned nb = static_cast<unsigned>(ceil_div(M, pl.rows));
  float* ws = rd->take(pl.parts * 3 * 256);
  float* cpart = rd->take(4 * (int64_t)nb);
  hipLaunchKernelGGL((grad::gemm_tn_skinny_kernel<3, true>), dim3(nb), dim3(256), 0, st, d_raw, 4, v2, C, ldc, ws, M,
                     pl.rows, cpart);
  CN_TRY(launch_status());
  CN_TRY(reduce(rd, ws, pl.parts, 3, 256, C, ldc, st));
  CN_TRY(reduce(rd, cpart, nb, 1, 3, g_rgb, 3, st));
  return reduce(rd, cpart + 3 * (int64_t)nb, nb, 1, 1, g_sig, 1, st);
}

// ---- the fused eval backward without float atomics (one code row, every wave inside one ray)

// The g_code sum of rows (n_rows x kCbStride, one per backward workgroup) as blocks of a ray launch
// (grad::gc_final_block: reduce()'s blocks for the same sum); rows null -> none.
static grad::GcFinal gc_final(const float* rows, int64_t n_rows, float* g_code) {
  if (!rows) return grad::GcFinal{nullptr, 0, nullptr, 0};
  const int64_t blocks = ceil_div(
      mlp::kCbStride, grad::reduce_block_elems(grad::reduce_groups(n_rows), grad::reduce_vec4(rows, mlp::kCbStride)));
  return grad::GcFinal{rows, n_rows, g_code, blocks};
}

static int64_t fused_ws_layout(int fmt_t, int64_t m, int64_t* ray_off, int64_t* q1_off, int64_t* rows_off) {
  const int64_t ws = fmt_t == CN_FMT_BF16X3_T ? 32 : 16;
  // the launch's grid is at most one workgroup per 128-sample tile and kMaxBwdBlocks
  const int64_t blocks = std::min<int64_t>(ceil_div(m, 128), mlp::kMaxBwdBlocks);
  const int64_t gc = blocks * mlp::kMaxBwdWaves * mlp::kCbStride;
  const int64_t rows = blocks * mlp::kCbStride;
  const int64_t rp = ceil_div(ceil_div(m, ws) * 6, 4) * 4;
  if (rows_off) *rows_off = gc;
  if (ray_off) *ray_off = gc + rows;
  if (q1_off) *q1_off = gc + rows + rp;
  return gc + rows + rp + 3 * m;
}

extern "C" int64_t cn_field_backward_fused_workspace_floats(int fmt_t, int64_t n_rays, int64_t n_samples) {
  if (!(fmt_t == CN_FMT_BF16X3_T || fmt_t == CN_FMT_F32_W16_T) || n_rays <= 0 || n_samples <= 0) return -1;
  return fused_ws_layout(fmt_t, n_rays * n_samples, nullptr, nullptr, nullptr);
}

extern "C" int cn_field_backward_fused_ws(int fmt_t, const float* packed_t, const uint32_t* masks,
                                          const float* d_raw, const float* pts, const float* ro, const float* rd,
                                          const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                                          const int64_t* code_index, int64_t n_codes, const float* freqs_xyz,
                                          const float* freqs_dir, float* g_code, float* d_pts, float* d_ro,
                                          float* d_rd, float* workspace, cn_stream_t stream) {
  mlp::FieldArgs a;
  CN_TRY(mlp::fused_backward_args(fmt_t, packed_t, masks, d_raw, pts, ro, rd, z, n_rays, n_samples, chunk_rows,
                                  code_index, n_codes, freqs_xyz, freqs_dir, g_code, d_pts, d_ro, d_rd, a));
  hipStream_t st = as_stream(stream);
  const int mode = pts ? mlp::kFromPts : mlp::kFromRayZ;
  const bool x3 = fmt_t == CN_FMT_BF16X3_T;
  const int wave_samples = x3 ? 32 : 16;
  // the deterministic form needs one code row (g_code: one row per workgroup) and every wave inside
  // one ray (the ray rows); otherwise the float-atomic kernel
  const bool det = workspace && n_codes == 1 && n_samples % wave_samples == 0;
  int64_t ray_off = 0, q1_off = 0, rows_off = 0;
  if (det) {
    fused_ws_layout(fmt_t, a.m, &ray_off, &q1_off, &rows_off);
    a.gc_part = workspace;
    a.ray_part = mode == mlp::kFromRayZ && (d_ro || d_rd) ? workspace + ray_off : nullptr;
    a.q1_part = d_rd ? workspace + q1_off : nullptr;
    if (!x3) a.gc_rows = workspace + rows_off;  // the fp32 kernel adds its waves' rows itself
  }
  CN_TRY(x3 ? mlp::launch_field_x3_bwd(mode, a, st) : mlp::launch_field_w16_bwd(mode, a, st));
  if (!det) return CN_OK;
  // one launch: the rays' sums; each workgroup's wave rows added in wave order (gc_rows: the fp32
  // kernel's own tail, x3 here); g_code += those rows in block order (the dW GEMMs' fixed-order
  // reduction: here for fp32, a launch of its own after this one for x3)
  float* gc_rows = workspace + rows_off;
  const int64_t ray_blocks = a.ray_part || a.q1_part ? ceil_div(n_rays, 4) : 0;
  const grad::GcFinal fin = gc_final(x3 ? nullptr : gc_rows, a.n_blocks, g_code);
  const int64_t row_blocks = x3 ? a.n_blocks : 0;
  hipLaunchKernelGGL(grad::ray_grad_reduce_kernel, dim3(static_cast<unsigned>(ray_blocks + row_blocks + fin.blocks)),
                     dim3(256), 0, st, a.ray_part, a.q1_part, ray_blocks ? n_rays : 0, n_samples, chunk_rows,
                     wave_samples, d_ro, d_rd, a.gc_part, 4, gc_rows, row_blocks, fin);
  CN_TRY(launch_status());
  return x3 ? reduce(nullptr, gc_rows, a.n_blocks, 1, mlp::kCbStride, g_code, mlp::kCbStride, st) : CN_OK;
}

// A render's two fields' deterministic eval backwards (the eval step's coarse and fine fields on the same
// rays, adding into the same d ro / d rd -- the pose's ray sink): one dX launch for both
// (field_w16_bwd2_kernel, whose workgroups also add up their waves' g_code rows) and one ray / g_code
// launch (ray_grad_reduce2_kernel), instead of two per field.  The rays' sums are added in the per-field
// calls' order with d_rd_between (the gradient that reached d rd between the two backwards) in its place,
// so d ro / d rd are bitwise those of: field 0's call, d_rd += d_rd_between, field 1's call.  Fields that
// cannot share run exactly that way.
extern "C" int cn_field_backward_fused_multi(int fmt_t, const cn_field_fused_bwd* fields, int n_fields,
                                             const float* d_rd_between, cn_stream_t stream) {
  CN_CHECK_ARG(fields && (n_fields == 1 || n_fields == 2));
  hipStream_t st = as_stream(stream);
  auto one = [&](const cn_field_fused_bwd& f) {
    return cn_field_backward_fused_ws(fmt_t, f.packed_t, f.masks, f.d_raw, f.pts, f.ro, f.rd, f.z, f.n_rays,
                                      f.n_samples, f.chunk_rows, f.code_index, f.n_codes, f.freqs_xyz, f.freqs_dir,
                                      f.g_code, f.d_pts, f.d_ro, f.d_rd, f.workspace, stream);
  };
  if (n_fields == 1) {
    CN_CHECK_ARG(!d_rd_between);
    return one(fields[0]);
  }
  const cn_field_fused_bwd &f0 = fields[0], &f1 = fields[1];
  CN_CHECK_ARG(!d_rd_between || (f0.d_rd && f0.d_rd == f1.d_rd && f0.n_rays == f1.n_rays));
  bool pair = fmt_t == CN_FMT_F32_W16_T && pair_enabled() && f0.n_rays == f1.n_rays && f0.d_ro == f1.d_ro &&
              f0.d_rd == f1.d_rd && !f0.pts && !f1.pts && !f0.d_pts && !f1.d_pts;
  for (const cn_field_fused_bwd* f : {&f0, &f1})
    pair = pair && f->workspace && f->n_codes == 1 && f->n_samples % 16 == 0 && f->ro && f->z;
  mlp::FieldArgs a[2];
  if (pair) {
    for (int k = 0; k < 2; ++k) {
      const cn_field_fused_bwd& f = fields[k];
      CN_TRY(mlp::fused_backward_args(fmt_t, f.packed_t, f.masks, f.d_raw, f.pts, f.ro, f.rd, f.z, f.n_rays,
                                      f.n_samples, f.chunk_rows, f.code_index, f.n_codes, f.freqs_xyz, f.freqs_dir,
                                      f.g_code, f.d_pts, f.d_ro, f.d_rd, a[k]));
      int64_t ray_off = 0, q1_off = 0, rows_off = 0;
      fused_ws_layout(fmt_t, a[k].m, &ray_off, &q1_off, &rows_off);
      a[k].gc_part = f.workspace;
      a[k].ray_part = (f.d_ro || f.d_rd) ? f.workspace + ray_off : nullptr;
      a[k].q1_part = f.d_rd ? f.workspace + q1_off : nullptr;
      a[k].gc_rows = f.workspace + rows_off;
    }
    const int rc = mlp::launch_field_w16_bwd2(mlp::kFromRayZ, a[0], a[1], st);
    if (rc == CN_EUNSUPPORTED) pair = false;
    else if (rc != CN_OK) return rc;
  }
  if (!pair) {
    CN_TRY(one(f0));
    if (d_rd_between) {
      const int64_t n = 3 * f0.n_rays;
      hipLaunchKernelGGL(grad::add_into_kernel, dim3(static_cast<unsigned>(ceil_div(n, 256))), dim3(256), 0, st,
                         f0.d_rd, d_rd_between, n);
      CN_TRY(launch_status());
    }
    return one(f1);
  }
  grad::RayRed rr[2];
  for (int k = 0; k < 2; ++k)
    rr[k] = grad::RayRed{a[k].ray_part, a[k].q1_part, fields[k].n_samples, fields[k].chunk_rows,
                         gc_final(a[k].gc_rows, a[k].n_blocks, fields[k].g_code), 16};
  const int64_t ray_blocks = (f0.d_ro || f0.d_rd) ? ceil_div(f0.n_rays, 4) : 0;
  hipLaunchKernelGGL(grad::ray_grad_reduce2_kernel,
                     dim3(static_cast<unsigned>(ray_blocks + rr[0].fin.blocks + rr[1].fin.blocks)), dim3(256), 0, st,
                     rr[0], rr[1], ray_blocks ? f0.n_rays : 0, d_rd_between, f0.d_ro, f0.d_rd);
  return launch_status();
}

// The code backward's first half (cn_code_bias_backward_act) of a render's fields in one launch.
extern "C" int cn_code_bias_backward_act_multi(const cn_code_act_job* jobs, int n_jobs, const float* z_s,
                                               const float* z_t, int64_t n_codes, cn_stream_t stream) {
  using namespace mlp;
  CN_CHECK_ARG(jobs && (n_jobs == 1 || n_jobs == 2) && z_s && z_t && n_codes > 0 && n_codes < (1ll << 31));
  grad::CodeDsJob j[2] = {};
  for (int k = 0; k < n_jobs; ++k) {
    CN_CHECK_ARG(jobs[k].params && jobs[k].code_act && jobs[k].g_code && jobs[k].workspace);
    for (int i = 0; i < CN_NUM_PARAMS; ++i) {
      CN_CHECK_ARG(jobs[k].params[i]);
      j[k].P.p[i] = jobs[k].params[i];
      j[k].G.p[i] = jobs[k].grads ? jobs[k].grads[i] : nullptr;
    }
    j[k].g = jobs[k].g_code;
    j[k].act = jobs[k].code_act;
    j[k].ws = jobs[k].workspace;
  }
  if (n_jobs == 1)
    hipLaunchKernelGGL(grad::code_ds_outer_kernel, dim3(static_cast<unsigned>(n_codes), grad::kCodeSlices), dim3(256), 0,
                       as_stream(stream), j[0].P, z_s, z_t, j[0].g, j[0].act, j[0].ws, j[0].G);
  else
    hipLaunchKernelGGL(grad::code_ds_outer2_kernel, dim3(static_cast<unsigned>(n_codes), 2 * grad::kCodeSlices),
                       dim3(256), 0, as_stream(stream), j[0], j[1], z_s, z_t);
  return launch_status();
}

extern "C" int64_t cn_field_backward_train_workspace_floats(int64_t m) {
  return m > 0 ? 5 * m * 256 + train_dw_ws_floats(m) : -1;
}

extern "C" int cn_field_backward_train(const float* packed_t, const float* const* params, const uint32_t* masks,
                                       const float* saved, const float* x_enc, const float* d_raw, const float* pts,
                                       const float* ro, const float* rd, const float* z, int64_t n_rays,
                                       int64_t n_samples, int64_t chunk_rows, const int64_t* code_index,
                                       int64_t n_codes, const float* freqs_xyz, const float* freqs_dir,
                                       float* workspace, float* const* grads, float* g_code, float* d_pts,
                                       float* d_ro, float* d_rd, cn_stream_t stream) {
  return cn_field_backward_train_fmt(CN_FMT_F32_W16_T, packed_t, params, masks, saved, x_enc, d_raw, pts, ro, rd, z,
                                     n_rays, n_samples, chunk_rows, code_index, n_codes, freqs_xyz, freqs_dir,
                                     workspace, grads, g_code, d_pts, d_ro, d_rd, stream);
}

// One field of a training backward: cn_field_backward_train_fmt's arguments and launch state, run in
// stages so that a render's two fields can share their launches (cn_field_backward_train_multi).
struct TrainBwd {
  bool x3 = false, wg = false, fold_code = false, jobs = false, rgb_role = false, dual_code = false, dirs = false;
  bool xenc_job = false;   // layer_xyz1's dW rides in the batched launch (CN_XENC_ROLE=1)
  int mode = 0;
  mlp::FieldArgs a = {};
  const float* saved = nullptr;
  const float* x_enc = nullptr;
  const float* d_raw = nullptr;
  float* const* grads = nullptr;
  float* g_code = nullptr;
  float* workspace = nullptr;
  const float* P[5] = {};
  Reducer red = {};
  TnBatch tb;
  grad::DirRole dir_role = {};
};

// layer_xyz1's dW reads the fp32 forward's own encodings (saved's encoding plane)
static bool train_bwd_xenc(const TrainBwd& t) { return !t.x_enc && !t.x3 && xenc_plane_enabled(); }

static int train_bwd_setup(int fmt_t, const cn_field_train_bwd& f, TrainBwd& t) {
  using namespace mlp;
  CN_CHECK_ARG(fmt_t == CN_FMT_F32_W16_T || fmt_t == CN_FMT_BF16X3_T);
  t.x3 = fmt_t == CN_FMT_BF16X3_T;
  CN_CHECK_ARG(f.packed_t && f.params && f.masks && f.saved && f.d_raw && f.rd && f.g_code && f.workspace);
  CN_CHECK_ARG(f.freqs_xyz && f.freqs_dir && f.n_rays > 0 && f.n_samples > 0 && f.chunk_rows > 0 && f.n_codes > 0);
  CN_CHECK_ARG(f.pts || (f.ro && f.z));
  CN_CHECK_ARG(!f.d_pts || f.pts);
  CN_CHECK_ARG(!f.d_ro || (f.ro && f.z && !f.pts));
  CN_CHECK_ARG(f.code_index || f.n_codes == 1 || f.n_codes == f.n_rays);
  for (int i = 0; i < CN_NUM_PARAMS; ++i) CN_CHECK_ARG(f.params[i]);
  // one code row per wave (32 samples x3, 16 samples w16)
  if (!(f.n_codes == 1 || f.n_samples % (t.x3 ? 32 : 16) == 0)) return CN_EUNSUPPORTED;
  const int64_t M = f.n_rays * f.n_samples;
  CN_CHECK_ARG(ceil_div(M, 128) <= 0x7fffffff);
  CN_CHECK_ARG(cn::aligned16(f.d_raw));  // float4 rows (include/codenerf.h)
  FieldArgs& a = t.a;
  a = {};
  a.packed = f.packed_t;
  a.code_index = f.code_index;
  a.n_codes = f.n_codes;
  a.pts = f.pts;
  a.ro = f.ro;
  a.rd = f.rd;
  a.z = f.z;
  a.n_rays = f.n_rays;
  a.n_samples = f.n_samples;
  a.chunk_rows = f.chunk_rows;
  a.m = M;
  for (int i = 0; i < 10; ++i) a.fx[i] = f.freqs_xyz[i];
  for (int i = 0; i < 4; ++i) a.fd[i] = f.freqs_dir[i];
  a.masks = const_cast<uint32_t*>(f.masks);
  a.d_raw = f.d_raw;
  a.g_code = f.g_code;
  a.d_pts = f.d_pts;
  a.d_ro = f.d_ro;
  a.d_rd = f.d_rd;
  a.dpre = f.workspace;
  t.mode = f.pts ? kFromPts : kFromRayZ;
  t.saved = f.saved;
  t.x_enc = f.x_enc;
  t.d_raw = f.d_raw;
  t.grads = f.grads;
  t.g_code = f.g_code;
  t.workspace = f.workspace;
  t.wg = f.grads && f.grads[0];
  // the bias gradients of layer_dir2 / layer_dir1 / layer_xyz1 are column sums of their dPre planes,
  // folded into the dW kernels below that stream those planes (deterministic partials), so the
  // fused backward sums none of them (a.gbias stays null).  With ONE code row (a chunk of one
  // object: every C3 step) g_code is column sums too -- of d feat (plane 2), of layer_xyz2's dPre
  // (plane 3) and of d raw -- folded the same way, so the step is deterministic in both precisions
  // (no float atomics anywhere in it) and the fused kernel skips its code sums (fp32) or leaves its
  // LDS sums unflushed (3xbf16).
  t.fold_code = t.wg && f.n_codes == 1;
  if (t.fold_code) a.g_code = nullptr;
  for (int k = 0; k < 5; ++k) t.P[k] = f.workspace + k * M * 256;
  t.red = Reducer{nullptr, f.workspace + 5 * M * 256, {}, 0};
  t.jobs = tn_jobs_enabled() && M >= 64 * 1024;
  // fc_rgb (h half): dW += d rgb^T v2 (+ g_code's rgb / sigma entries, folded, in the same pass); as the
  // batched launch's RGB role where that runs (fp32, folded code)
  t.rgb_role = t.jobs && t.fold_code && !t.x3;
  t.dual_code = t.rgb_role;  // the g_code sums also land in the bias gradients (below)
  t.dirs = t.jobs && !t.x3 && !t.x_enc && dirs_foldable(a);
  t.xenc_job = t.jobs && t.wg && train_bwd_xenc(t) && xenc_role_enabled();
  return CN_OK;
}

// After the dX launch, up to the batched dW launch: the launches before it and the jobs queued (t.tb;
// without the batched plan, the four 256 x 256 GEMMs run here one by one).
static int train_bwd_queue(TrainBwd& t, hipStream_t st) {
  using namespace mlp;
  t.red.st = st;
  const int64_t M = t.a.m;
  float* const* grads = t.grads;
  auto G = [&](int i) { return grads[i]; };
  auto B = [&](int i) { return grads[i]; };  // bias folded into this GEMM
  // biases: layer_dir2 / layer_dir1 / layer_xyz1 summed in the kernel; the others are g_code's
  // column sums (after the deferred reduction when g_code itself is folded)
  if (!t.fold_code) {
    hipLaunchKernelGGL(grad::gcode_bias_kernel, dim3(3), dim3(256), 0, st, t.g_code, t.a.n_codes, G(kBXyz2), G(kBOut),
                       G(kBRgb));
    CN_TRY(launch_status());
  }
  float* const gc_feat = t.fold_code ? t.g_code + kCbFeat : nullptr;
  float* const gc_xyz2 = t.fold_code ? t.g_code + kCbXyz2 : nullptr;
  float* const ws = nullptr;
  float* const bws = nullptr;
  Reducer* red = &t.red;
  const float* const* P = t.P;
  const float* h1 = t.saved;
  const float* h2 = t.saved + M * 256;
  const float* feat = t.saved + 2 * M * 256;
  const float* v1 = t.saved + 3 * M * 256;
  const float* v2 = t.saved + 4 * M * 256;
  const bool x3 = t.x3;
  if (t.rgb_role) {
  } else if (t.fold_code) {
    CN_TRY(rgb_dw_draw_sums(t.d_raw, v2, G(kWRgb), 512, M, t.g_code + kCbRgb, t.g_code + kCbSigma, st, red));
  } else {
    CN_TRY(gemm_tn(t.d_raw, 4, v2, 256, G(kWRgb), 512, M, 3, 256, st, x3, ws, nullptr, nullptr, red));
  }
  if (t.jobs) {
    // the four 256 x 256 layers as ONE whole-tile launch (TnBatch): layer_dir2, layer_dir1 [feat]
    // (+ its view-encoding columns by the DIRS fold where it applies), fc_out (+ sigma row),
    // layer_xyz2
    TnBatch& tb = t.tb;
    tb.n = 0;
    const float* c = tn_slot_cost();
    // with one code row the g_code entries summed here ARE the bias gradients of layer_xyz2, fc_out
    // and fc_rgb (gcode_bias_kernel's column sums over one row): the reductions add each sum to both
    // (bias2 / sig2), bitwise gcode_bias_kernel's 0 + g then b + that, and that launch is not needed
    float* const b_xyz2 = t.dual_code ? G(kBXyz2) : nullptr;
    float* const b_feat = t.dual_code ? G(kBOut) + 1 : nullptr;
    tb.p[tb.n++] = {P[0], v1, M, 0, G(kWDir2), 256, B(kBDir2), nullptr, nullptr, {}, c[0], nullptr, nullptr};
    tb.p[tb.n++] = {P[1], feat, M, t.dirs ? 2 : 0, G(kWDir1), 283, B(kBDir1), nullptr, nullptr, t.a, c[1], nullptr,
                    nullptr};
    tb.p[tb.n++] = {P[2], h2, M, 1, G(kWOut) + 512, 512, gc_feat, t.d_raw + 3, G(kWOut), {}, c[2], b_feat, nullptr};
    tb.p[tb.n++] = {P[3], h1, M, 0, G(kWXyz2), 512, gc_xyz2, nullptr, nullptr, {}, c[3], b_xyz2, nullptr};
    if (t.rgb_role)
      tb.p[tb.n++] = {t.d_raw, v2, M, 3, G(kWRgb), 512, t.g_code + kCbRgb, t.d_raw, t.g_code + kCbSigma, {}, c[4],
                      t.dual_code ? G(kBRgb) : nullptr, t.dual_code ? G(kBOut) : nullptr};
    if (t.xenc_job)   // layer_xyz1 from the forward's encoding plane (saved + 5 M 256)
      tb.p[tb.n++] = {P[4], t.saved + 5 * M * 256, M, 4, G(kWXyz1), 63, B(kBXyz1), nullptr, nullptr, {}, c[5], nullptr,
                      nullptr};
    return CN_OK;
  }
  // layer_dir2
  CN_TRY(gemm_tn(P[0], 256, v1, 256, G(kWDir2), 256, M, 256, 256, st, x3, ws, B(kBDir2), bws, red));
  // layer_dir1: [feat | dir enc]
  const int64_t dir1_budget =
      tn_ws_floats(M, 256, 256) + std::max(tn_ws_floats(M, 256, 27), enc_parts(M) * 256 * 27) + dirs_ws_floats(M);
  const int folded = x3 || t.x_enc ? CN_EUNSUPPORTED
                                   : dir1_dw_folded(P[1], feat, G(kWDir1), B(kBDir1), t.a, st, red, dir1_budget);
  if (folded != CN_OK) {
    if (folded != CN_EUNSUPPORTED) return folded;
    CN_TRY(gemm_tn(P[1], 256, feat, 256, G(kWDir1), 283, M, 256, 256, st, x3, ws, B(kBDir1), bws, red));
    if (t.x_enc)
      CN_TRY(gemm_tn(P[1], 256, t.x_enc + 63, 90, G(kWDir1) + 256, 283, M, 256, 27, st, x3, ws, nullptr, nullptr, red));
    else CN_TRY(gemm_tn_enc(1, P[1], t.a, G(kWDir1) + 256, 283, st, x3, ws, nullptr, nullptr, red));
  }
  // fc_out (h half): row 0 from d sigma, rows 1.. from d feat
  CN_TRY(gemm_tn(P[2], 256, h2, 256, G(kWOut) + 512, 512, M, 256, 256, st, x3, ws, gc_feat, bws, red, t.d_raw + 3,
                 G(kWOut)));
  // layer_xyz2 (h half)
  return gemm_tn(P[3], 256, h1, 256, G(kWXyz2), 512, M, 256, 256, st, x3, ws, gc_xyz2, bws, red);
}

// The DIRS fold's per-direction pass rides in layer_xyz1's encoding dW launch when that is a gemm_tn_enc /
// gemm_tn_xenc launch: one launch fewer per field and chunk.
static grad::DirRole* train_bwd_dir_out(TrainBwd& t) {
  return t.jobs && t.dirs && !t.x_enc && dir_in_enc_enabled() ? &t.dir_role : nullptr;
}

// After the batched launch: layer_dir1's view columns where the DIRS fold did not take them.
static int train_bwd_after_jobs(TrainBwd& t, hipStream_t st) {
  using namespace mlp;
  if (!t.jobs || t.dirs) return CN_OK;
  float* C = t.grads[kWDir1] + 256;
  if (t.x_enc) return gemm_tn(t.P[1], 256, t.x_enc + 63, 90, C, 283, t.a.m, 256, 27, st, t.x3, nullptr, nullptr, nullptr, &t.red);
  return gemm_tn_enc(1, t.P[1], t.a, C, 283, st, t.x3, nullptr, nullptr, nullptr, &t.red);
}


// layer_xyz1 (its own launch: as a role of the batched launch it ran no faster per CU -- it is compute
// work, not a bandwidth pass that could hide beside the GEMMs; r03m)
static int train_bwd_xyz1(TrainBwd& t, hipStream_t st) {
  using namespace mlp;
  float* C = t.grads[kWXyz1];
  float* bias = t.grads[kBXyz1];
  if (t.xenc_job) {   // its dW ran in the batched launch: the DIRS fold's per-direction pass alone
    if (t.dir_role.n == 0) return CN_OK;
    hipLaunchKernelGGL(grad::gemm_tn_xenc_kernel, dim3(t.dir_role.n), dim3(512), 0, st, nullptr, nullptr, 0, nullptr,
                       nullptr, 0, t.a, t.dir_role);
    return launch_status();
  }
  if (t.x_enc)
    return gemm_tn(t.P[4], 256, t.x_enc, 90, C, 63, t.a.m, 256, 63, st, t.x3, nullptr, bias, nullptr, &t.red);
  if (train_bwd_xenc(t)) return gemm_tn_xenc(t.P[4], t.saved + 5 * t.a.m * 256, t.a, C, 63, st, bias, &t.red, t.dir_role);
  return gemm_tn_enc(0, t.P[4], t.a, C, 63, st, t.x3, nullptr, bias, nullptr, &t.red, t.dir_role);
}

// Two fields' layer_xyz1 dW passes (gemm_tn_xenc each) as one gemm_tn_xenc2_kernel launch.
static int train_bwd_xyz1_pair(TrainBwd& t0, TrainBwd& t1, hipStream_t st) {
  using namespace mlp;
  grad::XencJob j[2];
  TrainBwd* t[2] = {&t0, &t1};
  unsigned blocks[2];
  if (t0.xenc_job && t1.xenc_job) {   // their dW ran in the batched launch: the DIRS passes alone
    for (int f = 0; f < 2; ++f) {
      j[f] = grad::XencJob{nullptr, nullptr, 0, nullptr, nullptr, 0, t[f]->a, t[f]->dir_role};
      blocks[f] = t[f]->dir_role.n;
    }
    if (blocks[0] + blocks[1] == 0) return CN_OK;
    hipLaunchKernelGGL(grad::gemm_tn_xenc2_kernel, dim3(blocks[0] + blocks[1]), dim3(512), 0, st, j[0], j[1], blocks[0]);
    return launch_status();
  }
  for (int f = 0; f < 2; ++f) {
    const int64_t m = t[f]->a.m, rows = enc_rows(m);
    const unsigned nb = static_cast<unsigned>(ceil_div(m, rows));
    float* bias = t[f]->grads[kBXyz1];
    j[f] = grad::XencJob{t[f]->P[4], t[f]->saved + 5 * m * 256, m, t[f]->red.take((int64_t)nb * 256 * 63),
                         bias ? t[f]->red.take((int64_t)nb * 256) : nullptr, rows, t[f]->a, t[f]->dir_role};
    blocks[f] = nb + t[f]->dir_role.n;
  }
  hipLaunchKernelGGL(grad::gemm_tn_xenc2_kernel, dim3(blocks[0] + blocks[1]), dim3(512), 0, st, j[0], j[1], blocks[0]);
  CN_TRY(launch_status());
  for (int f = 0; f < 2; ++f) {
    const unsigned nb = blocks[f] - t[f]->dir_role.n;
    CN_TRY(reduce(&t[f]->red, j[f].part, nb, 256, 63, t[f]->grads[kWXyz1], 63, st));
    if (j[f].bias_part) CN_TRY(reduce(&t[f]->red, j[f].bias_part, nb, 1, 256, t[f]->grads[kBXyz1], 256, st));
  }
  return CN_OK;
}

// After the deferred reduction: the biases formed from a folded g_code where no reduction did it.
static int train_bwd_tail(TrainBwd& t, hipStream_t st) {
  using namespace mlp;
  if (t.fold_code && !t.dual_code) {
    hipLaunchKernelGGL(grad::gcode_bias_kernel, dim3(3), dim3(256), 0, st, t.g_code, t.a.n_codes, t.grads[kBXyz2],
                       t.grads[kBOut], t.grads[kBRgb]);
    CN_TRY(launch_status());
  }
  return CN_OK;
}

static int train_bwd_dx(TrainBwd& t, hipStream_t st) {
  return t.x3 ? mlp::launch_field_x3_bwd(t.mode, t.a, st) : mlp::launch_field_w16_bwd(t.mode, t.a, st);
}

static int train_bwd_one(TrainBwd& t, hipStream_t st) {
  CN_TRY(train_bwd_dx(t, st));
  if (!t.wg) return CN_OK;
  CN_TRY(train_bwd_queue(t, st));
  if (t.jobs) CN_TRY(tn_batch_launch(t.tb, t.x3, st, &t.red, train_bwd_dir_out(t)));
  CN_TRY(train_bwd_after_jobs(t, st));
  CN_TRY(train_bwd_xyz1(t, st));
  CN_TRY(t.red.flush());
  return train_bwd_tail(t, st);
}

extern "C" int cn_field_backward_train_fmt(int fmt_t, const float* packed_t, const float* const* params,
                                           const uint32_t* masks, const float* saved, const float* x_enc,
                                           const float* d_raw, const float* pts, const float* ro, const float* rd,
                                           const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                                           const int64_t* code_index, int64_t n_codes, const float* freqs_xyz,
                                           const float* freqs_dir, float* workspace, float* const* grads,
                                           float* g_code, float* d_pts, float* d_ro, float* d_rd,
                                           cn_stream_t stream) {
  const cn_field_train_bwd f{packed_t, params, masks, saved, x_enc, d_raw, pts, ro, rd, z, n_rays, n_samples, chunk_rows,
                             code_index, n_codes, freqs_xyz, freqs_dir, workspace, grads, g_code, d_pts, d_ro, d_rd};
  return cn_field_backward_train_multi(fmt_t, &f, 1, stream);
}

// A render's fields in shared launches: both fields' dX chains in one field_w16_bwd2_kernel launch, their
// batched dW GEMMs in one gemm_tn256_jobs_kernel launch, their layer_xyz1 passes in one
// gemm_tn_xenc2_kernel launch and their deferred sums in one reduction launch -- every launch running
// each field's workgroups exactly as its own launch would, so every gradient is bitwise that of the
// per-field calls.  Pairs that cannot share (3xbf16, points input, small chunks without the batched dW
// plan, x_enc given, different kernel forms) run one after the other.
extern "C" int cn_field_backward_train_multi(int fmt_t, const cn_field_train_bwd* fields, int n_fields,
                                             cn_stream_t stream) {
  CN_CHECK_ARG(fields && (n_fields == 1 || n_fields == 2));
  hipStream_t st = as_stream(stream);
  TrainBwd t[2];
  for (int k = 0; k < n_fields; ++k) CN_TRY(train_bwd_setup(fmt_t, fields[k], t[k]));
  bool pair = n_fields == 2 && !t[0].x3 && pair_enabled();
  for (int k = 0; pair && k < 2; ++k)
    pair = t[k].wg && t[k].jobs && t[k].mode == mlp::kFromRayZ && train_bwd_xenc(t[k]);
  if (pair) {
    const int rc = mlp::launch_field_w16_bwd2(mlp::kFromRayZ, t[0].a, t[1].a, st);
    if (rc == CN_EUNSUPPORTED) pair = false;
    else if (rc != CN_OK) return rc;
  }
  if (!pair) {
    for (int k = 0; k < n_fields; ++k) CN_TRY(train_bwd_one(t[k], st));
    return CN_OK;
  }
  CN_TRY(train_bwd_queue(t[0], st));
  CN_TRY(train_bwd_queue(t[1], st));
  CN_TRY(tn_batch_launch2(t[0].tb, &t[0].red, train_bwd_dir_out(t[0]), t[1].tb, &t[1].red, train_bwd_dir_out(t[1]),
                          false, st));
  CN_TRY(train_bwd_after_jobs(t[0], st));
  CN_TRY(train_bwd_after_jobs(t[1], st));
  CN_TRY(train_bwd_xyz1_pair(t[0], t[1], st));
  CN_TRY(flush2(t[0].red, t[1].red));
  CN_TRY(train_bwd_tail(t[0], st));
  return train_bwd_tail(t[1], st);
}
