// Store-shape probe for the field kernels' HBM writes (WRITE_SIZE vs bytes written).
//
// Build:  hipcc --offload-arch=gfx950 -O3 tools/write_probe.hip -o tools/bin/write_probe
// Run:    rocprofv3 --kernel-trace --pmc WRITE_SIZE -- tools/bin/write_probe   (one pass per counter)
//
// Every kernel writes the same 2 GiB once per launch; the host prints each launch's time so the
// counter can be compared with what the store rate says HBM did.
//   lanes16     one float4 from lanes 0..15 per wave instruction (the raw output's shape)
//   lanes64     one float4 from all 64 lanes (the guide's calibrated shape)
//   plane_wb    the training planes' shape (csrc/mlp_f32.hip store_plane): a wave owns 16 rows of
//               1 KiB; instruction ob writes 16 B of lane (i = lane & 15, g = lane >> 4) at row i,
//               byte 16 g + 64 ob -- 16 rows x 64 B per instruction, 16 instructions per row block;
//               buffer stores with the default cache policy
//   plane_nt    the same with the non-temporal policy the kernels use (cpol 2)
//   plane_nt_4  the same, the 16 instructions issued 4 at a time between busy-work (the kernels
//               spread them over k-steps 4..7 of the next chunk)
//   rows_nt     one contiguous 1 KiB row per 64 lanes per instruction, NT (the alternative layout:
//               a wave writes whole rows)
//   lines_nt    the planes' layout written as whole 128-B lines: instruction k of a pair writes rows
//               8 h .. 8 h + 7 x bytes 128 k .. 128 k + 127 (lane i = lane & 15 < 8 its own block 2 k,
//               lane i >= 8 block 2 k + 1 of row i - 8: one row_ror:8 DPP exchange), NT
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void lanes16(f32x4* out, long n_vec) {
  const long wave = (long(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long i = wave * 16 + lane;
  if (lane < 16 && i < n_vec) out[i] = f32x4{1.f, 2.f, 3.f, float(lane)};
}

__global__ __launch_bounds__(256) void lanes64(f32x4* out, long n_vec) {
  const long wave = (long(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long i = wave * 64 + lane;
  if (i < n_vec) out[i] = f32x4{1.f, 2.f, 3.f, float(lane)};
}

// one wave = one 16 KiB block (16 rows x 1 KiB); a 256-thread block = 4 waves = 64 KiB
template <int CPOL, int SPREAD>
__global__ __launch_bounds__(256) void plane(float* out, long n_blocks) {
  const long wave = (long(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  if (wave >= n_blocks) return;
  const int lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + wave * 4096, 0, 16384, 0x00020000);
  const unsigned off = static_cast<unsigned>(lane & 15) * 1024u + 16u * (lane >> 4);
  float x = float(lane);
#pragma unroll
  for (int ob = 0; ob < 16; ++ob) {
    if (SPREAD && ob % 4 == 0 && ob) {
#pragma unroll
      for (int k = 0; k < 64; ++k) x = __builtin_fmaf(x, 1.0001f, 0.5f);   // busy-work between groups
    }
    const f32x4 v = f32x4{x, 2.f, 3.f, float(ob)};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, off + 64u * ob, 0, CPOL);
  }
}

// lines_nt: the DPP-exchanged form of the plane store (16 instructions per 16-row block as plane<>)
__global__ __launch_bounds__(256) void lines(float* out, long n_blocks) {
  const long wave = (long(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  if (wave >= n_blocks) return;
  const int lane = threadIdx.x & 63, i = lane & 15, g = lane >> 4;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + wave * 4096, 0, 16384, 0x00020000);
  const unsigned off = static_cast<unsigned>(i & 7) * 1024u + 64u * (i >> 3) + 16u * g;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float x = __builtin_amdgcn_update_dpp(0.0f, float(lane + k), 0x128, 0xf, 0xf, false);  // row_ror:8
    const f32x4 a = f32x4{x, 2.f, 3.f, float(k)};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a), r, off + 128u * k, 0, 2);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, a), r, off + 8192u + 128u * k, 0, 2);
  }
}

template <int CPOL>
__global__ __launch_bounds__(256) void rows(float* out, long n_blocks) {
  const long wave = (long(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  if (wave >= n_blocks) return;
  const int lane = threadIdx.x & 63;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out + wave * 4096, 0, 16384, 0x00020000);
#pragma unroll
  for (int row = 0; row < 16; ++row) {
    const f32x4 v = f32x4{float(lane), 2.f, 3.f, float(row)};
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), r, row * 1024u + 16u * lane, 0, CPOL);
  }
}

#define CHECK(x)                                                               \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

int main() {
  const long bytes = 2L << 30, n_vec = bytes / 16, n_blk = bytes / 16384;
  float* out;
  CHECK(hipMalloc(&out, bytes));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int reps = 3;
  const char* names[] = {"lanes16", "lanes64", "plane_wb", "plane_nt", "plane_nt_4", "rows_nt", "rows_wb", "lines_nt"};
  for (int which = 0; which < 8; ++which) {
    float best = 1e30f;
    for (int rep = 0; rep < reps + 1; ++rep) {
      CHECK(hipEventRecord(a));
      switch (which) {
        case 0: lanes16<<<n_vec / 16 / 4, 256>>>(reinterpret_cast<f32x4*>(out), n_vec); break;
        case 1: lanes64<<<n_vec / 64 / 4, 256>>>(reinterpret_cast<f32x4*>(out), n_vec); break;
        case 2: plane<0, 0><<<n_blk / 4, 256>>>(out, n_blk); break;
        case 3: plane<2, 0><<<n_blk / 4, 256>>>(out, n_blk); break;
        case 4: plane<2, 1><<<n_blk / 4, 256>>>(out, n_blk); break;
        case 5: rows<2><<<n_blk / 4, 256>>>(out, n_blk); break;
        case 6: rows<0><<<n_blk / 4, 256>>>(out, n_blk); break;
        default: lines<<<n_blk / 4, 256>>>(out, n_blk); break;
      }
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms;
      CHECK(hipEventElapsedTime(&ms, a, b));
      if (rep > 0 && ms < best) best = ms;  // launch 0 is warm-up
    }
    printf("%-11s %8.3f ms  %6.2f TB/s  (%ld MiB written per launch, %d launches)\n", names[which], best,
           bytes / (best * 1e-3) / 1e12, bytes >> 20, reps + 1);
  }
  CHECK(hipFree(out));
  return 0;
}
