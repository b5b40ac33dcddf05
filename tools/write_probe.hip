// Store-shape probe for the f32 field kernel's raw output (tools/write_probe.sh).
//
// field_w16_kernel stores its (samples, 4) fp32 raw output as ONE float4 per sample from the
// 16 lanes of a wave whose accumulator holds features 0..3 (256 contiguous bytes per wave
// instruction); rocprofv3's WRITE_SIZE reads 1.94x those bytes.  This probe writes the same
// 2 GiB with three shapes and times each (hipEvents) so the counter can be compared with what
// the store rate says HBM actually did:
//   lanes16   one float4 from lanes 0..15 per wave instruction (the kernel's shape)
//   lanes16x4 the same shape, four instructions per wave covering 1 KiB
//   lanes64   one float4 from all 64 lanes (the guide's calibrated shape)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void lanes16(f32x4* out, long n_vec) {
  const long wave = (long(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long i = wave * 16 + lane;
  if (lane < 16 && i < n_vec) out[i] = f32x4{1.f, 2.f, 3.f, float(lane)};
}

__global__ __launch_bounds__(256) void lanes16x4(f32x4* out, long n_vec) {
  const long wave = (long(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (lane < 16) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long i = wave * 64 + k * 16 + lane;
      if (i < n_vec) out[i] = f32x4{1.f, 2.f, 3.f, float(k)};
    }
  }
}

__global__ __launch_bounds__(256) void lanes64(f32x4* out, long n_vec) {
  const long wave = (long(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  const long i = wave * 64 + lane;
  if (i < n_vec) out[i] = f32x4{1.f, 2.f, 3.f, float(lane)};
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
  const long bytes = 2L << 30, n_vec = bytes / 16;
  f32x4* out;
  CHECK(hipMalloc(&out, bytes));
  hipEvent_t a, b;
  CHECK(hipEventCreate(&a));
  CHECK(hipEventCreate(&b));
  const int reps = 5;
  struct { const char* name; long vec_per_wave; int which; } shapes[] = {
      {"lanes16", 16, 0}, {"lanes16x4", 64, 1}, {"lanes64", 64, 2}};
  for (auto& s : shapes) {
    const long waves = n_vec / s.vec_per_wave;
    const long blocks = waves / 4;  // 4 waves per 256-thread block, exact for 2 GiB
    float best = 1e30f;
    for (int r = 0; r < reps + 1; ++r) {
      CHECK(hipEventRecord(a));
      if (s.which == 0) lanes16<<<blocks, 256>>>(out, n_vec);
      else if (s.which == 1) lanes16x4<<<blocks, 256>>>(out, n_vec);
      else lanes64<<<blocks, 256>>>(out, n_vec);
      CHECK(hipGetLastError());
      CHECK(hipEventRecord(b));
      CHECK(hipEventSynchronize(b));
      float ms;
      CHECK(hipEventElapsedTime(&ms, a, b));
      if (r > 0 && ms < best) best = ms;  // launch 0 is warm-up
    }
    printf("%-10s %8.3f ms  %6.2f TB/s  (%ld MiB written per launch)\n", s.name, best,
           bytes / (best * 1e-3) / 1e12, bytes >> 20);
  }
  CHECK(hipFree(out));
  return 0;
}
