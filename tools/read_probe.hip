// HBM read-rate probe: what a plain streaming read reaches on this box, to set beside the dW kernels'
// input streams (the encoding dW's "box read rate").
//
// Build:  hipcc --offload-arch=gfx950 -O3 tools/read_probe.hip -o tools/bin/read_probe
// Run:    tools/bin/read_probe        (prints one JSON line per kernel and size)
//
// Each kernel reads a 2 GiB (or 512 MiB, the encoding dW's per-call input size) buffer once per launch
// and writes one float per workgroup (so nothing is eliminated); median of 20 launches by HIP events.
//   f4_grid    one float4 per lane per iteration, a grid covering the buffer once (4 loads per lane in
//              flight: unrolled), 256-thread workgroups, 8 per CU
//   f4_stride  the same loads in a grid-stride loop over a persistent grid of 4 workgroups per CU
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void f4_grid(const f32x4* __restrict__ in, long n_vec, float* __restrict__ out) {
  const long base = (long(blockIdx.x) * 256 + threadIdx.x) * 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const long i = base + k;  // 4 consecutive float4 per lane: 64 B per lane, 16 KiB per workgroup
    if (i < n_vec) acc += __builtin_nontemporal_load(in + i);
  }
  __shared__ float red[256];
  red[threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int t = 0; t < 256; t += 64) s += red[t];
    out[blockIdx.x] = s;
  }
}

__global__ __launch_bounds__(256) void f4_stride(const f32x4* __restrict__ in, long n_vec, float* __restrict__ out) {
  const long stride = long(gridDim.x) * 256;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (long i = long(blockIdx.x) * 256 + threadIdx.x; i < n_vec; i += 4 * stride) {
    f32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const long j = i + k * stride;
      v[k] = j < n_vec ? __builtin_nontemporal_load(in + j) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) acc += v[k];
  }
  __shared__ float red[256];
  red[threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
  __syncthreads();
  if (threadIdx.x == 0) {
    float s = 0.f;
    for (int t = 0; t < 256; t += 64) s += red[t];
    out[blockIdx.x] = s;
  }
}

int main() {
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const long max_bytes = 2l << 30;
  f32x4* buf = nullptr;
  float* out = nullptr;
  if (hipMalloc(&buf, max_bytes) != hipSuccess || hipMalloc(&out, 64 << 20) != hipSuccess) {
    std::printf("{\"error\": \"hipMalloc\"}\n");
    return 1;
  }
  hipMemset(buf, 0, max_bytes);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (long bytes : {512l << 20, max_bytes}) {
    const long n_vec = bytes / 16;
    for (int kind = 0; kind < 2; ++kind) {
      const unsigned grid = kind == 0 ? static_cast<unsigned>((n_vec + 1023) / 1024) : static_cast<unsigned>(4 * cus);
      std::vector<float> ms;
      for (int it = 0; it < 23; ++it) {
        hipEventRecord(e0);
        if (kind == 0) hipLaunchKernelGGL(f4_grid, dim3(grid), dim3(256), 0, 0, buf, n_vec, out);
        else hipLaunchKernelGGL(f4_stride, dim3(grid), dim3(256), 0, 0, buf, n_vec, out);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float t = 0.f;
        hipEventElapsedTime(&t, e0, e1);
        if (it >= 3) ms.push_back(t);
      }
      std::sort(ms.begin(), ms.end());
      const double med = ms[ms.size() / 2];
      std::printf("{\"kernel\": \"%s\", \"bytes\": %ld, \"median_ms\": %.4f, \"min_ms\": %.4f, \"TBps\": %.3f, "
                  "\"TBps_best\": %.3f}\n",
                  kind == 0 ? "f4_grid" : "f4_stride", bytes, med, ms.front(), bytes / (med * 1e-3) / 1e12,
                  bytes / (ms.front() * 1e-3) / 1e12);
    }
  }
  hipFree(buf);
  hipFree(out);
  return 0;
}
