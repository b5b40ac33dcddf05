// Shared helpers for the gfx950 kernels of libcodenerf_hip.so.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "codenerf.h"

#define CN_CHECK_ARG(cond)          \
  do {                              \
    if (!(cond)) return CN_EINVAL;  \
  } while (0)

namespace cn {

constexpr int kWave = 64;

inline hipStream_t as_stream(cn_stream_t s) { return reinterpret_cast<hipStream_t>(s); }

// Launch status: hipGetLastError after a launch (sticky errors surface too).
inline int launch_status() {
  hipError_t e = hipGetLastError();
  return e == hipSuccess ? CN_OK : static_cast<int>(e);
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Grid for a grid-stride elementwise kernel: at most 256 CUs x 8 blocks.
// NULL counts as aligned (an optional output).
inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

inline unsigned elementwise_grid(int64_t n, int block) {
  int64_t g = ceil_div(n, block);
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return static_cast<unsigned>(g);
}

// Exact fp32 a*b then +c with two roundings (never contracted into an FMA):
// matches torch's separate mul and add kernels bit for bit.
__device__ __forceinline__ float mul_add_rn(float a, float b, float c) {
  return __fadd_rn(__fmul_rn(a, b), c);
}

// torch.nn.functional.softplus(x) with beta 1, threshold 20 (volumetric_render.py:32):
// log1p(e), e = expf(x), as log(u) + (e - (u - 1)) / u with u = fl(1 + e) -- the rounding of u
// compensated to first order -- on the hardware log2 (v_log_f32) instead of the libm log1pf, whose
// extended-precision path was ~60 of volume_render's ~220 VALU instructions per sample.
__device__ __forceinline__ float softplus20(float x) {
  if (x > 20.0f) return x;
  const float e = expf(x);
  const float u = 1.0f + e;
  const float c = (e - (u - 1.0f)) * __builtin_amdgcn_rcpf(u);
  return fmaf(__builtin_amdgcn_logf(u), 0.693147180559945309f, c);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.0f / (1.0f + expf(-x)); }

// sigmoid on the hardware exp2 / reciprocal (v_exp_f32, v_rcp_f32: 1 ulp each) instead of the
// libm expf and the IEEE division (~25 instructions).  The argument rounding of -x log2(e) moves
// e^-x by <= |x| 2^-24 relative, so the result stays within ~2e-7 of the exact sigmoid
// (saturated where |x| is large); volume_render's colours and their gradients use it.
__device__ __forceinline__ float sigmoid_hw(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.44269504088896341f));
}

}  // namespace cn
