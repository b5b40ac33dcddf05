// Positional encoding: PositionalEmbedder.embed (view_synthesis/nerf/position_embed.py:35-53).
//
// out row = [x (if include_input), sin(f_0 x), cos(f_0 x), sin(f_1 x), ...],
// each block d wide.  One lane per output element: consecutive lanes write
// consecutive floats of a row (coalesced stores; the d inputs of a row are
// re-read from L1).  Accurate sinf/cosf (full range reduction): x*2^k is exact
// in fp32 and the arguments reach 2^(L-1)|x|, where __sinf is far off.
#include "cn_common.h"

namespace {

struct Freqs {
  float f[32];
};

__global__ void posenc_kernel(const float* __restrict__ x, int64_t m, int d, Freqs F, int nf,
                              int inc, float* __restrict__ out) {
  const int width = d * (inc + 2 * nf);
  const int64_t n = m * width;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n;
       q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = q / width;
    const int c = static_cast<int>(q - row * width);
    const int blk = c / d, comp = c - blk * d;
    const float v = x[row * d + comp];
    float o;
    if (inc && blk == 0) {
      o = v;
    } else {
      const int b = blk - inc;
      const float arg = __fmul_rn(v, F.f[b >> 1]);
      o = (b & 1) ? cosf(arg) : sinf(arg);
    }
    out[q] = o;
  }
}

}  // namespace

extern "C" int cn_posenc(const float* x, int64_t m, int64_t d, const float* freqs,
                         int64_t num_freq, int include_input, float* out, cn_stream_t stream) {
  CN_CHECK_ARG(x && out && m > 0 && d > 0 && d <= 4096 && num_freq >= 0 && num_freq <= 32);
  CN_CHECK_ARG(num_freq == 0 || freqs);
  CN_CHECK_ARG(include_input || num_freq > 0);
  Freqs F = {};
  for (int i = 0; i < num_freq; ++i) F.f[i] = freqs[i];
  const int64_t n = m * d * ((include_input ? 1 : 0) + 2 * num_freq);
  hipLaunchKernelGGL(posenc_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0,
                     cn::as_stream(stream), x, m, static_cast<int>(d), F,
                     static_cast<int>(num_freq), include_input ? 1 : 0, out);
  return cn::launch_status();
}
