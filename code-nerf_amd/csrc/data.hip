// SRN views resident in HBM: the dataset's images are decoded
// once into one uint8 (n_views, h, w, c) tensor in device memory (SRN cars train: 122,900
// 96x96 RGBA views = 4.5 GB of the 288 GB) and each training / validation batch is
// unpacked on the device instead of re-reading PNGs (view_synthesis/datasets/dataset.py:60-94).
#include "cn_common.h"

namespace {

// dataset.py:77-80 per pixel of the batch's views: color = u8 / 255.0 (numpy float64, then
// float32: the quotient rounded once), mask = 1.0 where every channel != 255 else 0.0.
// One thread per pixel; a 4-channel pixel is one 32-bit load.
__global__ void srn_unpack_kernel(const uint8_t* __restrict__ images, int64_t n_views, int64_t hw, int64_t c,
                                  const int64_t* __restrict__ index, int64_t batch, float* __restrict__ color,
                                  float* __restrict__ mask) {
  const int64_t n = batch * hw;
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n; q += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = q / hw, p = q - b * hw;
    const int64_t v = index[b];
    const bool ok = v >= 0 && v < n_views;
    const uint8_t* px = images + ((ok ? v : 0) * hw + p) * c;
    bool all_not_white = true;
    for (int64_t k = 0; k < c; ++k) {
      const uint8_t u = px[k];
      all_not_white = all_not_white && (u != 255);
      if (color) color[q * c + k] = ok ? static_cast<float>(static_cast<double>(u) / 255.0) : __int_as_float(0x7fc00000);
    }
    if (mask) mask[q] = ok ? (all_not_white ? 1.0f : 0.0f) : __int_as_float(0x7fc00000);
  }
}

}  // namespace

extern "C" int cn_srn_unpack(const uint8_t* images, int64_t n_views, int64_t hw, int64_t channels,
                             const int64_t* view_index, int64_t batch, float* color, float* mask,
                             cn_stream_t stream) {
  CN_CHECK_ARG(images && view_index && n_views > 0 && hw > 0 && channels > 0 && channels <= 4 && batch > 0);
  CN_CHECK_ARG(color || mask);
  const int64_t n = batch * hw;
  hipLaunchKernelGGL(srn_unpack_kernel, dim3(cn::elementwise_grid(n, 256)), dim3(256), 0, cn::as_stream(stream),
                     images, n_views, hw, channels, view_index, batch, color, mask);
  return cn::launch_status();
}
