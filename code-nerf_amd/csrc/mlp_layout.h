// Packed-weight layout of the CodeNeRF MLP for the fp32 MFMA field kernel.
//
// The field kernel computes every layer as D = W * X^T with
// v_mfma_f32_32x32x2_f32: A = a 32-row block of W (lane l holds
// W[32*ob + (l & 31)][k(t, l >> 5)]), B = the activations (lane l holds sample
// l & 31 at input k(t, l >> 5)), D = 32 output features x 32 samples with the
// feature in registers: row(reg, lane) = (reg & 3) + 8*(reg >> 2) + 4*(lane >> 5).
// Because D is already in B's lane layout, a layer's output feeds the next
// layer's k-steps straight from registers; the only price is the permuted k
// order below, which the packing applies to W once.
//
// A fragment (layer, t, lane, ob) lives at off[layer] + (t*64 + lane)*nbp + ob,
// so a lane's A values for one k-step are nbp consecutive floats (ds_read_b128).
#pragma once

namespace cn {
namespace mlp {

constexpr int kHidden = 256;
constexpr int kCode = 256;
constexpr int kDimXyz = 63;
constexpr int kDimDir = 27;

enum Layer { kXyz1 = 0, kXyz2 = 1, kOut = 2, kDir1 = 3, kDir2 = 4, kRgb = 5, kNumLayers = 6 };

// k-steps (2 inputs each), real and padded 32-row output blocks per layer.
constexpr int kSteps[kNumLayers] = {32, 128, 128, 128 + 14, 128, 128};
constexpr int kBlocks[kNumLayers] = {8, 8, 9, 8, 8, 1};
constexpr int kBlocksPad[kNumLayers] = {8, 8, 12, 8, 8, 1};

constexpr int layer_floats(int l) { return kSteps[l] * 64 * kBlocksPad[l]; }
constexpr int layer_offset(int l) { return l == 0 ? 0 : layer_offset(l - 1) + layer_floats(l - 1); }

// Constant biases follow the fragments: b_xyz1, b_dir1, b_dir2 (256 each).
constexpr int kBiasXyz1 = layer_offset(kNumLayers);
constexpr int kBiasDir1 = kBiasXyz1 + 256;
constexpr int kBiasDir2 = kBiasDir1 + 256;
constexpr int kPackedFloats = kBiasDir2 + 256;

// Per-code bias row (CN_CODE_BIAS_STRIDE floats): the code halves of
// layer_xyz2 / fc_out / fc_rgb folded with their biases.
constexpr int kCbXyz2 = 0;     // 256
constexpr int kCbFeat = 256;   // 256 = fc_out rows 1..256
constexpr int kCbSigma = 512;  // 1   = fc_out row 0
constexpr int kCbRgb = 513;    // 3
constexpr int kCbStride = 520;

// Output feature held by accumulator register `reg` of block `ob` in lane half h.
__host__ __device__ constexpr int acc_row(int ob, int reg, int h) {
  return 32 * ob + (reg & 3) + 8 * (reg >> 2) + 4 * h;
}

// Input feature consumed at k-step t by lane half h when the input is a
// previous layer's accumulator (256 wide): k-step t = register (t & 15) of block t >> 4.
__host__ __device__ constexpr int k_from_acc(int t, int h) { return acc_row(t >> 4, t & 15, h); }

// Positional-encoding feature order (position_embed.py:44-53):
//   index d -> x_d; 3 + 6k + d -> sin(f_k x_d); 6 + 6k + d -> cos(f_k x_d).
// Each lane half computes sin AND cos of its own (k, d) pairs p = 2q + h, so
// one sincosf per pair per lane: k-steps [0, P) sines, [P, 2P) cosines, then
// the raw inputs, then zero padding.  P = 15 pairs (xyz, L=10) or 6 (dir, L=4).
__host__ __device__ constexpr int k_from_enc(int t, int h, int pairs_per_half) {
  const int P = pairs_per_half;
  if (t < 2 * P) {
    const int q = t < P ? t : t - P;
    const int p = 2 * q + h;
    const int k = p / 3, d = p % 3;
    return (t < P ? 3 : 6) + 6 * k + d;
  }
  const int raw = 2 * (t - 2 * P) + h;  // 0, 1 | 2, pad
  return raw < 3 ? (raw == 1 ? 2 : (raw == 2 ? 1 : 0)) : -1;
}

}  // namespace mlp
}  // namespace cn
