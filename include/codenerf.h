/*
 * codenerf.h — C ABI of libcodenerf_hip.so, the MI355X (gfx950) Code-NeRF renderer.
 *
 * Drop-in boundary for the ray-marching hot path of akashsharma02/code-nerf.
 * The reference is pure Python (PyTorch 1.8) with no FFI; each entry point
 * below replaces one of its tensor-in/tensor-out functions (cited file:line,
 * relative to the reference root).  The Python mirror (code-nerf_amd/codenerf)
 * binds these with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions (all entry points):
 *   - Pointers are DEVICE pointers to contiguous row-major fp32 (int64 for
 *     indices) unless marked "host".  The caller owns every buffer; nothing
 *     is allocated, freed or retained across calls.
 *   - Work is enqueued on `stream` (a hipStream_t; NULL = legacy default
 *     stream) and is asynchronous; no entry point synchronises the device,
 *     so all of them can be captured into a hipGraph.
 *   - Return value: 0 on success; a negative CN_E* for an argument error
 *     (nothing launched); a positive hipError_t from the launch.
 *   - Reentrant; one process per GPU (mirrors mp.spawn in train.py/eval.py).
 */
#ifndef CODENERF_H_
#define CODENERF_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* cn_stream_t; /* hipStream_t */

#define CN_OK 0
#define CN_EINVAL (-1)       /* bad size / null pointer / out-of-range argument */
#define CN_EUNSUPPORTED (-2) /* configuration outside what the kernels implement */

/* Architecture the fused MLP kernels implement (CodeNeRFModel, model.py:123-158,
 * as every runnable config instantiates it: hidden_size 256, code sizes 256,
 * num_encoding_fn_xyz 10, num_encoding_fn_dir 4, include_input_* True). */
#define CN_HIDDEN 256
#define CN_CODE 256
#define CN_DIM_XYZ 63
#define CN_DIM_DIR 27
#define CN_NUM_PARAMS 18        /* weight/bias tensors of CodeNeRFModel, state_dict order */
#define CN_CODE_BIAS_STRIDE 520 /* floats per code row: c_xyz2[256] c_feat[256] c_sigma c_rgb[3] pad[4] */

/* Packed-weight formats of the field kernel (cn_mlp_pack):
 *   CN_FMT_F32    fp32 fragments, v_mfma_f32_32x32x2_f32 (exact f32 products);
 *   CN_FMT_BF16X3 bf16 hi/lo fragments, Wh.Xh + Wh.Xl + Wl.Xh on
 *                 v_mfma_f32_32x32x16_bf16 with fp32 accumulation (~2^-17 relative
 *                 per product; 5.3x the fp32 MFMA rate). */
#define CN_FMT_F32 0
#define CN_FMT_BF16X3 1
/*   CN_FMT_BF16X3_T  the transposed 3xbf16 pack the fused backward streams
 *                    (cn_field_backward_x3); not a forward format. */
#define CN_FMT_BF16X3_T 2
/*   CN_FMT_F32_W16   fp32 fragments for v_mfma_f32_16x16x4_f32 at two waves per SIMD
 *                    (the inference kernel of precision "f32"; exact f32 products as
 *                    CN_FMT_F32, whose kernel remains the training forward). */
#define CN_FMT_F32_W16 3
/*   CN_FMT_F32_W16_T the transposed fp32 pack the fused fp32 backward streams
 *                    (cn_field_backward_fused); not a forward format. */
#define CN_FMT_F32_W16_T 4
/*   CN_FMT_BF16X3_W16 the same 3-product bf16 split as CN_FMT_BF16X3 on
 *                    v_mfma_f32_16x16x32_bf16 at two waves per SIMD (16 samples per wave;
 *                    cn_mlp_forward / cn_radiance_field only -- the mask-writing forward and
 *                    the fused backward take CN_FMT_BF16X3 / _T). */
#define CN_FMT_BF16X3_W16 5

const char* cn_version(void);
const char* cn_error_string(int code);

/* --- Rays: view_synthesis/nerf/ray_sampler.py -------------------------- */

/* RaySampler.__init__ directions, ray_sampler.py:35-51 (Q3: no +0.5).
 * dirs: (height, width, 3). */
int cn_ray_directions(int64_t height, int64_t width, float focal, float cx, float cy,
                      float* dirs, cn_stream_t stream);

/* RaySampler.get_bundle, ray_sampler.py:84-99: rd = R * d, ro = t.
 * dirs: (hw, 3); c2w: (batch, 4, 4); ro, rd: (batch, hw, 3). */
int cn_ray_bundle(const float* dirs, int64_t hw, const float* c2w, int64_t batch,
                  float* ro, float* rd, cn_stream_t stream);

/* RaySampler.sample gather, ray_sampler.py:77-80 (indices from the host RNG).
 * ro, rd: (batch, hw, 3); select_inds: (batch, sample_size) int64;
 * ro_out, rd_out: (batch*sample_size, 3). */
int cn_gather_rays(const float* ro, const float* rd, int64_t batch, int64_t hw,
                   const int64_t* select_inds, int64_t sample_size, float* ro_out,
                   float* rd_out, cn_stream_t stream);

/* --- Fused pose path (eval.py:22-38 pose_spherical + ray_sampler.py:53-99 sample
 *     + eval.py:147-148 target gather) ------------------- */

/* The pose from theta, phi, rho (batch) each (eval.py:33-37), or given as c2w (batch, 4, 4)
 * when theta is NULL, then ONLY the selected rays:
 * select_inds (batch, sample_size) int64 (the sample gather, ray_sampler.py:77-80), or NULL
 * with sample_size == hw for the whole bundle (get_bundle).  dirs: (hw, 3) from
 * cn_ray_directions.  ro, rd: (batch*sample_size, 3); c2w_out (batch, 4, 4) or NULL;
 * target (batch, hw, target_channels) gathered into target_out (batch*sample_size,
 * target_channels) when both are non-NULL.  Out-of-range indices give NaN rows. */
int cn_pose_rays(const float* theta, const float* phi, const float* rho, const float* c2w, int64_t batch,
                 const float* dirs,
                 int64_t hw, const int64_t* select_inds, int64_t sample_size, const float* target,
                 int64_t target_channels, float* c2w_out, float* ro, float* rd, float* target_out,
                 cn_stream_t stream);

/* Backward of cn_pose_rays from g_ro / g_rd (batch*sample_size, 3; either may be NULL, not
 * both): d_c2w (batch, 4, 4) WRITTEN (rows 0..2; row 3 zero) and/or d_theta, d_phi, d_rho
 * (batch) WRITTEN (any may be NULL) through the analytic d c2w / d(theta, phi, rho). */
int cn_pose_rays_backward(const float* theta, const float* phi, const float* rho, int64_t batch,
                          const float* dirs, int64_t hw, const int64_t* select_inds, int64_t sample_size,
                          const float* g_ro, const float* g_rd, float* d_c2w, float* d_theta, float* d_phi,
                          float* d_rho, cn_stream_t stream);

/* Device replacement of ray_sampler.py:41-42's np.random.permutation(hw)[:sample_size]
 * per image (throughput mode; same distribution, not the same draws): Philox4x32-10 keyed
 * by seed, counter (pixel, image, offset).  select_inds: (batch, sample_size) int64.
 * hw <= 16384 (one workgroup sorts an image's keys in LDS), else CN_EUNSUPPORTED. */
int cn_random_select(int64_t batch, int64_t hw, int64_t sample_size, uint64_t seed, uint64_t offset,
                     int64_t* select_inds, cn_stream_t stream);

/* The eval pose metric, eval.py:161-162: twist = SE3.Log(inverse(gt) @ cam)
 * (utils/lieutils.py:709-718) and err = ||twist||_2 per pose.  gt_c2w, cam_c2w: (batch, 4, 4);
 * twist (batch, 6) = (w, v) and/or err (batch). */
int cn_pose_error(const float* gt_c2w, const float* cam_c2w, int64_t batch, float* twist, float* err,
                  cn_stream_t stream);

/* --- SRN data resident in HBM (view_synthesis/datasets/dataset.py:60-94) --
 * images: (n_views, hw, channels) uint8, the decoded and cropped views; view_index: (batch) int64.
 * color (batch, hw, channels) = u8 / 255.0 (rounded once to fp32, as numpy's float64 quotient
 * cast to float32) and/or mask (batch, hw) = 1.0 where every channel != 255, else 0.0. */
int cn_srn_unpack(const uint8_t* images, int64_t n_views, int64_t hw, int64_t channels,
                  const int64_t* view_index, int64_t batch, float* color, float* mask, cn_stream_t stream);

/* --- Points: view_synthesis/nerf/point_sampler.py ---------------------- */

/* PointSampler.sample_uniform, point_sampler.py:49-71.
 * z_bins/lower/upper: (nc) from PointSampler.__init__ (:33-47);
 * t_rand: (n_rays, nc) or NULL (no perturbation);
 * z_out: (n_rays, nc); pts_out: (n_rays, nc, 3) or NULL. */
int cn_sample_uniform(const float* ro, const float* rd, int64_t n_rays, const float* z_bins,
                      const float* lower, const float* upper, int64_t nc, const float* t_rand,
                      float* z_out, float* pts_out, cn_stream_t stream);

/* pts = ro + rd * z for per-ray depth lists (point_sampler.py:70 and :118).
 * ro, rd: (n_rays, 3); z: (n_rays, n_samples); pts: (n_rays, n_samples, 3). */
int cn_ray_points(const float* ro, const float* rd, const float* z, int64_t n_rays,
                  int64_t n_samples, float* pts, cn_stream_t stream);

/* PointSampler.sample_pdf, point_sampler.py:73-120.
 * weights: row r at weights + r*w_stride, nc-2 values (the coarse weights[..., 1:-1]);
 * z: (n_rays, nc) sorted; u: row r at u + r*u_stride, nf values (u_stride 0 = one
 * row for every ray, e.g. the host's torch.linspace(0, 1, nf)), or NULL for an
 * in-kernel linspace;
 * z_out: (n_rays, nc+nf) sorted; pts_out: (n_rays, nc+nf, 3) or NULL.  nc <= 256, nf <= 256. */
int cn_sample_pdf(const float* ro, const float* rd, const float* weights, int64_t w_stride,
                  const float* z, int64_t n_rays, int64_t nc, int64_t nf, const float* u,
                  int64_t u_stride, float* z_out, float* pts_out, cn_stream_t stream);

/* --- Encoding: view_synthesis/nerf/position_embed.py ------------------- */

/* PositionalEmbedder.embed, position_embed.py:35-53.
 * x: (m, d); freqs: HOST array of num_freq floats (frequency_bands, :17-33);
 * out: (m, d*(include_input + 2*num_freq)).  num_freq <= 32. */
int cn_posenc(const float* x, int64_t m, int64_t d, const float* freqs, int64_t num_freq,
              int include_input, float* out, cn_stream_t stream);

/* --- Volume integration: view_synthesis/nerf/volumetric_render.py ------ */

/* volume_render, volumetric_render.py:36-66.
 * raw: (n_rays, n_samples, 4); z: (n_rays, n_samples); rd: (n_rays, 3);
 * rgb: (n_rays, 3); disp, acc, depth: (n_rays); weights: (n_rays, n_samples) or NULL.
 * raw, z and weights are read / written with 16-B vector accesses: 16-B aligned, or CN_EINVAL. */
int cn_volume_render(const float* raw, const float* z, const float* rd, int64_t n_rays,
                     int64_t n_samples, float* rgb, float* disp, float* acc, float* weights,
                     float* depth, cn_stream_t stream);

/* --- Code-conditioned MLP: view_synthesis/models/model.py -------------- */

/* Every field entry point below stores raw / reads d_raw as one 16-B row per sample: raw and d_raw
 * must be 16-B aligned, or the call returns CN_EINVAL without a launch. */

/* Floats needed for one packed model of format fmt (cn_mlp_pack output); -1 for a bad fmt. */
int64_t cn_mlp_packed_floats(int fmt);

/* Pack a CodeNeRFModel state_dict (model.py:145-156) into the MFMA fragment
 * layout the field kernel streams.  params: HOST array of CN_NUM_PARAMS device
 * pointers in state_dict order (layer_xyz1.weight, layer_xyz1.bias, layer_xyz2.*,
 * fc_out.*, shape_code_layer1.*, shape_code_layer2.*, texture_code_layer1.*,
 * layer_dir1.*, layer_dir2.*, fc_rgb.*). */
int cn_mlp_pack(const float* const* params, int fmt, float* packed, cn_stream_t stream);

/* The per-object terms of CodeNeRFModel.forward that the reference recomputes
 * for every sample (model.py:174-177 and the code halves of :180-192), once
 * per code row: out row i = [W_xyz2[:,256:] zs1 + b_xyz2 | W_out[:,256:] zs2 + b_out |
 * W_rgb[:,256:] zt1 + b_rgb | 0 0 0 0] with zs1/zs2/zt1 the relu'd code layers.
 * z_s, z_t: (n_codes, 256); code_bias: (n_codes, CN_CODE_BIAS_STRIDE). */
int cn_code_bias(const float* const* params, const float* z_s, const float* z_t,
                 int64_t n_codes, float* code_bias, cn_stream_t stream);

/* Everything a step needs from a model's weights and codes before its fp32 field kernels, in ONE
 * launch (what the reference recomputes inside every CodeNeRFModel.forward, model.py:160-194):
 * code_bias as cn_code_bias (NULL: skipped), packed / packed_t as cn_mlp_pack with CN_FMT_F32_W16
 * / CN_FMT_F32_W16_T (each NULL: skipped), and zero[0 .. n_zero) set to 0 (the fused backward's
 * g_code accumulator).  Bitwise the outputs of the separate calls. */
int cn_field_prepare(const float* const* params, const float* z_s, const float* z_t, int64_t n_codes,
                     float* code_bias, float* packed, float* packed_t, float* zero, int64_t n_zero,
                     cn_stream_t stream);

/* One model's part of cn_field_prepare_models: the arguments of cn_field_prepare, and code_act
 * (optional, with code_bias; (n_codes, 768)): the code layers' activations s1 | s2 | t1 after the
 * ReLU (model.py:174-177) as this launch formed them, for cn_code_bias_backward_act. */
typedef struct cn_field_prep {
  const float* const* params;
  float* code_bias;
  float* packed;
  float* packed_t;
  float* zero;
  int64_t n_zero;
  float* code_act;
} cn_field_prep;

/* cn_field_prepare for n_models (1 or 2) models on the same codes in ONE launch: a render's coarse
 * and fine fields (nerf/__init__.py:74-91 runs both on one object's codes) prepared together before
 * the coarse field.  Bitwise each model's cn_field_prepare. */
int cn_field_prepare_models(const cn_field_prep* models, int n_models, const float* z_s, const float* z_t,
                            int64_t n_codes, cn_stream_t stream);

/* CodeNeRFModel.forward(z_s, z_t, x), model.py:160-194, for pre-encoded rows.
 * x: (m, 90) = [xyz 63 | dir 27]; code row of row i = code_index ? code_index[i]
 * : (n_codes == 1 ? 0 : i); raw: (m, 4) = [rgb_raw(3), sigma_raw]. */
int cn_mlp_forward(const float* packed, int fmt, const float* code_bias, const int64_t* code_index,
                   int64_t n_codes, const float* x, int64_t m, float* raw, cn_stream_t stream);

/* forward_pass, nerf/__init__.py:94-134: embed + MLP for a ray chunk list.
 * Points come from pts (n_rays, n_samples, 3) if non-NULL, else pts = ro + rd*z
 * with z: (n_rays, n_samples).  rays are cut into consecutive chunks of
 * chunk_rows (util.get_minibatches) and Q1 applies per chunk: sample row
 * k = r*S + s of a chunk of Rc rays takes the view direction of ray k mod Rc.
 * freqs_xyz (10) / freqs_dir (4): HOST arrays.  code row of ray r as in
 * cn_mlp_forward (with r for i).  raw: (n_rays, n_samples, 4). */
int cn_radiance_field(const float* packed, int fmt, const float* code_bias, const int64_t* code_index,
                      int64_t n_codes, const float* pts, const float* ro, const float* rd,
                      const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                      const float* freqs_xyz, const float* freqs_dir, float* raw,
                      cn_stream_t stream);

/* --- Backward (autograd through the eval / train step) ------------------
 * The gradients loss.backward() takes through the path in the reference's
 * test-time optimisation (view_synthesis/eval.py) and training step:
 * pose -> get_bundle -> sample -> sample_uniform / sample_pdf (depths
 * detached, point_sampler.py:115) -> forward_pass -> CodeNeRFModel.forward
 * -> volume_render.  All fp32. */

/* cn_radiance_field in fp32 that also stores the post-activation hidden rows
 * the backward needs: save = (5, M, 256) planes h1, h2, feat, v1, v2 with
 * M = n_rays * n_samples (layer_xyz1, layer_xyz2, fc_out[1:], layer_dir1,
 * layer_dir2 of model.py:179-191).  packed must be an fp32 (CN_FMT_F32) pack. */
int cn_radiance_field_train(const float* packed, const float* code_bias, const int64_t* code_index,
                            int64_t n_codes, const float* pts, const float* ro, const float* rd,
                            const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                            const float* freqs_xyz, const float* freqs_dir, float* raw, float* save,
                            cn_stream_t stream);

/* cn_mlp_forward in fp32 that also stores the (5, m, 256) activations (as above). */
int cn_mlp_forward_train(const float* packed, const float* code_bias, const int64_t* code_index,
                         int64_t n_codes, const float* x, int64_t m, float* raw, float* save,
                         cn_stream_t stream);

/* The (M, 90) rows forward_pass hands CodeNeRFModel.forward (nerf/__init__.py:116-132):
 * [posenc(pts) 63 | posenc(Q1 view dir) 27].  pts, or ro + z. */
int cn_encode_inputs(const float* pts, const float* ro, const float* rd, const float* z, int64_t n_rays,
                     int64_t n_samples, int64_t chunk_rows, const float* freqs_xyz, const float* freqs_dir,
                     float* x, cn_stream_t stream);

/* Floats of scratch cn_field_backward needs for M sample rows. */
int64_t cn_field_backward_workspace_floats(int64_t m);
/* Offset (floats) of the (M, 90) dL/dx rows inside that scratch after cn_field_backward. */
int64_t cn_field_backward_dx_offset(int64_t m);

/* Backward of forward_pass + CodeNeRFModel.forward (model.py:160-194) from
 * d_raw (M, 4).  saved / x_enc from cn_radiance_field_train / cn_encode_inputs.
 * grads: 18 pointers (model.py parameter order, same as params) ACCUMULATED
 * into (+=), or NULL for no parameter gradients; the code-layer parameters
 * (shape/texture_code_layer*) and the code halves of layer_xyz2 / fc_out /
 * fc_rgb get their gradients from cn_code_bias_backward instead.
 * g_code: (n_codes, CN_CODE_BIAS_STRIDE) accumulated gradient of the
 * per-object code terms (cn_code_bias layout), or NULL.
 * d_pts (M, 3) is written when the inputs were pts; d_ro / d_rd (n_rays, 3) are
 * ACCUMULATED into (view-direction and, for ro + z inputs, point gradients).
 * With d_pts, d_ro and d_rd all NULL, pts / ro / rd / z / freqs may be NULL too
 * (rows from cn_mlp_forward_train: n_rays = M, n_samples = 1).  On return
 * workspace[2*260*M, 2*260*M + 90*M) holds dL/dx_enc (M, 90). */
int cn_field_backward(const float* const* params, const float* saved, const float* x_enc,
                      const float* d_raw, const float* pts, const float* ro, const float* rd,
                      const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                      const int64_t* code_index, int64_t n_codes, const float* freqs_xyz,
                      const float* freqs_dir, float* workspace, float* const* grads, float* g_code,
                      float* d_pts, float* d_ro, float* d_rd, cn_stream_t stream);

/* cn_field_backward with the GEMMs' arithmetic chosen by fmt: CN_FMT_F32 (exact-product
 * fp32 MFMA, what cn_field_backward runs) or CN_FMT_BF16X3 (every dX / dW GEMM as
 * Ah.Bh + Ah.Bl + Al.Bh on bf16 MFMA with fp32 accumulation, ~2^-17 relative error per
 * product; the training step).  Same arguments, outputs and workspace otherwise. */
int cn_field_backward_fmt(int fmt, const float* const* params, const float* saved, const float* x_enc,
                          const float* d_raw, const float* pts, const float* ro, const float* rd,
                          const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                          const int64_t* code_index, int64_t n_codes, const float* freqs_xyz,
                          const float* freqs_dir, float* workspace, float* const* grads, float* g_code,
                          float* d_pts, float* d_ro, float* d_rd, cn_stream_t stream);

/* --- Fused 3xbf16 backward (eval-step gradients, frozen weights) ---------
 * The gradients eval.py's loss.backward() takes into the codes and the pose
 * (eval.py:141-160; the reference's weight gradients are never read there).
 * Forward: cn_radiance_field_masks = cn_radiance_field on a CN_FMT_BF16X3 pack
 * that also writes the ReLU masks of layer_xyz1 / layer_xyz2 / layer_dir1 /
 * layer_dir2 (cn_field_mask_words(M) uint32 words).  Backward: one launch from
 * d_raw (M, 4) through the whole field on a CN_FMT_BF16X3_T pack of the same
 * weights: g_code (n_codes, CN_CODE_BIAS_STRIDE) ACCUMULATED as in
 * cn_field_backward (feed cn_code_bias_backward for dz_s / dz_t), d_pts (M, 3)
 * written for pts inputs, d_ro / d_rd (n_rays, 3) ACCUMULATED.  Needs one code
 * row per 32 consecutive samples (n_codes == 1, or n_samples % 32 == 0), else
 * CN_EUNSUPPORTED (use cn_field_backward). */
int64_t cn_field_mask_words(int64_t m);
int cn_radiance_field_masks(const float* packed, const float* code_bias, const int64_t* code_index,
                            int64_t n_codes, const float* pts, const float* ro, const float* rd,
                            const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                            const float* freqs_xyz, const float* freqs_dir, float* raw, uint32_t* masks,
                            cn_stream_t stream);
int cn_field_backward_x3(const float* packed_t, const uint32_t* masks, const float* d_raw, const float* pts,
                         const float* ro, const float* rd, const float* z, int64_t n_rays, int64_t n_samples,
                         int64_t chunk_rows, const int64_t* code_index, int64_t n_codes,
                         const float* freqs_xyz, const float* freqs_dir, float* g_code, float* d_pts,
                         float* d_ro, float* d_rd, cn_stream_t stream);

/* The same pair in either arithmetic.  fmt CN_FMT_BF16X3 (as above) or CN_FMT_F32_W16: the
 * fp32 16x16x4 inference kernel (exact fp32 products, the reference's arithmetic) that also
 * writes its ReLU masks (cn_field_mask_words_fmt(fmt, M) words).  The backward takes the
 * matching transposed pack (fmt_t CN_FMT_BF16X3_T / CN_FMT_F32_W16_T) and needs one code row
 * per wave: n_codes == 1, or n_samples % 32 (bf16x3) / % 16 (fp32) == 0. */
int64_t cn_field_mask_words_fmt(int fmt, int64_t m);
int cn_radiance_field_masks_fmt(int fmt, const float* packed, const float* code_bias, const int64_t* code_index,
                                int64_t n_codes, const float* pts, const float* ro, const float* rd,
                                const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                                const float* freqs_xyz, const float* freqs_dir, float* raw, uint32_t* masks,
                                cn_stream_t stream);
int cn_field_backward_fused(int fmt_t, const float* packed_t, const uint32_t* masks, const float* d_raw,
                            const float* pts, const float* ro, const float* rd, const float* z, int64_t n_rays,
                            int64_t n_samples, int64_t chunk_rows, const int64_t* code_index, int64_t n_codes,
                            const float* freqs_xyz, const float* freqs_dir, float* g_code, float* d_pts,
                            float* d_ro, float* d_rd, cn_stream_t stream);
/* The same backward without float atomics (eval.py:145-160's backward, bit-reproducible): with
 * n_codes == 1 and n_samples % 32 (bf16x3) / % 16 (fp32) == 0 the kernel writes per-workgroup g_code
 * rows and per-wave / per-sample ray-gradient terms into workspace
 * (cn_field_backward_fused_workspace_floats(fmt_t, n_rays, n_samples) floats, 16-B aligned), and two
 * short launches add them into g_code, d_ro and d_rd in a fixed order (g_code / d_ro / d_rd are still
 * ACCUMULATED).  Other shapes, or workspace NULL, run cn_field_backward_fused. */
int64_t cn_field_backward_fused_workspace_floats(int fmt_t, int64_t n_rays, int64_t n_samples);
int cn_field_backward_fused_ws(int fmt_t, const float* packed_t, const uint32_t* masks, const float* d_raw,
                               const float* pts, const float* ro, const float* rd, const float* z, int64_t n_rays,
                               int64_t n_samples, int64_t chunk_rows, const int64_t* code_index, int64_t n_codes,
                               const float* freqs_xyz, const float* freqs_dir, float* g_code, float* d_pts,
                               float* d_ro, float* d_rd, float* workspace, cn_stream_t stream);
/* The eval step's two fields (eval.py:153-167: predict_radiance_and_render's coarse and fine fields on the
 * same rays; the fine depths are detached, point_sampler.py:115, so the two backwards are independent) in
 * shared launches: each field the arguments of one cn_field_backward_fused_ws call, both adding into the
 * same d_ro / d_rd.  fp32, rays + depths, one code row, whole waves per ray: one dX launch and one ray /
 * g_code launch for both; d_ro / d_rd and g_code bitwise those of field 0's call,
 * then d_rd += d_rd_between (optional, n_rays x 3: the rays' gradient that arrives between the two
 * backwards -- the coarse volume render's), then field 1's call -- which is how fields that cannot share
 * run.  n_fields 1 or 2 (d_rd_between: 2 only). */
typedef struct cn_field_fused_bwd {
  const float* packed_t;
  const uint32_t* masks;
  const float* d_raw;
  const float* pts;
  const float* ro;
  const float* rd;
  const float* z;
  int64_t n_rays, n_samples, chunk_rows;
  const int64_t* code_index;
  int64_t n_codes;
  const float* freqs_xyz;
  const float* freqs_dir;
  float* g_code;
  float* d_pts;
  float* d_ro;
  float* d_rd;
  float* workspace;
} cn_field_fused_bwd;
int cn_field_backward_fused_multi(int fmt_t, const cn_field_fused_bwd* fields, int n_fields, const float* d_rd_between,
                                  cn_stream_t stream);

/* --- Fused fp32 training step (train.py:92-114; weights trained) ------------------
 * Forward: cn_radiance_field on a CN_FMT_F32_W16 pack that also writes the ReLU masks
 * (cn_field_mask_words_fmt(CN_FMT_F32_W16, M) words), the (5, M, 256) post-activation planes
 * h1, h2, feat, v1, v2 (cn_radiance_field_train's layout) and after them, at save + 5 M 256, the
 * (M, 64) encoding plane: the positional encodings layer_xyz1 multiplied, 16 per lane group in the
 * kernel's k-step order (column c' -> PositionalEmbedder column of the mlp_common.h map, one padding
 * slot).  save holds cn_field_train_saved_floats(CN_FMT_F32_W16, M) floats.
 * Backward: the fused dX chain of cn_field_backward_fused on the CN_FMT_F32_W16_T pack (g_code,
 * d_pts / d_ro / d_rd as there; g_code required) that also writes every layer's masked input
 * gradient into workspace (cn_field_backward_train_workspace_floats(M) floats), then the weight
 * and bias gradients dW = dPre^T X as split-M fp32 MFMA GEMMs over those planes, saved and x_enc
 * (cn_encode_inputs; or x_enc NULL: the forward's own encodings from saved's encoding plane, fp32,
 * or generated inside the dW kernels, bf16x3), reduced
 * deterministically (cn_gemm_tn_ws) through the rest of workspace: grads (18 pointers, or NULL for none) ACCUMULATED as in
 * cn_field_backward (the code-layer parameters and code halves come from cn_code_bias_backward).
 * One code row per 16-sample wave: n_codes == 1 or n_samples % 16 == 0, else CN_EUNSUPPORTED. */
int cn_radiance_field_train_w16(const float* packed, const float* code_bias, const int64_t* code_index,
                                int64_t n_codes, const float* pts, const float* ro, const float* rd,
                                const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                                const float* freqs_xyz, const float* freqs_dir, float* raw, float* save,
                                uint32_t* masks, cn_stream_t stream);
/* The same pair for either precision: fmt CN_FMT_F32_W16 (fp32 16x16x4) or CN_FMT_BF16X3 (3xbf16
 * 32x32x16; masks cn_field_mask_words_fmt(CN_FMT_BF16X3, M) words, the same fp32 planes), and
 * fmt_t the matching transposed pack (CN_FMT_F32_W16_T / CN_FMT_BF16X3_T; the bf16x3 dW GEMMs
 * are 3xbf16 too).  bf16x3: one code row per 32-sample wave (n_codes == 1 or n_samples % 32 == 0);
 * its save buffer holds 5 * M * 256 + 256 floats (the last row is scratch for padding lanes).
 * cn_field_train_saved_floats: the save buffer's floats for fmt and M (-1: bad arguments). */
int64_t cn_field_train_saved_floats(int fmt, int64_t m);
int cn_radiance_field_train_fmt(int fmt, const float* packed, const float* code_bias, const int64_t* code_index,
                                int64_t n_codes, const float* pts, const float* ro, const float* rd,
                                const float* z, int64_t n_rays, int64_t n_samples, int64_t chunk_rows,
                                const float* freqs_xyz, const float* freqs_dir, float* raw, float* save,
                                uint32_t* masks, cn_stream_t stream);
int64_t cn_field_backward_train_workspace_floats(int64_t m);
int cn_field_backward_train(const float* packed_t, const float* const* params, const uint32_t* masks,
                            const float* saved, const float* x_enc, const float* d_raw, const float* pts,
                            const float* ro, const float* rd, const float* z, int64_t n_rays, int64_t n_samples,
                            int64_t chunk_rows, const int64_t* code_index, int64_t n_codes,
                            const float* freqs_xyz, const float* freqs_dir, float* workspace,
                            float* const* grads, float* g_code, float* d_pts, float* d_ro, float* d_rd,
                            cn_stream_t stream);
int cn_field_backward_train_fmt(int fmt_t, const float* packed_t, const float* const* params,
                                const uint32_t* masks, const float* saved, const float* x_enc, const float* d_raw,
                                const float* pts, const float* ro, const float* rd, const float* z, int64_t n_rays,
                                int64_t n_samples, int64_t chunk_rows, const int64_t* code_index, int64_t n_codes,
                                const float* freqs_xyz, const float* freqs_dir, float* workspace,
                                float* const* grads, float* g_code, float* d_pts, float* d_ro, float* d_rd,
                                cn_stream_t stream);
/* A render's fields' training backwards in shared launches (replaces two cn_field_backward_train_fmt
 * calls for predict_radiance_and_render's coarse and fine fields, nerf/__init__.py:81-89 under
 * train.py:112's loss.backward(): the fine depths are detached, point_sampler.py:115, so the two
 * backwards are independent).  Each field: the arguments of cn_field_backward_train_fmt, with its own
 * workspace.  With two fp32 fields on rays + depths that both take the batched dW plan and the forward's
 * encoding plane (every runnable training config): ONE dX launch, ONE batched dW launch (layer_xyz1's
 * dW among its jobs), ONE DIRS-pass launch and ONE reduction launch for both, each running every field's
 * workgroups as its own launch would -- the gradients are bitwise those of the per-field calls.  Otherwise the fields run one after
 * the other.  n_fields 1 or 2. */
typedef struct cn_field_train_bwd {
  const float* packed_t;
  const float* const* params;
  const uint32_t* masks;
  const float* saved;
  const float* x_enc;
  const float* d_raw;
  const float* pts;
  const float* ro;
  const float* rd;
  const float* z;
  int64_t n_rays, n_samples, chunk_rows;
  const int64_t* code_index;
  int64_t n_codes;
  const float* freqs_xyz;
  const float* freqs_dir;
  float* workspace;
  float* const* grads;
  float* g_code;
  float* d_pts;
  float* d_ro;
  float* d_rd;
} cn_field_train_bwd;
int cn_field_backward_train_multi(int fmt_t, const cn_field_train_bwd* fields, int n_fields, cn_stream_t stream);

/* Backward of cn_code_bias (the code layers, model.py:174-177, and the code
 * halves of layer_xyz2 / fc_out / fc_rgb) from g_code.  dz_s / dz_t (n_codes, 256)
 * are written (either may be NULL); grads as in cn_field_backward (accumulated). */
int cn_code_bias_backward(const float* const* params, const float* z_s, const float* z_t, int64_t n_codes,
                          const float* g_code, float* dz_s, float* dz_t, float* const* grads,
                          cn_stream_t stream);
/* The same backward in two launches with a caller-provided workspace
 * (cn_code_bias_backward_workspace_floats(n_codes) floats): each code's layers and
 * reductions are formed once, split over 64 workgroups, instead of once per workgroup.
 * Bitwise the same results as cn_code_bias_backward.  accumulate_dz = 1: dz_s / dz_t +=
 * the code gradients instead of = (the training step points them at the code tables'
 * gradient rows, so the coarse and fine fields' code gradients add up in place --
 * ShapeTextureEmbedding.forward in model.py:102-105 is the lookup they flow back to). */
int64_t cn_code_bias_backward_workspace_floats(int64_t n_codes);
/* The code backward on the forward's code-layer activations (code_act of cn_field_prepare_models),
 * first half: ds1 / ds2 / dt1 (ReLU-masked by code_act) into the workspace
 * (cn_code_bias_backward_workspace_floats) and the code layers' / code halves' parameter gradients
 * added into grads (optional) -- no code layer is recomputed.  cn_code_dz forms dz from it. */
int cn_code_bias_backward_act(const float* const* params, const float* z_s, const float* z_t, int64_t n_codes,
                              const float* code_act, const float* g_code, float* const* grads, float* workspace,
                              cn_stream_t stream);
/* cn_code_bias_backward_act of a render's 1 or 2 fields on the same codes in ONE launch (each job: the
 * arguments of one cn_code_bias_backward_act call; bitwise those calls' results). */
typedef struct cn_code_act_job {
  const float* const* params;
  const float* code_act;
  const float* g_code;
  float* const* grads;
  float* workspace;
} cn_code_act_job;
int cn_code_bias_backward_act_multi(const cn_code_act_job* jobs, int n_jobs, const float* z_s, const float* z_t,
                                    int64_t n_codes, cn_stream_t stream);
/* One field's part of cn_code_dz: its parameters, g_code and cn_code_bias_backward_act's workspace. */
typedef struct cn_code_dz_job {
  const float* const* params;
  const float* g_code;
  const float* workspace;
} cn_code_dz_job;
/* dz_s / dz_t (n_codes, 256; either may be NULL) of 1 or 2 jobs on the same codes (a render's coarse and
 * fine fields, nerf/__init__.py:74-91), summed in job order; accumulate = 1: added to what dz holds. */
int cn_code_dz(const cn_code_dz_job* jobs, int n_jobs, int64_t n_codes, float* dz_s, float* dz_t, int accumulate,
               cn_stream_t stream);
int cn_code_bias_backward_ws(const float* const* params, const float* z_s, const float* z_t, int64_t n_codes,
                             const float* g_code, float* dz_s, float* dz_t, float* const* grads, float* workspace,
                             int accumulate_dz, cn_stream_t stream);

/* Backward of volume_render (volumetric_render.py:36-66) w.r.t. raw and rd
 * (z is detached in the reference).  Any of g_rgb (R,3), g_disp, g_acc, g_depth
 * (R), g_weights (R,S) may be NULL (zero).  d_raw (R,S,4) and d_rd (R,3, may be
 * NULL) are written -- d_rd added to instead with accumulate_rd = 1 (a running sum
 * of the rays' gradients over their consumers).  raw, z and d_raw 16-B aligned, or
 * CN_EINVAL. */
int cn_volume_render_backward(const float* raw, const float* z, const float* rd, int64_t n_rays,
                              int64_t n_samples, const float* g_rgb, const float* g_disp,
                              const float* g_acc, const float* g_weights, const float* g_depth,
                              float* d_raw, float* d_rd, int accumulate_rd, cn_stream_t stream);

/* Backward of get_bundle (ray_sampler.py:95-98): d_c2w (batch, 4, 4) rows 0..2
 * ACCUMULATED from g_ro / g_rd (batch*hw, 3), either may be NULL (not both). */
int cn_ray_bundle_backward(const float* dirs, int64_t hw, int64_t batch, const float* g_ro,
                           const float* g_rd, float* d_c2w, cn_stream_t stream);

/* Backward of the sample gather (ray_sampler.py:77-80): scatter-add g_ro / g_rd
 * (batch*sample_size, 3) into d_ro / d_rd (batch*hw, 3). */
int cn_gather_rays_backward(const float* g_ro, const float* g_rd, int64_t batch, int64_t hw,
                            const int64_t* select_inds, int64_t sample_size, float* d_ro, float* d_rd,
                            cn_stream_t stream);

/* Backward of cn_posenc (position_embed.py:35-53): dx (m, d) from g_enc (m, d*(inc + 2*num_freq)). */
int cn_posenc_backward(const float* x, int64_t m, int64_t d, const float* freqs, int64_t num_freq,
                       int include_input, const float* g_enc, float* dx, cn_stream_t stream);

/* Backward of cn_ray_points (z detached, point_sampler.py:115): d_ro += sum_s g_pts,
 * d_rd += sum_s g_pts * z; either output may be NULL (not both). */
int cn_ray_points_backward(const float* g_pts, const float* z, int64_t n_rays, int64_t n_samples,
                           float* d_ro, float* d_rd, cn_stream_t stream);

/* --- The step's scalar loss (train.py:103-108, eval.py:157-163) ---------------
 * out[6] = [mse(rgb_coarse, target[:, :3]), mse(rgb_fine, target[:, :3]),
 *           lambda * (||z_s|| + ||z_t||), their sum, ||z_s||, ||z_t||] (fp32, device), with
 * ||z|| = sqrt(expand * sum z^2) over n_code values (a code row expanded over `expand` rays,
 * eval; or whole tables with expand 1, train).  rgb_*: (n_rays, 3), either may be NULL;
 * target rows of target_stride floats (the first 3 are rgb).  n_code 0: no regulariser.
 * workspace: cn_render_loss_workspace_doubles(n_code) doubles (0: may be NULL) for the
 * multi-workgroup sums of large code tensors. */
int64_t cn_render_loss_workspace_doubles(int64_t n_code);
int cn_render_loss(const float* rgb_coarse, const float* rgb_fine, const float* target,
                   int64_t target_stride, int64_t n_rays, const float* z_s, const float* z_t,
                   int64_t n_code, int64_t expand, float regularizer_lambda, double* workspace, float* out,
                   cn_stream_t stream);
/* The same, plus psnr[0] = mse2psnr of the fine loss (of the coarse one without rgb_fine) in
 * float64 on the device -- utils/util.py:216-227 (-10 log10(mse), mse 0 -> 1e-5), the psnr
 * train.py:105 / eval.py:160 log -- so the caller needs no launches and no read-back for it. */
int cn_render_loss_psnr(const float* rgb_coarse, const float* rgb_fine, const float* target,
                        int64_t target_stride, int64_t n_rays, const float* z_s, const float* z_t,
                        int64_t n_code, int64_t expand, float regularizer_lambda, double* workspace,
                        float* out, double* psnr, cn_stream_t stream);
/* Its backward for an upstream gradient *grad_total (device scalar) of the sum, reading
 * the forward's out as stats: d_rgb_* (n_rays, 3) and d_z_* (n_code) WRITTEN (any NULL);
 * accumulate_z = 1: d_z_* added to (the codes' running gradient). */
int cn_render_loss_backward(const float* rgb_coarse, const float* rgb_fine, const float* target,
                            int64_t target_stride, int64_t n_rays, const float* z_s, const float* z_t,
                            int64_t n_code, int64_t expand, float regularizer_lambda, const float* stats,
                            const float* grad_total, float* d_rgb_coarse, float* d_rgb_fine, float* d_z_s,
                            float* d_z_t, int accumulate_z, cn_stream_t stream);

/* --- Training step: the optimiser (train.py:111-114, utils/util.py:147-172) ---
 * torch.optim.AdamW.step (decoupled weight decay; amsgrad / maximize off) over ONE
 * flat fp32 buffer holding every trained parameter, with its gradient and both
 * moments in three more buffers of the same layout (all 16-B aligned).  The update
 * runs over n_segments ranges [seg_begin[k], seg_end[k]) (HOST int64 arrays, float
 * offsets, multiples of 4, ascending, disjoint); segment k has its own lr[k],
 * weight_decay[k] (HOST double arrays) and step[k] (HOST int64, the step number
 * after this update, >= 1) -- normally one segment per param group; elements in no
 * segment are not touched.  Per element, in torch's _single_tensor_adam order with
 * each op rounded to fp32:
 *   p = p (1 - lr wd); m = lerp(m, g, 1 - beta1); v = v beta2 + ((1 - beta2) g) g;
 *   p = p + (-lr / (1 - beta1^step)) m / (sqrt(v) / sqrt(1 - beta2^step) + eps). */
int cn_adamw_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n_segments,
                  const int64_t* seg_begin, const int64_t* seg_end, const double* lr, const double* weight_decay,
                  const int64_t* step, double beta1, double beta2, double eps, cn_stream_t stream);

/* The same update with its per-segment scalars read from DEVICE memory, so a captured graph can
 * replay it with fresh ones: scalars = 3 floats per segment {1 - lr wd, -lr / (1 - beta1^step),
 * (1 - beta2^step)^0.5}, as cn_adamw_scalars folds them (host, the same double arithmetic as
 * cn_adamw_step).  Replaces optimizer.step() inside the captured eval iteration
 * (codenerf.evaluate.GraphedEvalStep; eval.py:165-167). */
int cn_adamw_scalars(int64_t n_segments, const double* lr, const double* weight_decay, const int64_t* step,
                     double beta1, double beta2, float* out);
int cn_adamw_step_dev(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n_segments,
                      const int64_t* seg_begin, const int64_t* seg_end, const float* scalars, double beta1,
                      double beta2, double eps, cn_stream_t stream);

/* fp32 MFMA GEMMs the backward is built from (row-major, leading dims in floats):
 *   cn_gemm_nn: C[M][N] = A[M][K] B[K][N], zeroed where mask[m][n] <= 0 (mask may be NULL); K <= 288;
 *   cn_gemm_tn: C[N][K] += sum_m A[M][N] B[M][K] (accumulates). */
int cn_gemm_nn(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
               const float* mask, int64_t ldm, int64_t M, int64_t N, int64_t K, cn_stream_t stream);
int cn_gemm_tn(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M,
               int64_t N, int64_t K, cn_stream_t stream);
/* The same two products as 3xbf16 (split operands on v_mfma_f32_32x32x16_bf16, fp32
 * accumulation; the GEMMs of cn_field_backward_fmt(CN_FMT_BF16X3)). */
int cn_gemm_nn_x3(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                  const float* mask, int64_t ldm, int64_t M, int64_t N, int64_t K, cn_stream_t stream);
int cn_gemm_tn_x3(const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc, int64_t M,
                  int64_t N, int64_t K, cn_stream_t stream);
/* cn_gemm_tn (fmt CN_FMT_F32) or cn_gemm_tn_x3 (CN_FMT_BF16X3), deterministic: each workgroup
 * stores its partial N x K tile into workspace (cn_gemm_tn_workspace_floats(M, N, K) floats) and
 * a second pass adds the partials to C in a fixed order, so the result is bitwise reproducible
 * (the float-atomic flush of cn_gemm_tn is not). */
int64_t cn_gemm_tn_workspace_floats(int64_t M, int64_t N, int64_t K);
int cn_gemm_tn_ws(int fmt, const float* A, int64_t lda, const float* B, int64_t ldb, float* C, int64_t ldc,
                  int64_t M, int64_t N, int64_t K, float* workspace, cn_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* CODENERF_H_ */
