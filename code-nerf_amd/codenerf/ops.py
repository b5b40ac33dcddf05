"""Tensor-level wrappers of the C ABI: validate, allocate outputs, launch on the current stream.

Every function here is one entry point of include/codenerf.h; the reference
function it replaces is named in its docstring.  Inputs must be CUDA (HIP)
fp32 tensors; shape errors raise AssertionError like the reference's asserts,
and a failed launch raises ``CodeNerfError``.  Nothing here falls back to
PyTorch compute.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import check, ptr, stream_of

Tensor = torch.Tensor


def _cuda(t: Tensor, name: str, dtype=torch.float32) -> Tensor:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a tensor")
    if t.device.type != "cuda":
        raise ValueError(f"{name} must be on a HIP device (got {t.device}); the MI355X path has no CPU fallback")
    if t.dtype != dtype:
        raise TypeError(f"{name} must be {dtype} (got {t.dtype})")
    return t.contiguous()


def _aligned16(t: Tensor) -> Tensor:
    """t itself when its data pointer is 16-B aligned (what the kernels' vector accesses need; every
    fresh allocation is), else an aligned copy (a contiguous view at an odd element offset)."""
    return t if t.data_ptr() % 16 == 0 else t.clone()


def _lib_ready():
    return _lib.load()


# ------------------------------------------------------------------ rays


def ray_directions(height: int, width: int, focal: float, cx: float, cy: float, device) -> Tensor:
    """RaySampler.__init__ directions (ray_sampler.py:35-51) -> (H, W, 3)."""
    lib = _lib_ready()
    out = torch.empty(height, width, 3, device=device, dtype=torch.float32)
    check(lib.cn_ray_directions(height, width, focal, cx, cy, ptr(out), stream_of(out)), "cn_ray_directions")
    return out


def ray_bundle(dirs: Tensor, c2w: Tensor) -> Tuple[Tensor, Tensor]:
    """RaySampler.get_bundle (ray_sampler.py:84-99): (H,W,3), (B,4,4) -> ro, rd (B,H,W,3)."""
    lib = _lib_ready()
    dirs = _cuda(dirs, "directions")
    c2w = _cuda(c2w, "tform_cam2world")
    assert c2w.dim() == 3 and c2w.shape[-2:] == (4, 4), "tform_cam2world must be (batch, 4, 4)"
    h, w = dirs.shape[0], dirs.shape[1]
    b = c2w.shape[0]
    ro = torch.empty(b, h, w, 3, device=dirs.device, dtype=torch.float32)
    rd = torch.empty_like(ro)
    check(lib.cn_ray_bundle(ptr(dirs), h * w, ptr(c2w), b, ptr(ro), ptr(rd), stream_of(dirs)), "cn_ray_bundle")
    return ro, rd


def gather_rays(ro: Tensor, rd: Tensor, select_inds: Tensor) -> Tuple[Tensor, Tensor]:
    """RaySampler.sample gather (ray_sampler.py:77-80): (B,HW,3) x2, (B,S) -> (B*S,3) x2."""
    lib = _lib_ready()
    ro, rd = _cuda(ro, "ray_origins"), _cuda(rd, "ray_directions")
    sel = _cuda(select_inds, "select_inds", torch.int64)
    b, s = sel.shape
    hw = ro.numel() // (3 * b)
    o = torch.empty(b * s, 3, device=ro.device, dtype=torch.float32)
    d = torch.empty_like(o)
    check(lib.cn_gather_rays(ptr(ro), ptr(rd), b, hw, ptr(sel), s, ptr(o), ptr(d), stream_of(o)), "cn_gather_rays")
    return o, d


# ------------------------------------------------------------------ fused pose path


def pose_rays(dirs: Tensor, theta: Optional[Tensor] = None, phi: Optional[Tensor] = None,
              rho: Optional[Tensor] = None, c2w: Optional[Tensor] = None, select_inds: Optional[Tensor] = None,
              target: Optional[Tensor] = None):
    """pose_spherical (eval.py:22-38) -> sample (ray_sampler.py:53-99) -> target gather
    (eval.py:147-148) in one launch.  theta, phi, rho (B,) each, or c2w (B,4,4); select_inds
    (B,S) int64 or None (whole bundle); target (B,HW,C) or None -> ro, rd (B*S,3), c2w (B,4,4),
    target rows (B*S,C) | None."""
    lib = _lib_ready()
    dirs = _cuda(dirs, "directions")
    hw = dirs.numel() // 3
    assert (theta is None) != (c2w is None), "give exactly one of (theta, phi, rho) and c2w"
    if theta is not None:
        theta, phi, rho = (_cuda(t, n).reshape(-1) for t, n in ((theta, "theta"), (phi, "phi"), (rho, "rho")))
        b = theta.numel()
        assert phi.numel() == b and rho.numel() == b, "theta, phi and rho must have one value per pose"
    else:
        c2w = _cuda(c2w, "tform_cam2world")
        assert c2w.dim() == 3 and c2w.shape[-2:] == (4, 4), "tform_cam2world must be (batch, 4, 4)"
        b = c2w.shape[0]
    if select_inds is not None:
        select_inds = _cuda(select_inds, "select_inds", torch.int64)
        assert select_inds.dim() == 2 and select_inds.shape[0] == b, "select_inds must be (batch, sample_size)"
        s = select_inds.shape[1]
    else:
        s = hw
    ch = 0
    tgt_out = None
    if target is not None:
        target = _cuda(target, "target")
        assert target.shape[0] == b and target.numel() % (b * hw) == 0, "target must be (batch, H*W, C)"
        ch = target.numel() // (b * hw)
        tgt_out = torch.empty(b * s, ch, device=dirs.device, dtype=torch.float32)
    ro = torch.empty(b * s, 3, device=dirs.device, dtype=torch.float32)
    rd = torch.empty_like(ro)
    c2w_out = torch.empty(b, 4, 4, device=dirs.device, dtype=torch.float32)
    check(lib.cn_pose_rays(ptr(theta), ptr(phi), ptr(rho), ptr(c2w), b, ptr(dirs), hw, ptr(select_inds), s,
                           ptr(target), ch, ptr(c2w_out), ptr(ro), ptr(rd), ptr(tgt_out), stream_of(ro)),
          "cn_pose_rays")
    return ro, rd, c2w_out, tgt_out


def pose_rays_backward(dirs: Tensor, batch: int, g_ro: Optional[Tensor], g_rd: Optional[Tensor],
                       theta: Optional[Tensor] = None, phi: Optional[Tensor] = None, rho: Optional[Tensor] = None,
                       select_inds: Optional[Tensor] = None, want_c2w: bool = False, out=None):
    """Backward of pose_rays -> (d_theta, d_phi, d_rho (B,) each | None, d_c2w (B,4,4) | None).  ``out``:
    three (B,) contiguous device tensors the angle gradients are written into (e.g. the optimiser's
    gradient slots)."""
    lib = _lib_ready()
    dirs = _cuda(dirs, "directions")
    hw = dirs.numel() // 3
    s = hw if select_inds is None else select_inds.shape[1]
    g_ro, g_rd = _opt(g_ro, "g_ro"), _opt(g_rd, "g_rd")
    angles = theta is not None
    if out is not None and angles:
        assert all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.numel() == batch for t in out)
        d = list(out)
    else:
        d = [torch.empty(batch, device=dirs.device, dtype=torch.float32) if angles else None for _ in range(3)]
    d_c2w = torch.empty(batch, 4, 4, device=dirs.device, dtype=torch.float32) if want_c2w else None
    check(lib.cn_pose_rays_backward(ptr(theta), ptr(phi), ptr(rho), batch, ptr(dirs), hw, ptr(select_inds), s,
                                    ptr(g_ro), ptr(g_rd), ptr(d_c2w), ptr(d[0]), ptr(d[1]), ptr(d[2]),
                                    stream_of(dirs)), "cn_pose_rays_backward")
    return (d[0], d[1], d[2]), d_c2w


def random_select(batch: int, hw: int, sample_size: int, seed: int, offset: int, device) -> Tensor:
    """On-device np.random.permutation(hw)[:sample_size] per image (ray_sampler.py:41-42, same
    distribution; Philox4x32-10) -> (batch, sample_size) int64."""
    lib = _lib_ready()
    out = torch.empty(batch, sample_size, device=device, dtype=torch.int64)
    check(lib.cn_random_select(batch, hw, sample_size, seed & (2 ** 64 - 1), offset & (2 ** 64 - 1), ptr(out),
                               stream_of(out)), "cn_random_select")
    return out


def pose_error(gt_c2w: Tensor, cam_c2w: Tensor) -> Tuple[Tensor, Tensor]:
    """eval.py:161-162: (SE3.Log(inverse(gt) @ cam) (B,6), its 2-norm (B,))."""
    lib = _lib_ready()
    gt, cam = _cuda(gt_c2w, "gt_pose").reshape(-1, 4, 4), _cuda(cam_c2w, "cam_pose").reshape(-1, 4, 4)
    assert gt.shape == cam.shape, "poses must both be (batch, 4, 4)"
    b = gt.shape[0]
    twist = torch.empty(b, 6, device=gt.device, dtype=torch.float32)
    err = torch.empty(b, device=gt.device, dtype=torch.float32)
    check(lib.cn_pose_error(ptr(gt), ptr(cam), b, ptr(twist), ptr(err), stream_of(gt)), "cn_pose_error")
    return twist, err


# ------------------------------------------------------------------ points


def sample_uniform(ro: Tensor, rd: Tensor, z_bins: Tensor, lower: Tensor, upper: Tensor,
                   t_rand: Optional[Tensor] = None, want_pts: bool = True):
    """PointSampler.sample_uniform (point_sampler.py:49-71) -> pts (R,Nc,3) | None, z (R,Nc)."""
    lib = _lib_ready()
    ro, rd = _cuda(ro, "ro"), _cuda(rd, "rd")
    n, nc = ro.shape[0], z_bins.shape[-1]
    if t_rand is not None:
        t_rand = _cuda(t_rand, "t_rand")
        assert t_rand.shape == (n, nc), "t_rand must be (num_rays, num_coarse)"
    z = torch.empty(n, nc, device=ro.device, dtype=torch.float32)
    pts = torch.empty(n, nc, 3, device=ro.device, dtype=torch.float32) if want_pts else None
    if n:      # no rays: empty outputs, as torch's ops give (the C ABI refuses n_rays == 0)
        check(lib.cn_sample_uniform(ptr(ro), ptr(rd), n, ptr(z_bins), ptr(lower), ptr(upper), nc, ptr(t_rand),
                                    ptr(z), ptr(pts), stream_of(z)), "cn_sample_uniform")
    return pts, z


def ray_points(ro: Tensor, rd: Tensor, z: Tensor) -> Tensor:
    """pts = ro + rd * z (point_sampler.py:70, :118): (R,3) x2, (R,S) -> (R,S,3)."""
    lib = _lib_ready()
    ro, rd, z = _cuda(ro, "ro"), _cuda(rd, "rd"), _cuda(z, "z_vals")
    n, s = z.shape
    assert ro.shape == (n, 3) and rd.shape == (n, 3), "ro / rd must be (num_rays, 3)"
    pts = torch.empty(n, s, 3, device=z.device, dtype=torch.float32)
    if n * s:
        check(lib.cn_ray_points(ptr(ro), ptr(rd), ptr(z), n, s, ptr(pts), stream_of(z)), "cn_ray_points")
    return pts


def sample_pdf(ro: Tensor, rd: Tensor, weights: Tensor, z: Tensor, num_fine: int,
               u: Optional[Tensor] = None, want_pts: bool = True):
    """PointSampler.sample_pdf (point_sampler.py:73-120) -> pts (R,Nc+Nf,3) | None, z (R,Nc+Nf).

    ``weights`` may be the strided view ``w[..., 1:-1]`` of a contiguous (R, Nc) tensor;
    ``u`` is (R, Nf) per-ray draws or one (Nf,) row shared by every ray.
    """
    lib = _lib_ready()
    ro, rd, z = _cuda(ro, "ro"), _cuda(rd, "rd"), _cuda(z, "z_vals")
    n, nc = z.shape
    assert nc - 2 == weights.shape[-1], f"Weights size {weights.shape} should match {nc - 1}"
    if weights.device.type != "cuda" or weights.dtype != torch.float32 or weights.stride(-1) != 1:
        weights = _cuda(weights, "weights")
    w_stride = weights.stride(0)
    u_stride = 0
    if u is not None:
        u = _cuda(u, "u")
        assert u.shape in ((n, num_fine), (num_fine,)), "u must be (num_rays, num_fine) or (num_fine,)"
        u_stride = num_fine if u.dim() == 2 else 0
    zo = torch.empty(n, nc + num_fine, device=z.device, dtype=torch.float32)
    pts = torch.empty(n, nc + num_fine, 3, device=z.device, dtype=torch.float32) if want_pts else None
    if n:
        check(lib.cn_sample_pdf(ptr(ro), ptr(rd), ptr(weights), w_stride, ptr(z), n, nc, num_fine, ptr(u), u_stride,
                                ptr(zo), ptr(pts), stream_of(zo)), "cn_sample_pdf")
    return pts, zo


# ------------------------------------------------------------------ encoding


def posenc(x: Tensor, freqs: Sequence[float], include_input: bool) -> Tensor:
    """PositionalEmbedder.embed (position_embed.py:35-53): (M, D) -> (M, D*(inc + 2L))."""
    lib = _lib_ready()
    x = _cuda(x, "tensor")
    assert x.dim() == 2, "tensor must be (N, num_dim)"
    m, d = x.shape
    out = torch.empty(m, d * (int(include_input) + 2 * len(freqs)), device=x.device, dtype=torch.float32)
    if m:
        check(lib.cn_posenc(ptr(x), m, d, _lib.host_floats(freqs), len(freqs), int(include_input), ptr(out),
                            stream_of(x)), "cn_posenc")
    return out


# ------------------------------------------------------------------ volume integration


def volume_render(raw: Tensor, z: Tensor, rd: Tensor, want_weights: bool = True):
    """volume_render (volumetric_render.py:36-66) -> rgb, disp, acc, weights, depth."""
    lib = _lib_ready()
    raw, z, rd = _cuda(raw, "radiance_field"), _cuda(z, "depth_values"), _cuda(rd, "ray_directions")
    raw, z = _aligned16(raw), _aligned16(z)
    n, s = z.shape
    assert raw.shape == (n, s, 4), "radiance_field must be (num_rays, num_samples, 4)"
    assert rd.shape == (n, 3), "ray_directions must be (num_rays, 3)"
    dev = raw.device
    rgb = torch.empty(n, 3, device=dev, dtype=torch.float32)
    disp = torch.empty(n, device=dev, dtype=torch.float32)
    acc = torch.empty_like(disp)
    depth = torch.empty_like(disp)
    w = torch.empty(n, s, device=dev, dtype=torch.float32) if want_weights else None
    if n:
        check(lib.cn_volume_render(ptr(raw), ptr(z), ptr(rd), n, s, ptr(rgb), ptr(disp), ptr(acc), ptr(w), ptr(depth),
                                   stream_of(raw)), "cn_volume_render")
    if w is not None and s == 1:
        w = w[:, :0]          # the reference's S == 1 weights are (R, 0) (see volume.hip)
    return rgb, disp, acc, w, depth


# ------------------------------------------------------------------ MLP


def _fmt(precision: str) -> int:
    if precision not in _lib.FORMATS:
        raise ValueError(f"precision must be one of {sorted(_lib.FORMATS)}, got {precision!r}")
    return _lib.FORMATS[precision]


def mlp_packed_floats(precision: str = "f32") -> int:
    return int(_lib_ready().cn_mlp_packed_floats(_fmt(precision)))


def mlp_pack(params: Sequence[Tensor], precision: str = "f32") -> Tensor:
    """Pack a CodeNeRFModel state_dict (model.py:145-156, state_dict order) for the field kernel.

    precision "f32": fp32 fragments for v_mfma_f32_32x32x2_f32; "bf16x3": bf16 hi/lo
    fragments for the 3-product split on v_mfma_f32_32x32x16_bf16 (include/codenerf.h);
    "bf16x3_t": the transposed 3xbf16 pack of the fused backward.
    """
    lib = _lib_ready()
    assert len(params) == _lib.CN_NUM_PARAMS, "expected the 18 CodeNeRFModel weight/bias tensors"
    params = [_cuda(p.detach(), f"param{i}") for i, p in enumerate(params)]
    out = torch.empty(mlp_packed_floats(precision), device=params[0].device, dtype=torch.float32)
    arr, keep = _lib.pointer_array(params)
    check(lib.cn_mlp_pack(arr, _fmt(precision), ptr(out), stream_of(out)), "cn_mlp_pack")
    del keep
    return out


def code_bias(params: Sequence[Tensor], z_s: Tensor, z_t: Tensor) -> Tensor:
    """Per-code folded terms of CodeNeRFModel.forward (model.py:174-192) -> (n_codes, 520)."""
    lib = _lib_ready()
    params = [_cuda(p.detach(), f"param{i}") for i, p in enumerate(params)]
    z_s, z_t = _cuda(z_s.detach(), "z_s"), _cuda(z_t.detach(), "z_t")
    assert z_s.shape == z_t.shape and z_s.dim() == 2 and z_s.shape[1] == 256, "codes must be (n, 256)"
    out = torch.empty(z_s.shape[0], _lib.CN_CODE_BIAS_STRIDE, device=z_s.device, dtype=torch.float32)
    arr, keep = _lib.pointer_array(params)
    check(lib.cn_code_bias(arr, ptr(z_s), ptr(z_t), z_s.shape[0], ptr(out), stream_of(out)), "cn_code_bias")
    del keep
    return out


def field_prepare(params: Sequence[Tensor], z_s: Tensor, z_t: Tensor, pack: bool = True, pack_t: bool = True,
                  n_zero: int = 0):
    """cn_field_prepare: code_bias(params, z_s, z_t), the fp32 forward / backward packs ("f32_w16",
    "f32_w16_t"; each only if asked) and a zeroed (n_zero,) buffer in ONE launch -> (cb, packed or None,
    packed_t or None, zero or None); bitwise the separate calls' outputs."""
    lib = _lib_ready()
    params = [_cuda(p.detach(), f"param{i}") for i, p in enumerate(params)]
    z_s, z_t = _cuda(z_s.detach(), "z_s"), _cuda(z_t.detach(), "z_t")
    assert z_s.shape == z_t.shape and z_s.dim() == 2 and z_s.shape[1] == 256, "codes must be (n, 256)"
    dev = z_s.device
    cb = torch.empty(z_s.shape[0], _lib.CN_CODE_BIAS_STRIDE, device=dev, dtype=torch.float32)
    nf = mlp_packed_floats("f32_w16")
    packed = torch.empty(nf, device=dev, dtype=torch.float32) if pack else None
    packed_t = torch.empty(nf, device=dev, dtype=torch.float32) if pack_t else None
    zero = torch.empty(n_zero, device=dev, dtype=torch.float32) if n_zero else None
    arr, keep = _lib.pointer_array(params)
    check(lib.cn_field_prepare(arr, ptr(z_s), ptr(z_t), z_s.shape[0], ptr(cb), ptr(packed), ptr(packed_t), ptr(zero),
                               n_zero, stream_of(cb)), "cn_field_prepare")
    del keep
    return cb, packed, packed_t, zero


def field_prepare_models(models: Sequence[Tuple[Sequence[Tensor], bool, bool, int]], z_s: Tensor, z_t: Tensor,
                         want_act: bool = False):
    """cn_field_prepare_models: field_prepare for one or two models (params, pack, pack_t, n_zero) on the
    same codes in ONE launch -> [(cb, packed or None, packed_t or None, zero or None)] per model; bitwise
    each model's field_prepare.  ``want_act``: each tuple also carries the code-layer activations
    (n_codes, 768) (code_ds_outer's operand) as a fifth entry."""
    lib = _lib_ready()
    assert 1 <= len(models) <= 2, "one or two models"
    z_s, z_t = _cuda(z_s.detach(), "z_s"), _cuda(z_t.detach(), "z_t")
    assert z_s.shape == z_t.shape and z_s.dim() == 2 and z_s.shape[1] == 256, "codes must be (n, 256)"
    dev = z_s.device
    nf = mlp_packed_floats("f32_w16")
    outs, keep = [], []
    preps = (_lib.FieldPrep * len(models))()
    for k, (params, pack, pack_t, n_zero) in enumerate(models):
        params = [_cuda(p.detach(), f"param{i}") for i, p in enumerate(params)]
        cb = torch.empty(z_s.shape[0], _lib.CN_CODE_BIAS_STRIDE, device=dev, dtype=torch.float32)
        packed = torch.empty(nf, device=dev, dtype=torch.float32) if pack else None
        packed_t = torch.empty(nf, device=dev, dtype=torch.float32) if pack_t else None
        zero = torch.empty(n_zero, device=dev, dtype=torch.float32) if n_zero else None
        act = torch.empty(z_s.shape[0], 768, device=dev, dtype=torch.float32) if want_act else None
        arr, k_arr = _lib.pointer_array(params)
        keep += [params, arr, k_arr]
        preps[k] = _lib.FieldPrep(arr, ptr(cb), ptr(packed), ptr(packed_t), ptr(zero), n_zero, ptr(act))
        outs.append((cb, packed, packed_t, zero, act) if want_act else (cb, packed, packed_t, zero))
    check(lib.cn_field_prepare_models(preps, len(models), ptr(z_s), ptr(z_t), z_s.shape[0], stream_of(z_s)),
          "cn_field_prepare_models")
    del keep
    return outs


def xenc_columns():
    """The fp32 training forward's encoding plane (cn_field_train_saved_floats): column c' (0..63) ->
    PositionalEmbedder column (position_embed.py:44-53), -1 for the padding slot (mlp_common.h
    xenc_col: lane group g = c' // 16 holds layer_xyz1's k-steps t = c' % 16)."""
    out = []
    for cp in range(64):
        t, g = cp & 15, cp >> 4
        i, p = t & 7, 4 * (t & 7) + g
        if p < 30:
            out.append((3 if t < 8 else 6) + 6 * (p // 3) + p % 3)
        else:
            out.append((0 if g == 2 else 2) if t < 8 else (1 if g == 2 else -1))
    return out


def mlp_forward(packed: Tensor, cb: Tensor, x: Tensor, code_index: Optional[Tensor] = None,
                precision: str = "f32") -> Tensor:
    """CodeNeRFModel.forward on pre-encoded rows (model.py:160-194): (M, 90) -> (M, 4)."""
    lib = _lib_ready()
    x = _cuda(x, "x")
    assert x.dim() == 2 and x.shape[1] == 90, "x must be (M, 63 + 27)"
    m = x.shape[0]
    n_codes = cb.shape[0]
    if code_index is not None:
        code_index = _cuda(code_index, "code_index", torch.int64)
    else:
        assert n_codes in (1, m), "codes must be one row or one row per sample"
    raw = torch.empty(m, 4, device=x.device, dtype=torch.float32)
    if m:
        check(lib.cn_mlp_forward(ptr(packed), _fmt(precision), ptr(cb), ptr(code_index), n_codes, ptr(x), m, ptr(raw),
                                 stream_of(x)),
              "cn_mlp_forward")
    return raw


def radiance_field(packed: Tensor, cb: Tensor, rd: Tensor, n_samples: int, chunk_rows: int,
                   freqs_xyz: Sequence[float], freqs_dir: Sequence[float], pts: Optional[Tensor] = None,
                   ro: Optional[Tensor] = None, z: Optional[Tensor] = None,
                   code_index: Optional[Tensor] = None, precision: str = "f32") -> Tensor:
    """forward_pass (nerf/__init__.py:94-134) fused with the MLP -> raw (R, S, 4)."""
    lib = _lib_ready()
    rd = _cuda(rd, "rd")
    n = rd.shape[0]
    if pts is not None:
        pts = _cuda(pts, "pts")
        assert pts.shape == (n, n_samples, 3), "pts must be (num_rays, num_samples, 3)"
    else:
        ro, z = _cuda(ro, "ro"), _cuda(z, "z")
        assert z.shape == (n, n_samples)
    n_codes = cb.shape[0]
    if code_index is not None:
        code_index = _cuda(code_index, "code_index", torch.int64)
    else:
        assert n_codes in (1, n), "codes must be one row or one row per ray"
    assert len(freqs_xyz) == 10 and len(freqs_dir) == 4, "the field kernel implements L_xyz=10, L_dir=4"
    raw = torch.empty(n, n_samples, 4, device=rd.device, dtype=torch.float32)
    if n:
        check(lib.cn_radiance_field(ptr(packed), _fmt(precision), ptr(cb), ptr(code_index), n_codes, ptr(pts), ptr(ro),
                                    ptr(rd), ptr(z), n, n_samples, chunk_rows, _lib.host_floats(freqs_xyz),
                                    _lib.host_floats(freqs_dir), ptr(raw), stream_of(rd)), "cn_radiance_field")
    return raw


# ------------------------------------------------------------------ backward (A14)


def _opt(t: Optional[Tensor], name: str) -> Optional[Tensor]:
    return None if t is None else _cuda(t, name)


def volume_render_backward(raw: Tensor, z: Tensor, rd: Tensor, g_rgb=None, g_disp=None, g_acc=None,
                           g_weights=None, g_depth=None, want_rd: bool = True,
                           d_rd_into: Optional[Tensor] = None) -> Tuple[Tensor, Optional[Tensor]]:
    """Gradient of volume_render (volumetric_render.py:36-66) -> d_raw (R,S,4), d_rd (R,3) or None.
    ``d_rd_into`` (a contiguous (R, 3) device tensor): d rd ADDED into it (accumulate_rd) and returned."""
    lib = _lib_ready()
    raw, z, rd = _cuda(raw, "radiance_field"), _cuda(z, "depth_values"), _cuda(rd, "ray_directions")
    raw, z = _aligned16(raw), _aligned16(z)
    n, s = z.shape
    assert raw.shape == (n, s, 4) and rd.shape == (n, 3)
    g_rgb, g_disp, g_acc, g_depth = (_opt(g_rgb, "g_rgb"), _opt(g_disp, "g_disp"), _opt(g_acc, "g_acc"),
                                     _opt(g_depth, "g_depth"))
    if g_weights is not None and g_weights.shape[-1] != s:   # S == 1: the reference's weights are (R, 0)
        g_weights = None
    g_weights = _opt(g_weights, "g_weights")
    d_raw = torch.empty_like(raw)
    if d_rd_into is not None:
        assert d_rd_into.is_cuda and d_rd_into.is_contiguous() and d_rd_into.shape == (n, 3)
        d_rd = d_rd_into
    else:
        d_rd = torch.empty_like(rd) if want_rd else None
    if n == 0:      # no rays: empty gradients (the C ABI refuses n_rays == 0), as the forward
        return d_raw, d_rd
    check(lib.cn_volume_render_backward(ptr(raw), ptr(z), ptr(rd), n, s, ptr(g_rgb), ptr(g_disp), ptr(g_acc),
                                        ptr(g_weights), ptr(g_depth), ptr(d_raw), ptr(d_rd),
                                        int(d_rd_into is not None), stream_of(raw)), "cn_volume_render_backward")
    return d_raw, d_rd


def ray_bundle_backward(dirs: Tensor, batch: int, g_ro: Optional[Tensor], g_rd: Optional[Tensor]) -> Tensor:
    """Gradient of get_bundle (ray_sampler.py:95-98) w.r.t. tform_cam2world -> (B, 4, 4)."""
    lib = _lib_ready()
    dirs = _cuda(dirs, "directions")
    hw = dirs.numel() // 3
    g_ro, g_rd = _opt(g_ro, "g_ro"), _opt(g_rd, "g_rd")
    d = torch.zeros(batch, 4, 4, device=dirs.device, dtype=torch.float32)
    if g_ro is None and g_rd is None:
        return d
    check(lib.cn_ray_bundle_backward(ptr(dirs), hw, batch, ptr(g_ro), ptr(g_rd), ptr(d), stream_of(d)),
          "cn_ray_bundle_backward")
    return d


def gather_rays_backward(g_ro: Optional[Tensor], g_rd: Optional[Tensor], batch: int, hw: int,
                         select_inds: Tensor) -> Tuple[Tensor, Tensor]:
    """Gradient of the sample gather (ray_sampler.py:77-80) -> d ro, d rd (B, HW, 3)."""
    lib = _lib_ready()
    sel = _cuda(select_inds, "select_inds", torch.int64)
    g_ro, g_rd = _opt(g_ro, "g_ro"), _opt(g_rd, "g_rd")
    d_ro = torch.zeros(batch, hw, 3, device=sel.device, dtype=torch.float32)
    d_rd = torch.zeros_like(d_ro)
    check(lib.cn_gather_rays_backward(ptr(g_ro), ptr(g_rd), batch, hw, ptr(sel), sel.shape[1], ptr(d_ro), ptr(d_rd),
                                      stream_of(sel)), "cn_gather_rays_backward")
    return d_ro, d_rd


def radiance_field_train(packed: Tensor, cb: Tensor, rd: Tensor, n_samples: int, chunk_rows: int,
                         freqs_xyz: Sequence[float], freqs_dir: Sequence[float], pts: Optional[Tensor] = None,
                         ro: Optional[Tensor] = None, z: Optional[Tensor] = None,
                         code_index: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """fp32 radiance_field that also keeps the activations -> raw (R,S,4), saved (5, R*S, 256)."""
    lib = _lib_ready()
    rd = _cuda(rd, "rd")
    n = rd.shape[0]
    if pts is not None:
        pts = _cuda(pts, "pts")
        assert pts.shape == (n, n_samples, 3)
    else:
        ro, z = _cuda(ro, "ro"), _cuda(z, "z")
        assert z.shape == (n, n_samples)
    if code_index is not None:
        code_index = _cuda(code_index, "code_index", torch.int64)
    raw = torch.empty(n, n_samples, 4, device=rd.device, dtype=torch.float32)
    saved = torch.empty(5, n * n_samples, 256, device=rd.device, dtype=torch.float32)
    if n * n_samples == 0:
        return raw, saved
    check(lib.cn_radiance_field_train(ptr(packed), ptr(cb), ptr(code_index), cb.shape[0], ptr(pts), ptr(ro), ptr(rd),
                                      ptr(z), n, n_samples, chunk_rows, _lib.host_floats(freqs_xyz),
                                      _lib.host_floats(freqs_dir), ptr(raw), ptr(saved), stream_of(rd)),
          "cn_radiance_field_train")
    return raw, saved


def radiance_field_train_w16(packed: Tensor, cb: Tensor, rd: Tensor, n_samples: int, chunk_rows: int,
                             freqs_xyz: Sequence[float], freqs_dir: Sequence[float], pts: Optional[Tensor] = None,
                             ro: Optional[Tensor] = None, z: Optional[Tensor] = None,
                             code_index: Optional[Tensor] = None, precision: str = "f32"):
    """Training forward -> raw (R,S,4), saved (5, R*S, 256), ReLU masks (the fused training backward's
    inputs): precision "f32" on the fp32 16x16x4 kernel (packed "f32_w16"), "bf16x3" on the 3xbf16
    kernel (packed "bf16x3")."""
    fmt = _lib.CN_FMT_BF16X3 if precision == "bf16x3" else _lib.CN_FMT_F32_W16
    lib = _lib_ready()
    rd = _cuda(rd, "rd")
    n = rd.shape[0]
    if pts is not None:
        pts = _cuda(pts, "pts")
        assert pts.shape == (n, n_samples, 3)
    else:
        ro, z = _cuda(ro, "ro"), _cuda(z, "z")
        assert z.shape == (n, n_samples)
    if code_index is not None:
        code_index = _cuda(code_index, "code_index", torch.int64)
    m = n * n_samples
    raw = torch.empty(n, n_samples, 4, device=rd.device, dtype=torch.float32)
    if m == 0:
        return (raw, torch.empty(5, 0, 256, device=rd.device, dtype=torch.float32),
                torch.empty(0, device=rd.device, dtype=torch.int32))
    # the planes (+ fp32: the encoding plane) + one scratch row (cn_radiance_field_train_fmt); ``saved`` is
    # the (5, m, 256) planes view, the backward finds the encoding plane after them in the same storage
    buf = torch.empty(int(lib.cn_field_train_saved_floats(fmt, m)), device=rd.device, dtype=torch.float32)
    saved = buf[:5 * m * 256].view(5, m, 256)
    masks = torch.empty(int(lib.cn_field_mask_words_fmt(fmt, m)), device=rd.device, dtype=torch.int32)
    check(lib.cn_radiance_field_train_fmt(fmt, ptr(packed), ptr(cb), ptr(code_index), cb.shape[0], ptr(pts), ptr(ro),
                                          ptr(rd), ptr(z), n, n_samples, chunk_rows, _lib.host_floats(freqs_xyz),
                                          _lib.host_floats(freqs_dir), ptr(raw), ptr(saved), ptr(masks),
                                          stream_of(rd)), "cn_radiance_field_train_fmt")
    return raw, saved, masks


def field_backward_train(packed_t: Tensor, params: Sequence[Tensor], masks: Tensor, saved: Tensor,
                         x_enc: Optional[Tensor],
                         d_raw: Tensor, n_rays: int, n_samples: int, chunk_rows: int, n_codes: int,
                         freqs_xyz: Sequence[float], freqs_dir: Sequence[float], rd: Tensor,
                         pts: Optional[Tensor] = None, ro: Optional[Tensor] = None, z: Optional[Tensor] = None,
                         code_index: Optional[Tensor] = None, param_grads: Optional[Sequence[Tensor]] = None,
                         want_pts: bool = False, want_ro: bool = False, want_rd: bool = False,
                         precision: str = "f32", g_code: Optional[Tensor] = None):
    """Fused training backward (one dX launch + deterministic dW GEMMs) -> dict g_code / d_pts / d_ro / d_rd.
    precision "f32" (packed_t "f32_w16_t") or "bf16x3" (packed_t "bf16x3_t", 3xbf16 dW GEMMs).
    ``g_code``: a zeroed (n_codes, CN_CODE_BIAS_STRIDE) accumulator (field_prepare's), else allocated."""
    return field_backward_train_multi([dict(
        packed_t=packed_t, params=params, masks=masks, saved=saved, x_enc=x_enc, d_raw=d_raw, n_rays=n_rays,
        n_samples=n_samples, chunk_rows=chunk_rows, n_codes=n_codes, freqs_xyz=freqs_xyz, freqs_dir=freqs_dir, rd=rd,
        pts=pts, ro=ro, z=z, code_index=code_index, param_grads=param_grads, want_pts=want_pts, want_ro=want_ro,
        want_rd=want_rd, g_code=g_code)], precision)[0]


def field_backward_train_multi(fields: Sequence[dict], precision: str = "f32"):
    """The training backwards of a render's fields (field_backward_train's keyword arguments, one dict
    per field, 1 or 2) through ONE cn_field_backward_train_multi call: with two fp32 fields on rays +
    depths, one dX launch, one batched dW launch (layer_xyz1's dW among its jobs), one DIRS-pass launch
    and one reduction launch for both, every gradient bitwise that of the per-field calls -> one result
    dict per field."""
    assert len(fields) in (1, 2)
    fmt_t = _lib.CN_FMT_BF16X3_T if precision == "bf16x3" else _lib.CN_FMT_F32_W16_T
    lib = _lib_ready()
    outs, structs, keep = [], [], []
    stream = None
    for f in fields:
        n_rays, n_samples, n_codes = f["n_rays"], f["n_samples"], f["n_codes"]
        m = n_rays * n_samples
        params = [_cuda(p.detach(), f"param{i}") for i, p in enumerate(f["params"])]
        d_raw = _aligned16(_cuda(f["d_raw"], "d_raw"))
        saved, x_enc = f["saved"], f.get("x_enc")
        assert d_raw.numel() == 4 * m and saved.shape == (5, m, 256) and (x_enc is None or x_enc.shape == (m, 90))
        if m and precision != "bf16x3" and x_enc is None:
            # the fp32 backward reads the forward's encoding plane at saved + 5 M 256 (cn_field_backward_train_fmt):
            # ``saved`` must be radiance_field_train_w16's view of its whole save buffer, not a copy of the planes
            need = 4 * int(lib.cn_field_train_saved_floats(_lib.CN_FMT_F32_W16, m))
            assert saved.is_contiguous() and saved.storage_offset() == 0 and \
                saved.untyped_storage().nbytes() >= need, \
                "field_backward_train: saved must be the training forward's own buffer (planes + encoding plane)"
        dev = d_raw.device
        rd, pts, ro, z = _opt(f["rd"], "rd"), _opt(f.get("pts"), "pts"), _opt(f.get("ro"), "ro"), _opt(f.get("z"), "z")
        code_index = f.get("code_index")
        if code_index is not None:
            code_index = _cuda(code_index, "code_index", torch.int64)
        ws = torch.empty(max(0, int(lib.cn_field_backward_train_workspace_floats(m))), device=dev, dtype=torch.float32)
        g_code = f.get("g_code")
        if g_code is None:
            g_code = torch.zeros(n_codes, _lib.CN_CODE_BIAS_STRIDE, device=dev, dtype=torch.float32)
        else:
            assert g_code.shape == (n_codes, _lib.CN_CODE_BIAS_STRIDE) and g_code.is_contiguous()
        d_pts = torch.empty(n_rays, n_samples, 3, device=dev, dtype=torch.float32) if f.get("want_pts") else None
        d_ro = torch.zeros(n_rays, 3, device=dev, dtype=torch.float32) if f.get("want_ro") else None
        d_rd = torch.zeros(n_rays, 3, device=dev, dtype=torch.float32) if f.get("want_rd") else None
        outs.append({"g_code": g_code, "d_pts": d_pts, "d_ro": d_ro, "d_rd": d_rd})
        if m == 0:      # no samples: nothing accumulates (the C ABI refuses n_rays == 0)
            continue
        arr, k1 = _lib.pointer_array(params)
        garr, k2 = (None, None)
        pg = f.get("param_grads")
        if pg is not None:
            assert len(pg) == _lib.CN_NUM_PARAMS and all(g.is_contiguous() for g in pg)
            garr, k2 = _lib.pointer_array(list(pg))
        fx, fd = _lib.host_floats(f["freqs_xyz"]), _lib.host_floats(f["freqs_dir"])
        keep += [params, d_raw, ws, arr, k1, garr, k2, fx, fd, rd, pts, ro, z, code_index]
        structs.append(_lib.FieldTrainBwd(
            ptr(f["packed_t"]), arr, ptr(f["masks"]), ptr(saved), ptr(x_enc), ptr(d_raw), ptr(pts), ptr(ro), ptr(rd),
            ptr(z), n_rays, n_samples, f["chunk_rows"], ptr(code_index), n_codes,
            ctypes.cast(fx, ctypes.POINTER(ctypes.c_float)), ctypes.cast(fd, ctypes.POINTER(ctypes.c_float)), ptr(ws),
            garr, ptr(g_code), ptr(d_pts), ptr(d_ro), ptr(d_rd)))
        stream = stream_of(d_raw)
    if structs:
        jobs = (_lib.FieldTrainBwd * len(structs))(*structs)
        check(lib.cn_field_backward_train_multi(fmt_t, jobs, len(structs), stream), "cn_field_backward_train_multi")
    del keep
    return outs


def mlp_forward_train(packed: Tensor, cb: Tensor, x: Tensor, code_index: Optional[Tensor] = None
                      ) -> Tuple[Tensor, Tensor]:
    """fp32 mlp_forward that also keeps the activations -> raw (M,4), saved (5, M, 256)."""
    lib = _lib_ready()
    x = _cuda(x, "x")
    assert x.dim() == 2 and x.shape[1] == 90
    m = x.shape[0]
    if code_index is not None:
        code_index = _cuda(code_index, "code_index", torch.int64)
    raw = torch.empty(m, 4, device=x.device, dtype=torch.float32)
    saved = torch.empty(5, m, 256, device=x.device, dtype=torch.float32)
    check(lib.cn_mlp_forward_train(ptr(packed), ptr(cb), ptr(code_index), cb.shape[0], ptr(x), m, ptr(raw),
                                   ptr(saved), stream_of(x)), "cn_mlp_forward_train")
    return raw, saved


def encode_inputs(rd: Tensor, n_samples: int, chunk_rows: int, freqs_xyz: Sequence[float],
                  freqs_dir: Sequence[float], pts: Optional[Tensor] = None, ro: Optional[Tensor] = None,
                  z: Optional[Tensor] = None) -> Tensor:
    """forward_pass's MLP input rows (nerf/__init__.py:116-132) -> (R*S, 90)."""
    lib = _lib_ready()
    rd = _cuda(rd, "rd")
    n = rd.shape[0]
    pts, ro, z = _opt(pts, "pts"), _opt(ro, "ro"), _opt(z, "z")
    x = torch.empty(n * n_samples, 90, device=rd.device, dtype=torch.float32)
    if n * n_samples == 0:
        return x
    check(lib.cn_encode_inputs(ptr(pts), ptr(ro), ptr(rd), ptr(z), n, n_samples, chunk_rows,
                               _lib.host_floats(freqs_xyz), _lib.host_floats(freqs_dir), ptr(x), stream_of(rd)),
          "cn_encode_inputs")
    return x


def field_backward(params: Sequence[Tensor], saved: Tensor, x_enc: Tensor, d_raw: Tensor, n_rays: int,
                   n_samples: int, chunk_rows: int, n_codes: int, freqs_xyz=None, freqs_dir=None,
                   rd: Optional[Tensor] = None, pts: Optional[Tensor] = None, ro: Optional[Tensor] = None,
                   z: Optional[Tensor] = None, code_index: Optional[Tensor] = None,
                   param_grads: Optional[Sequence[Tensor]] = None, want_code: bool = False,
                   want_pts: bool = False, want_ro: bool = False, want_rd: bool = False, want_x: bool = False,
                   precision: str = "f32"):
    """Backward of forward_pass + CodeNeRFModel.forward -> dict of d_pts / d_ro / d_rd / g_code / d_x.

    ``param_grads``: 18 zero-or-running fp32 buffers the parameter gradients accumulate into.
    ``precision``: the GEMMs' arithmetic, "f32" (exact products) or "bf16x3" (split bf16 MFMA).
    """
    lib = _lib_ready()
    m = n_rays * n_samples
    params = [_cuda(p.detach(), f"param{i}") for i, p in enumerate(params)]
    d_raw = _aligned16(_cuda(d_raw, "d_raw"))
    assert d_raw.numel() == 4 * m and saved.shape == (5, m, 256) and (x_enc is None or x_enc.shape == (m, 90))
    dev = d_raw.device
    rd, pts, ro, z = _opt(rd, "rd"), _opt(pts, "pts"), _opt(ro, "ro"), _opt(z, "z")
    if code_index is not None:
        code_index = _cuda(code_index, "code_index", torch.int64)
    ws = torch.empty(max(0, int(lib.cn_field_backward_workspace_floats(m))), device=dev, dtype=torch.float32)
    out = {}
    g_code = torch.zeros(n_codes, _lib.CN_CODE_BIAS_STRIDE, device=dev, dtype=torch.float32) if want_code else None
    d_pts = torch.empty(n_rays, n_samples, 3, device=dev, dtype=torch.float32) if want_pts else None
    d_ro = torch.zeros(n_rays, 3, device=dev, dtype=torch.float32) if want_ro else None
    d_rd = torch.zeros(n_rays, 3, device=dev, dtype=torch.float32) if want_rd else None
    if m == 0:      # no samples: zero sums (the C ABI refuses n_rays == 0)
        out.update(g_code=g_code, d_pts=d_pts, d_ro=d_ro, d_rd=d_rd)
        if want_x:
            out["d_x"] = torch.empty(0, 90, device=dev, dtype=torch.float32)
        return out
    arr, keep = _lib.pointer_array(params)
    garr, gkeep = (None, None)
    if param_grads is not None:
        assert len(param_grads) == _lib.CN_NUM_PARAMS and all(g.is_contiguous() for g in param_grads)
        garr, gkeep = _lib.pointer_array(list(param_grads))
    fx = _lib.host_floats(freqs_xyz) if freqs_xyz is not None else None
    fd = _lib.host_floats(freqs_dir) if freqs_dir is not None else None
    check(lib.cn_field_backward_fmt(_lib.FORMATS[precision], arr, ptr(saved), ptr(x_enc), ptr(d_raw), ptr(pts), ptr(ro), ptr(rd), ptr(z), n_rays,
                                n_samples, chunk_rows, ptr(code_index), n_codes, fx, fd, ptr(ws), garr, ptr(g_code),
                                ptr(d_pts), ptr(d_ro), ptr(d_rd), stream_of(d_raw)), "cn_field_backward_fmt")
    del keep, gkeep
    out.update(g_code=g_code, d_pts=d_pts, d_ro=d_ro, d_rd=d_rd)
    if want_x:
        off = int(lib.cn_field_backward_dx_offset(m))
        out["d_x"] = ws[off: off + 90 * m].view(m, 90)
    return out


def code_bias_backward(params: Sequence[Tensor], z_s: Tensor, z_t: Tensor, g_code: Tensor,
                       param_grads: Optional[Sequence[Tensor]] = None, want_z: bool = True,
                       single_launch: bool = False, dz_into: Optional[Tuple[Tensor, Tensor]] = None):
    """Backward of code_bias (model.py:174-177 + the code halves) -> dz_s, dz_t (n_codes, 256) or None.
    The two-launch form (cn_code_bias_backward_ws) unless single_launch (cn_code_bias_backward):
    bitwise the same results.  ``dz_into`` (two contiguous (n_codes, 256) device tensors, two-launch
    form): the code gradients are ADDED into them (accumulate_dz) and returned."""
    lib = _lib_ready()
    params = [_cuda(p.detach(), f"param{i}") for i, p in enumerate(params)]
    z_s, z_t, g_code = _cuda(z_s.detach(), "z_s"), _cuda(z_t.detach(), "z_t"), _cuda(g_code, "g_code")
    n = z_s.shape[0]
    if dz_into is not None:
        assert not single_launch, "dz_into: the two-launch form"
        for d in dz_into:
            assert d.is_cuda and d.dtype == torch.float32 and d.is_contiguous() and d.shape == z_s.shape, \
                "dz_into: contiguous (n_codes, 256) fp32 device tensors"
        dz_s, dz_t = dz_into
    else:
        dz_s = torch.empty_like(z_s) if want_z else None
        dz_t = torch.empty_like(z_t) if want_z else None
    arr, keep = _lib.pointer_array(params)
    garr, gkeep = (None, None)
    if param_grads is not None:
        garr, gkeep = _lib.pointer_array(list(param_grads))
    if single_launch:
        check(lib.cn_code_bias_backward(arr, ptr(z_s), ptr(z_t), n, ptr(g_code), ptr(dz_s), ptr(dz_t), garr,
                                        stream_of(g_code)), "cn_code_bias_backward")
    else:
        ws = torch.empty(lib.cn_code_bias_backward_workspace_floats(n), device=g_code.device, dtype=torch.float32)
        check(lib.cn_code_bias_backward_ws(arr, ptr(z_s), ptr(z_t), n, ptr(g_code), ptr(dz_s), ptr(dz_t), garr,
                                           ptr(ws), int(dz_into is not None), stream_of(g_code)),
              "cn_code_bias_backward_ws")
    del keep, gkeep
    return dz_s, dz_t


def code_ds_outer(params: Sequence[Tensor], z_s: Tensor, z_t: Tensor, code_act: Tensor, g_code: Tensor,
                  param_grads: Optional[Sequence[Tensor]] = None) -> Tensor:
    """cn_code_bias_backward_act: the code backward's first half on the forward's code-layer activations
    (field_prepare_models(..., want_act=True)) -> its workspace (the masked ds1 / ds2 / dt1, for code_dz);
    the code layers' and code halves' gradients are added into ``param_grads``."""
    lib = _lib_ready()
    params = [_cuda(p.detach(), f"param{i}") for i, p in enumerate(params)]
    z_s, z_t, g_code = _cuda(z_s.detach(), "z_s"), _cuda(z_t.detach(), "z_t"), _cuda(g_code, "g_code")
    code_act = _cuda(code_act, "code_act")
    n = z_s.shape[0]
    assert code_act.numel() == n * 768, "code_act: (n_codes, 768)"
    ws = torch.empty(lib.cn_code_bias_backward_workspace_floats(n), device=g_code.device, dtype=torch.float32)
    arr, keep = _lib.pointer_array(params)
    garr, gkeep = _lib.pointer_array(list(param_grads)) if param_grads is not None else (None, None)
    check(lib.cn_code_bias_backward_act(arr, ptr(z_s), ptr(z_t), n, ptr(code_act), ptr(g_code), garr, ptr(ws),
                                        stream_of(g_code)), "cn_code_bias_backward_act")
    del keep, gkeep
    return ws


def code_ds_outer_multi(jobs, z_s: Tensor, z_t: Tensor):
    """code_ds_outer of a render's 1 or 2 fields on the same codes in ONE launch
    (cn_code_bias_backward_act_multi); jobs: [(params, code_act, g_code, param_grads | None)] -> the
    workspaces, one per job (bitwise code_ds_outer's)."""
    lib = _lib_ready()
    assert 1 <= len(jobs) <= 2, "one or two jobs"
    z_s, z_t = _cuda(z_s.detach(), "z_s"), _cuda(z_t.detach(), "z_t")
    n = z_s.shape[0]
    structs, keep, outs = [], [], []
    for params, code_act, g_code, param_grads in jobs:
        params = [_cuda(p.detach(), f"param{i}") for i, p in enumerate(params)]
        g_code, code_act = _cuda(g_code, "g_code"), _cuda(code_act, "code_act")
        assert code_act.numel() == n * 768, "code_act: (n_codes, 768)"
        ws = torch.empty(lib.cn_code_bias_backward_workspace_floats(n), device=g_code.device, dtype=torch.float32)
        arr, k1 = _lib.pointer_array(params)
        garr, k2 = _lib.pointer_array(list(param_grads)) if param_grads is not None else (None, None)
        keep += [params, g_code, code_act, arr, k1, garr, k2]
        structs.append(_lib.CodeActJob(arr, ptr(code_act), ptr(g_code), garr, ptr(ws)))
        outs.append(ws)
    js = (_lib.CodeActJob * len(structs))(*structs)
    check(lib.cn_code_bias_backward_act_multi(js, len(structs), ptr(z_s), ptr(z_t), n, stream_of(z_s)),
          "cn_code_bias_backward_act_multi")
    del keep
    return outs


def code_dz(jobs: Sequence[Tuple[Sequence[Tensor], Tensor, Tensor]], n_codes: int,
            dz_into: Optional[Tuple[Tensor, Tensor]] = None):
    """cn_code_dz: dz_s, dz_t of one or two fields' code backwards [(params, g_code, code_ds_outer's
    workspace)] on the same codes, summed in job order -> fresh (n_codes, 256) tensors, or ADDED into
    ``dz_into`` (contiguous (n_codes, 256) device tensors) and those returned."""
    lib = _lib_ready()
    assert 1 <= len(jobs) <= 2, "one or two jobs"
    dev = jobs[0][1].device
    if dz_into is not None:
        for d in dz_into:
            assert d.is_cuda and d.dtype == torch.float32 and d.is_contiguous() and d.shape == (n_codes, 256), \
                "dz_into: contiguous (n_codes, 256) fp32 device tensors"
        dz_s, dz_t = dz_into
    else:
        dz_s = torch.empty(n_codes, 256, device=dev, dtype=torch.float32)
        dz_t = torch.empty(n_codes, 256, device=dev, dtype=torch.float32)
    arr = (_lib.CodeDzJob * len(jobs))()
    keep = []
    for k, (params, g_code, ws) in enumerate(jobs):
        params = [_cuda(p.detach(), f"param{i}") for i, p in enumerate(params)]
        pa, pk = _lib.pointer_array(params)
        keep += [params, pa, pk]
        arr[k] = _lib.CodeDzJob(pa, ptr(_cuda(g_code, "g_code")), ptr(ws))
    check(lib.cn_code_dz(arr, len(jobs), n_codes, ptr(dz_s), ptr(dz_t), int(dz_into is not None), stream_of(dz_s)),
          "cn_code_dz")
    del keep
    return dz_s, dz_t


def gemm_nn(a: Tensor, b: Tensor, mask: Optional[Tensor] = None, precision: str = "f32") -> Tensor:
    """C = A B (masked where mask <= 0) on the fp32 (or 3xbf16) MFMA tile kernel."""
    lib = _lib_ready()
    # A may be a row-strided view (lda > k, unit column stride), as the field backward's
    # (M, 257)-in-rows-of-260 gradient buffers are
    if not (a.is_cuda and a.dtype == torch.float32 and a.dim() == 2 and a.stride(1) == 1 and a.stride(0) >= a.shape[1]):
        a = _cuda(a, "A")
    b = _cuda(b, "B")
    (m, k), (k2, n) = a.shape, b.shape
    assert k == k2
    mask = _opt(mask, "mask")
    c = torch.empty(m, n, device=a.device, dtype=torch.float32)
    fn, name = (lib.cn_gemm_nn_x3, "cn_gemm_nn_x3") if precision == "bf16x3" else (lib.cn_gemm_nn, "cn_gemm_nn")
    check(fn(ptr(a), a.stride(0), ptr(b), n, ptr(c), n, ptr(mask), n, m, n, k, stream_of(a)), name)
    return c


def gemm_tn(a: Tensor, b: Tensor, c: Optional[Tensor] = None, precision: str = "f32",
            deterministic: bool = False) -> Tensor:
    """C += A^T B on the fp32 (or 3xbf16) MFMA tile kernel (C zero-initialised when not given).
    deterministic: partial tiles + a fixed-order reduction (cn_gemm_tn_ws) instead of float atomics."""
    lib = _lib_ready()
    a, b = _cuda(a, "A"), _cuda(b, "B")
    (m, n), (m2, k) = a.shape, b.shape
    assert m == m2
    if c is None:
        c = torch.zeros(n, k, device=a.device, dtype=torch.float32)
    if deterministic:
        ws = torch.empty(lib.cn_gemm_tn_workspace_floats(m, n, k), device=a.device, dtype=torch.float32)
        fmt = _lib.FORMATS["bf16x3" if precision == "bf16x3" else "f32"]
        check(lib.cn_gemm_tn_ws(fmt, ptr(a), n, ptr(b), k, ptr(c), k, m, n, k, ptr(ws), stream_of(a)), "cn_gemm_tn_ws")
        return c
    fn, name = (lib.cn_gemm_tn_x3, "cn_gemm_tn_x3") if precision == "bf16x3" else (lib.cn_gemm_tn, "cn_gemm_tn")
    check(fn(ptr(a), n, ptr(b), k, ptr(c), k, m, n, k, stream_of(a)), name)
    return c


def posenc_backward(x: Tensor, freqs: Sequence[float], include_input: bool, g_enc: Tensor) -> Tensor:
    """Gradient of PositionalEmbedder.embed (position_embed.py:35-53) w.r.t. its input."""
    lib = _lib_ready()
    x, g_enc = _cuda(x, "x"), _cuda(g_enc, "g_enc")
    d = x.shape[-1]
    m = x.numel() // d
    assert g_enc.numel() == m * d * (int(include_input) + 2 * len(freqs))
    dx = torch.empty_like(x)
    check(lib.cn_posenc_backward(ptr(x), m, d, _lib.host_floats(freqs), len(freqs), int(include_input), ptr(g_enc),
                                 ptr(dx), stream_of(x)), "cn_posenc_backward")
    return dx


def ray_points_backward(g_pts: Tensor, z: Tensor, want_ro: bool = True, want_rd: bool = True):
    """Gradient of pts = ro + rd z (point_sampler.py:70, :118; z detached) -> d_ro, d_rd (R, 3)."""
    lib = _lib_ready()
    g_pts, z = _cuda(g_pts, "g_pts"), _cuda(z, "z")
    n, s = z.shape
    assert g_pts.shape == (n, s, 3)
    d_ro = torch.zeros(n, 3, device=z.device, dtype=torch.float32) if want_ro else None
    d_rd = torch.zeros(n, 3, device=z.device, dtype=torch.float32) if want_rd else None
    if want_ro or want_rd:
        check(lib.cn_ray_points_backward(ptr(g_pts), ptr(z), n, s, ptr(d_ro), ptr(d_rd), stream_of(z)),
              "cn_ray_points_backward")
    return d_ro, d_rd


# ------------------------------------------------------------------ fused 3xbf16 backward (eval step)


def radiance_field_masks(packed: Tensor, cb: Tensor, rd: Tensor, n_samples: int, chunk_rows: int,
                         freqs_xyz: Sequence[float], freqs_dir: Sequence[float], pts: Optional[Tensor] = None,
                         ro: Optional[Tensor] = None, z: Optional[Tensor] = None,
                         code_index: Optional[Tensor] = None, precision: str = "bf16x3") -> Tuple[Tensor, Tensor]:
    """radiance_field that also writes the ReLU masks of the fused backward -> raw (R,S,4), masks (uint32
    words as int32).  precision "bf16x3" (packed "bf16x3") or "f32" (packed "f32_w16": the fp32
    16x16x4 kernel)."""
    fmt = _lib.CN_FMT_BF16X3 if precision == "bf16x3" else _lib.CN_FMT_F32_W16
    lib = _lib_ready()
    rd = _cuda(rd, "rd")
    n = rd.shape[0]
    if pts is not None:
        pts = _cuda(pts, "pts")
        assert pts.shape == (n, n_samples, 3)
    else:
        ro, z = _cuda(ro, "ro"), _cuda(z, "z")
        assert z.shape == (n, n_samples)
    if code_index is not None:
        code_index = _cuda(code_index, "code_index", torch.int64)
    m = n * n_samples
    raw = torch.empty(n, n_samples, 4, device=rd.device, dtype=torch.float32)
    if m == 0:
        return raw, torch.empty(0, device=rd.device, dtype=torch.int32)
    masks = torch.empty(int(lib.cn_field_mask_words_fmt(fmt, m)), device=rd.device, dtype=torch.int32)
    check(lib.cn_radiance_field_masks_fmt(fmt, ptr(packed), ptr(cb), ptr(code_index), cb.shape[0], ptr(pts), ptr(ro),
                                          ptr(rd), ptr(z), n, n_samples, chunk_rows, _lib.host_floats(freqs_xyz),
                                          _lib.host_floats(freqs_dir), ptr(raw), ptr(masks), stream_of(rd)),
          "cn_radiance_field_masks_fmt")
    return raw, masks


def fused_backward_supported(n_codes: int, n_samples: int, code_index: Optional[Tensor] = None,
                             precision: str = "bf16x3") -> bool:
    """cn_field_backward_fused needs one code row per wave: 32 consecutive samples (bf16x3) or 16 (f32)."""
    return n_codes == 1 or n_samples % (32 if precision == "bf16x3" else 16) == 0


def field_backward_x3_acc_floats(n_codes: int, n_rays: int, want_ro: bool, want_rd: bool) -> int:
    """Floats of field_backward_x3's zeroed accumulator buffer: g_code, then d ro / d rd if wanted."""
    return n_codes * _lib.CN_CODE_BIAS_STRIDE + 3 * n_rays * (int(want_ro) + int(want_rd))


def field_backward_x3(packed_t: Tensor, masks: Tensor, d_raw: Tensor, n_rays: int, n_samples: int,
                      chunk_rows: int, n_codes: int, freqs_xyz: Sequence[float], freqs_dir: Sequence[float],
                      rd: Tensor, pts: Optional[Tensor] = None, ro: Optional[Tensor] = None,
                      z: Optional[Tensor] = None, code_index: Optional[Tensor] = None, want_pts: bool = False,
                      want_ro: bool = False, want_rd: bool = False, precision: str = "bf16x3",
                      acc: Optional[Tensor] = None, ray_into: Optional[Tuple[Tensor, Tensor]] = None,
                      deterministic: bool = True):
    """Fused backward of forward_pass + CodeNeRFModel.forward (frozen weights) -> g_code / d_pts / d_ro / d_rd.
    precision "bf16x3" (packed_t "bf16x3_t") or "f32" (packed_t "f32_w16_t", masks of the f32_w16 forward).
    ``acc``: a zeroed buffer of field_backward_x3_acc_floats(...) floats for the accumulated outputs
    (field_prepare's), else one is allocated and filled.  ``ray_into`` ((R, 3) d ro, d rd device tensors,
    with want_ro and want_rd): the ray gradients are ADDED into those instead.  ``deterministic`` (default):
    with one code row and S % 32 (bf16x3) / % 16 (f32) == 0, cn_field_backward_fused_ws's form without
    float atomics, so repeated backwards give the same bits (False: the float-atomic kernel)."""
    fmt_t = _lib.CN_FMT_BF16X3_T if precision == "bf16x3" else _lib.CN_FMT_F32_W16_T
    lib = _lib_ready()
    m = n_rays * n_samples
    d_raw = _aligned16(_cuda(d_raw, "d_raw"))
    assert d_raw.numel() == 4 * m
    dev = d_raw.device
    rd, pts, ro, z = _opt(rd, "rd"), _opt(pts, "pts"), _opt(ro, "ro"), _opt(z, "z")
    if code_index is not None:
        code_index = _cuda(code_index, "code_index", torch.int64)
    # the accumulated outputs share one zero-filled buffer (one fill launch instead of three)
    nc = n_codes * _lib.CN_CODE_BIAS_STRIDE
    n_acc = field_backward_x3_acc_floats(n_codes, n_rays, want_ro, want_rd)
    if acc is None:
        acc = torch.zeros(n_acc, device=dev, dtype=torch.float32)
    else:
        assert acc.numel() == n_acc and acc.is_contiguous()
    g_code = acc[:nc].view(n_codes, _lib.CN_CODE_BIAS_STRIDE)
    d_ro = acc[nc:nc + 3 * n_rays].view(n_rays, 3) if want_ro else None
    d_rd = acc[acc.numel() - 3 * n_rays:].view(n_rays, 3) if want_rd else None
    if ray_into is not None:
        assert want_ro and want_rd and all(t.is_cuda and t.is_contiguous() and t.shape == (n_rays, 3) for t in ray_into)
        d_ro, d_rd = ray_into
    d_pts = torch.empty(n_rays, n_samples, 3, device=dev, dtype=torch.float32) if want_pts else None
    if m == 0:      # no samples: zero sums (the C ABI refuses n_rays == 0)
        return {"g_code": g_code, "d_pts": d_pts, "d_ro": d_ro, "d_rd": d_rd}
    # one code row, every wave inside one ray: the deterministic form (no float atomics; its partials in a
    # workspace, summed in a fixed order by two short launches), else the float-atomic kernel
    ws = None
    if deterministic and n_codes == 1 and n_samples % (32 if precision == "bf16x3" else 16) == 0:
        ws = torch.empty(int(lib.cn_field_backward_fused_workspace_floats(fmt_t, n_rays, n_samples)), device=dev,
                         dtype=torch.float32)
    check(lib.cn_field_backward_fused_ws(fmt_t, ptr(packed_t), ptr(masks), ptr(d_raw), ptr(pts), ptr(ro), ptr(rd),
                                         ptr(z), n_rays, n_samples, chunk_rows, ptr(code_index), n_codes,
                                         _lib.host_floats(freqs_xyz), _lib.host_floats(freqs_dir), ptr(g_code),
                                         ptr(d_pts), ptr(d_ro), ptr(d_rd), ptr(ws), stream_of(d_raw)),
          "cn_field_backward_fused_ws")
    return {"g_code": g_code, "d_pts": d_pts, "d_ro": d_ro, "d_rd": d_rd}


def field_backward_x3_multi(fields: Sequence[dict], d_rd_between: Optional[Tensor] = None):
    """The eval step's two fields' fused backwards (field_backward_x3's keyword arguments, one dict per
    field, both adding into the same ``ray_into`` d ro / d rd) through ONE cn_field_backward_fused_multi
    call: fp32, one code row, whole waves per ray -> one dX launch, one ray / g_code-row launch and one
    g_code reduction for both.  d ro / d rd end bitwise as field 0's call, then d rd += ``d_rd_between``,
    then field 1's call.  -> one result dict per field."""
    assert len(fields) == 2
    lib = _lib_ready()
    fmt_t = _lib.CN_FMT_F32_W16_T
    structs, keep, outs = [], [], []
    stream = None
    for f in fields:
        assert f.get("precision", "f32") == "f32" and f.get("ray_into") is not None and f.get("acc") is not None
        n_rays, n_samples, n_codes = f["n_rays"], f["n_samples"], f["n_codes"]
        assert n_codes == 1 and n_samples % 16 == 0 and f.get("pts") is None and not f.get("want_pts")
        m = n_rays * n_samples
        d_raw = _aligned16(_cuda(f["d_raw"], "d_raw"))
        assert d_raw.numel() == 4 * m and m > 0
        dev = d_raw.device
        rd, ro, z = _opt(f["rd"], "rd"), _opt(f.get("ro"), "ro"), _opt(f.get("z"), "z")
        acc = f["acc"]
        assert acc.numel() == field_backward_x3_acc_floats(n_codes, n_rays, True, True) and acc.is_contiguous()
        g_code = acc[:_lib.CN_CODE_BIAS_STRIDE].view(1, _lib.CN_CODE_BIAS_STRIDE)
        d_ro, d_rd = f["ray_into"]
        assert all(t.is_cuda and t.is_contiguous() and t.shape == (n_rays, 3) for t in (d_ro, d_rd))
        ws = torch.empty(int(lib.cn_field_backward_fused_workspace_floats(fmt_t, n_rays, n_samples)), device=dev,
                         dtype=torch.float32)
        fx, fd = _lib.host_floats(f["freqs_xyz"]), _lib.host_floats(f["freqs_dir"])
        keep += [d_raw, rd, ro, z, ws, fx, fd]
        structs.append(_lib.FieldFusedBwd(
            ptr(f["packed_t"]), ptr(f["masks"]), ptr(d_raw), None, ptr(ro), ptr(rd), ptr(z), n_rays, n_samples,
            f["chunk_rows"], None, 1, ctypes.cast(fx, ctypes.POINTER(ctypes.c_float)),
            ctypes.cast(fd, ctypes.POINTER(ctypes.c_float)), ptr(g_code), None, ptr(d_ro), ptr(d_rd), ptr(ws)))
        outs.append({"g_code": g_code, "d_pts": None, "d_ro": d_ro, "d_rd": d_rd})
        stream = stream_of(d_raw)
    if d_rd_between is not None:
        d_rd_between = _cuda(d_rd_between, "d_rd_between").contiguous()
        assert d_rd_between.shape == outs[0]["d_rd"].shape
    js = (_lib.FieldFusedBwd * 2)(*structs)
    check(lib.cn_field_backward_fused_multi(fmt_t, js, 2, ptr(d_rd_between), stream), "cn_field_backward_fused_multi")
    del keep
    return outs


# ------------------------------------------------------------------ training step: optimiser


def adamw_step(param: Tensor, grad: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor, segments,
               beta1: float, beta2: float, eps: float) -> None:
    """torch.optim.AdamW.step (train.py:113) on flat fp32 buffers, in place (cn_adamw_step).

    ``segments``: [(begin, end, lr, weight_decay, step)] float ranges (multiples of 4).
    """
    lib = _lib_ready()
    bufs = [_cuda(t, name) for t, name in ((param, "param"), (grad, "grad"), (exp_avg, "exp_avg"),
                                          (exp_avg_sq, "exp_avg_sq"))]
    n = param.numel()
    assert all(b.data_ptr() == t.data_ptr() and b.numel() == n for b, t in zip(bufs, (param, grad, exp_avg, exp_avg_sq))), \
        "flat optimiser buffers must be contiguous and of one size"
    assert segments and all(b % 4 == 0 and e % 4 == 0 and 0 <= b < e <= n for b, e, *_ in segments)
    k = len(segments)

    def arr(ct, vals):
        return (ct * k)(*vals)
    check(lib.cn_adamw_step(ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), k,
                            arr(ctypes.c_int64, [int(s[0]) for s in segments]),
                            arr(ctypes.c_int64, [int(s[1]) for s in segments]),
                            arr(ctypes.c_double, [float(s[2]) for s in segments]),
                            arr(ctypes.c_double, [float(s[3]) for s in segments]),
                            arr(ctypes.c_int64, [int(s[4]) for s in segments]),
                            float(beta1), float(beta2), float(eps), stream_of(param)), "cn_adamw_step")


def adamw_scalars(segments, beta1: float, beta2: float, out) -> None:
    """The per-segment scalars of adamw_step_dev, folded on the host exactly as cn_adamw_step folds
    them: ``out`` a float32 buffer of 3 * len(segments) (a pinned tensor's numpy view)."""
    lib = _lib_ready()
    k = len(segments)
    assert k >= 1 and out.size >= 3 * k

    def arr(ct, vals):
        return (ct * k)(*vals)
    check(lib.cn_adamw_scalars(k, arr(ctypes.c_double, [float(s[2]) for s in segments]),
                               arr(ctypes.c_double, [float(s[3]) for s in segments]),
                               arr(ctypes.c_int64, [int(s[4]) for s in segments]), float(beta1), float(beta2),
                               ctypes.c_void_p(out.ctypes.data)), "cn_adamw_scalars")


def adamw_step_dev(param: Tensor, grad: Tensor, exp_avg: Tensor, exp_avg_sq: Tensor, segments, scalars: Tensor,
                   beta1: float, beta2: float, eps: float) -> None:
    """adamw_step with the per-segment scalars in device memory (``scalars``: float32, 3 per
    segment): the graph-capturable form (cn_adamw_step_dev)."""
    lib = _lib_ready()
    bufs = [_cuda(t, name) for t, name in ((param, "param"), (grad, "grad"), (exp_avg, "exp_avg"),
                                          (exp_avg_sq, "exp_avg_sq"))]
    n = param.numel()
    assert all(b.data_ptr() == t.data_ptr() and b.numel() == n for b, t in zip(bufs, (param, grad, exp_avg, exp_avg_sq)))
    k = len(segments)
    assert k >= 1 and scalars.numel() >= 3 * k and scalars.dtype == torch.float32 and scalars.is_cuda
    assert all(b % 4 == 0 and e % 4 == 0 and 0 <= b < e <= n for b, e, *_ in segments)

    def arr(ct, vals):
        return (ct * k)(*vals)
    check(lib.cn_adamw_step_dev(ptr(param), ptr(grad), ptr(exp_avg), ptr(exp_avg_sq), k,
                                arr(ctypes.c_int64, [int(s[0]) for s in segments]),
                                arr(ctypes.c_int64, [int(s[1]) for s in segments]), ptr(scalars),
                                float(beta1), float(beta2), float(eps), stream_of(param)), "cn_adamw_step_dev")


# ------------------------------------------------------------------ the step's loss


def render_loss(rgb_coarse: Optional[Tensor], rgb_fine: Optional[Tensor], target: Tensor,
                z_s: Optional[Tensor] = None, z_t: Optional[Tensor] = None, expand: int = 1,
                regularizer_lambda: float = 0.0, psnr: Optional[Tensor] = None) -> Tensor:
    """train.py:103-108 / eval.py:157-163 in one launch -> (6,) [loss_coarse, loss_fine, regulariser,
    total, ||z_s||, ||z_t||]; ``||z||`` over z's elements times ``expand`` (expanded rows).
    ``psnr`` (a float64 device scalar): also mse2psnr of the fine loss, written by the same launch."""
    lib = _lib_ready()
    rc, rf = _opt(rgb_coarse, "rgb_coarse"), _opt(rgb_fine, "rgb_fine")
    target = _cuda(target, "target")
    n = (rc if rc is not None else rf).shape[0]
    assert target.shape[0] == n and target.dim() == 2 and target.shape[1] >= 3, "target must be (R, >=3)"
    zs, zt = _opt(z_s, "z_s"), _opt(z_t, "z_t")
    n_code = 0 if zs is None else zs.numel()
    assert zt is None or zt.numel() == n_code, "z_s and z_t must have the same size"
    out = torch.empty(6, device=target.device, dtype=torch.float32)
    nws = int(lib.cn_render_loss_workspace_doubles(n_code))
    ws = torch.empty(nws, device=target.device, dtype=torch.float64) if nws > 0 else None
    if psnr is not None:
        assert psnr.is_cuda and psnr.dtype == torch.float64 and psnr.numel() == 1, "psnr: a float64 device scalar"
        check(lib.cn_render_loss_psnr(ptr(rc), ptr(rf), ptr(target), target.shape[1], n, ptr(zs), ptr(zt), n_code,
                                      expand, regularizer_lambda, ptr(ws), ptr(out), ptr(psnr), stream_of(out)),
              "cn_render_loss_psnr")
        return out
    check(lib.cn_render_loss(ptr(rc), ptr(rf), ptr(target), target.shape[1], n, ptr(zs), ptr(zt), n_code, expand,
                             regularizer_lambda, ptr(ws), ptr(out), stream_of(out)), "cn_render_loss")
    return out


def render_loss_backward(rgb_coarse, rgb_fine, target, z_s, z_t, expand, regularizer_lambda, stats, grad_total,
                         want=(True, True, True, True), dz_into: Optional[Tuple[Tensor, Tensor]] = None):
    """Backward of render_loss -> (d_rgb_coarse, d_rgb_fine, d_z_s, d_z_t), None where not wanted.
    ``dz_into`` (two contiguous device tensors of z_s's / z_t's size): d z ADDED into them and returned."""
    lib = _lib_ready()
    rc, rf = _opt(rgb_coarse, "rgb_coarse"), _opt(rgb_fine, "rgb_fine")
    target = _cuda(target, "target")
    n = (rc if rc is not None else rf).shape[0]
    zs, zt = _opt(z_s, "z_s"), _opt(z_t, "z_t")
    n_code = 0 if zs is None else zs.numel()
    outs = [torch.empty_like(t) if (w and t is not None) else None for w, t in zip(want, (rc, rf, zs, zt))]
    if dz_into is not None:
        for d in dz_into:
            assert d.is_cuda and d.dtype == torch.float32 and d.is_contiguous() and d.numel() == n_code
        outs[2], outs[3] = dz_into
    check(lib.cn_render_loss_backward(ptr(rc), ptr(rf), ptr(target), target.shape[1], n, ptr(zs), ptr(zt), n_code,
                                      expand, regularizer_lambda, ptr(stats), ptr(_cuda(grad_total, "grad")),
                                      *[ptr(o) for o in outs], int(dz_into is not None), stream_of(target)),
          "cn_render_loss_backward")
    return tuple(outs)


# ------------------------------------------------------------------ SRN data resident in HBM


def srn_unpack(images: Tensor, view_index: Tensor, want_color: bool = True, want_mask: bool = True):
    """dataset.py:77-80 for a batch of resident uint8 views (n, h, w, c) -> color (B, h, w, c) float,
    mask (B, h, w, 1) float (either None when not wanted)."""
    lib = _lib_ready()
    images = _cuda(images, "images", torch.uint8)
    idx = _cuda(view_index, "view_index", torch.int64).reshape(-1)
    n, h, w, c = images.shape
    b = idx.numel()
    color = torch.empty(b, h, w, c, device=images.device, dtype=torch.float32) if want_color else None
    mask = torch.empty(b, h, w, 1, device=images.device, dtype=torch.float32) if want_mask else None
    check(lib.cn_srn_unpack(ptr(images), n, h * w, c, ptr(idx), b, ptr(color), ptr(mask), stream_of(images)),
          "cn_srn_unpack")
    return color, mask
