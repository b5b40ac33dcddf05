"""Tensor-level wrappers of the C ABI: validate, allocate outputs, launch on the current stream.

Every function here is one entry point of include/codenerf.h; the reference
function it replaces is named in its docstring.  Inputs must be CUDA (HIP)
fp32 tensors; shape errors raise AssertionError like the reference's asserts,
and a failed launch raises ``CodeNerfError``.  Nothing here falls back to
PyTorch compute.
"""
from __future__ import annotations

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
    check(lib.cn_sample_pdf(ptr(ro), ptr(rd), ptr(weights), w_stride, ptr(z), n, nc, num_fine, ptr(u), u_stride, ptr(zo),
                            ptr(pts), stream_of(zo)), "cn_sample_pdf")
    return pts, zo


# ------------------------------------------------------------------ encoding


def posenc(x: Tensor, freqs: Sequence[float], include_input: bool) -> Tensor:
    """PositionalEmbedder.embed (position_embed.py:35-53): (M, D) -> (M, D*(inc + 2L))."""
    lib = _lib_ready()
    x = _cuda(x, "tensor")
    assert x.dim() == 2, "tensor must be (N, num_dim)"
    m, d = x.shape
    out = torch.empty(m, d * (int(include_input) + 2 * len(freqs)), device=x.device, dtype=torch.float32)
    check(lib.cn_posenc(ptr(x), m, d, _lib.host_floats(freqs), len(freqs), int(include_input), ptr(out),
                        stream_of(x)), "cn_posenc")
    return out


# ------------------------------------------------------------------ volume integration


def volume_render(raw: Tensor, z: Tensor, rd: Tensor, want_weights: bool = True):
    """volume_render (volumetric_render.py:36-66) -> rgb, disp, acc, weights, depth."""
    lib = _lib_ready()
    raw, z, rd = _cuda(raw, "radiance_field"), _cuda(z, "depth_values"), _cuda(rd, "ray_directions")
    n, s = z.shape
    assert raw.shape == (n, s, 4), "radiance_field must be (num_rays, num_samples, 4)"
    assert rd.shape == (n, 3), "ray_directions must be (num_rays, 3)"
    dev = raw.device
    rgb = torch.empty(n, 3, device=dev, dtype=torch.float32)
    disp = torch.empty(n, device=dev, dtype=torch.float32)
    acc = torch.empty_like(disp)
    depth = torch.empty_like(disp)
    w = torch.empty(n, s, device=dev, dtype=torch.float32) if want_weights else None
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
    fragments for the 3-product split on v_mfma_f32_32x32x16_bf16 (include/codenerf.h).
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
    check(lib.cn_radiance_field(ptr(packed), _fmt(precision), ptr(cb), ptr(code_index), n_codes, ptr(pts), ptr(ro), ptr(rd), ptr(z),
                                n, n_samples, chunk_rows, _lib.host_floats(freqs_xyz), _lib.host_floats(freqs_dir),
                                ptr(raw), stream_of(rd)), "cn_radiance_field")
    return raw
