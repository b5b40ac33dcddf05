"""``torch.library`` operators in namespace ``codenerf``.

Each operator is one entry point of libcodenerf_hip.so (through codenerf.ops);
the differentiable ones register their backward kernels with
``register_autograd``, so ``torch.ops.codenerf.*`` composes with autograd and
with torch.compile's fake-tensor tracing like any aten op.

    import codenerf.torch_ops  # registers the ops
    rgb, disp, acc, w, depth = torch.ops.codenerf.volume_render(raw, z, rd)

Ops: ray_bundle, sample_uniform, sample_pdf, posenc, codenerf_mlp (inference,
either precision), codenerf_mlp_train (fp32 + saved activations,
differentiable), volume_render, render_rays (the fused coarse -> resample ->
fine pipeline of predict_radiance_and_render), and the *_backward ops.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import _lib, ops

_NS = "codenerf"


def _op(name, **kw):
    return torch.library.custom_op(f"{_NS}::{name}", mutates_args=(), device_types="cuda", **kw)


# ------------------------------------------------------------------ rays / points / encoding


@_op("ray_bundle")
def ray_bundle(directions: Tensor, c2w: Tensor) -> Tuple[Tensor, Tensor]:
    """RaySampler.get_bundle (ray_sampler.py:84-99): (H,W,3), (B,4,4) -> ro, rd (B,H,W,3)."""
    return ops.ray_bundle(directions, c2w)


@ray_bundle.register_fake
def _(directions, c2w):
    shape = (c2w.shape[0],) + tuple(directions.shape)
    return directions.new_empty(shape), directions.new_empty(shape)


@_op("ray_bundle_backward")
def ray_bundle_backward(directions: Tensor, batch: int, g_ro: Optional[Tensor], g_rd: Optional[Tensor]) -> Tensor:
    return ops.ray_bundle_backward(directions, batch, g_ro, g_rd)


@ray_bundle_backward.register_fake
def _(directions, batch, g_ro, g_rd):
    return directions.new_empty(batch, 4, 4)


def _rb_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0])
    ctx.batch = inputs[1].shape[0]


def _rb_backward(ctx, g_ro, g_rd):
    (dirs,) = ctx.saved_tensors
    return None, ray_bundle_backward(dirs, ctx.batch, _c(g_ro), _c(g_rd))


ray_bundle.register_autograd(_rb_backward, setup_context=_rb_setup)


@_op("sample_uniform")
def sample_uniform(ro: Tensor, rd: Tensor, z_bins: Tensor, lower: Tensor, upper: Tensor,
                   t_rand: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """PointSampler.sample_uniform (point_sampler.py:49-71) -> pts (R,Nc,3), z (R,Nc)."""
    return ops.sample_uniform(ro, rd, z_bins, lower, upper, t_rand)


@sample_uniform.register_fake
def _(ro, rd, z_bins, lower, upper, t_rand=None):
    n, nc = ro.shape[0], z_bins.shape[-1]
    return ro.new_empty(n, nc, 3), ro.new_empty(n, nc)


@_op("sample_pdf")
def sample_pdf(ro: Tensor, rd: Tensor, weights: Tensor, z: Tensor, num_fine: int,
               u: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """PointSampler.sample_pdf (point_sampler.py:73-120) -> pts (R,Nc+Nf,3), z (R,Nc+Nf) (detached)."""
    return ops.sample_pdf(ro, rd, weights, z, num_fine, u)


@sample_pdf.register_fake
def _(ro, rd, weights, z, num_fine, u=None):
    n, s = z.shape[0], z.shape[1] + num_fine
    return ro.new_empty(n, s, 3), ro.new_empty(n, s)


@_op("posenc")
def posenc(x: Tensor, freqs: List[float], include_input: bool) -> Tensor:
    """PositionalEmbedder.embed (position_embed.py:35-53)."""
    return ops.posenc(x, freqs, include_input)


@posenc.register_fake
def _(x, freqs, include_input):
    return x.new_empty(x.shape[0], x.shape[1] * (int(include_input) + 2 * len(freqs)))


@_op("posenc_backward")
def posenc_backward(x: Tensor, freqs: List[float], include_input: bool, g_enc: Tensor) -> Tensor:
    return ops.posenc_backward(x, freqs, include_input, g_enc)


@posenc_backward.register_fake
def _(x, freqs, include_input, g_enc):
    return torch.empty_like(x)


def _pe_setup(ctx, inputs, output):
    ctx.save_for_backward(inputs[0])
    ctx.freqs, ctx.inc = inputs[1], inputs[2]


def _pe_backward(ctx, g):
    (x,) = ctx.saved_tensors
    return posenc_backward(x, ctx.freqs, ctx.inc, g.contiguous()), None, None


posenc.register_autograd(_pe_backward, setup_context=_pe_setup)


# ------------------------------------------------------------------ volume integration


@_op("volume_render")
def volume_render(raw: Tensor, z: Tensor, rd: Tensor) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """volume_render (volumetric_render.py:36-66) -> rgb, disp, acc, weights, depth."""
    rgb, disp, acc, w, depth = ops.volume_render(raw, z, rd)
    return rgb, disp, acc, w.clone() if w.shape[-1] != z.shape[-1] else w, depth


@volume_render.register_fake
def _(raw, z, rd):
    n, s = z.shape
    return (raw.new_empty(n, 3), raw.new_empty(n), raw.new_empty(n), raw.new_empty(n, 0 if s == 1 else s),
            raw.new_empty(n))


@_op("volume_render_backward")
def volume_render_backward(raw: Tensor, z: Tensor, rd: Tensor, g_rgb: Optional[Tensor], g_disp: Optional[Tensor],
                           g_acc: Optional[Tensor], g_weights: Optional[Tensor],
                           g_depth: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
    return ops.volume_render_backward(raw, z, rd, g_rgb, g_disp, g_acc, g_weights, g_depth, want_rd=True)


@volume_render_backward.register_fake
def _(raw, z, rd, *grads):
    return torch.empty_like(raw), torch.empty_like(rd)


def _vr_setup(ctx, inputs, output):
    ctx.save_for_backward(*inputs)


def _vr_backward(ctx, g_rgb, g_disp, g_acc, g_w, g_depth):
    raw, z, rd = ctx.saved_tensors
    d_raw, d_rd = volume_render_backward(raw, z, rd, _c(g_rgb), _c(g_disp), _c(g_acc), _c(g_w), _c(g_depth))
    return d_raw, None, d_rd


volume_render.register_autograd(_vr_backward, setup_context=_vr_setup)


# ------------------------------------------------------------------ code-conditioned MLP


def _code_rows(z_s, z_t):
    if z_s.dim() == 2 and z_s.stride(0) == 0 and z_t.stride(0) == 0:
        return z_s[:1], z_t[:1]
    return z_s, z_t


@_op("codenerf_mlp")
def codenerf_mlp(z_s: Tensor, z_t: Tensor, x: Tensor, params: List[Tensor], precision: str = "f32") -> Tensor:
    """CodeNeRFModel.forward (model.py:160-194) on encoded rows; params in state_dict order."""
    cs, ct = _code_rows(z_s, z_t)
    fmt = _lib.kernel_format(precision)
    return ops.mlp_forward(ops.mlp_pack(params, fmt), ops.code_bias(params, cs, ct), x, precision=fmt)


@codenerf_mlp.register_fake
def _(z_s, z_t, x, params, precision="f32"):
    return x.new_empty(x.shape[0], 4)


@_op("codenerf_mlp_train")
def codenerf_mlp_train(z_s: Tensor, z_t: Tensor, x: Tensor, params: List[Tensor]) -> Tuple[Tensor, Tensor]:
    """fp32 CodeNeRFModel.forward that also returns the (5, M, 256) activations its backward reads."""
    return ops.mlp_forward_train(ops.mlp_pack(params, "f32"), ops.code_bias(params, z_s, z_t), x)


@codenerf_mlp_train.register_fake
def _(z_s, z_t, x, params):
    return x.new_empty(x.shape[0], 4), x.new_empty(5, x.shape[0], 256)


@_op("codenerf_mlp_backward")
def codenerf_mlp_backward(z_s: Tensor, z_t: Tensor, x: Tensor, params: List[Tensor], saved: Tensor,
                          g_raw: Tensor) -> Tuple[Tensor, Tensor, Tensor, List[Tensor]]:
    """-> d x, d z_s, d z_t, d params (state_dict order)."""
    m = x.shape[0]
    pg = [torch.zeros_like(p) for p in params]
    r = ops.field_backward(params, saved, x, g_raw.contiguous(), m, 1, m, z_s.shape[0], param_grads=pg,
                           want_code=True, want_x=True)
    dz_s, dz_t = ops.code_bias_backward(params, z_s, z_t, r["g_code"], pg)
    return r["d_x"].clone(), dz_s, dz_t, pg


@codenerf_mlp_backward.register_fake
def _(z_s, z_t, x, params, saved, g_raw):
    return torch.empty_like(x), torch.empty_like(z_s), torch.empty_like(z_t), [torch.empty_like(p) for p in params]


def _mlp_setup(ctx, inputs, output):
    z_s, z_t, x, params = inputs
    ctx.n_params = len(params)
    ctx.save_for_backward(z_s, z_t, x, output[1], *params)


def _mlp_backward(ctx, g_raw, _g_saved):
    z_s, z_t, x, saved, *params = ctx.saved_tensors
    dx, dzs, dzt, pg = codenerf_mlp_backward(z_s, z_t, x, params, saved, g_raw)
    return dzs, dzt, dx, pg


codenerf_mlp_train.register_autograd(_mlp_backward, setup_context=_mlp_setup)


# ------------------------------------------------------------------ fused render


class _ParamModel:
    """The model interface codenerf.nerf's field dispatch needs, over a bare parameter list."""

    def __init__(self, params, precision):
        self._params, self.precision = list(params), precision

    def param_list(self):
        return self._params

    def kernel_format(self):
        return _lib.kernel_format(self.precision)

    def packed(self):
        return ops.mlp_pack(self._params, self.kernel_format())

    def code_bias(self, z_s, z_t):
        return ops.code_bias(self._params, z_s, z_t)


_SAMPLERS = {}


def _samplers(nc, nf, near, far, spacing, perturb, l_xyz, l_dir, include_input, log_sampling, device):
    from .nerf import PointSampler, PositionalEmbedder
    key = (nc, nf, near, far, spacing, perturb, l_xyz, l_dir, include_input, log_sampling, str(device))
    if key not in _SAMPLERS:
        ps = PointSampler(nc, max(nf, 1), near, far, spacing_mode=spacing, perturb=perturb, dtype=torch.float32,
                          device=device)
        emb = (PositionalEmbedder(l_xyz, log_sampling, include_input, torch.float32, device),
               PositionalEmbedder(l_dir, log_sampling, include_input, torch.float32, device))
        _SAMPLERS[key] = (ps, emb)
    return _SAMPLERS[key]


@_op("render_rays")
def render_rays(ro: Tensor, rd: Tensor, z_s: Tensor, z_t: Tensor, coarse_params: List[Tensor],
                fine_params: List[Tensor], near: float, far: float, num_coarse: int, num_fine: int,
                spacing_mode: str, perturb: bool, num_encoding_fn_xyz: int, num_encoding_fn_dir: int,
                include_input: bool, log_sampling: bool, chunk_rows: int, t_rand: Optional[Tensor] = None,
                u_fine: Optional[Tensor] = None, precision: str = "f32"
                ) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """predict_radiance_and_render (nerf/__init__.py:74-91) over a whole ray list, Q1 chunking by chunk_rows.

    -> rgb_coarse (R,3), rgb_fine (R,3), depth_fine (R), acc_fine (R), weights_coarse (R,Nc),
    z_fine (R,Nc+Nf).  num_fine == 0 renders coarse only (fine outputs are empty).
    """
    from . import nerf
    ps, emb = _samplers(num_coarse, num_fine, near, far, spacing_mode, perturb, num_encoding_fn_xyz,
                        num_encoding_fn_dir, include_input, log_sampling, ro.device)
    coarse_only = num_fine == 0
    out = nerf.render_rays(ro, rd, z_s, z_t, ps, emb, _ParamModel(coarse_params, precision),
                           None if coarse_only else _ParamModel(fine_params, precision), chunk_rows,
                           t_rand=t_rand, u=u_fine, coarse_only=coarse_only)
    n = ro.shape[0]
    if coarse_only:
        return (out["rgb_coarse"], ro.new_empty(0, 3), ro.new_empty(0), ro.new_empty(0), out["weights_coarse"],
                ro.new_empty(0, num_coarse))
    return (out["rgb_coarse"], out["rgb_fine"], out["depth_fine"], out["acc_fine"], out["weights_coarse"],
            out["z_fine"].view(n, num_coarse + num_fine))


@render_rays.register_fake
def _(ro, rd, z_s, z_t, coarse_params, fine_params, near, far, num_coarse, num_fine, *rest, **kw):
    n = ro.shape[0]
    if num_fine == 0:
        return (ro.new_empty(n, 3), ro.new_empty(0, 3), ro.new_empty(0), ro.new_empty(0), ro.new_empty(n, num_coarse),
                ro.new_empty(0, num_coarse))
    return (ro.new_empty(n, 3), ro.new_empty(n, 3), ro.new_empty(n), ro.new_empty(n), ro.new_empty(n, num_coarse),
            ro.new_empty(n, num_coarse + num_fine))


def _c(t):
    return None if t is None else t.contiguous()
