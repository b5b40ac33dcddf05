"""torch.autograd.Function wrappers of the HIP ops.

Each wrapper runs the HIP forward; when no input requires grad it returns the
plain op result and records nothing.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from . import ops


def _needs_grad(*ts) -> bool:
    return torch.is_grad_enabled() and any(isinstance(t, torch.Tensor) and t.requires_grad for t in ts)


def _no_backward(name):
    raise NotImplementedError(f"backward of {name} on the gfx950 path is not built yet")


def ray_bundle_autograd(dirs, c2w):
    if not _needs_grad(c2w):
        return ops.ray_bundle(dirs, c2w.detach())
    _no_backward("ray_bundle")


def gather_rays_autograd(ro, rd, sel):
    if not _needs_grad(ro, rd):
        return ops.gather_rays(ro.detach(), rd.detach(), sel)
    _no_backward("gather_rays")


def sample_points_autograd(ro, rd, z):
    """pts = ro + rd * z for sorted depths z (detached, point_sampler.py:70,115-118)."""
    if not _needs_grad(ro, rd):
        return ops.ray_points(ro.detach(), rd.detach(), z.detach())
    _no_backward("sample points")


def posenc_autograd(x, freqs: Sequence[float], include_input: bool):
    if not _needs_grad(x):
        return ops.posenc(x.detach(), freqs, include_input)
    _no_backward("posenc")


def volume_render_autograd(raw, z, rd):
    if not _needs_grad(raw, rd):
        return ops.volume_render(raw.detach(), z.detach(), rd.detach())
    _no_backward("volume_render")


def mlp_forward_autograd(model, z_s, z_t, x):
    _no_backward("CodeNeRFModel.forward")


def radiance_field_autograd(model, rd, z_s, z_t, chunk_rows, fx, fd, pts=None, ro=None, z=None):
    _no_backward("forward_pass")
