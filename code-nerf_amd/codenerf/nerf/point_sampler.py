"""PointSampler on the gfx950 kernels (view_synthesis/nerf/point_sampler.py:7-120).

The per-config depth bins (Nc floats) are set up once on the host with the
reference's formulas (quirk Q2 spacing names kept), then copied to the device.
Uniform draws come from torch's device RNG unless injected (``t_rand`` /
``u``), which is how the parity tests replay the reference's draws.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from .. import ops


class PointSampler(object):

    def __init__(self, num_samples_coarse, num_samples_fine, near: float, far: float, spacing_mode: str,
                 perturb: bool, dtype, device):
        assert near >= 0 and far > near, "Near and far ranges should be positive values, and far > near"
        assert num_samples_coarse > 0 and num_samples_fine > 0, "Number of samples must be greater than 0"
        self.num_samples_coarse = num_samples_coarse
        self.num_samples_fine = num_samples_fine
        self.near, self.far = near, far
        self.spacing_mode = spacing_mode
        self.perturb = perturb
        self.dtype = torch.float32
        self.device = torch.device(device)
        t = torch.linspace(0.0, 1.0, num_samples_coarse, dtype=torch.float32)
        if spacing_mode == "lindisp":                      # Q2: linear in depth
            z = near * (1.0 - t) + far * t
        else:                                              # "lindepth": linear in disparity
            z = 1.0 / (1.0 / near * (1.0 - t) + 1.0 / far * t)
        mids = 0.5 * (z[1:] + z[:-1])
        self.t_vals = t.to(self.device)
        self.z_vals = z.to(self.device)
        self.mids = mids.to(self.device)
        self.upper = torch.cat((mids, z[-1:])).to(self.device)
        self.lower = torch.cat((z[:1], mids)).to(self.device)
        # u of the unperturbed inverse-CDF pass (point_sampler.py:95), built by torch
        # on the host once: the same bits as the reference's linspace
        self.u_lin = torch.linspace(0.0, 1.0, steps=num_samples_fine, dtype=torch.float32).to(self.device)

    def sample_uniform(self, ro: torch.Tensor, rd: torch.Tensor, t_rand: Optional[torch.Tensor] = None,
                       want_pts: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
        """point_sampler.py:49-71 -> pts (R, Nc, 3), z_vals (R, Nc)."""
        if self.perturb and t_rand is None:
            t_rand = torch.rand(ro.shape[-2], self.num_samples_coarse, dtype=torch.float32, device=ro.device)
        from ..autograd import sample_points_autograd
        pts, z = ops.sample_uniform(ro.detach(), rd.detach(), self.z_vals, self.lower, self.upper,
                                    t_rand if self.perturb else None, want_pts=False)
        return (sample_points_autograd(ro, rd, z) if want_pts else None), z

    def sample_pdf(self, ro: torch.Tensor, rd: torch.Tensor, weights: torch.Tensor, z_vals: torch.Tensor,
                   u: Optional[torch.Tensor] = None, want_pts: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
        """point_sampler.py:73-120 -> pts (R, Nc+Nf, 3), z_vals (R, Nc+Nf) sorted (samples detached, :115)."""
        assert self.num_samples_coarse - 2 == weights.shape[-1], \
            f"Weights size {weights.shape} should match {self.num_samples_coarse - 1}"
        if self.perturb and u is None:
            u = torch.rand(weights.shape[0], self.num_samples_fine, dtype=torch.float32, device=weights.device)
        _, z = ops.sample_pdf(ro.detach(), rd.detach(), weights.detach(), z_vals.detach(), self.num_samples_fine,
                              u if self.perturb else self.u_lin, want_pts=False)
        from ..autograd import sample_points_autograd
        return (sample_points_autograd(ro, rd, z) if want_pts else None), z
