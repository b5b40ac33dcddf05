"""volume_render on the gfx950 kernel (view_synthesis/nerf/volumetric_render.py:36-66)."""
from __future__ import annotations

import torch


def volume_render(radiance_field: torch.Tensor, depth_values: torch.Tensor, ray_directions: torch.Tensor):
    """-> rgb_map (R,3), disp_map (R), acc_map (R), weights (R,S), depth_map (R)."""
    from ..autograd import volume_render_autograd
    return volume_render_autograd(radiance_field, depth_values, ray_directions)
