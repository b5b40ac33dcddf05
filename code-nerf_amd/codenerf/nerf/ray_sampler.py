"""RaySampler on the gfx950 kernels (view_synthesis/nerf/ray_sampler.py:7-99).

Directions are generated once on the device (cn_ray_directions); get_bundle
rotates them by the c2w poses (cn_ray_bundle); sample draws the pixel subset
with the host numpy RNG exactly as the reference does (bit-identical
``select_inds`` for the same seed) and gathers on the device (cn_gather_rays).
"""
from __future__ import annotations

from typing import Tuple, Union

import numpy as np
import torch

from .. import ops


class RaySampler(object):

    def __init__(self, height: int, width: int, intrinsics: Union[torch.Tensor, np.ndarray], sample_size: int,
                 device, datatype):
        assert height > 0 and width > 0, "Height and width must be positive integers"
        assert sample_size > 0 and sample_size <= height * width, \
            "Sample size must be a positive number less than height * width"
        self.height, self.width, self.sample_size = height, width, sample_size
        self.device = torch.device(device)
        if isinstance(intrinsics, np.ndarray):
            intrinsics = torch.from_numpy(intrinsics).to(datatype)
        assert intrinsics.shape == torch.Size([4, 4]), "Incorrect intrinsics shape"
        k = intrinsics.detach().to("cpu", torch.float32)
        self.intrinsics = intrinsics.to(self.device)
        self.focal_length = float(k[0, 0])
        self.cx = float(k[0, 2])
        self.cy = float(k[1, 2])
        self.directions = ops.ray_directions(height, width, self.focal_length, self.cx, self.cy, self.device)

    def sample(self, tform_cam2world: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, np.ndarray]:
        """ray_sampler.py:53-82 -> ro, rd (B*S, 3), select_inds (B, S) numpy."""
        batch = tform_cam2world.shape[0]
        n = self.height * self.width
        pixel_range = np.arange(0, n)
        select_inds = np.asarray([np.random.permutation(pixel_range)[: self.sample_size] for _ in range(batch)])
        ro, rd = self.get_bundle(tform_cam2world)
        sel = torch.from_numpy(select_inds.astype(np.int64)).to(self.device, non_blocking=True)
        from ..autograd import gather_rays_autograd
        o, d = gather_rays_autograd(ro, rd, sel)
        return o, d, select_inds

    def get_bundle(self, tform_cam2world: torch.Tensor):
        """ray_sampler.py:84-99 -> ro, rd (B, H, W, 3)."""
        from ..autograd import ray_bundle_autograd
        return ray_bundle_autograd(self.directions, tform_cam2world.to(self.device, torch.float32))
