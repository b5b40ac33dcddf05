"""RaySampler on the gfx950 kernels (view_synthesis/nerf/ray_sampler.py:7-99).

Directions are generated once on the device (cn_ray_directions).  ``sample`` draws the
pixel subset with the host numpy RNG exactly as the reference does (bit-identical
``select_inds`` for the same seed) and then computes ONLY those rays on the device:
one cn_pose_rays launch does get_bundle + the gather (the reference rotates all H*W
directions, then gathers).  ``get_bundle`` still returns the whole (B, H, W, 3) bundle.

``sample_spherical`` is the eval step's pose path fused:
pose_spherical(theta, phi, rho) (eval.py:22-38) -> sample -> the target-pixel gather
(eval.py:147-148) in one launch, with the analytic gradient into theta, phi, rho in one
more.  ``rng="device"`` replaces the host permutation by an on-device Philox draw
(cn_random_select; same distribution, different draws -- throughput mode).
"""
from __future__ import annotations

from typing import Optional, Tuple, Union

import numpy as np
import torch

from .. import ops


class RaySampler(object):

    def __init__(self, height: int, width: int, intrinsics: Union[torch.Tensor, np.ndarray], sample_size: int,
                 device, datatype, rng: str = "numpy", seed: int = 0):
        assert height > 0 and width > 0, "Height and width must be positive integers"
        assert sample_size > 0 and sample_size <= height * width, \
            "Sample size must be a positive number less than height * width"
        assert rng in ("numpy", "device"), "rng must be 'numpy' (the reference's draws) or 'device' (Philox)"
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
        self.rng, self.seed, self._draws = rng, seed, 0

    def select_inds(self, batch: int):
        """ray_sampler.py:41-42: per image np.random.permutation(H*W)[:S] -> (numpy (B,S) | None,
        device int64 (B,S)).  rng="device": Philox on the device (no host copy, numpy None)."""
        n = self.height * self.width
        if self.rng == "device":
            sel = ops.random_select(batch, n, self.sample_size, self.seed, self._draws, self.device)
            self._draws += 1
            return None, sel
        select_inds = self.draw_host(batch)
        sel = torch.from_numpy(select_inds.astype(np.int64))
        if self.device.type == "cuda":  # pinned: the copy is enqueued, not a host-side wait on the stream
            sel = sel.pin_memory()
        sel = sel.to(self.device, non_blocking=True)
        return select_inds, sel

    def draw_host(self, batch: int) -> np.ndarray:
        """ray_sampler.py:41-42's numpy draw alone: per image np.random.permutation(H*W)[:S]."""
        pixel_range = np.arange(0, self.height * self.width)
        return np.asarray([np.random.permutation(pixel_range)[: self.sample_size] for _ in range(batch)])

    def sample(self, tform_cam2world: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor, np.ndarray]:
        """ray_sampler.py:53-82 -> ro, rd (B*S, 3), select_inds (B, S) (numpy; a device tensor with
        rng="device")."""
        from ..autograd import pose_rays_autograd
        batch = tform_cam2world.shape[0]
        select_inds, sel = self.select_inds(batch)
        c2w = tform_cam2world.to(self.device, torch.float32)
        ro, rd, _, _ = pose_rays_autograd(self.directions, c2w=c2w, sel=sel)
        return ro, rd, (sel if select_inds is None else select_inds)

    def sample_pixels(self, tform_cam2world: torch.Tensor, color: torch.Tensor):
        """train.py:76-80 fused: sample(tform_cam2world) and the target pixels
        ``color.flatten(1, 2)[k, select_inds[k], :]`` concatenated over the images, in one launch.
        color: (B, H, W, C) -> ro, rd (B*S, 3), select_inds, target rows (B*S, C)."""
        from ..autograd import pose_rays_autograd
        batch = tform_cam2world.shape[0]
        select_inds, sel = self.select_inds(batch)
        c2w = tform_cam2world.to(self.device, torch.float32)
        target = color.reshape(batch, self.height * self.width, -1)
        ro, rd, _, tgt = pose_rays_autograd(self.directions, c2w=c2w, sel=sel, target=target)
        return ro, rd, (sel if select_inds is None else select_inds), tgt

    def sample_spherical(self, theta: torch.Tensor, phi: torch.Tensor, rho: torch.Tensor,
                         target: Optional[torch.Tensor] = None, sel: Optional[torch.Tensor] = None):
        """eval.py:145-148 fused: cam_pose = pose_spherical(theta, phi, rho); ro, rd, select_inds =
        sample(cam_pose); target_pixels = target[..., select_inds, :].  theta, phi, rho: (B,) each
        (the reference's (1,) leaves); target: (B, H*W, C) or (H*W, C) for B = 1.
        ``sel``: (B, S') device indices drawn by the caller (a captured eval step, whose host draw
        happens outside the graph; S' = sample_size, or a rank's share of them in the ray-sharded
        eval step); else drawn here.
        -> ro, rd (B*S, 3), select_inds, cam_pose (B, 4, 4) (no grad), target rows (B*S, C) | None.
        Inside evaluate.eval_step_loss (autograd.eval_ray_sinks) the rays' consumers add their gradients
        in place and return none for ro / rd; elsewhere the rays' gradients flow through autograd."""
        from ..autograd import pose_rays_autograd
        batch = theta.numel()
        if sel is None:
            select_inds, sel = self.select_inds(batch)
        else:
            assert sel.dim() == 2 and sel.shape[0] == batch and 0 < sel.shape[1] <= self.sample_size, \
                "sel must be (B, S') with S' <= sample_size"
            select_inds = None
        if target is not None:
            target = target.reshape(batch, self.height * self.width, -1)
        ro, rd, cam, tgt = pose_rays_autograd(self.directions, theta, phi, rho, sel=sel, target=target)
        return ro, rd, (sel if select_inds is None else select_inds), cam, tgt

    def get_bundle(self, tform_cam2world: torch.Tensor):
        """ray_sampler.py:84-99 -> ro, rd (B, H, W, 3)."""
        from ..autograd import ray_bundle_autograd
        return ray_bundle_autograd(self.directions, tform_cam2world.to(self.device, torch.float32))
