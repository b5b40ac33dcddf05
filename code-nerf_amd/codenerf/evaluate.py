"""Test-time optimisation of pose + latent codes (eval.py:22-38, :41-205) on the gfx950 kernels.

The reference's eval loop renders a random ray batch from the current pose
estimate, takes the MSE against the target pixels plus a code regulariser,
and steps an optimiser over (z_s, z_t, theta, phi, rho).  Here every stage of
that step -- ray bundle, gather, sampling, the fused field, compositing and
all of their backwards -- runs on the HIP kernels (codenerf.autograd); torch
supplies the 4x4 pose algebra, the scalar losses and the optimiser.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch

from . import nerf
from .utils import mse2psnr


def pose_spherical(theta: torch.Tensor, phi: torch.Tensor, rho: torch.Tensor) -> torch.Tensor:
    """eval.py:22-38: camera on a sphere of radius rho looking at the origin -> (4, 4) c2w."""
    c2w = torch.eye(n=4, device=theta.device)
    st, ct, sp, cp = torch.sin(theta), torch.cos(theta), torch.sin(phi), torch.cos(phi)
    c2w[0, 0], c2w[1, 0] = -sp, cp
    c2w[0, 1], c2w[1, 1], c2w[2, 1] = -st * cp, -st * sp, ct
    c2w[0, 2], c2w[1, 2], c2w[2, 2] = ct * cp, ct * sp, st
    c2w[0, 3], c2w[1, 3], c2w[2, 3] = rho * ct * cp, rho * ct * sp, rho * st
    return c2w


def eval_step_loss(theta, phi, rho, shape_code, texture_code, target_pixels, samplers, embedders, models,
                   regularizer_lambda: float) -> Tuple[torch.Tensor, Dict[str, float]]:
    """One iteration's forward of eval.py:145-160 -> (loss, logs).

    ``target_pixels``: (H*W, 4) image of the object; rays are drawn by
    ``RaySampler.sample`` (host numpy RNG, as the reference).
    """
    ray_sampler, point_sampler = samplers
    cam_pose = pose_spherical(theta, phi, rho)[None, :]
    ro, rd, select_inds = ray_sampler.sample(tform_cam2world=cam_pose)
    sel = torch.as_tensor(select_inds, device=target_pixels.device)
    tp = target_pixels[None][..., sel, :].squeeze()
    z_s, z_t = shape_code.expand(ro.shape[0], -1), texture_code.expand(ro.shape[0], -1)
    rgb_c, rgb_f = nerf.predict_radiance_and_render((ro, rd), point_sampler, embedders, models["nerf_coarse"],
                                                    models["nerf_fine"], (z_s, z_t))
    lc = torch.nn.functional.mse_loss(rgb_c[..., :3], tp[..., :3])
    lf = torch.nn.functional.mse_loss(rgb_f[..., :3], tp[..., :3])
    reg = regularizer_lambda * (torch.norm(z_s, p=2) + torch.norm(z_t, p=2))
    loss = lc + lf + reg
    # eval.py:159 reads the fine loss back every iteration (psnr); the other terms are read only when logged
    return loss, {"nerf_loss_coarse": lc.detach(), "nerf_loss_fine": lf.detach(), "embedding_loss": reg.detach(),
                  "psnr": mse2psnr(lf.item())}


def test_time_optimize(target_pixels: torch.Tensor, samplers, embedders, models, init_codes,
                       iterations: int, val_lr: float = 1e-2, angle_lr: float = 1e-2, radius_lr: float = 1e-2,
                       regularizer_lambda: float = 1e-5, optimizer: str = "AdamW",
                       init_pose: Tuple[float, float, float] = (1.57, 0.0, 1.30),
                       freeze_models: bool = True, log_every: Optional[int] = None):
    """eval.py:121-171: optimise codes + (theta, phi, rho) against one image.

    ``freeze_models``: the reference leaves the MLP weights requiring grad, so its
    backward also forms weight gradients that its optimiser never reads; they
    do not change the result, and freezing skips those GEMMs.
    Returns (shape_code, texture_code, (theta, phi, rho), history).
    """
    dev = target_pixels.device
    z_s0, z_t0 = init_codes
    shape_code = z_s0.to(dev).mean(dim=0, keepdim=True).clone().detach().requires_grad_(True)
    texture_code = z_t0.to(dev).mean(dim=0, keepdim=True).clone().detach().requires_grad_(True)
    theta = torch.tensor([init_pose[0]], device=dev).requires_grad_(True)
    phi = torch.tensor([init_pose[1]], device=dev).requires_grad_(True)
    rho = torch.tensor([init_pose[2]], device=dev).requires_grad_(True)
    opt = getattr(torch.optim, optimizer)([
        {"params": [shape_code, texture_code]},
        {"params": [theta, phi], "lr": angle_lr},
        {"params": [rho], "lr": radius_lr},
    ], lr=val_lr)
    saved = {}
    if freeze_models:
        for k, m in models.items():
            saved[k] = [p.requires_grad for p in m.parameters()]
            m.requires_grad_(False)
    history = []
    try:
        for it in range(iterations):
            for m in models.values():
                m.train()
            loss, logs = eval_step_loss(theta, phi, rho, shape_code, texture_code, target_pixels, samplers,
                                        embedders, models, regularizer_lambda)
            opt.zero_grad()
            loss.backward()
            opt.step()
            logs["total_loss"] = loss.detach()
            history.append(logs)
            if log_every and (it % log_every == 0 or it == iterations - 1):
                print(f"[val-optim {it}] " + " ".join(f"{k}={float(v):.5f}" for k, v in logs.items()))
    finally:
        for k, flags in saved.items():
            for p, f in zip(models[k].parameters(), flags):
                p.requires_grad_(f)
    history = [{k: float(v) for k, v in h.items()} for h in history]
    return shape_code, texture_code, (theta, phi, rho), history
