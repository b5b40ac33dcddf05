"""Test-time optimisation of pose + latent codes and the validation render (eval.py:22-38, :82-205)
on the gfx950 kernels.

The reference's eval loop renders a random ray batch from the current pose estimate, takes
the MSE against the target pixels plus a code regulariser, and steps an optimiser over
(z_s, z_t, theta, phi, rho); after the last iteration it renders the whole view from the
optimised pose with ``parallel_image_render`` and reports its PSNR.  Here one eval
iteration is: the fused pose path (``RaySampler.sample_spherical``: pose_spherical +
sample + target gather, one launch; its backward one more), the hierarchical render and its
backward on the HIP kernels (codenerf.autograd), the fused loss (cn_render_loss, one
launch each way), the pose metric (cn_pose_error) and, for ``val_type: AdamW``, the flat
one-launch AdamW (codenerf.optim).  torch only routes the tensors.
"""
from __future__ import annotations

import warnings
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from . import nerf, ops
from .autograd import backward_from
from .utils import mse2psnr


def pose_spherical(theta: torch.Tensor, phi: torch.Tensor, rho: torch.Tensor) -> torch.Tensor:
    """eval.py:22-38: camera on a sphere of radius rho looking at the origin -> (4, 4) c2w.
    (Host-side helper with the reference's torch ops; the eval step itself builds the pose inside
    cn_pose_rays.)"""
    c2w = torch.eye(n=4, device=theta.device)
    st, ct, sp, cp = torch.sin(theta), torch.cos(theta), torch.sin(phi), torch.cos(phi)
    c2w[0, 0], c2w[1, 0] = -sp, cp
    c2w[0, 1], c2w[1, 1], c2w[2, 1] = -st * cp, -st * sp, ct
    c2w[0, 2], c2w[1, 2], c2w[2, 2] = ct * cp, ct * sp, st
    c2w[0, 3], c2w[1, 3], c2w[2, 3] = rho * ct * cp, rho * ct * sp, rho * st
    return c2w


def eval_step_loss(theta, phi, rho, shape_code, texture_code, target_pixels, samplers, embedders, models,
                   regularizer_lambda: float, gt_pose: Optional[torch.Tensor] = None,
                   t_rand: Optional[torch.Tensor] = None, u: Optional[torch.Tensor] = None,
                   sel: Optional[torch.Tensor] = None,
                   rows_total: Optional[int] = None) -> Tuple[torch.Tensor, Dict[str, object]]:
    """One iteration's forward of eval.py:145-163 -> (loss, logs).

    ``target_pixels``: (H*W, C) image of the object; rays are drawn by the ray sampler's RNG
    (host numpy as the reference, or rng="device").  ``gt_pose`` (4, 4): the view's pose, for
    the logged pose error (eval.py:161-162).  ``t_rand`` / ``u``: injected stratified / fine
    uniforms (parity tests), else drawn on the device.  ``sel``: (1, S) device ray indices drawn
    by the caller (GraphedEvalStep), else the ray sampler draws them.  ``rows_total``: this call renders
    one rank's share of an iteration of ``rows_total`` rays (sharded_eval_step): the regulariser
    expands the codes over all ``rows_total`` rows and the loss is weighted by share / rows_total, so
    the ranks' losses sum to the whole iteration's.  logs: device tensors (read back only when
    logged; the per-share means when sharded); eval.py:159's per-iteration psnr is read back by the
    caller once the backward and the optimiser step are enqueued (``step_psnr``)."""
    from .autograd import eval_ray_sinks
    ray_sampler, point_sampler = samplers
    with eval_ray_sinks():            # the rays' gradients summed in place (autograd.RaySink)
        ro, rd, select_inds, cam_pose, tp = ray_sampler.sample_spherical(theta, phi, rho, target=target_pixels,
                                                                         sel=sel)
    n = ro.shape[0]
    # the code rows, with their gradient summed in place (code_rows_with_sink), expanded over the rays
    from .models.model import CodeRows, code_rows_with_sink
    shape_code, texture_code = code_rows_with_sink(shape_code, texture_code)
    z_s, z_t = shape_code.expand(n, -1), texture_code.expand(n, -1)
    if shape_code.dim() == 2 and shape_code.shape[0] == 1:
        z_s._cn_code_rows = z_t._cn_code_rows = CodeRows(shape_code, texture_code, None)
    # predict_radiance_and_render (nerf/__init__.py:74-91) over the whole ray batch; the two fields' backwards
    # in shared launches (autograd.FieldPair: the loss below reaches both)
    from .autograd import paired_fields
    with paired_fields():
        out = nerf.render_rays(ro, rd, z_s, z_t, point_sampler, embedders, models["nerf_coarse"],
                               models["nerf_fine"], chunk_rows=n, t_rand=t_rand, u=u)
    rgb_c, rgb_f = out["rgb_coarse"], out["rgb_fine"]
    # mse(coarse) + mse(fine) + lambda (||z_s|| + ||z_t||), the codes expanded over the n rays
    psnr = torch.empty((), dtype=torch.float64, device=tp.device)   # eval.py:159's psnr, by the loss launch
    expand = n if rows_total is None else rows_total
    loss, stats = nerf_loss(rgb_c, rgb_f, tp, shape_code, texture_code, expand, regularizer_lambda, psnr=psnr)
    if expand != n:
        loss = loss * (n / expand)
    logs = {"nerf_loss_coarse": stats[0], "nerf_loss_fine": stats[1], "embedding_loss": stats[2], "psnr": psnr}
    if gt_pose is not None:
        logs["pose_error"] = ops.pose_error(gt_pose.reshape(1, 4, 4), cam_pose)[1][0]
    logs["cam_pose"] = cam_pose
    return loss, logs


def step_psnr(logs: Dict[str, object]) -> float:
    """eval.py:159: psnr of the fine MSE (mse2psnr, util.py:216-227); one read-back."""
    return mse2psnr(logs["nerf_loss_fine"].item())


def step_psnr_tensor(logs: Dict[str, object]) -> torch.Tensor:
    """eval.py:159's psnr on the device (no read-back; float() it when logged): the loss launch's own
    (eval_step_loss), else formed from the fine MSE."""
    if "psnr" in logs:
        return logs["psnr"]
    from .train import psnr_tensor
    return psnr_tensor(logs["nerf_loss_fine"])


def sync_shard_state(samplers, src: int = 0, group=None) -> None:
    """Put the ranks of a ray-sharded eval (sharded_eval_step) in step with rank ``src``: its random
    streams -- numpy's global state (the ray draw, ray_sampler.py:41-42), torch's CPU and
    current-device generators (the stratified / fine uniforms), the ray sampler's device-Philox
    counter -- and its ray sampler's camera (focal, principal point: eval.py:66-76 builds each rank's
    samplers from its own first validation batch, while a sharded step renders ONE view, rank
    ``src``'s).  One object broadcast; the other ranks continue with rank ``src``'s streams."""
    import numpy as np
    rs = samplers[0]
    rank = dist.get_rank(group)
    state = [None]
    if rank == src:
        cuda = torch.cuda.get_rng_state() if torch.cuda.is_available() and torch.cuda.is_initialized() else None
        state = [dict(np=np.random.get_state(), cpu=torch.get_rng_state(), cuda=cuda, draws=(rs.seed, rs._draws),
                      camera=(rs.height, rs.width, rs.focal_length, rs.cx, rs.cy), k=rs.intrinsics.cpu())]
    dist.broadcast_object_list(state, src=src, group=group)
    if rank == src:
        return
    st = state[0]
    np.random.set_state(st["np"])
    torch.set_rng_state(st["cpu"])
    if st["cuda"] is not None:
        torch.cuda.set_rng_state(st["cuda"])
    rs.seed, rs._draws = st["draws"]
    h, w, focal, cx, cy = st["camera"]
    assert (h, w) == (rs.height, rs.width), "ray-sharded eval: the ranks' images differ in size"
    if (focal, cx, cy) != (rs.focal_length, rs.cx, rs.cy):
        rs.focal_length, rs.cx, rs.cy = focal, cx, cy
        rs.intrinsics = st["k"].to(rs.device)
        rs.directions = ops.ray_directions(h, w, focal, cx, cy, rs.device)


def shard_draws(samplers, n_rays: int):
    """The random inputs of one ray-sharded eval iteration, drawn in full on every rank in the order
    the unsharded step draws them (eval_step_loss: the ray subset, then render_rays' stratified and
    fine uniforms from torch's device generator) -> (sel (1, n_rays) device int64, t_rand | None,
    u | None).  With the ranks' streams in step (sync_shard_state), every rank holds the same draws."""
    rs, ps = samplers
    assert n_rays == rs.sample_size, "one view's sample_size rays per iteration (eval.py:145)"
    _, sel = rs.select_inds(1)
    t_rand = u = None
    if ps.perturb:
        t_rand = torch.rand(n_rays, ps.num_samples_coarse, dtype=torch.float32, device=sel.device)
        u = torch.rand(n_rays, ps.num_samples_fine, dtype=torch.float32, device=sel.device)
    return sel, t_rand, u


def shard_of(n_rays: int, world: int, rank: int) -> slice:
    """Rank ``rank``'s rows of an ``n_rays`` iteration: parallel_image_render's Q5 split
    (utils.split_sizes: truncating, the last rank takes the remainder)."""
    from .utils import split_sizes
    per, _ = split_sizes(n_rays, world)
    start = sum(per[:rank])
    return slice(start, start + per[rank])


def _allreduce_sum(optimizer, params, group) -> None:
    """Sum the parameters' gradients over the group: the flat AdamW's one all-reduce (no average),
    else one all-reduce of the gradients concatenated."""
    from .optim import AdamW
    if isinstance(optimizer, AdamW):
        optimizer.allreduce_grads(group, average=False)
        return
    for p in params:              # a parameter without a gradient on this rank reduces zeros
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    grads = [p.grad for p in params]
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, group=group)
    torch._foreach_copy_(grads, [f.view_as(g) for f, g in zip(flat.split([g.numel() for g in grads]), grads)])


def sharded_eval_step(theta, phi, rho, shape_code, texture_code, target_pixels, samplers, embedders, models,
                      optimizer, regularizer_lambda: float, gt_pose: Optional[torch.Tensor] = None,
                      group=None) -> Tuple[torch.Tensor, Dict[str, object]]:
    """One test-time-optimisation iteration with its ray batch split over the ranks (SURVEY.md 8(e)'s
    optional sharded C5 mode, a build extension: eval.py runs one independent optimisation per rank,
    Q6, which stays the default).  Every rank draws the iteration's rays and uniforms in full
    (shard_draws; the streams put in step by sync_shard_state), renders its Q5 share of the rays, weights
    its loss by share / rays (eval_step_loss ``rows_total``), runs the backward, and ONE all-reduce
    sums the code / pose gradients (515 floats; a second one the two MSE terms for the logs); the
    optimiser step then runs on identical gradients, so the parameters stay identical on every rank.
    Semantics: the gradient of the whole batch's loss, except that each share is rendered as its own
    chunk, so the Q1 view-direction map (nerf/__init__.py:127-128) pairs samples with rays of the
    share rather than of the whole batch -- the reason this mode is reported beside, not instead of,
    the reference's.  -> (total loss, logs) of the whole iteration; logs as eval_step_loss's."""
    rs, _ = samplers
    n_rays = rs.sample_size
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    sel, t_rand, u = shard_draws(samplers, n_rays)
    sl = shard_of(n_rays, world, rank)
    n = sl.stop - sl.start
    loss, logs = eval_step_loss(theta, phi, rho, shape_code, texture_code, target_pixels, samplers, embedders,
                                models, regularizer_lambda, gt_pose=gt_pose,
                                t_rand=None if t_rand is None else t_rand[sl], u=None if u is None else u[sl],
                                sel=sel[:, sl], rows_total=n_rays)
    optimizer.zero_grad()
    backward_from(loss)
    params = [shape_code, texture_code, theta, phi, rho]
    _allreduce_sum(optimizer, params, group)
    mse = torch.stack([logs["nerf_loss_coarse"], logs["nerf_loss_fine"]]) * (n / n_rays)
    dist.all_reduce(mse, group=group)
    optimizer.step()
    from .train import psnr_tensor
    logs.update(nerf_loss_coarse=mse[0], nerf_loss_fine=mse[1], psnr=psnr_tensor(mse[1]))
    return mse[0] + mse[1] + logs["embedding_loss"], logs


class GraphedEvalStep:
    """One test-time-optimisation iteration's forward and backward (eval.py:145-160) captured ONCE
    as a HIP graph (torch.cuda.CUDAGraph, i.e. hipGraph on ROCm) and replayed every iteration: the
    ~60 launches of the fused pose path, the hierarchical render, the fused loss and their
    backward -- and the Python that issues them -- become one graph launch.

    Per ``step()``: the host draws the ray subset exactly as the reference does
    (np.random.permutation per iteration, ray_sampler.py:41-42) into a pinned buffer and folds
    the AdamW step's bias-corrected scalars (counting the step as ``optimizer.step()`` would) into
    another; both are copied to fixed device buffers on the stream (outside the graph), then one
    replay renders, takes the loss and its gradients into the optimiser's flat gradient buffer
    (zeroed inside the graph, as ``zero_grad`` would) and applies the flat AdamW update
    (cn_adamw_step_dev, scalars read from device memory).  With ``optimizer_in_graph=False`` the
    caller runs ``optimizer.step()`` after the replay instead.
    The pinned buffers alternate between two sets, each reused only once the copy that read it two
    steps earlier has finished: the host never waits for the replay it just launched, so it draws
    and enqueues the next iteration while the GPU runs this one.  (A first form copied from ONE
    pinned set inside the graph and had to wait for each replay to end before refilling it: the
    GPU then idled for the host's wake-up, draw and graph launch every iteration -- slower than
    the eager loop)
    The stratified / fine-sample uniforms come from torch's device generator, whose graph-safe
    state advances per replay; the warm-up iterations' draws are rolled back (the generator state
    is restored before capture), so replay i draws what eager iteration i would.

    Needs the flat codenerf.optim.AdamW over (shape_code, texture_code, theta, phi, rho), frozen
    model weights (the packed weights stay cached across replays) and ``rng="numpy"``.
    ``t_rand`` / ``u``: fixed uniforms (parity tests), captured as static inputs."""

    def __init__(self, theta, phi, rho, shape_code, texture_code, target_pixels, samplers, embedders, models,
                 optimizer, regularizer_lambda: float, gt_pose: Optional[torch.Tensor] = None,
                 t_rand: Optional[torch.Tensor] = None, u: Optional[torch.Tensor] = None, warmup: int = 2,
                 optimizer_in_graph: bool = True):
        from .optim import AdamW
        rs = samplers[0]
        assert rs.rng == "numpy", "GraphedEvalStep draws the rays on the host (rng='numpy')"
        assert isinstance(optimizer, AdamW), "GraphedEvalStep needs codenerf.optim.AdamW (flat gradients)"
        assert theta.numel() == 1, "one view per eval step (eval.py:145)"
        dev = target_pixels.device
        self.rs, self.opt, self._next = rs, optimizer, None
        self.h_sel = [torch.zeros(1, rs.sample_size, dtype=torch.int64).pin_memory() for _ in range(2)]
        self.d_sel = torch.zeros(1, rs.sample_size, dtype=torch.int64, device=dev)
        self.copied = [None, None]             # events: the copies that last read each pinned set
        self.k = 0
        args = (theta, phi, rho, shape_code, texture_code, target_pixels, samplers, embedders, models,
                regularizer_lambda)
        kw = dict(gt_pose=gt_pose, t_rand=t_rand, u=u, sel=self.d_sel)
        grads = self.opt.flat_buffers()["grad"]
        # gradients accumulate into the flat slices (attached, not None) inside the graph
        self.opt.zero_grad(set_to_none=False)
        self.opt_in_graph = optimizer_in_graph
        if optimizer_in_graph:
            n_seg = len(self.opt._plan(advance=False))
            self.h_scal = [torch.zeros(3 * n_seg, dtype=torch.float32).pin_memory() for _ in range(2)]
            self.d_scal = torch.zeros(3 * n_seg, dtype=torch.float32, device=dev)

        def body(with_opt: bool):
            grads.zero_()
            loss, logs = eval_step_loss(*args, **kw)
            backward_from(loss)
            if with_opt:
                self.opt.graph_step(self.d_scal)
            return loss, logs

        rng_state = torch.cuda.get_rng_state(dev)
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):          # warm-up outside the capture (lazy inits, weight packs);
            for _ in range(warmup):            # never the update: it would move the parameters
                body(False)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        torch.cuda.set_rng_state(rng_state, dev)  # the warm-up's t_rand / u draws never happened
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss, self.logs = body(optimizer_in_graph)
        torch.cuda.synchronize(dev)

    def step(self) -> Tuple[torch.Tensor, Dict[str, object]]:
        """This iteration's rays (host numpy, the reference's call; drawn by prefetch() if it ran),
        then the replay.  -> (loss, logs): the graph's static output tensors, valid until the next
        step()."""
        sel = self._next if self._next is not None else self.rs.draw_host(1)
        self._next = None
        k = self.k
        self.k ^= 1
        if self.copied[k] is not None:
            self.copied[k].synchronize()       # the copies of two steps ago have read this set
        self.h_sel[k].numpy()[:] = sel
        self.d_sel.copy_(self.h_sel[k], non_blocking=True)
        if self.opt_in_graph:
            self.opt.graph_scalars(self.h_scal[k].numpy())
            self.d_scal.copy_(self.h_scal[k], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self.copied[k] = ev
        self.graph.replay()
        return self.loss, self.logs

    def prefetch(self) -> None:
        """Draw the NEXT iteration's rays now, while the GPU runs this one (the same numpy calls in
        the same order; call it only when another step() follows)."""
        self._next = self.rs.draw_host(1)


def nerf_loss(rgb_c, rgb_f, target, shape_code, texture_code, expand: int, regularizer_lambda: float, psnr=None):
    """eval.py:157-163 -> (loss, stats (6,)) through cn_render_loss (one launch each way); ``psnr``: the
    fine loss's mse2psnr written by the same launch."""
    from .autograd import render_loss_autograd
    return render_loss_autograd(rgb_c, rgb_f, target, shape_code, texture_code, expand, regularizer_lambda,
                                psnr=psnr)


def _optimizer(kind: str, groups, lr: float):
    if kind == "AdamW":
        from .optim import AdamW
        return AdamW(groups, lr=lr)
    return getattr(torch.optim, kind)(groups, lr=lr)


def test_time_optimize(target_pixels: torch.Tensor, samplers, embedders, models, init_codes,
                       iterations: int, val_lr: float = 1e-2, angle_lr: float = 1e-2, radius_lr: float = 1e-2,
                       regularizer_lambda: float = 1e-5, optimizer: str = "AdamW",
                       init_pose: Tuple[float, float, float] = (1.57, 0.0, 1.30),
                       freeze_models: bool = True, log_every: Optional[int] = None,
                       gt_pose: Optional[torch.Tensor] = None, graph: bool = False, shard_rays: bool = False,
                       group=None):
    """eval.py:121-180: optimise codes + (theta, phi, rho) against one image.

    ``init_codes``: the embedding tables (z_s, z_t); the start point is their mean (eval.py:121-127).
    ``freeze_models``: the reference leaves the MLP weights requiring grad, so its backward also
    forms weight gradients that its optimiser never reads; they do not change the result, and
    freezing skips those GEMMs.
    ``graph``: run the iterations as replays of one captured HIP graph (GraphedEvalStep; needs
    frozen models, val_type AdamW and the numpy ray draw) -- the same arithmetic and draws.  Off by
    default: the eager loop is GPU-bound (C5 3.585 ms eager vs 3.592 ms replayed, DESIGN.md section 8
    item 3); the graph pays only where the host is the bottleneck.
    ``shard_rays`` (with an initialised process group of more than one rank): every iteration's ray
    batch split over the ranks (sharded_eval_step; the caller puts the ranks' random streams in step
    first, sync_shard_state) -- one optimisation shared by all ranks instead of one per rank (Q6).

    Returns (shape_code, texture_code, (theta, phi, rho), history, cam_pose of the last iteration).
    """
    dev = target_pixels.device
    z_s0, z_t0 = init_codes
    shape_code = z_s0.to(dev).mean(dim=0, keepdim=True).clone().detach().requires_grad_(True)
    texture_code = z_t0.to(dev).mean(dim=0, keepdim=True).clone().detach().requires_grad_(True)
    theta = torch.tensor([init_pose[0]], device=dev).requires_grad_(True)
    phi = torch.tensor([init_pose[1]], device=dev).requires_grad_(True)
    rho = torch.tensor([init_pose[2]], device=dev).requires_grad_(True)
    opt = _optimizer(optimizer, [
        {"params": [shape_code, texture_code]},
        {"params": [theta, phi], "lr": angle_lr},
        {"params": [rho], "lr": radius_lr},
    ], val_lr)
    saved = {}
    if freeze_models:
        for k, m in models.items():
            saved[k] = [p.requires_grad for p in m.parameters()]
            m.requires_grad_(False)
    history, cam_pose = [], None
    sharded = bool(shard_rays) and dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1
    assert not (sharded and graph), "graph=True runs one rank's whole batch; shard_rays needs the eager step"
    try:
        graphed = None
        if graph:
            assert freeze_models and optimizer == "AdamW", "graph=True needs frozen models and val_type AdamW"
            for m in models.values():
                m.train()
            graphed = GraphedEvalStep(theta, phi, rho, shape_code, texture_code, target_pixels, samplers,
                                      embedders, models, opt, regularizer_lambda, gt_pose=gt_pose)
        for it in range(iterations):
            if graphed is not None:
                loss, logs = graphed.step()        # forward, backward and the AdamW update
                if it + 1 < iterations:
                    graphed.prefetch()             # host draw overlapping this replay
                # the graph's outputs are overwritten by the next replay
                loss, logs = loss.detach().clone(), {k: v.clone() for k, v in logs.items()}
                cam_pose = logs.pop("cam_pose")
            elif sharded:
                for m in models.values():
                    m.train()
                loss, logs = sharded_eval_step(theta, phi, rho, shape_code, texture_code, target_pixels, samplers,
                                               embedders, models, opt, regularizer_lambda, gt_pose=gt_pose,
                                               group=group)
                cam_pose = logs.pop("cam_pose")
            else:
                for m in models.values():
                    m.train()
                loss, logs = eval_step_loss(theta, phi, rho, shape_code, texture_code, target_pixels, samplers,
                                            embedders, models, regularizer_lambda, gt_pose=gt_pose)
                cam_pose = logs.pop("cam_pose")
                opt.zero_grad()
                backward_from(loss)
                opt.step()
            logs["psnr"] = step_psnr_tensor(logs)       # read back with the history (below) or when logged
            logs["total_loss"] = loss.detach()
            history.append(logs)
            if log_every and ((it != 0 and it % log_every == 0) or it == iterations - 1):
                print(f"[VALOPT] Iter: {it:>8} " + " ".join(f"{k}: {float(v):>4.4f}" for k, v in logs.items()))
    finally:
        for k, flags in saved.items():
            for p, f in zip(models[k].parameters(), flags):
                p.requires_grad_(f)
    history = [{k: float(v) for k, v in h.items()} for h in history]
    return shape_code, texture_code, (theta, phi, rho), history, cam_pose


def _pose_lr(o, key: str) -> float:
    """eval.py:135-136 reads optimizer.angle_lr / radius_lr; srn-cars-code.yml lacks both, so
    the reference raises there.  This build substitutes val_lr -- and says so."""
    if isinstance(o, dict) and key in o:
        return o[key]
    if not isinstance(o, dict) and hasattr(o, key):
        return getattr(o, key)
    warnings.warn(f"optimizer.{key} is not in the config (the reference's eval.py:135-136 raises for it, SURVEY "
                  f"Q8); using optimizer.val_lr = {o.val_lr}", stacklevel=3)
    return o.val_lr


def validation_batch(cfg, dataloader, iteration: int) -> Dict[str, torch.Tensor]:
    """eval.py:103-109: ``set_epoch(iteration)`` when distributed, then the SIXTH batch of a fresh
    iterator over the validation loader (``islice(iter(loader), 5, None)``).  Every rank draws its
    own; ``validate`` then broadcasts rank 0's (eval.py:111-115)."""
    from itertools import islice
    if getattr(cfg, "is_distributed", False):
        dataloader.sampler.set_epoch(iteration)
    return next(islice(iter(dataloader), 5, None))


def eval_loop(rank: int, cfg, device=None, resident: bool = True, verbose: bool = True):
    """eval.py:41-79: seeds ``(rank + 1) + experiment.randomseed``, the val loader and the train split
    (for the code-table size), models / optimiser / checkpoint, the samplers and embedders from the
    first validation batch, then ``experiment.iterations // val_batch_size`` validations -> their
    results (validate's dicts; rank 0 holds loss / psnr / pose_error)."""
    from .checkpoint import load_checkpoint
    from .datasets import prepare_dataloader
    from .train import log_losses, prepare_models, prepare_optimizer, seed_rank
    seed_rank(rank, cfg)
    device = torch.device("cuda", rank) if device is None else torch.device(device)
    torch.cuda.set_device(device)
    dataloader, _ = prepare_dataloader("val", cfg, device if resident else None)
    _, train_dataset = prepare_dataloader("train", cfg, None)
    models = prepare_models(cfg, train_dataset.num_objects, device)
    optimizer, _ = prepare_optimizer(cfg, models)
    load_checkpoint(cfg, models, optimizer)
    first = next(iter(dataloader))
    (height, width), intrinsic = first["color"][0].shape[:2], first["intrinsic"][0]
    samplers = nerf.prepare_samplers(cfg, height, width, intrinsic.cpu(), torch.float32, device)
    embedders = nerf.prepare_embedders(cfg, torch.float32, device)
    results = []
    for iteration in range(int(cfg.experiment.iterations) // int(cfg.dataset.val_batch_size)):
        val_data = validation_batch(cfg, dataloader, iteration)
        res = validate(cfg, val_data, models, samplers, embedders, device,
                       log_every=cfg.experiment.val_print_every if verbose else None)
        if verbose and "psnr" in res:
            print(log_losses("val", iteration, 0.0, {"loss": res["loss"], "psnr": res["psnr"]}))
        results.append(res)
    return results


def validate(cfg, val_data: Dict[str, torch.Tensor], models, samplers, embedders, device,
             log_every: Optional[int] = None, shard_rays: Optional[bool] = None) -> Dict[str, object]:
    """eval.py:82-205 for one loaded validation view (``color`` (1,H,W,C), ``pose`` (1,4,4)):

    1. rank 0's view is broadcast to every rank (eval.py:111-115);
    2. test-time optimisation of the codes (from the mean of the trained tables) and the pose
       (eval.py:121-180);
    3. the whole view rendered from the optimised pose with ``parallel_image_render`` (sharded
       over the ranks, one all-gather) and its MSE / PSNR against the target on rank 0
       (eval.py:182-205).
    ``shard_rays`` (default: the config's ``experiment.val_shard_rays``, else False = the reference's
    Q6): with several ranks, step 2 runs as ONE optimisation with every iteration's rays split over the
    ranks (sharded_eval_step), every rank continuing with rank 0's random streams and camera
    (sync_shard_state).
    Returns {"history", "rgb" (H*W,3) on rank 0, "loss", "psnr", "pose_error", "codes", "pose"}."""
    is_distributed = bool(getattr(cfg, "is_distributed", False))
    if shard_rays is None:
        shard_rays = bool(getattr(cfg.experiment, "val_shard_rays", False))
    shard_rays = shard_rays and is_distributed
    color = val_data["color"].to(device, torch.float32)
    gt_pose = val_data["pose"].to(device, torch.float32)
    if is_distributed:
        color, gt_pose = color.contiguous(), gt_pose.contiguous()
        dist.broadcast(color, 0)
        dist.broadcast(gt_pose, 0)
        if shard_rays:
            sync_shard_state(samplers, 0)
    emb = models["embedding"]
    emb = getattr(emb, "module", emb)
    all_s, all_t = emb.get_all_embeddings(device=device)
    e, o = cfg.experiment, cfg.optimizer
    zs, zt, (th, ph, rh), history, cam_pose = test_time_optimize(
        color.reshape(-1, color.shape[-1]), samplers, embedders, models, (all_s.detach(), all_t.detach()),
        e.val_iterations, val_lr=o.val_lr, angle_lr=_pose_lr(o, "angle_lr"), radius_lr=_pose_lr(o, "radius_lr"),
        regularizer_lambda=e.regularizer_lambda, optimizer=getattr(o, "val_type", "AdamW"), log_every=log_every,
        gt_pose=gt_pose, shard_rays=shard_rays)
    rgb = nerf.parallel_image_render(cfg, cam_pose, [zs.detach(), zt.detach()], models, samplers, embedders,
                                     device)
    out = {"history": history, "rgb": rgb, "codes": (zs.detach(), zt.detach()),
           "pose": (th.detach().item(), ph.detach().item(), rh.detach().item()), "cam_pose": cam_pose}
    rank0 = (not is_distributed) or dist.get_rank() == 0
    if rank0:
        assert rgb is not None, "Main process must contain rgb"
        target = color.reshape(-1, color.shape[-1])
        stats = ops.render_loss(None, rgb, target)
        out["loss"] = float(stats[1])
        out["psnr"] = mse2psnr(out["loss"])
        out["pose_error"] = float(ops.pose_error(gt_pose.reshape(1, 4, 4), cam_pose)[1][0])
    return out


# ---------------------------------------------------------------- process launch (eval.py:208-242)

def _eval_rank(rank: int, cfg) -> None:
    eval_loop(rank, cfg)


def main(cfg, backend: Optional[str] = None, port: int = 29500) -> None:
    """eval.py:222-242: ``eval_loop`` on ``cfg.gpus`` ranks (one spawned process per GPU, RCCL) or on
    one (codenerf.train.launch)."""
    from .train import launch
    launch(_eval_rank, cfg, backend=backend, port=port)


if __name__ == "__main__":
    import argparse
    from .config import load_config
    parser = argparse.ArgumentParser()
    parser.add_argument("-c", "--config", type=str, required=True, help="Path to (.yml) config file.")
    parser.add_argument("--load-checkpoint", type=str, required=True, help="Path to load saved checkpoint from.")
    parser.add_argument("-g", "--gpus", default=1, type=int, help="Number of gpus per node")
    parser.add_argument("--distributed", action="store_true", dest="is_distributed",
                        help="Run the models in DataDistributedParallel")
    a = parser.parse_args()
    main(load_config(a.config, gpus=a.gpus, is_distributed=a.is_distributed, load_checkpoint=a.load_checkpoint))
