"""Benchmark: rendered rays/s on SRN-cars 128x128 at 64 samples/ray (BASELINE.json metric, config C2).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--hierarchical]

One step renders N full 128x128 images (16384 rays each, 64 coarse samples per
ray, srn-cars-code near 0.8 / far 1.8, lindepth, 4096-ray chunks) through the
gfx950 path: ray bundle -> per-object code terms -> depths -> fused
encode+MLP field kernel -> compositing.  The field kernel runs the
3xbf16 split (Wh.Xh + Wh.Xl + Wl.Xh on bf16 MFMA, fp32 accumulation; fp32-level
accuracy, parity-tested at the same 1e-4 as the fp32 kernel) by default;
``--precision f32`` selects the exact-product fp32 MFMA kernel, which is also
timed beside it and reported under ``f32_kernel``.  With N ranks every image
is split over the ranks exactly like the reference's parallel_image_render
(nerf/__init__.py:179-218) and the rendered pixels are all-gathered to rank 0
over RCCL; per-rank work is fixed (16384 rays), so scaling is weak.

Inputs are synthetic (no dataset/checkpoint offline): hash-initialised
CodeNeRFModel weights of the reference architecture, one latent code pair,
spherical poses.  Everything is resident in HBM before timing.

JSON line fields beyond the driver contract: ``roofline`` (the field kernel,
timed by HIP events on its stream inside the timed steps), ``cpu_baseline``
(the CPU oracle -- the reference's op sequence in torch fp32 -- on this host,
rank 0, one full image), ``psnr_vs_ref`` (our image vs that CPU render).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "code-nerf_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

H = W = 128
FOCAL = 131.25
NC, NF = 64, 64
NEAR, FAR = 0.8, 1.8
CHUNK = 4096
FLOP_PER_SAMPLE = 572_416          # hoisted CodeNeRF MLP per sample-evaluation
PEAK_FP32_MFMA_TFLOPS = 157.3      # MI355X dense fp32 matrix peak (MI355X_MICROARCH.md)
PEAK_BF16_MFMA_TFLOPS = 2516.6     # MI355X dense bf16 matrix peak (guide: ~2.5 PF dense)
KERNELS = {"f32": ("field_kernel<kFromRayZ> (fused posenc + CodeNeRF MLP, fp32 MFMA)", 1, PEAK_FP32_MFMA_TFLOPS),
           "bf16x3": ("field_x3_kernel<kFromRayZ> (fused posenc + CodeNeRF MLP, 3xbf16 MFMA)", 3,
                      PEAK_BF16_MFMA_TFLOPS)}


def pose(theta, phi, rho):
    """eval.py:22-38 pose_spherical (host, float32)."""
    import math
    st, ct, sp, cp = math.sin(theta), math.cos(theta), math.sin(phi), math.cos(phi)
    m = torch.eye(4)
    m[0, 0], m[1, 0] = -sp, cp
    m[0, 1], m[1, 1], m[2, 1] = -st * cp, -st * sp, ct
    m[0, 2], m[1, 2], m[2, 2] = ct * cp, ct * sp, st
    m[0, 3], m[1, 3], m[2, 3] = rho * ct * cp, rho * ct * sp, rho * st
    return m


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--hierarchical", action="store_true", help="also time the 64+64 (C3) render")
    ap.add_argument("--precision", default="bf16x3", choices=sorted(KERNELS))
    ap.add_argument("--no-f32-compare", action="store_true", help="skip the fp32-kernel side measurement")
    ap.add_argument("--eval-iters", type=int, default=10,
                    help="C5: time this many test-time-optimisation iterations (0 = skip)")
    ap.add_argument("--train-iters", type=int, default=3,
                    help="C3 training: time this many train.py iterations (4 x 4096 rays each; 0 = skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = max(world, 1)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)

    import codenerf
    from codenerf import synthetic
    from codenerf.models import CodeNeRFModel
    from codenerf.nerf import PointSampler, PositionalEmbedder, RaySampler, gather_rows, render_rays
    from codenerf.utils import split_sizes
    codenerf.load_library()

    k = synthetic.srn_intrinsics(H, FOCAL)
    rs = RaySampler(H, W, k, sample_size=4096, device=dev, datatype=torch.float32)
    ps = PointSampler(NC, NF, NEAR, FAR, "lindepth", False, torch.float32, dev)
    emb = (PositionalEmbedder(10, True, True, torch.float32, dev), PositionalEmbedder(4, True, True, torch.float32, dev))
    models = []
    for seed in (0, 1):
        m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
        m.load_state_dict(synthetic.codenerf_params(seed))
        m.precision = args.precision
        models.append(m.to(dev).eval())
    zs = synthetic.latent_codes(5, 1).to(dev)
    zt = synthetic.latent_codes(6, 1).to(dev)
    poses = torch.stack([pose(0.5 + 0.3 * i, 0.3, 1.3) for i in range(n)]).to(dev)
    n_img_rays = H * W
    per, _ = split_sizes(n_img_rays, n)
    start = sum(per[:rank])
    chunk = min(CHUNK, per[rank])
    rays_per_rank = per[rank] * n
    for mm in models:
        mm.packed()                              # weights packed once (frozen, as in eval)

    timing = {"field_ms": 0.0, "field_launches": 0}

    def step(record: bool, coarse_only: bool = True):
        with torch.no_grad():
            ro, rd = rs.get_bundle(poses)                    # (n, H, W, 3)
            ro = ro.reshape(n, -1, 3)[:, start:start + per[rank]].reshape(-1, 3)
            rd = rd.reshape(n, -1, 3)[:, start:start + per[rank]].reshape(-1, 3)
            r = ro.shape[0]
            hook = {} if record else None
            out = render_rays(ro, rd, zs.expand(r, -1), zt.expand(r, -1), ps, emb, models[0], models[1],
                              chunk_rows=chunk, coarse_only=coarse_only, events=hook)
            rgb = out["rgb_coarse" if coarse_only else "rgb_fine"]
            if world > 1:
                rgb = gather_rows(rgb, [per[rank] * n] * n, rank)
                if rgb is not None and len(set(per)) == 1:        # (rank, image, row) -> (image, rank, row)
                    rgb = rgb.view(n, n, per[0], 3).transpose(0, 1).reshape(n * n_img_rays, 3)
            if record:
                timing["pending"] = timing.get("pending", []) + hook["field"]
            return rgb

    def timed(k_steps, w_steps, coarse_only=True):
        for _ in range(w_steps):
            step(False, coarse_only)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        timing["pending"] = []
        t0 = time.perf_counter()
        for _ in range(k_steps):
            img = step(True, coarse_only)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([dt], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        ms = [a.elapsed_time(b) for a, b in timing["pending"]]
        return dt, ms, img

    dt, field_ms, img = timed(args.steps, args.warmup, coarse_only=True)
    total_rays = n_img_rays * n * args.steps
    value = total_rays / dt
    field_avg_ms = sum(field_ms) / max(1, len(field_ms))
    samples_per_launch = rays_per_rank * NC
    flop_per_launch = samples_per_launch * FLOP_PER_SAMPLE
    algo_tf = flop_per_launch / (field_avg_ms * 1e-3) / 1e12       # fp32-equivalent algorithmic rate
    kname, passes, peak = KERNELS[args.precision]
    achieved_tf = passes * algo_tf                                  # MFMA flops the hardware executes

    extra = {}
    if args.precision != "f32" and not args.no_f32_compare:
        for mm in models:
            mm.precision = "f32"
            mm.packed()
        dtf, fms, _ = timed(max(1, args.steps // 2), 1, coarse_only=True)
        f_ms = sum(fms) / max(1, len(fms))
        extra["f32_kernel"] = {"value": n_img_rays * n * max(1, args.steps // 2) / dtf, "unit": "rays/s",
                               "field_avg_ms": f_ms,
                               "achieved_tflops": flop_per_launch / (f_ms * 1e-3) / 1e12,
                               "peak": PEAK_FP32_MFMA_TFLOPS}
        for mm in models:
            mm.precision = args.precision
    if args.hierarchical:
        dth, _, _ = timed(max(1, args.steps // 2), 1, coarse_only=False)
        extra["hierarchical_64_64_rays_per_s"] = n_img_rays * n * max(1, args.steps // 2) / dth

    if args.eval_iters > 0:
        extra["eval_c5"] = eval_bench(dev, rs, emb, models, args.eval_iters)
    if args.train_iters > 0:
        extra["train_c3"] = train_bench(dev, k, args.train_iters, world)

    traffic = None
    tpath = os.path.join(ROOT, "profiles", "field_kernel_traffic.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            tj = json.load(f)
            traffic = tj.get(args.precision, {}).get("hbm_bytes_per_launch")

    result = {
        "metric": "rendered rays/sec (128x128, 64 samples/ray)",
        "value": value,
        "unit": "rays/s",
        "n_gpus": n,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "bf16x3" if args.precision == "bf16x3" else "f32",
        "data": "synthetic (hash-initialised CodeNeRFModel weights, one latent code pair, spherical poses)",
        "config": {"workload": "C2: srn-cars-code 128x128 image per rank-step, 64 coarse samples/ray, "
                               "chunk 4096, lindepth near 0.8 far 1.8, fused HIP render",
                   "images_per_step": n, "rays_per_image": n_img_rays, "samples_per_ray": NC,
                   "parallelism": f"ray-sharded x{n} + RCCL all-gather" if n > 1 else "single GPU"},
        "roofline": {"kernel": kname, "bound": "mfma", "achieved": achieved_tf, "peak": peak,
                     "unit": "TFLOP/s", "frac": achieved_tf / peak, "traffic": traffic,
                     "avg_launch_ms": field_avg_ms, "flop_per_launch": flop_per_launch,
                     "mfma_passes": passes, "fp32_equiv_tflops": algo_tf},
    }
    result.update(extra)

    if rank == 0 and not args.no_cpu_baseline:
        result["cpu_baseline"], result["psnr_vs_ref"] = cpu_baseline(img, k, poses, n)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


def eval_bench(dev, rs, emb, models, iters):
    """C5 (srn-cars-code-3080-val.yml): one eval.py:141-165 iteration = 2048 random rays, 64+64
    perturbed samples, forward + backward through the HIP kernels into (codes, theta, phi, rho),
    AdamW step.  Weights frozen (their grads are never read by the reference's optimiser)."""
    import numpy as np
    from codenerf.evaluate import eval_step_loss
    from codenerf.nerf import PointSampler
    ps = PointSampler(NC, NF, NEAR, FAR, "lindepth", True, torch.float32, dev)
    rs.sample_size = 2048
    target = torch.rand(H * W, 4, generator=torch.Generator().manual_seed(3)).to(dev)
    mods = {"nerf_coarse": models[0], "nerf_fine": models[1]}
    saved = [(m, m.precision) for m in models]
    for m in models:
        m.requires_grad_(False)
    zs = (torch.randn(1, 256, generator=torch.Generator().manual_seed(4)) * 0.3).to(dev).requires_grad_(True)
    zt = (torch.randn(1, 256, generator=torch.Generator().manual_seed(5)) * 0.3).to(dev).requires_grad_(True)
    th = torch.tensor([1.57], device=dev).requires_grad_(True)
    ph = torch.tensor([0.0], device=dev).requires_grad_(True)
    rh = torch.tensor([1.3], device=dev).requires_grad_(True)
    opt = torch.optim.AdamW([{"params": [zs, zt]}, {"params": [th, ph]}, {"params": [rh]}], lr=1e-2)
    np.random.seed(0)

    def it():
        loss, _ = eval_step_loss(th, ph, rh, zs, zt, target, (rs, ps), emb, mods, 1e-5)
        opt.zero_grad()
        loss.backward()
        opt.step()

    for _ in range(2):
        it()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        it()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / iters
    for m, prec in saved:
        m.requires_grad_(True)
        m.precision = prec
    return {"ms_per_iter": dt * 1e3, "rays_per_s": 2048 / dt, "rays_per_iter": 2048, "samples": "64+64 perturbed",
            "note": "forward with ReLU masks + one fused backward launch per field (3xbf16, frozen weights); "
                    "host-side numpy ray permutation and eval.py's per-iteration psnr read-back included"}


def train_bench(dev, k, iters, world):
    """C3 training (srn-cars-code.yml; train.py:64-114): one iteration = 4 images x 4096 random rays,
    chunk 4096 -> 4 optimiser steps, each 64+64 perturbed samples per ray with per-object codes from a
    2458-object table, fwd + bwd into both MLPs and both code tables, flat AdamW (one launch), LambdaLR,
    and with N ranks one RCCL all-reduce of the flat gradient per step (DDP's average)."""
    import numpy as np
    from types import SimpleNamespace as NS
    from codenerf import nerf as N, train as T
    n_objects, batch = 2458, 4
    cfg = NS(is_distributed=world > 1,
             models=NS(embedding=NS(shape_code_size=256, texture_code_size=256), nerf_coarse=NS(hidden_size=256),
                       nerf_fine=NS(hidden_size=256)),
             nerf=NS(embedder=NS(num_encoding_fn_xyz=10, include_input_xyz=True, log_sampling_xyz=True,
                                 num_encoding_fn_dir=4, include_input_dir=True, log_sampling_dir=True,
                                 use_viewdirs=True),
                     ray_sampler=NS(num_random_rays=4096),
                     point_sampler=NS(num_coarse=NC, num_fine=NF, near_limit=NEAR, far_limit=FAR,
                                      spacing_mode="lindepth", perturb=True),
                     train=NS(chunksize=4096)),
             optimizer=NS(type="AdamW", lr=1e-4, embedding_lr=1e-3, scheduler_gamma=0.1,
                          scheduler_step_size=5000000),
             experiment=NS(regularizer_lambda=1e-5))
    rank = dist.get_rank() if world > 1 else 0
    torch.manual_seed(rank + 1)                   # train.py:29-31: each rank draws its own rays
    np.random.seed(rank + 1)
    models = T.prepare_models(cfg, n_objects, dev)
    opt, sched = T.prepare_optimizer(cfg, models)
    samplers = N.prepare_samplers(cfg, H, W, k, torch.float32, dev)
    embedders = N.prepare_embedders(cfg, torch.float32, dev)
    g = torch.Generator().manual_seed(7 + rank)
    data = {"color": torch.rand(batch, H, W, 4, generator=g).to(dev),
            "pose": torch.stack([pose(0.4 + 0.5 * i, 0.3, 1.3) for i in range(batch)]).to(dev),
            "object_id": torch.randint(0, n_objects, (batch,), generator=g).to(dev)}
    T.train_iteration(cfg, data, models, opt, sched, samplers, embedders)        # warm-up
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        logs = T.train_iteration(cfg, data, models, opt, sched, samplers, embedders)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    # the optimiser kernel alone: 20 back-to-back cn_adamw_step launches over the whole flat
    # buffer (one segment per group, as a step builds them) between HIP events on its stream
    from codenerf import ops
    n_params = sum(p.numel() for m in models.values() for p in m.parameters())
    f = opt.flat_buffers()
    st = opt.group_starts
    segs = [[st[i], st[i + 1], float(gr["lr"]), float(gr["weight_decay"]), 1000]
            for i, gr in enumerate(opt.param_groups)]
    flat_copy = {kk: v.clone() for kk, v in f.items()}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        ops.adamw_step(flat_copy["param"], flat_copy["grad"], flat_copy["exp_avg"], flat_copy["exp_avg_sq"], segs,
                       0.9, 0.999, 1e-8)
    e1.record()
    torch.cuda.synchronize()
    adamw_ms = e0.elapsed_time(e1) / 20
    rays = batch * 4096 * iters * world
    return {"ms_per_iter": dt / iters * 1e3, "rays_per_s": rays / dt, "rays_per_iter_per_rank": batch * 4096,
            "optimizer_steps_per_iter": batch, "samples": "64+64 perturbed", "objects": n_objects,
            "params": n_params, "loss": float(logs[-1]["total_loss"]),
            "adamw": {"kernel_ms": adamw_ms, "bytes": 28 * n_params,
                      "gbps": 28 * n_params / (adamw_ms * 1e-3) / 1e9},
            "note": "fp32 training field kernel (activations kept), layer-wise 3xbf16 MFMA backward GEMMs, "
                    "flat AdamW; train.py's per-chunk psnr read-back included"}


def cpu_baseline(img, k, poses, n):
    """The CPU oracle (reference op sequence, torch fp32) on this host: one full C2 image."""
    from oracle import codenerf_oracle as O
    from codenerf import synthetic
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    d = O.ray_directions(H, W, k)
    ro, rd = O.ray_bundle(d, poses[:1].cpu())
    ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
    nr = ro.shape[0]
    zs, zt = synthetic.latent_codes(5, 1).expand(nr, -1), synthetic.latent_codes(6, 1).expand(nr, -1)
    pc, pf = synthetic.codenerf_params(0), synthetic.codenerf_params(1)
    t0 = time.perf_counter()
    with torch.no_grad():
        out = O.render_image(ro, rd, zs, zt, O.Sampling(NC, NF, NEAR, FAR), O.EmbedCfg(), pc, pf, CHUNK,
                             coarse_only=True)
    dt = time.perf_counter() - t0
    ref = out["rgb_coarse"]
    mine = img[:nr].float().cpu() if img is not None else None
    psnr = None
    if mine is not None and mine.shape == ref.shape:
        mse = float(((mine - ref) ** 2).mean())
        psnr = O.mse2psnr(mse)
    return ({"value": nr / dt, "unit": "rays/s", "cores": threads, "kind": "port",
             "sample": f"one full 128x128 image (16384 rays x 64 coarse samples, chunk 4096), {dt:.1f} s"}, psnr)


if __name__ == "__main__":
    main()
