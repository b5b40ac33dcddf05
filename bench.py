"""Benchmark: rendered rays/s on SRN-cars 128x128 at 64 samples/ray (BASELINE.json metric, config C2).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--images-per-step B] [--no-cpu-baseline]

One step renders B novel 128x128 views of one held-out car per rank (default B = 16; 16384 rays
each, 64 coarse samples per ray, srn-cars-code near 0.8 / far 1.8, lindepth, 4096-ray chunks)
through the gfx950 path: ray bundle -> per-object code terms -> depths -> fused encode+MLP field
kernel -> compositing, in the reference's precision (fp32: exact-product fp32 MFMA).  That is the
headline ``value`` / ``dtype`` / ``roofline``.  Beside it, on the same batch: the opt-in 3xbf16
field kernel (``bf16x3``, its own roofline against the bf16 MFMA peak), the C3 64+64 hierarchical
render, the C4 chairs render sharded over the ranks, one C5 eval step and one C3 training
iteration, and the CPU baseline.

Ranks: under torch.distributed.run (WORLD_SIZE set) each process is one rank.  Otherwise
``--gpus N`` > 1 spawns N worker processes itself (as the reference's mp.spawn, train.py:159-179)
before this process touches the GPU, and refuses to run when fewer than N GPUs are visible.
With N ranks every view is split over the ranks exactly like parallel_image_render
(nerf/__init__.py:179-218) and the rendered pixels are all-gathered to rank 0 over RCCL; per-rank
work is fixed (B views' worth of rays), so C2 scaling is weak.

Inputs are synthetic (no dataset/checkpoint offline): hash-initialised CodeNeRFModel weights of the
reference architecture, one latent code pair, spherical poses.  Everything is resident in HBM
before timing.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
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
KERNELS = {"f32": ("field_w16_kernel<kFromRayZ> (fused posenc + CodeNeRF MLP, fp32 v_mfma_f32_16x16x4_f32, "
                    "2 waves/SIMD)", 1, PEAK_FP32_MFMA_TFLOPS),
           "f32_v1": ("field_kernel<kFromRayZ> (fused posenc + CodeNeRF MLP, fp32 v_mfma_f32_32x32x2_f32, "
                      "1 wave/SIMD)", 1, PEAK_FP32_MFMA_TFLOPS),
           "bf16x3": ("field_x3_kernel<kFromRayZ> (fused posenc + CodeNeRF MLP, 3xbf16 32x32x16 MFMA, "
                      "1 wave/SIMD)", 3, PEAK_BF16_MFMA_TFLOPS),
           "bf16x3_w16": ("field_x3w_kernel<kFromRayZ> (fused posenc + CodeNeRF MLP, 3xbf16 16x16x32 MFMA, "
                          "2 waves/SIMD)", 3, PEAK_BF16_MFMA_TFLOPS)}


def pose(theta, phi, rho):
    """eval.py:22-38 pose_spherical (host, float32)."""
    st, ct, sp, cp = math.sin(theta), math.cos(theta), math.sin(phi), math.cos(phi)
    m = torch.eye(4)
    m[0, 0], m[1, 0] = -sp, cp
    m[0, 1], m[1, 1], m[2, 1] = -st * cp, -st * sp, ct
    m[0, 2], m[1, 2], m[2, 2] = ct * cp, ct * sp, st
    m[0, 3], m[1, 3], m[2, 3] = rho * ct * cp, rho * ct * sp, rho * st
    return m


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--images-per-step", type=int, default=16,
                    help="views of the car rendered per rank per step (16 x 16384 rays: ~90 ms of fp32 work)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="headline + bf16x3 only (profiling runs)")
    ap.add_argument("--precision", default="f32", choices=sorted(KERNELS),
                    help="headline field-kernel arithmetic (f32 = the reference's precision)")
    ap.add_argument("--eval-iters", type=int, default=40,
                    help="C5: time this many test-time-optimisation iterations (0 = skip)")
    ap.add_argument("--train-iters", type=int, default=8,
                    help="C3 training: time this many train.py iterations (4 x 4096 rays each; 0 = skip)")
    ap.add_argument("--backend", default="nccl", choices=("nccl", "gloo"),
                    help="process-group backend for N > 1 (nccl = RCCL; gloo: test harness only)")
    ap.add_argument("--quiet", action="store_true", help="return the result without printing it (tests)")
    return ap.parse_args(argv)


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawned(local_rank: int, argv, n: int, port: int):
    os.environ.update(RANK=str(local_rank), LOCAL_RANK=str(local_rank), WORLD_SIZE=str(n),
                      MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    run(parse_args(argv))


def main():
    args = parse_args()
    if "WORLD_SIZE" in os.environ:
        world = int(os.environ["WORLD_SIZE"])
        if args.gpus not in (1, world):
            raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks")
        run(args)
        return
    if args.gpus <= 1:
        run(args)
        return
    # spawn one process per GPU before this process touches the GPU (device_count does not
    # initialise HIP on this image); never re-exec a process that has
    visible = torch.cuda.device_count()
    if visible < args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} needs {args.gpus} visible GPUs, found {visible}")
    import torch.multiprocessing as mp
    mp.start_processes(_spawned, args=(sys.argv[1:], args.gpus, free_port()), nprocs=args.gpus, join=True,
                       start_method="spawn")


def run(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    n = max(world, 1)
    rccl_world = 1
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        # the launcher's env:// rendezvous, or a file:// one (CODENERF_INIT_METHOD: the multi-rank tests)
        init = os.environ.get("CODENERF_INIT_METHOD") or None
        if args.backend == "nccl":
            dist.init_process_group("nccl", init_method=init, rank=rank, world_size=world,
                                    device_id=torch.device("cuda", local))
            rccl_world = dist.get_world_size()
        else:       # gloo: the multi-rank test harness (ranks sharing one GPU; tests/test_gpu_multirank.py)
            dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    dev = torch.device("cuda", local)

    import codenerf
    from codenerf import synthetic
    from codenerf.models import CodeNeRFModel
    from codenerf.nerf import PointSampler, PositionalEmbedder, RaySampler, gather_views, render_rays
    from codenerf.utils import split_sizes
    codenerf.load_library()
    info = codenerf.build_info()

    B = args.images_per_step
    k = synthetic.srn_intrinsics(H, FOCAL)
    rs = RaySampler(H, W, k, sample_size=4096, device=dev, datatype=torch.float32)
    ps = PointSampler(NC, NF, NEAR, FAR, "lindepth", False, torch.float32, dev)
    emb = (PositionalEmbedder(10, True, True, torch.float32, dev), PositionalEmbedder(4, True, True, torch.float32, dev))
    models = []
    for seed in (0, 1):
        m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
        m.load_state_dict(synthetic.codenerf_params(seed))
        models.append(m.to(dev).eval())
    zs = synthetic.latent_codes(5, 1).to(dev)
    zt = synthetic.latent_codes(6, 1).to(dev)
    # B*n views on a turntable around the car; rank r renders its Q5 slice of every view
    views = B * n
    poses = torch.stack([pose(0.5 + 0.7 * math.sin(0.37 * i), 2 * math.pi * i / views, 1.3)
                         for i in range(views)]).to(dev)
    n_img_rays = H * W
    per, _ = split_sizes(n_img_rays, n)
    start = sum(per[:rank])
    chunk = min(CHUNK, per[rank])
    rays_per_rank = per[rank] * views

    def set_precision(prec):
        for mm in models:
            mm.precision = prec
            mm.packed()                          # weights packed once per format (frozen, as in eval)

    timing = {}

    def render_step(record: bool, coarse_only: bool, ps_=ps, poses_=poses, per_=per, start_=start, chunk_=chunk):
        with torch.no_grad():
            nv = poses_.shape[0]
            ro, rd = rs.get_bundle(poses_)                    # (views, H, W, 3)
            ro = ro.reshape(nv, -1, 3)[:, start_:start_ + per_[rank]].reshape(-1, 3)
            rd = rd.reshape(nv, -1, 3)[:, start_:start_ + per_[rank]].reshape(-1, 3)
            r = ro.shape[0]
            hook = {} if record else None
            key = "rgb_coarse" if coarse_only else "rgb_fine"
            if per_[rank] % chunk_ == 0:
                # the views' slices concatenated: every chunk lies inside one view, so one pass has
                # parallel_image_render's per-view chunking (the Q1 view-direction map) exactly
                rgb = render_rays(ro, rd, zs.expand(r, -1), zt.expand(r, -1), ps_, emb, models[0], models[1],
                                  chunk_rows=chunk_, coarse_only=coarse_only, events=hook)[key]
            else:
                # a ragged last chunk per view (e.g. 3 ranks: 5461 rays per view): chunking restarts at
                # every view as parallel_image_render's does, so one pass per view
                p_ = per_[rank]
                rgb = torch.cat([render_rays(ro[v * p_:(v + 1) * p_], rd[v * p_:(v + 1) * p_], zs.expand(p_, -1),
                                             zt.expand(p_, -1), ps_, emb, models[0], models[1], chunk_rows=chunk_,
                                             coarse_only=coarse_only, events=hook)[key] for v in range(nv)])
            if world > 1:
                rgb = gather_views(rgb, per_, rank, nv)          # rank 0: (views, H*W, 3)
                if rgb is not None:
                    rgb = rgb.reshape(nv * n_img_rays, 3)
            if record:
                timing["pending"] += hook["field"]
            return rgb

    def timed(k_steps, w_steps, fn):
        for _ in range(w_steps):
            fn(False)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        timing["pending"] = []
        t0 = time.perf_counter()
        img = None
        for _ in range(k_steps):
            img = fn(True)
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

    samples_per_launch = rays_per_rank * NC
    flop_per_launch = samples_per_launch * FLOP_PER_SAMPLE

    def roofline(prec, field_ms):
        kname, passes, peak = KERNELS[prec]
        avg = sum(field_ms) / max(1, len(field_ms))
        algo_tf = flop_per_launch / (avg * 1e-3) / 1e12       # algorithmic (fp32-equivalent) rate
        achieved = passes * algo_tf                           # MFMA flops the hardware executes
        return {"kernel": kname, "bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                "frac": achieved / peak, "traffic": traffic_of(prec, samples_per_launch), "avg_launch_ms": avg,
                "launches_timed": len(field_ms), "flop_per_launch": flop_per_launch,
                "samples_per_launch": samples_per_launch, "flop_per_sample": FLOP_PER_SAMPLE,
                "mfma_passes": passes, "fp32_equiv_tflops": algo_tf,
                "timing": "HIP events on the launching (current) stream around every field launch of the timed steps",
                "traffic_source": traffic_source(prec)}

    # ---- headline: C2 in the reference's precision
    set_precision(args.precision)
    dt, field_ms, img = timed(args.steps, args.warmup, lambda rec: render_step(rec, True))
    total_rays = n_img_rays * views * args.steps
    value = total_rays / dt
    result = {
        "metric": "rendered rays/sec (128x128, 64 samples/ray)",
        "value": value,
        "unit": "rays/s",
        "n_gpus": n,
        "rccl_world_size": rccl_world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3,
        "timed_s": dt,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.precision == "f32" else args.precision,
        "data": "synthetic (hash-initialised CodeNeRFModel weights, one latent code pair, spherical poses)",
        "config": {"workload": "C2: srn-cars-code, one held-out car, 128x128 views, 64 coarse samples/ray, "
                               "chunk 4096, lindepth near 0.8 far 1.8, perturb=False (parity mode: the "
                               "deterministic depths the golden renders pin; the perturbed form is the "
                               "'perturbed' line), fused HIP render",
                   "perturb": False,
                   "images_per_step": views, "images_per_rank_step": B, "rays_per_image": n_img_rays,
                   "samples_per_ray": NC,
                   "parallelism": f"ray-sharded x{n} + RCCL all-gather" if n > 1 else "single GPU"},
        "roofline": roofline(args.precision, field_ms),
        "build": {"cn_version": info["version"], "tree_src": info["tree_src"]},
    }
    psnr_img = {args.precision: img}

    # ---- the other field-kernel format on the same batch
    other = "bf16x3" if args.precision == "f32" else "f32"
    set_precision(other)
    dto, fms_o, img_o = timed(args.steps, args.warmup, lambda rec: render_step(rec, True))
    psnr_img[other] = img_o
    result[other] = {"value": total_rays / dto, "unit": "rays/s", "ms_per_step": dto / args.steps * 1e3,
                     "dtype": other, "roofline": roofline(other, fms_o),
                     "note": ("opt-in 3-product bf16 split (Wh.Xh + Wh.Xl + Wl.Xh, fp32 accumulate): narrower than "
                              "the reference's fp32; parity-tested at the same tolerances incl. trained-magnitude "
                              "weights (tests/test_gpu_configs.py)") if other == "bf16x3" else "reference precision"}
    if args.precision == "f32":
        # the previous fp32 kernel (32x32x2, one wave per SIMD; still the training forward)
        set_precision("f32_v1")
        dtv, fms_v, img_v = timed(args.steps, args.warmup, lambda rec: render_step(rec, True))
        psnr_img["f32_v1"] = img_v
        result["f32_v1"] = {"value": total_rays / dtv, "unit": "rays/s", "ms_per_step": dtv / args.steps * 1e3,
                            "dtype": "f32", "roofline": roofline("f32_v1", fms_v),
                            "note": "round-1 fp32 kernel, kept as the forward of the layer-wise training path (models whose inference and training precisions differ)"}
    set_precision(args.precision)

    if not args.no_extras:
        # ---- C2 as srn-cars-code.yml's validation render configures it (perturb: True, Q4): stratified
        # depths from the device RNG (torch.rand_like on the GPU, point_sampler.py:61-65)
        ps_p = PointSampler(NC, NF, NEAR, FAR, "lindepth", True, torch.float32, dev)
        kp = max(1, args.steps // 4)
        dtp, fp_, _ = timed(kp, 1, lambda rec: render_step(rec, True, ps_p))
        result["perturbed"] = {"value": total_rays / args.steps * kp / dtp, "unit": "rays/s",
                               "ms_per_step": dtp / kp * 1e3, "steps": kp, "dtype": args.precision,
                               "field_launch_ms_avg": sum(fp_) / max(1, len(fp_)),
                               "note": "C2 with perturb=True (stratified depths drawn on the device per step)"}
        # ---- C3: 64+64 hierarchical render, same views
        k3 = max(1, args.steps // 4)
        dth, f3, _ = timed(k3, 1, lambda rec: render_step(rec, False))
        result["hierarchical_64_64"] = {"value": n_img_rays * views * k3 / dth, "unit": "rays/s",
                                        "ms_per_step": dth / k3 * 1e3, "steps": k3, "dtype": args.precision,
                                        "field_launch_ms_avg": sum(f3) / max(1, len(f3)),
                                        "samples_per_ray": "64 coarse + 128 fine (64+64 merged)"}
        # ---- C4: chairs (Nc 32 / Nf 128, near 1.25 far 2.75), B views each sharded over the ranks
        ps4 = PointSampler(32, 128, 1.25, 2.75, "lindepth", False, torch.float32, dev)
        poses4 = torch.stack([pose(0.5 + 0.7 * math.sin(0.37 * i), 2 * math.pi * i / B, 2.0)
                              for i in range(B)]).to(dev)
        dt4, f4, _ = timed(k3, 1, lambda rec: render_step(rec, False, ps4, poses4, per, start, chunk))
        result["c4_chairs_sharded"] = {"value": n_img_rays * B * k3 / dt4, "unit": "rays/s", "scaling": "strong",
                                       "ms_per_step": dt4 / k3 * 1e3, "steps": k3, "views_per_step": B,
                                       "rays_per_rank_per_view": per[rank], "dtype": args.precision,
                                       "samples_per_ray": "32 coarse + 160 fine",
                                       "field_launch_ms_avg": sum(f4) / max(1, len(f4))}
        if args.eval_iters > 0:
            result["eval_c5"] = {p: eval_bench(dev, rs, emb, models, args.eval_iters, p) for p in ("f32", "bf16x3")}
            result["eval_c5_chairs"] = eval_bench(dev, rs, emb, models, args.eval_iters, "f32", shape="chairs")
            # the HIP-graph form at N = 1 only: C5 is a per-replica loop, and a capture beside a live
            # RCCL communicator (its watchdog thread queries events) is a risk the scaling lines need not take
            if world == 1:
                for p in ("f32", "bf16x3"):
                    result["eval_c5"][p]["graph"] = eval_bench(dev, rs, emb, models, args.eval_iters, p, graph=True)
            else:
                # the optional ray-sharded mode: one C5 optimisation strong-scaled over the ranks
                result["eval_c5_sharded"] = eval_bench(dev, rs, emb, models, args.eval_iters, "f32", sharded=True)
            set_precision(args.precision)
        if args.train_iters > 0:
            result["train_c3"] = train_bench(dev, k, args.train_iters, world, "f32")
            result["train_c3"]["bf16x3"] = train_bench(dev, k, args.train_iters, world, "bf16x3")
            # the reference's own runnable training configurations, fp32
            result["train_cars_code"] = train_bench(dev, k, args.train_iters, world, "f32", shape="cars_code")
            result["train_3080"] = train_bench(dev, k, 4 * args.train_iters, world, "f32", shape="3080")

    if world > 1 and rank == 0 and psnr_img[args.precision] is not None:
        result.update(multi_rank_check(psnr_img[args.precision], rs, poses[:1], per, zs, zt, ps, emb, models))
    if rank == 0 and world == 1 and not args.no_cpu_baseline:   # the CPU baseline: rank 0 at N=1 only
        cb, ref_img = cpu_baseline(k, poses[:1])
        result["cpu_baseline"] = cb
        from oracle.codenerf_oracle import mse2psnr
        for prec, im in psnr_img.items():
            if im is not None:
                mse = float(((im[:n_img_rays].float().cpu() - ref_img) ** 2).mean())
                result.setdefault("psnr_vs_ref", {})[prec] = mse2psnr(mse)
    if rank == 0 and not args.quiet:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return result if rank == 0 else None


def multi_rank_check(img, rs, pose1, per, zs, zt, ps, emb, models):
    """After the timed region, N > 1, rank 0: the gathered first view of the headline's last step
    against the same view rendered on this GPU alone, (a) with the N-rank split and per-rank chunking
    (parallel_image_render's semantics: must be identical) and (b) as one 4096-ray-chunked image (the
    single-GPU render: differs by the Q1 view-direction map wherever the chunking differs)."""
    from codenerf.nerf import render_rays
    n_img = H * W
    with torch.no_grad():
        ro, rd = rs.get_bundle(pose1)
        ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
        parts, s0 = [], 0
        for p in per:
            sl = slice(s0, s0 + p)
            parts.append(render_rays(ro[sl], rd[sl], zs.expand(p, -1), zt.expand(p, -1), ps, emb, models[0],
                                     models[1], chunk_rows=min(CHUNK, p), coarse_only=True)["rgb_coarse"])
            s0 += p
        sharded = torch.cat(parts)
        single = render_rays(ro, rd, zs.expand(n_img, -1), zt.expand(n_img, -1), ps, emb, models[0], models[1],
                             chunk_rows=CHUNK, coarse_only=True)["rgb_coarse"]
    got = img[:n_img]
    return {"multi_rank_maxdiff": float((got - sharded).abs().max()),
            "multi_rank_vs_single_chunking_maxdiff": float((got - single).abs().max()),
            "multi_rank_note": "gathered view 0 vs the same view rendered on rank 0 alone with the N-rank split "
                               "and per-rank chunks (expected 0) and with one 4096-ray chunking (Q1 view-dir map)"}


def traffic_of(prec, samples):
    """HBM bytes per launch from the PMC passes (profiles/field_kernel_traffic.json: FETCH_SIZE and
    WRITE_SIZE in separate rocprofv3 passes, gfx950-corrected), scaled from per-sample bytes."""
    tpath = os.path.join(ROOT, "profiles", "field_kernel_traffic.json")
    if not os.path.exists(tpath):
        return None
    with open(tpath) as f:
        per_sample = json.load(f).get(prec, {}).get("hbm_bytes_per_sample")
    return None if per_sample is None else per_sample * samples


def traffic_source(prec):
    """Where `traffic` comes from: it is NOT a counter read in this run (PMC passes cannot share a
    run with the timing), but the per-sample HBM bytes of the kernel's own PMC passes, scaled."""
    tpath = os.path.join(ROOT, "profiles", "field_kernel_traffic.json")
    if not os.path.exists(tpath):
        return None
    with open(tpath) as f:
        rec = json.load(f).get(prec, {})
    return (f"rocprofv3 FETCH_SIZE / WRITE_SIZE passes ({rec.get('measured_round', '?')}, {rec.get('raw', '?')}), "
            "per-sample bytes x this launch's samples; profiles/field_kernel_traffic.json")


# The eval shapes: C5 (srn-cars-code-3080-val.yml:47-52, BASELINE config 5) and the chairs eval of
# srn-chairs-code.yml:47-54 (4096 rays, 32 + 128, near 1.25 / far 2.75).
EVAL_SHAPES = {"c5": dict(rays=2048, nc=64, nf=64, near=NEAR, far=FAR, rho=1.3),
               "chairs": dict(rays=4096, nc=32, nf=128, near=1.25, far=2.75, rho=2.0)}


def eval_bench(dev, rs, emb, models, iters, precision, graph=False, sharded=False, shape="c5"):
    """C5 (srn-cars-code-3080-val.yml): one eval.py:141-167 iteration = 2048 random rays, 64+64
    perturbed samples, forward + backward through the HIP kernels into (codes, theta, phi, rho),
    AdamW step.  Weights frozen (their grads are never read by the reference's optimiser).
    ``sharded`` (N > 1): the optional ray-sharded mode -- ONE optimisation, each iteration's 2048 rays
    split over the ranks, the gradients summed by one all-reduce (codenerf.evaluate.sharded_eval_step);
    timed between barriers, the max over ranks."""
    import numpy as np
    from codenerf.autograd import backward_from
    from codenerf.evaluate import GraphedEvalStep, eval_step_loss, step_psnr_tensor
    from codenerf.nerf import PointSampler
    from codenerf.optim import AdamW
    sh = EVAL_SHAPES[shape]
    n_rays = sh["rays"]
    ps = PointSampler(sh["nc"], sh["nf"], sh["near"], sh["far"], "lindepth", True, torch.float32, dev)
    rs.sample_size = n_rays
    target = torch.rand(H * W, 4, generator=torch.Generator().manual_seed(3)).to(dev)
    mods = {"nerf_coarse": models[0], "nerf_fine": models[1]}
    saved = [(m, m.precision) for m in models]
    for m in models:
        m.requires_grad_(False)
        m.precision = precision
    zs = (torch.randn(1, 256, generator=torch.Generator().manual_seed(4)) * 0.3).to(dev).requires_grad_(True)
    zt = (torch.randn(1, 256, generator=torch.Generator().manual_seed(5)) * 0.3).to(dev).requires_grad_(True)
    th = torch.tensor([1.57], device=dev).requires_grad_(True)
    ph = torch.tensor([0.0], device=dev).requires_grad_(True)
    rh = torch.tensor([sh["rho"]], device=dev).requires_grad_(True)
    # test_time_optimize's optimiser for val_type AdamW: the flat one-launch AdamW
    opt = AdamW([{"params": [zs, zt]}, {"params": [th, ph]}, {"params": [rh]}], lr=1e-2)
    np.random.seed(0)

    if sharded:
        from codenerf.evaluate import sharded_eval_step, sync_shard_state
        sync_shard_state((rs, ps), 0)         # every rank draws rank 0's rays and uniforms

        def it():
            _, logs = sharded_eval_step(th, ph, rh, zs, zt, target, (rs, ps), emb, mods, opt, 1e-5)
            step_psnr_tensor(logs)
    elif graph:
        # the iteration's forward + backward captured once as a HIP graph (GraphedEvalStep);
        # the numpy draw, the replay, the flat AdamW and the psnr read-back per iteration
        graphed = GraphedEvalStep(th, ph, rh, zs, zt, target, (rs, ps), emb, mods, opt, 1e-5)

        def it():
            _, logs = graphed.step()  # forward + backward + the flat AdamW update, one replay
            graphed.prefetch()  # the next iteration's numpy draw while the GPU replays this one
            step_psnr_tensor(logs)  # eval.py:159's psnr, on the device
    else:
        def it():
            loss, logs = eval_step_loss(th, ph, rh, zs, zt, target, (rs, ps), emb, mods, 1e-5)
            opt.zero_grad()
            backward_from(loss)
            opt.step()
            step_psnr_tensor(logs)  # eval.py:159's per-iteration psnr, on the device (no read-back)

    warm_up(it, dev, collective=sharded)
    if sharded:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(iters):
        it()
    torch.cuda.synchronize()
    if sharded:
        dist.barrier()
    dt = (time.perf_counter() - t0) / iters
    if sharded:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    for m, prec in saved:
        m.requires_grad_(True)
        m.precision = prec
    note = ("3xbf16 forward with ReLU masks + one fused 3xbf16 backward launch per field" if precision == "bf16x3"
            else "fp32 16x16x4 forward with ReLU masks + one fused fp32 backward launch per field")
    if graph:
        note += "; forward + backward + AdamW replayed as one captured HIP graph (GraphedEvalStep)"
    # the MLP work of one iteration: forward + dX (2 x 572,416 FLOP; frozen weights, no dW) per sample
    # evaluation, 64 coarse + 128 merged fine samples per ray, as train_bench's accounting
    flop_iter = 2.0 * FLOP_PER_SAMPLE * n_rays * (2 * sh["nc"] + sh["nf"])
    tflops = flop_iter / dt / 1e12
    peak = PEAK_FP32_MFMA_TFLOPS if precision == "f32" else PEAK_BF16_MFMA_TFLOPS / 3.0
    extra = {"mlp_tflop_per_iter": flop_iter / 1e12, "achieved_tflops": tflops, "frac_of_peak": tflops / peak}
    if sharded:
        world = dist.get_world_size()
        note += (f"; ray-sharded over {world} ranks (one optimisation; {n_rays} / {world} rays per rank and iteration, "
                 "one all-reduce of the 515 code / pose gradient floats; each share is its own Q1 chunk, so this "
                 "mode is reported beside the reference's per-rank optimisation, Q6)")
        extra.update(scaling="strong", n_ranks=world, rays_per_rank_per_iter=n_rays // world,
                     frac_of_peak=tflops / (peak * world))
    return {"ms_per_iter": dt * 1e3, "rays_per_s": n_rays / dt, "rays_per_iter": n_rays,
            "samples": f"{sh['nc']}+{sh['nf']} perturbed", "near_far": [sh["near"], sh["far"]],
            "dtype": precision, **extra,
            "note": note + "; fused pose path + loss; host-side numpy ray permutation included; eval.py's "
                           "per-iteration psnr formed on the device"}


# The training shapes: C3 (BASELINE config 3: srn-cars-code.yml with 64 + 64), and the reference's own
# runnable configurations srn-cars-code.yml:18,45-48,63 (4 images x 4096 rays, 32 + 128, chunk 4096) and
# srn-cars-code-3080.yml:18,45-48,62 (1 image x 4096 rays, 64 + 128, chunk 1024).
TRAIN_SHAPES = {"c3": dict(batch=4, nc=64, nf=64, chunk=4096),
                "cars_code": dict(batch=4, nc=32, nf=128, chunk=4096),
                "3080": dict(batch=1, nc=64, nf=128, chunk=1024)}


def warm_up(step, dev, min_s: float = 0.15, min_steps: int = 2, collective: bool = False) -> int:
    """Untimed iterations until at least ``min_s`` seconds of them have run (and ``min_steps``): the side
    lines start after host-side work (packs, another line's teardown) with the GPU's clock down -- a C5
    trace shows the first six iterations at 3.73 .. 3.46 ms before the steady 3.40 ms
    (gpurun_out/r06d) -- and a fixed two-iteration warm-up timed that ramp.  -> iterations run."""
    if collective:
        # steps with a collective in them (sharded eval, multi-rank training): every rank runs the same count
        for _ in range(max(min_steps, 6)):
            step()
        torch.cuda.synchronize(dev)
        return max(min_steps, 6)
    n, t0 = 0, time.perf_counter()
    while n < min_steps or time.perf_counter() - t0 < min_s:
        step()
        n += 1
        if n >= min_steps:
            torch.cuda.synchronize(dev)
    return n


def train_bench(dev, k, iters, world, precision=None, shape="c3"):
    """Training (train.py:64-114) at one of TRAIN_SHAPES: one iteration = batch images x 4096 random
    rays, cut into chunks -> one optimiser step per chunk, each Nc + Nf perturbed samples per ray with
    per-object codes from a 2458-object table, fwd + bwd into both MLPs and both code tables, flat AdamW
    (one launch), LambdaLR, and with N ranks one RCCL all-reduce of the flat gradient per step (DDP's
    average)."""
    import numpy as np
    from types import SimpleNamespace as NS
    from codenerf import nerf as N, train as T
    sh = TRAIN_SHAPES[shape]
    n_objects, batch = 2458, sh["batch"]
    cfg = NS(is_distributed=world > 1,
             models=NS(embedding=NS(shape_code_size=256, texture_code_size=256), nerf_coarse=NS(hidden_size=256),
                       nerf_fine=NS(hidden_size=256)),
             nerf=NS(embedder=NS(num_encoding_fn_xyz=10, include_input_xyz=True, log_sampling_xyz=True,
                                 num_encoding_fn_dir=4, include_input_dir=True, log_sampling_dir=True,
                                 use_viewdirs=True),
                     ray_sampler=NS(num_random_rays=4096),
                     point_sampler=NS(num_coarse=sh["nc"], num_fine=sh["nf"], near_limit=NEAR, far_limit=FAR,
                                      spacing_mode="lindepth", perturb=True),
                     train=NS(chunksize=sh["chunk"])),
             optimizer=NS(type="AdamW", lr=1e-4, embedding_lr=1e-3, scheduler_gamma=0.1,
                          scheduler_step_size=5000000),
             experiment=NS(regularizer_lambda=1e-5))
    rank = dist.get_rank() if world > 1 else 0
    torch.manual_seed(rank + 1)                   # train.py:29-31: each rank draws its own rays
    np.random.seed(rank + 1)
    models = T.prepare_models(cfg, n_objects, dev)
    precision = precision or os.environ.get("CODENERF_PRECISION", "f32")
    for key in ("nerf_coarse", "nerf_fine"):       # field kernels and dW GEMMs in one precision
        models[key].precision = models[key].train_precision = precision
    opt, sched = T.prepare_optimizer(cfg, models)
    samplers = N.prepare_samplers(cfg, H, W, k, torch.float32, dev)
    embedders = N.prepare_embedders(cfg, torch.float32, dev)
    g = torch.Generator().manual_seed(7 + rank)
    oid = torch.randint(0, n_objects, (batch,), generator=g)
    data = {"color": torch.rand(batch, H, W, 4, generator=g).to(dev),
            "pose": torch.stack([pose(0.4 + 0.5 * i, 0.3, 1.3) for i in range(batch)]).to(dev),
            "object_id": oid.to(dev), "object_id_host": oid.numpy()}   # as the resident loader hands them
    warm_up(lambda: T.train_iteration(cfg, data, models, opt, sched, samplers, embedders), dev, collective=world > 1)
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
    # the MLP work of one iteration per rank: forward + dX + dW (3 x 572,416 FLOP) per sample evaluation,
    # (64 coarse + 128 merged fine) samples per ray; against the dense MFMA peak of the precision's pipe
    # (3xbf16: three bf16 products per fp32 one, so its figure is in fp32-equivalent TFLOP/s)
    flop_iter = 3.0 * FLOP_PER_SAMPLE * batch * 4096 * (2 * sh["nc"] + sh["nf"])
    tflops = flop_iter / (dt / iters) / 1e12
    peak = PEAK_FP32_MFMA_TFLOPS if precision == "f32" else PEAK_BF16_MFMA_TFLOPS / 3.0
    steps = batch * 4096 // sh["chunk"]
    return {"ms_per_iter": dt / iters * 1e3, "rays_per_s": rays / dt, "rays_per_iter_per_rank": batch * 4096,
            "mlp_tflop_per_iter": flop_iter / 1e12, "achieved_tflops": tflops, "frac_of_peak": tflops / peak,
            "optimizer_steps_per_iter": steps, "chunk": sh["chunk"],
            "samples": f"{sh['nc']}+{sh['nf']} perturbed ({2 * sh['nc'] + sh['nf']} field samples per ray)",
            "tiles_per_cu": {"coarse": sh["chunk"] * sh["nc"] // 128 / 256,
                             "fine": sh["chunk"] * (sh["nc"] + sh["nf"]) // 128 / 256},
            "objects": n_objects,
            "params": n_params, "loss": float(logs[-1]["total_loss"]), "dtype": precision,
            "adamw": {"kernel_ms": adamw_ms, "bytes": 28 * n_params,
                      "gbps": 28 * n_params / (adamw_ms * 1e-3) / 1e9},
            "note": (("fp32 16x16x4" if precision == "f32" else "3xbf16 32x32x16") +
                     " training forward (activation planes + ReLU masks kept), ONE fused dX backward launch per field"
                     " (masked layer-input gradients kept), deterministic split-M dW GEMMs (encodings generated "
                     "in-kernel, bias and one-object code sums folded in), fused loss, flat AdamW; train.py's "
                     "per-chunk psnr formed on the device (read when logged), no host sync inside an iteration")}


def cgroup_cpus():
    """The cgroup v2 CPU quota of this job (cpu.max "quota period") in CPUs, or None."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else max(1, int(int(quota) / int(period)))
    except (OSError, ValueError):
        return None


def cpu_share() -> dict:
    """The host-core figures the CPU baseline states: OMP_NUM_THREADS, the affinity mask, the cgroup
    quota, os.cpu_count(), and the threads timed = the job's real share of the host: the affinity
    mask, capped by the cgroup quota when one is set (on the GPU box os.cpu_count() and the mask can
    show the whole machine while the job's share is a fraction of it)."""
    env = os.environ.get("OMP_NUM_THREADS")
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = cgroup_cpus()
    threads = min(aff, quota) if quota else aff
    return {"omp_threads": int(env) if env and env.isdigit() else None, "affinity_cores": aff,
            "cgroup_cpus": quota, "os_cpu_count": os.cpu_count(), "threads_timed": threads}


def cpu_threads() -> int:
    return cpu_share()["threads_timed"]


def cpu_baseline(k, pose1):
    """The CPU oracle (the reference's op sequence, torch fp32) on this host, median of 3:
    C2 = 3 full 128x128 images (64 coarse samples), C3 = 3 samples of one 4096-ray chunk at 64+64."""
    from oracle import codenerf_oracle as O
    from codenerf import synthetic
    share = cpu_share()
    threads = share["threads_timed"]
    torch.set_num_threads(threads)
    d = O.ray_directions(H, W, k)
    ro, rd = O.ray_bundle(d, pose1.cpu())
    ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
    nr = ro.shape[0]
    zs, zt = synthetic.latent_codes(5, 1).expand(nr, -1), synthetic.latent_codes(6, 1).expand(nr, -1)
    pc, pf = synthetic.codenerf_params(0), synthetic.codenerf_params(1)
    c2, ref = [], None
    with torch.no_grad():
        # one untimed warm-up chunk (thread pool start, page-in of the weights, the host's clock ramp):
        # the r05 line's first timed image was 52 % slower than its last without it
        O.render_image(ro[:CHUNK], rd[:CHUNK], zs[:CHUNK], zt[:CHUNK], O.Sampling(NC, NF, NEAR, FAR), O.EmbedCfg(),
                       pc, pf, CHUNK, coarse_only=True)
        for _ in range(3):
            t0 = time.perf_counter()
            out = O.render_image(ro, rd, zs, zt, O.Sampling(NC, NF, NEAR, FAR), O.EmbedCfg(), pc, pf, CHUNK,
                                 coarse_only=True)
            c2.append(time.perf_counter() - t0)
            ref = out["rgb_coarse"]
        c3 = []
        for _ in range(3):
            t0 = time.perf_counter()
            O.render_image(ro[:CHUNK], rd[:CHUNK], zs[:CHUNK], zt[:CHUNK], O.Sampling(NC, NF, NEAR, FAR), O.EmbedCfg(),
                           pc, pf, CHUNK)
            c3.append(time.perf_counter() - t0)
    m2, m3 = sorted(c2)[1], sorted(c3)[1]

    def spread(ts, rays):
        return {"min": rays / max(ts), "median": rays / sorted(ts)[1], "max": rays / min(ts),
                "spread": (max(ts) - min(ts)) / sorted(ts)[1]}
    return ({"value": nr / m2, "unit": "rays/s", "cores": threads, "kind": "port",
             "sample": f"C2: median of 3 full 128x128 images (16384 rays x 64 coarse samples, chunk 4096) after "
                       f"one untimed warm-up chunk: {', '.join(f'{t:.2f}' for t in c2)} s",
             "rays_per_s": spread(c2, nr),
             "hierarchical_64_64": {"value": CHUNK / m3, "unit": "rays/s", "rays_per_s": spread(c3, CHUNK),
                                    "sample": f"C3: median of 3 renders of one 4096-ray chunk at 64+64: "
                                              f"{', '.join(f'{t:.2f}' for t in c3)} s"},
             "host": host_cpu(), "host_cores": share}, ref)


def host_cpu() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


if __name__ == "__main__":
    main()
