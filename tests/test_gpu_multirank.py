"""The product's multi-rank code with TWO ranks running the HIP kernels (VERDICT r03
"what's missing" 2): two freshly spawned processes (start_method "spawn", as bench.py and
codenerf.train.launch start ranks) form a world-size-2 gloo group, both on the test box's one GPU
(RCCL refuses two ranks on one device; on a node every rank has its own GPU and the group is RCCL).
This torch build's gloo takes device tensors in every collective the product uses (tools/gloo_probe.py,
profiles/r04/gloo_probe.jsonl), so the product code runs unchanged on the gloo group.

(a) parallel_image_render (nerf/__init__.py:137-226) of C4 chairs with 2 ranks: rank 0's gathered
    image vs the reference's 2-rank image (render_chairs.npz ``n2_rgb``) at 1e-4;
(b) two ranks each run train_minibatch (train.py:96-114) on their own 4096-ray chunk, with the flat
    gradient all-reduce (AdamW.allreduce_grads, DDP's average, util.py:139-142): both end with the same
    parameters, bit-identical to one process that averages the two chunks' gradients before ONE step;
(c) bench.py at 2 ranks (--backend gloo): gather_views + multi_rank_check -> multi_rank_maxdiff == 0,
    including 3 ranks, whose 5461-ray slices need the per-view chunk restart.
"""
import json
import os
import socket
import sys
from types import SimpleNamespace as NS

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawn(fn, world, *args):
    import torch.multiprocessing as mp
    mp.start_processes(fn, args=(world, _port()) + args, nprocs=world, join=True, start_method="spawn")


def _init(rank, world, port):
    import torch.distributed as dist
    import codenerf
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    codenerf.load_library()
    return dev


def _chairs_worker(rank, world, port, out_path):
    import torch.distributed as dist
    from codenerf import synthetic
    from codenerf.nerf import PointSampler, RaySampler, parallel_image_render
    from test_gpu_configs import model_from
    from test_gpu_parity import load
    from test_gpu_train import embedders
    dev = _init(rank, world, port)
    try:
        g = load("render_chairs.npz", dev)
        rs = RaySampler(128, 128, g["intrinsics"].cpu(), sample_size=4096, device=dev, datatype=torch.float32)
        ps = PointSampler(32, 128, 1.25, 2.75, "lindepth", False, torch.float32, dev)
        models = {"nerf_coarse": model_from(dev, synthetic.codenerf_params(0), "f32"),
                  "nerf_fine": model_from(dev, synthetic.codenerf_params(1), "f32")}
        cfg = NS(is_distributed=True, gpus=world, nerf=NS(validation=NS(chunksize=4096)))
        rgb = parallel_image_render(cfg, g["pose"], [g["z_s"], g["z_t"]], models, (rs, ps), embedders(dev), dev)
        if rank == 0:
            torch.save({"rgb": rgb.cpu()}, out_path)
        else:
            assert rgb is None
    finally:
        dist.destroy_process_group()


def test_parallel_image_render_two_ranks(tmp_path):
    from conftest import GOLDEN, margin
    import numpy as np
    out = str(tmp_path / "chairs.pt")
    _spawn(_chairs_worker, 2, out)
    rgb = torch.load(out, weights_only=True)["rgb"]
    ref = torch.from_numpy(np.load(os.path.join(GOLDEN, "render_chairs.npz"))["n2_rgb"])
    assert rgb.shape == ref.shape == (128 * 128, 3)
    margin("chairs_c4_two_processes[f32]", "rgb_f gathered", (rgb.double() - ref.double()).abs().max().item(), 1e-4)


def _chunk(dev, n, seed):
    g = torch.Generator().manual_seed(seed)
    ro = (torch.randn(n, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 1.3])).to(dev)
    rd = (torch.randn(n, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, -1.0])).to(dev)
    ids = torch.full((n,), 1, dtype=torch.int64, device=dev)
    return ro, rd, ids, torch.rand(n, 4, generator=g).to(dev)


def _setup(dev, distributed):
    from codenerf import train as T
    from codenerf.nerf import PointSampler
    from test_gpu_train import _opt_cfg, _train_models
    torch.manual_seed(0)
    models = _train_models(dev, 3)
    cfg = _opt_cfg()
    cfg.is_distributed = distributed
    opt, sched = T.prepare_optimizer(cfg, models)
    ps = PointSampler(64, 64, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device=dev)
    return models, opt, sched, ps


def _train_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from codenerf import train as T
    from test_gpu_train import embedders
    dev = _init(rank, world, port)
    try:
        models, opt, sched, ps = _setup(dev, True)
        if rank == 1:       # a different start on rank 1: prepare_optimizer's broadcast must undo it
            with torch.no_grad():
                models["nerf_fine"].fc_rgb.weight.add_(1.0)
        opt.broadcast_params(0)
        ro, rd, ids, tgt = _chunk(dev, 4096, 10 + rank)
        for _ in range(2):
            T.train_minibatch(models, opt, sched, ps, embedders(dev), ro, rd, ids, tgt, 1e-5, is_distributed=True)
        torch.cuda.synchronize()
        torch.save({f"{k}.{n}": p.detach().cpu() for k, m in models.items() for n, p in m.named_parameters()},
                   os.path.join(out_dir, f"params{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_train_allreduce_two_ranks(tmp_path):
    """Two data-parallel chunk steps on 2 ranks vs one process averaging both chunks' gradients."""
    from codenerf import train as T
    from test_gpu_train import embedders
    _spawn(_train_worker, 2, str(tmp_path))
    got = [torch.load(str(tmp_path / f"params{r}.pt"), weights_only=True) for r in range(2)]
    dev = torch.device("cuda", 0)
    models, opt, sched, ps = _setup(dev, False)
    chunks = [_chunk(dev, 4096, 10 + r) for r in range(2)]
    keep = NS(step=lambda: None)
    for _ in range(2):
        grads = []
        opt.step = lambda closure=None: None             # capture each chunk's gradients, no update
        for ro, rd, ids, tgt in chunks:
            T.train_minibatch(models, opt, keep, ps, embedders(dev), ro, rd, ids, tgt, 1e-5)
            opt._sync_grads()
            grads.append(opt.flat_buffers()["grad"].clone())
        del opt.step
        flat = opt.flat_buffers()["grad"]
        flat.copy_(grads[0] + grads[1])                   # gloo SUM, then / world (AdamW.allreduce_grads)
        flat.div_(2)
        opt.step()
        sched.step()
    torch.cuda.synchronize()
    want = {f"{k}.{n}": p.detach().cpu() for k, m in models.items() for n, p in m.named_parameters()}
    for k in want:
        assert torch.equal(got[0][k], got[1][k]), ("ranks differ", k)
        assert torch.equal(got[0][k], want[k]), ("vs the averaged single process", k)


def _bench_worker(rank, world, port, out_dir):
    os.environ.update(RANK=str(rank), LOCAL_RANK="0", WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    sys.path.insert(0, ROOT)
    import bench
    res = bench.run(bench.parse_args(["--steps", "2", "--warmup", "1", "--images-per-step", "2", "--no-extras",
                                      "--no-cpu-baseline", "--backend", "gloo", "--quiet"]))
    if rank == 0:
        with open(os.path.join(out_dir, "bench.json"), "w") as f:
            json.dump(res, f)


@pytest.mark.parametrize("world", [2, 3])
def test_bench_gather_views_multi_rank(tmp_path, world):
    """bench.py's N-rank headline: every view split over the ranks (Q5), rendered with per-view
    chunking, gathered (gather_views) -- view 0 equals the same view rendered in one process with
    the same split and chunking, bit for bit."""
    from conftest import margin
    _spawn(_bench_worker, world, str(tmp_path))
    res = json.load(open(tmp_path / "bench.json"))
    assert res["n_gpus"] == world and res["value"] > 0
    margin(f"bench_multi_rank_n{world}[f32]", "multi_rank_maxdiff", res["multi_rank_maxdiff"], 0.0)
