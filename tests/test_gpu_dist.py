"""The RCCL branch of the pixel gather (nerf/__init__.py:212-224 -> codenerf.nerf.gather_rows) on the one
GPU of the test box: a world-size-1 "nccl" (RCCL) process group, so ``all_gather_into_tensor`` runs
for real; parallel_image_render in distributed mode on top of it.  World sizes 2-4 are covered on
CPU with gloo (tests/test_distributed_cpu.py); 8-GPU runs are the driver's."""

import pytest
import torch
import torch.distributed as dist

from test_gpu_parity import dev, embedders, load, maxdiff  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture
def rccl_world1(dev):
    store = dist.HashStore()   # one process: an in-memory store, no port to pick
    dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=dev)
    try:
        yield dist.get_world_size()
    finally:
        dist.destroy_process_group()


def test_gather_rows_rccl(dev, rccl_world1):
    from codenerf.nerf import gather_rows
    assert dist.get_backend() == "nccl" and rccl_world1 == 1
    rows = torch.randn(1237, 3, device=dev)
    out = gather_rows(rows, [1237], 0)
    assert torch.equal(out, rows)


def test_parallel_image_render_rccl(dev, rccl_world1):
    """parallel_image_render with is_distributed=True over RCCL equals the reference's 1-rank image."""
    from types import SimpleNamespace as NS
    from codenerf import synthetic
    from codenerf.models import CodeNeRFModel
    from codenerf.nerf import PointSampler, RaySampler, parallel_image_render
    g = load("render_small.npz", dev)
    rs = RaySampler(12, 16, g["intrinsics"].cpu(), sample_size=64, device=dev, datatype=torch.float32)
    ps = PointSampler(8, 8, 0.8, 1.8, "lindepth", False, torch.float32, dev)
    models = {}
    for key, seed in (("nerf_coarse", 0), ("nerf_fine", 1)):
        m = CodeNeRFModel(256, 1, 256, 256, 10, 4)
        m.load_state_dict(synthetic.codenerf_params(seed))
        models[key] = m.to(dev)
    cfg = NS(is_distributed=True, gpus=1, nerf=NS(validation=NS(chunksize=50)))
    rgb = parallel_image_render(cfg, g["pose"], [g["z_s"], g["z_t"]], models, (rs, ps), embedders(dev), dev)
    assert maxdiff(rgb, g["nc8_n1_rgb"]) <= 1e-4


def _train_setup(dev, seed=0):
    from test_gpu_train import _opt_cfg, _train_models
    torch.manual_seed(seed)
    return _train_models(dev, 3)


def _chunk(dev, n=256, obj=1, seed=4):
    g = torch.Generator().manual_seed(seed)
    ro = (torch.randn(n, 3, generator=g) * 0.1 + torch.tensor([0.0, 0.0, 1.3])).to(dev)
    rd = (torch.randn(n, 3, generator=g) * 0.2 + torch.tensor([0.0, 0.0, -1.0])).to(dev)
    ids = torch.full((n,), obj, dtype=torch.int64, device=dev)
    return ro, rd, ids, torch.rand(n, 4, generator=g).to(dev)


def test_adamw_allreduce_broadcast_rccl(dev, rccl_world1):
    """codenerf.optim.AdamW's data-parallel pieces over RCCL (world 1: the collectives run): the
    flat all-reduce leaves the averaged gradients (here: themselves) and the flags' None-ness, the
    broadcast leaves the parameters; a step after them equals a step without them."""
    from codenerf.optim import AdamW
    g = torch.Generator().manual_seed(0)
    base = [torch.randn(64, 32, generator=g), torch.randn(7, generator=g), torch.randn(3, 5, generator=g)]
    runs = []
    for collective in (False, True):
        ps = [torch.nn.Parameter(t.clone().to(dev)) for t in base]
        opt = AdamW([{"params": ps[:2]}, {"params": ps[2:], "lr": 1e-3}], lr=1e-4)
        if collective:
            opt.broadcast_params(0)
        gg = torch.Generator().manual_seed(1)
        for it in range(3):
            opt.zero_grad()
            for i, p in enumerate(ps):
                gr = torch.randn(p.shape, generator=gg).to(dev)
                if not (it == 1 and i == 1):      # parameter 1 has no gradient in step 1
                    p.grad = gr
            if collective:
                opt.allreduce_grads()
                assert (ps[1].grad is None) == (it == 1)
            opt.step()
        torch.cuda.synchronize()
        runs.append([p.detach().clone() for p in ps])
    for a, b in zip(*runs):
        assert torch.equal(a, b)


def test_ddp_drop_in_rccl(dev, rccl_world1):
    """INTEGRATION.md's drop-in under the reference's DDP (util.py:139-142): the three modules wrapped in
    torch.nn.parallel.DistributedDataParallel on an RCCL group, stepped by torch.optim.AdamW (the
    reference's optimiser, util.py:147-172) through train_minibatch (train.py:96-114): every
    gradient reaches DDP's hooks (its reducer all-reduces them) and the gradients and the updated
    parameters equal the unwrapped path's bit for bit (world 1: the average is the gradient)."""
    from torch.distributed.algorithms.ddp_comm_hooks import default_hooks
    from torch.nn.parallel import DistributedDataParallel as DDP
    from codenerf import train as T
    from codenerf.nerf import PointSampler
    from test_gpu_train import embedders as embs
    ps = PointSampler(16, 16, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device=dev)
    out = []
    for wrap in (False, True):
        models = _train_setup(dev)
        if wrap:
            models = {k: DDP(m, device_ids=[dev.index]) for k, m in models.items()}
        groups = [{"params": list(models["nerf_coarse"].parameters())},
                  {"params": list(models["nerf_fine"].parameters())},
                  {"params": list(models["embedding"].parameters()), "lr": 1e-3}]
        opt = torch.optim.AdamW(groups, lr=1e-4)
        sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda e: 0.1 ** (e / 5000000))
        hooked = []
        if wrap:   # DDP's reducer all-reduces the buckets; count the communication hook's calls
            def hook(state, bucket):
                hooked.append(bucket.buffer().numel())
                return default_hooks.allreduce_hook(None, bucket)
            for m in models.values():
                m.register_comm_hook(None, hook)
        grads = []
        for step in range(2):
            ro, rd, ids, tgt = _chunk(dev, obj=step + 1, seed=4 + step)
            T.train_minibatch(models, opt, sched, ps, embs(dev), ro, rd, ids, tgt, 1e-5, is_distributed=wrap)
            grads.append({f"{k}.{n}": p.grad.detach().clone() for k, m in models.items()
                          for n, p in (m.module if wrap else m).named_parameters() if p.grad is not None})
        torch.cuda.synchronize()
        params = {f"{k}.{n}": p.detach().clone() for k, m in models.items()
                  for n, p in (m.module if wrap else m).named_parameters()}
        out.append((grads, params, hooked))
    (g0, p0, _), (g1, p1, hooked) = out
    n_params = sum(v.numel() for v in p1.values())
    assert sum(hooked) == 2 * n_params, (sum(hooked), n_params)   # every gradient went through the reducer
    for a, b in zip(g0, g1):
        assert a.keys() == b.keys()
        for k in a:
            assert torch.equal(a[k], b[k]), k
    for k in p0:
        assert torch.equal(p0[k], p1[k]), k


def test_train_minibatch_no_host_sync_rccl(dev, rccl_world1):
    """The data-parallel chunk step (train.py:96-114 + util.py:139-142's gradient average) over RCCL
    runs with no host synchronisation: AdamW.allreduce_grads issues ONE all-reduce of the flat
    gradient with its has-grad flags appended (a cached device tensor) and reads nothing back when
    every parameter holds a gradient; torch's sync debug mode "error" raises on any sync."""
    import numpy as np
    from codenerf import train as T
    from codenerf.nerf import PointSampler
    from test_gpu_train import _opt_cfg, embedders as embs
    models = _train_setup(dev)
    cfg = _opt_cfg()
    cfg.is_distributed = True
    opt, sched = T.prepare_optimizer(cfg, models)
    ps = PointSampler(16, 16, 0.8, 1.8, spacing_mode="lindepth", perturb=False, dtype=torch.float32, device=dev)
    e = embs(dev)
    chunks = []
    for step in range(3):
        ro, rd, ids, tgt = _chunk(dev, obj=1, seed=4 + step)
        ids._cn_host_ids = np.full(ids.shape[0], 1, dtype=np.int64)
        chunks.append((ro, rd, ids, tgt))
    T.train_minibatch(models, opt, sched, ps, e, *chunks[0], 1e-5, is_distributed=True)   # first call: caches
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        for c in chunks[1:]:
            out = T.train_minibatch(models, opt, sched, ps, e, *c, 1e-5, is_distributed=True)
    finally:
        torch.cuda.set_sync_debug_mode(0)
    torch.cuda.synchronize()
    assert np.isfinite(float(out["psnr"])) and np.isfinite(float(out["total_loss"]))
