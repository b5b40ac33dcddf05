"""parallel_image_render over gloo with 2 and 3 CPU ranks.

The reference's multi-rank image (render_small.npz, produced by its own
parallel_image_render with 2 / 3 ranks) must come back on rank 0 from the
package's sharding + all-gather, with each rank holding the Q5 share.
"""
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN, rendezvous


def _launch(world, nc, nf, tmp_path):
    import dist_worker
    out = str(tmp_path / f"r{world}.npz")
    mp.start_processes(dist_worker.run, args=(world, rendezvous(), nc, nf, out), nprocs=world, join=True,
                       start_method="spawn")
    return np.load(out)


@pytest.mark.parametrize("world,nc,nf", [(2, 8, 8), (3, 8, 8), (2, 32, 128)])
def test_parallel_image_render_gloo(world, nc, nf, tmp_path):
    from codenerf.utils import split_sizes
    res = _launch(world, nc, nf, tmp_path)
    g = np.load(os.path.join(GOLDEN, "render_small.npz"))
    per, _ = split_sizes(12 * 16, world)
    assert list(res["rows"]) == list(per) == list(g[f"nc{nc}_n{world}_split"])
    assert np.abs(res["rgb"] - g[f"nc{nc}_n{world}_rgb"]).max() <= 1e-5


def _gather_worker(rank, world, rdv, out_path, single_tensor):
    import torch.distributed as dist
    from codenerf.nerf import gather_rows
    from codenerf.utils import split_sizes
    dist.init_process_group("gloo", init_method=rdv, rank=rank, world_size=world)
    try:
        per, _ = split_sizes(1001, world)
        start = sum(per[:rank])
        rows = torch.arange(start, start + per[rank], dtype=torch.float32)[:, None].repeat(1, 3)
        out = gather_rows(rows, per, rank, single_tensor=single_tensor)
        if rank == 0:
            np.save(out_path, out.numpy())
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("single_tensor", [True, False])
@pytest.mark.parametrize("world", [2, 3, 4])
def test_gather_rows_uneven_shares(world, single_tensor, tmp_path):
    """gather_rows' two branches: all_gather_into_tensor (the default, RCCL's form, run on gloo here) and
    the list all_gather, with uneven Q5 shares."""
    out = str(tmp_path / "g.npy")
    mp.start_processes(_gather_worker, args=(world, rendezvous(), out, single_tensor), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    assert got.shape == (1001, 3)
    assert np.array_equal(got[:, 0], np.arange(1001, dtype=np.float32))


def _views_worker(rank, world, rdv, n_pix, n_views, out_path):
    import torch.distributed as dist
    from codenerf.nerf import gather_views
    from codenerf.utils import split_sizes
    dist.init_process_group("gloo", init_method=rdv, rank=rank, world_size=world)
    try:
        per, _ = split_sizes(n_pix, world)
        start = sum(per[:rank])
        # pixel value = 1000 * view + pixel id, this rank's slice of every view, view-major (bench.py)
        v = torch.arange(n_views, dtype=torch.float32)[:, None] * 1000
        px = torch.arange(start, start + per[rank], dtype=torch.float32)[None, :]
        rows = (v + px).reshape(-1, 1).repeat(1, 3)
        out = gather_views(rows, per, rank, n_views)
        if rank == 0:
            np.save(out_path, out.numpy())
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_pix", [(2, 16384), (3, 1000), (4, 16384), (4, 1001)])
def test_gather_views_layout(world, n_pix, tmp_path):
    """bench.py's multi-view gather (every view split over the ranks as parallel_image_render splits
    one, nerf/__init__.py:179-218, rank 0 re-interleaving the blocks), with uneven Q5 shares."""
    out = str(tmp_path / "v.npy")
    mp.start_processes(_views_worker, args=(world, rendezvous(), n_pix, 5, out), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    want = (np.arange(5, dtype=np.float32)[:, None] * 1000 + np.arange(n_pix, dtype=np.float32)[None, :])
    assert got.shape == (5, n_pix, 3)
    assert np.array_equal(got[..., 0], want) and np.array_equal(got[..., 2], want)


def _shard_sync_worker(rank, world, rdv, out_path):
    import torch.distributed as dist
    from types import SimpleNamespace as NS
    from codenerf.evaluate import shard_of, sync_shard_state
    dist.init_process_group("gloo", init_method=rdv, rank=rank, world_size=world)
    try:
        np.random.seed(100 + rank)              # per-rank streams, as eval.py seeds them ((r + 1) + seed)
        torch.manual_seed(200 + rank)
        rs = NS(seed=7, _draws=3 + rank, height=8, width=8, focal_length=70.0, cx=4.0, cy=5.0,
                intrinsics=torch.eye(4), device=torch.device("cpu"))
        sync_shard_state((rs, None), 0)
        draw = np.random.permutation(64)[:16]   # the ray draw every rank makes next (shard_draws)
        u = torch.rand(5)
        sl = shard_of(16, world, rank)
        rows = torch.zeros(16)
        rows[sl] = 1.0 + rank
        dist.all_reduce(rows)                   # every row owned by exactly one rank
        torch.save({"draw": torch.from_numpy(draw), "u": u, "draws": rs._draws, "rows": rows,
                    "share": sl.stop - sl.start}, f"{out_path}.{rank}")
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ray_sharded_eval_state_sync(world, tmp_path):
    """The ray-sharded eval step's host logic (codenerf.evaluate.sharded_eval_step): after
    sync_shard_state every rank continues with rank 0's numpy / torch streams and ray-sampler counter,
    so all ranks draw the same rays and uniforms; shard_of gives each row to exactly one rank with
    parallel_image_render's Q5 split."""
    from codenerf.utils import split_sizes
    out = str(tmp_path / "s")
    mp.start_processes(_shard_sync_worker, args=(world, rendezvous(), out), nprocs=world, join=True,
                       start_method="spawn")
    got = [torch.load(f"{out}.{r}", weights_only=True) for r in range(world)]
    for g in got[1:]:
        assert torch.equal(g["draw"], got[0]["draw"]) and torch.equal(g["u"], got[0]["u"])
        assert g["draws"] == 3
    np.random.seed(100)
    assert np.array_equal(got[0]["draw"].numpy(), np.random.permutation(64)[:16])
    per, _ = split_sizes(16, world)
    assert [g["share"] for g in got] == per
    want = torch.cat([torch.full((p,), 1.0 + r) for r, p in enumerate(per)])
    assert torch.equal(got[0]["rows"], want)
