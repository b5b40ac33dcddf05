"""parallel_image_render over gloo with 2 and 3 CPU ranks.

The reference's multi-rank image (render_small.npz, produced by its own
parallel_image_render with 2 / 3 ranks) must come back on rank 0 from the
package's sharding + all-gather, with each rank holding the Q5 share.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(world, nc, nf, tmp_path):
    import dist_worker
    out = str(tmp_path / f"r{world}.npz")
    mp.start_processes(dist_worker.run, args=(world, _free_port(), nc, nf, out), nprocs=world, join=True,
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


def _gather_worker(rank, world, port, out_path):
    import torch.distributed as dist
    from codenerf.nerf import gather_rows
    from codenerf.utils import split_sizes
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        per, _ = split_sizes(1001, world)
        start = sum(per[:rank])
        rows = torch.arange(start, start + per[rank], dtype=torch.float32)[:, None].repeat(1, 3)
        out = gather_rows(rows, per, rank)
        if rank == 0:
            np.save(out_path, out.numpy())
        else:
            assert out is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_gather_rows_uneven_shares(world, tmp_path):
    out = str(tmp_path / "g.npy")
    mp.start_processes(_gather_worker, args=(world, _free_port(), out), nprocs=world, join=True,
                       start_method="spawn")
    got = np.load(out)
    assert got.shape == (1001, 3)
    assert np.array_equal(got[:, 0], np.arange(1001, dtype=np.float32))
