"""The RCCL branch of the pixel gather (nerf/__init__.py:212-224 -> codenerf.nerf.gather_rows) on the one
GPU of the test box: a world-size-1 "nccl" (RCCL) process group, so ``all_gather_into_tensor`` runs
for real; parallel_image_render in distributed mode on top of it.  World sizes 2-4 are covered on
CPU with gloo (tests/test_distributed_cpu.py); 8-GPU runs are the driver's."""
import socket

import pytest
import torch
import torch.distributed as dist

from test_gpu_parity import dev, embedders, load, maxdiff  # noqa: F401

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def rccl_world1(dev):
    store = dist.TCPStore("127.0.0.1", _port(), 1, True)
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
