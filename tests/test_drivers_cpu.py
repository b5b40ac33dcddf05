"""The drivers' process launch and per-rank state on the CPU (gloo, world size 2):

* ``codenerf.train.launch`` / ``main`` (train.py:145-179, eval.py:208-242): one spawned process per
  rank, a gloo group of ``cfg.gpus`` ranks, ``fn(rank, cfg)`` in each -- here a stub body that runs
  the drivers' own seeding (``seed_rank``: ``(rank + 1) + randomseed``) and batch draw
  (``next_train_batch``: ``set_epoch(iteration)`` then a fresh iterator, train.py:67-70) over the
  reference's loader on a synthetic SRN tree;
* checkpoints keep EVERY rank's generator states: after a resume the ranks draw what
  they would have drawn without the interruption -- different rays per rank, as the reference's
  per-rank seeds intend -- and a checkpoint holding one rank's state restores none at world size 2;
* the LogBook's batched read-back and bounded history.
"""
import json
import os
import sys
from types import SimpleNamespace as NS

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import GOLDEN, rendezvous

sys.path.insert(0, GOLDEN)
import srn_tree  # noqa: E402


def _cfg(base, out_dir, gpus=2):
    from codenerf.config import Cfg
    return Cfg(gpus=gpus, is_distributed=True, load_checkpoint="", out_dir=out_dir,
               experiment=dict(randomseed=55, iterations=4),
               dataset=dict(type="SRNDataset", basedir=base, train_batch_size=1, val_batch_size=1))


def _stub_body(rank, cfg):
    """What train()'s body does before any GPU work, recorded per rank."""
    import torch.distributed as dist
    from codenerf.datasets import prepare_dataloader
    from codenerf.train import next_train_batch, seed_rank
    seed = seed_rank(rank, cfg)
    draws = {"np": np.random.rand(3).tolist(), "torch": torch.rand(3).tolist()}
    loader, ds = prepare_dataloader("train", cfg, None)
    batches = []
    for it in range(3):
        b = next_train_batch(cfg, loader, it)
        batches.append({"object_id": b["object_id"].tolist(), "pose0": float(b["pose"][0, 0, 3])})
    rec = {"rank": rank, "world": dist.get_world_size(), "backend": dist.get_backend(), "seed": seed,
           "draws": draws, "batches": batches, "n": len(ds)}
    with open(os.path.join(cfg.out_dir, f"rank{rank}.json"), "w") as f:
        json.dump(rec, f)


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    return srn_tree.write_tree(str(tmp_path_factory.mktemp("srn")))


def test_launch_spawns_ranks_with_reference_seeds_and_epochs(tree, tmp_path):
    from codenerf.datasets import SRNDataset
    from codenerf.train import launch
    cfg = _cfg(tree, str(tmp_path))
    launch(_stub_body, cfg, backend="gloo", init_method=rendezvous())
    recs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(2)]
    ds = SRNDataset(tree, "train")
    for r, rec in enumerate(recs):
        assert rec["rank"] == r and rec["world"] == 2 and rec["backend"] == "gloo"
        assert rec["seed"] == (r + 1) + 55                           # train.py:28-31
        np.random.seed(rec["seed"])
        torch.manual_seed(rec["seed"])
        assert rec["draws"]["np"] == np.random.rand(3).tolist()
        assert rec["draws"]["torch"] == torch.rand(3).tolist()
        # train.py:67-70: set_epoch(iteration) then the first index of the rank's share
        for it, b in enumerate(rec["batches"]):
            s = torch.utils.data.DistributedSampler(ds, num_replicas=2, rank=r, drop_last=False)
            s.set_epoch(it)
            idx = next(iter(s))
            assert b["object_id"] == [ds[idx]["object_id"]], (r, it)
            assert b["pose0"] == pytest.approx(float(ds[idx]["pose"][0, 3]), abs=0)
    assert recs[0]["draws"] != recs[1]["draws"]


def test_launch_single_process_when_not_distributed(tree, tmp_path):
    from codenerf.train import launch
    seen = []
    cfg = _cfg(tree, str(tmp_path), gpus=2) | {"is_distributed": False}
    launch(lambda rank, c: seen.append((rank, c.gpus)), cfg)
    assert seen == [(0, 2)]                                          # train.py:178-179


def _ckpt_worker(rank, world, rdv, path, out_dir, per_rank):
    import torch.distributed as dist
    from codenerf import checkpoint as C
    from codenerf.models import CodeNeRFModel, ShapeTextureEmbedding
    from collections import OrderedDict
    dist.init_process_group("gloo", init_method=rdv, rank=rank, world_size=world)
    try:
        np.random.seed(rank + 1 + 55)
        torch.manual_seed(rank + 1 + 55)
        g = torch.Generator().manual_seed(9)                          # the same models on every rank
        models = OrderedDict([("embedding", ShapeTextureEmbedding(3, 256, 256)),
                              ("nerf_coarse", CodeNeRFModel(256, 3, 256, 256, 10, 4))])
        with torch.no_grad():
            for m in models.values():
                for p in m.parameters():
                    p.copy_(torch.randn(p.shape, generator=g))
        opt = torch.optim.AdamW([p for m in models.values() for p in m.parameters()], lr=1e-4)
        np.random.rand(5)                                             # some draws before the save
        torch.rand(5)
        start = C.rng_state(None)
        np.random.rand(2)
        now = C.rng_state(None)
        states = C.gather_rng_states({"now": now, "iter_start": start})
        if rank == 0:
            if per_rank:
                C.save_checkpoint(path, 3, models, opt, cursor=(3, 1), rng_ranks=states)
            else:
                C.save_checkpoint(path, 3, models, opt, next_iter=4)  # one process's state only
        dist.barrier()
        want_now = (np.random.rand(4).tolist(), torch.rand(4).tolist())
        C.set_rng_state(start)
        want_start = np.random.rand(4).tolist()
        np.random.seed(1234)                                           # a fresh process's seeding
        torch.manual_seed(1234)
        fresh = (np.random.rand(4).tolist(), torch.rand(4).tolist())
        np.random.seed(1234)
        torch.manual_seed(1234)
        extras = {}
        it = C.load_checkpoint(NS(load_checkpoint=path, is_distributed=True), models, opt, extras=extras)
        p = C.resume_point(extras, None, it, rank=rank, world_size=world)
        rec = {"iteration": p.iteration, "chunk": p.chunk, "has_rng": p.rng is not None}
        if p.rng is not None:
            C.set_rng_state(p.iter_rng)
            rec["start"] = np.random.rand(4).tolist()
            C.set_rng_state(p.rng)
        rec["draws"] = (np.random.rand(4).tolist(), torch.rand(4).tolist())
        rec["want_now"], rec["want_start"], rec["fresh"] = want_now, want_start, fresh
        with open(os.path.join(out_dir, f"ck{rank}.json"), "w") as f:
            json.dump(rec, f)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("per_rank", [True, False])
def test_checkpoint_rng_is_per_rank(tmp_path, per_rank):
    path = str(tmp_path / "checkpoint    3.ckpt")
    mp.start_processes(_ckpt_worker, args=(2, rendezvous(), path, str(tmp_path), per_rank), nprocs=2, join=True,
                       start_method="spawn")
    recs = [json.load(open(tmp_path / f"ck{r}.json")) for r in range(2)]
    for r in recs:
        if per_rank:
            # the cursor and each rank's own streams: the continuation of the uninterrupted draws
            assert (r["iteration"], r["chunk"], r["has_rng"]) == (3, 1, True)
            assert r["draws"] == r["want_now"] and r["start"] == r["want_start"]
        else:
            # one rank's state is never handed to every rank: each keeps its own seeding
            assert (r["iteration"], r["chunk"], r["has_rng"]) == (4, 0, False)
            assert r["draws"] == r["fresh"]
    if per_rank:
        assert recs[0]["draws"] != recs[1]["draws"]                   # the ranks still sample different rays
    ck = torch.load(path, weights_only=True)
    if per_rank:
        assert ck["cn_cursor"].tolist() == [3, 1] and len(ck["cn_rng_ranks"]) == 2 and "cn_next_iter" not in ck
        assert torch.equal(ck["cn_rng"]["numpy_keys"], ck["cn_rng_ranks"][0]["now"]["numpy_keys"])


def test_cursor_at_iteration_end_keeps_next_iter(tmp_path):
    """A save after an iteration's last chunk is also readable the pre-cursor way (cn_next_iter)."""
    from codenerf import checkpoint as C
    from codenerf.models import ShapeTextureEmbedding
    models = {"embedding": ShapeTextureEmbedding(2, 256, 256)}
    opt = torch.optim.AdamW(models["embedding"].parameters(), lr=1e-3)
    path = tmp_path / "c.ckpt"
    C.save_checkpoint(path, 6, models, opt, cursor=(7, 0), rng_ranks=[{"now": C.rng_state(None),
                                                                      "iter_start": C.rng_state(None)}])
    ck = torch.load(str(path), weights_only=True)
    assert ck["cn_next_iter"] == 7 and ck["cn_cursor"].tolist() == [7, 0]
    extras = {}
    it = C.load_checkpoint(NS(load_checkpoint=str(path)), models, opt, extras=extras)
    assert C.resume_state(extras, None, it) == 7
    p = C.resume_point(extras, None, it)
    assert (p.iteration, p.chunk, p.iter_rng) == (7, 0, None) and p.rng is not None


def test_logbook_batches_and_bounds():
    from codenerf.train import LogBook
    book = LogBook(keep=5, flush_every=4)
    for i in range(11):
        book.add({"loss": torch.tensor(float(i)), "psnr": torch.tensor(i / 3, dtype=torch.float64), "n": i})
        assert len(book.pending) == (i + 1) % 4
    assert book.count == 11
    got = book.as_list()
    assert [g["loss"] for g in got] == [6.0, 7.0, 8.0, 9.0, 10.0]
    assert got[-1]["psnr"] == 10 / 3 and got[-1]["n"] == 10.0
    assert book.last() == got[-1]
