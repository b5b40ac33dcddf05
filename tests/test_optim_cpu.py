"""Flat-buffer AdamW host logic on the CPU.

The update itself is one HIP kernel (cn_adamw_step; tests/test_gpu_train.py holds it
against torch.optim.AdamW).  Here: the flat layout (values kept, 256-B aligned views,
gradients landing in the flat buffer), zero_grad semantics, the refusal to update
without a GPU, and the data-parallel pieces -- the gradient average and the
start-of-training parameter broadcast -- over gloo with 2 ranks.
"""

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import rendezvous


SHAPES = [(256, 63), (256,), (3, 512), (3,), (40, 256)]


def _params(seed=0):
    g = torch.Generator().manual_seed(seed)
    return [torch.nn.Parameter(torch.randn(*s, generator=g)) for s in SHAPES]


def _opt(ps):
    from codenerf.optim import AdamW
    return AdamW([{"params": ps[:4]}, {"params": ps[4:], "lr": 1e-3}], lr=1e-4)


def test_flat_layout_keeps_values_and_aliases():
    from codenerf.optim import ALIGN
    ps = _params()
    before = [p.detach().clone() for p in ps]
    opt = _opt(ps)
    f = opt.flat_buffers()
    assert set(f) == {"param", "grad", "exp_avg", "exp_avg_sq"}
    starts = opt.group_starts
    assert len(starts) == 3 and starts[0] == 0 and starts[-1] <= f["param"].numel()
    for p, b in zip(ps, before):
        assert torch.equal(p.detach(), b)
        assert (p.data_ptr() - f["param"].data_ptr()) // 4 % ALIGN == 0
    with torch.no_grad():
        f["param"].add_(1.0)                      # the parameters are views of the buffer
    assert torch.equal(ps[2].detach(), before[2] + 1.0)


def test_gradients_land_in_the_flat_buffer():
    ps = _params()
    opt = _opt(ps)
    opt.zero_grad()
    assert all(p.grad is None for p in ps)
    sum((p * p).sum() for p in ps[:3]).backward()     # ps[3], ps[4] get no gradient
    missing = opt._sync_grads()
    assert [id(p) for p in missing] == [id(p) for p in ps[3:]]
    f = opt.flat_buffers()
    for p in ps[:3]:
        assert p.grad.data_ptr() - f["grad"].data_ptr() == p.data_ptr() - f["param"].data_ptr()
        assert torch.equal(p.grad, 2 * p.detach())
    opt.zero_grad(set_to_none=False)
    assert all(p.grad is not None and not p.grad.any() for p in ps)


def test_step_needs_the_gpu():
    ps = _params()
    opt = _opt(ps)
    for p in ps:
        p.grad = torch.ones_like(p)
    with pytest.raises(ValueError, match="no CPU fallback"):
        opt.step()


def test_graph_scalars_refuses_changed_segments():
    """A captured graph_step bakes its segment bounds into the launch: a later lr change that merges
    two groups' segments must stop graph_scalars instead of shifting scalars onto the wrong slices."""
    ps = _params()
    opt = _opt(ps)
    for p in ps:
        p.grad = torch.ones_like(p)
    opt._sync_grads()
    opt._graph_bounds = [(b, e) for b, e, *_ in opt._plan(advance=False)]   # as graph_step records them
    assert len(opt._graph_bounds) == 2
    opt.param_groups[1]["lr"] = opt.param_groups[0]["lr"]                  # the two groups now merge
    with pytest.raises(RuntimeError, match="need a new capture"):
        opt.graph_scalars(np.zeros(6, dtype=np.float32))


def test_refuses_unsupported_options():
    from codenerf.optim import AdamW
    with pytest.raises(NotImplementedError):
        AdamW(_params(), amsgrad=True)
    with pytest.raises(TypeError):
        AdamW([torch.nn.Parameter(torch.zeros(3, dtype=torch.float64))])


def test_state_dict_matches_torch_layout():
    ps = _params()
    opt = _opt(ps)
    ref = torch.optim.AdamW([{"params": _params()[:4]}, {"params": _params()[4:], "lr": 1e-3}], lr=1e-4)
    a, b = opt.state_dict(), ref.state_dict()
    assert a["state"] == {} and [g["params"] for g in a["param_groups"]] == [g["params"] for g in b["param_groups"]]
    assert set(a["param_groups"][0]) == set(b["param_groups"][0])


def _dp_worker(rank, world, rdv, out):
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=rdv, rank=rank, world_size=world)
    try:
        ps = _params(seed=rank)                  # replicas start apart (train.py:29-31 seeds by rank)
        opt = _opt(ps)
        opt.broadcast_params(0)
        steps = []
        # three rounds of has-grad patterns: (missing on rank 1 only, missing everywhere), the same
        # again (the cached flags), then a new one (missing on rank 0 only)
        for missing_here, missing_all in (({3} if rank == 1 else set(), {1}), ({3} if rank == 1 else set(), {1}),
                                          ({2} if rank == 0 else set(), set())):
            for i, p in enumerate(ps):
                p.grad = None if (i in missing_here or i in missing_all) else torch.full_like(p, float(rank + 1))
            opt.allreduce_grads()
            for i in missing_all:
                assert ps[i].grad is None
            steps.append(torch.cat([(p.grad if p.grad is not None else torch.full_like(p, -7.0)).reshape(-1)
                                    for p in ps]).numpy())
        np.savez(out.format(rank), params=torch.cat([p.detach().reshape(-1) for p in ps]).numpy(),
                 grads=np.stack(steps))
        # the torch-optimiser fallback: ranks with DIFFERENT missing gradients issue the same
        # all-reduce sizes (no hang) and the same flags
        from types import SimpleNamespace
        from codenerf import train as T
        qs = _params(seed=10 + rank)
        mods = {"m": SimpleNamespace(parameters=lambda: iter(qs))}
        T.broadcast_parameters(mods)
        for q in qs:
            q.grad = torch.full_like(q, float(rank + 1))
        qs[rank].grad = None                     # rank 0 lacks q0, rank 1 lacks q1
        qs[4].grad = None                        # nobody has q4
        T._average_gradients(torch.optim.SGD(qs, lr=0.1), mods)
        np.savez(out.format(rank) + ".fallback.npz",
                 params=torch.cat([q.detach().reshape(-1) for q in qs]).numpy(),
                 g0=qs[0].grad.numpy(), g1=qs[1].grad.numpy(), g2=qs[2].grad.numpy(), none4=qs[4].grad is None)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_allreduce_and_broadcast_gloo(world, tmp_path):
    """AdamW.allreduce_grads (util.py:139-142's DDP average): one SUM all-reduce of the flat gradient
    with the has-grad flags in its tail, divided by the world size -- the arithmetic on every backend;
    a gradient missing on a rank counts as zero, one missing everywhere stays None; changing patterns
    between steps (the per-pattern flag cache) reduce correctly."""
    out = str(tmp_path / "r{}.npz")
    mp.start_processes(_dp_worker, args=(world, rendezvous(), out), nprocs=world, join=True, start_method="spawn")
    res = [np.load(out.format(r)) for r in range(world)]
    ref = torch.cat([p.detach().reshape(-1) for p in _params(seed=0)]).numpy()
    sizes = [int(np.prod(s)) for s in SHAPES]
    offs = np.concatenate([[0], np.cumsum(sizes)])
    full = np.float32(sum(range(1, world + 1))) / np.float32(world)
    exp = np.stack([np.full(offs[-1], full, np.float32) for _ in range(3)])
    for st in (0, 1):
        exp[st, offs[3]:offs[4]] = np.float32(sum(r + 1 for r in range(world) if r != 1)) / np.float32(world)
        exp[st, offs[1]:offs[2]] = -7.0       # no rank had it: grad None
    exp[2, offs[2]:offs[3]] = np.float32(sum(r + 1 for r in range(world) if r != 0)) / np.float32(world)
    for r in res:
        assert np.array_equal(r["params"], ref)
        assert np.array_equal(r["grads"], exp)
    if world != 2:
        return
    f0, f1 = np.load(out.format(0) + ".fallback.npz"), np.load(out.format(1) + ".fallback.npz")
    ref10 = torch.cat([q.detach().reshape(-1) for q in _params(seed=10)]).numpy()
    assert np.array_equal(f0["params"], ref10) and np.array_equal(f1["params"], ref10)   # broadcast from rank 0
    for f in (f0, f1):
        assert np.all(f["g0"] == 1.0) and np.all(f["g1"] == 0.5) and np.all(f["g2"] == 1.5) and bool(f["none4"])
