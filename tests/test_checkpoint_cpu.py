"""Checkpoint interop on the CPU: the reference's checkpoint format
(train.py:129-138) and its loader's rules (utils/util.py:175-213).

A checkpoint as the reference's DDP training writes it -- ``module.``-prefixed state_dicts of
CodeNeRFModel x2 + ShapeTextureEmbedding and a torch.optim.AdamW state after real steps -- loads
into this build's modules and flat AdamW; what this build saves has the reference's keys and
loads back with torch.load(weights_only=True).
"""
from collections import OrderedDict
from types import SimpleNamespace as NS

import pytest
import torch


def _models(seed):
    from codenerf.models import CodeNeRFModel, ShapeTextureEmbedding
    torch.manual_seed(seed)
    return OrderedDict([("embedding", ShapeTextureEmbedding(5, 256, 256)),
                        ("nerf_coarse", CodeNeRFModel(256, 5, 256, 256, 10, 4)),
                        ("nerf_fine", CodeNeRFModel(256, 5, 256, 256, 10, 4))])


def _groups(models):
    return [{"params": list(models["nerf_coarse"].parameters())},
            {"params": list(models["nerf_fine"].parameters())},
            {"params": list(models["embedding"].parameters()), "lr": 1e-3}]


def _reference_checkpoint(path, ddp_prefix=True, iteration=7):
    """What train.py:129-137 writes (DDP-wrapped modules carry 'module.'), after 2 AdamW steps."""
    models = _models(1)
    opt = torch.optim.AdamW(_groups(models), lr=1e-4)
    g = torch.Generator().manual_seed(3)
    for _ in range(2):
        opt.zero_grad()
        for m in models.values():
            for p in m.parameters():
                p.grad = torch.randn(p.shape, generator=g)
        opt.step()
    pre = "module." if ddp_prefix else ""
    ckpt = {"iter": iteration}
    for name in ("nerf_coarse", "nerf_fine", "embedding"):
        ckpt[f"model_{name}_state_dict"] = OrderedDict((pre + k, v) for k, v in models[name].state_dict().items())
    ckpt["optimizer_state_dict"] = opt.state_dict()
    torch.save(ckpt, str(path))
    return models, opt


@pytest.mark.parametrize("ddp_prefix", [True, False])
def test_load_reference_checkpoint(tmp_path, ddp_prefix):
    from codenerf.checkpoint import load_checkpoint
    from codenerf.optim import AdamW
    path = tmp_path / "checkpoint    5.ckpt"
    ref_models, ref_opt = _reference_checkpoint(path, ddp_prefix)
    models = _models(2)
    opt = AdamW(_groups(models), lr=1e-4)
    it = load_checkpoint(NS(load_checkpoint=str(path), is_distributed=False), models, opt)
    assert it == 7
    for name in models:
        for (k, a), (k2, b) in zip(models[name].state_dict().items(), ref_models[name].state_dict().items()):
            assert k == k2 and torch.equal(a, b), (name, k)
    ref_sd, sd = ref_opt.state_dict(), opt.state_dict()
    assert [g["lr"] for g in sd["param_groups"]] == [g["lr"] for g in ref_sd["param_groups"]]
    assert set(sd["state"]) == set(ref_sd["state"])
    for i, st in ref_sd["state"].items():
        assert float(sd["state"][i]["step"]) == float(st["step"])
        assert torch.equal(sd["state"][i]["exp_avg"], st["exp_avg"])
        assert torch.equal(sd["state"][i]["exp_avg_sq"], st["exp_avg_sq"])
    # the moments live in the flat buffers the one-launch update reads
    p0 = next(models["nerf_coarse"].parameters())
    assert opt.state[p0]["exp_avg"].data_ptr() != ref_sd["state"][0]["exp_avg"].data_ptr()
    f = opt.flat_buffers()["exp_avg"]
    assert f.data_ptr() <= opt.state[p0]["exp_avg"].data_ptr() < f.data_ptr() + 4 * f.numel()


def test_load_rules(tmp_path):
    """Only an existing regular .ckpt file is read; anything else leaves the models alone, start 0."""
    from codenerf.checkpoint import load_checkpoint
    models = _models(2)
    before = {k: v.clone() for k, v in models["nerf_fine"].state_dict().items()}
    opt = torch.optim.AdamW(_groups(models), lr=1e-4)
    wrong = tmp_path / "model.pt"
    _reference_checkpoint(wrong)
    for p in (str(wrong), str(tmp_path / "missing.ckpt"), str(tmp_path), ""):
        assert load_checkpoint(NS(load_checkpoint=p, is_distributed=False), models, opt) == 0
    for k, v in models["nerf_fine"].state_dict().items():
        assert torch.equal(v, before[k])


def test_save_has_reference_keys(tmp_path):
    from codenerf.checkpoint import load_checkpoint, save_checkpoint
    from codenerf.optim import AdamW
    models = _models(4)
    opt = AdamW(_groups(models), lr=1e-4)
    path = tmp_path / "checkpoint   12.ckpt"
    save_checkpoint(path, 12, models, opt)
    ck = torch.load(str(path), weights_only=True)
    # the reference's keys, plus this build's resume keys (cn_*), which the reference's loader ignores
    assert {k for k in ck if not k.startswith("cn_")} == {"iter", "model_nerf_coarse_state_dict",
                                                         "model_nerf_fine_state_dict", "model_embedding_state_dict",
                                                         "optimizer_state_dict"}
    assert set(ck) - {"iter", "model_nerf_coarse_state_dict", "model_nerf_fine_state_dict",
                      "model_embedding_state_dict", "optimizer_state_dict"} == {"cn_rng"}
    assert list(ck["model_nerf_coarse_state_dict"]) == list(models["nerf_coarse"].state_dict())
    assert list(ck["model_embedding_state_dict"]) == ["shape_embedding.weight", "texture_embedding.weight"]
    fresh = _models(5)
    assert load_checkpoint(NS(load_checkpoint=str(path)), fresh, torch.optim.AdamW(_groups(fresh), lr=1e-4)) == 12
    for name in models:
        for (k, a), b in zip(models[name].state_dict().items(), fresh[name].state_dict().values()):
            assert torch.equal(a, b), (name, k)


def test_save_ddp_prefix_and_rng_roundtrip(tmp_path):
    """save_checkpoint(ddp_prefix=True) writes the keys the reference's distributed training writes
    (DDP's ``module.``; its distributed load expects them); load_checkpoint strips them again.  The
    RNG streams saved with ``rng`` come back through resume_state."""
    import numpy as np
    from codenerf.checkpoint import load_checkpoint, resume_state, save_checkpoint
    models = _models(4)
    opt = torch.optim.AdamW(_groups(models), lr=1e-4)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lambda e: 0.5 ** e)
    for _ in range(3):
        sched.step()
    path = tmp_path / "checkpoint    3.ckpt"
    np.random.seed(7)
    torch.manual_seed(7)
    save_checkpoint(path, 3, models, opt, scheduler=sched, next_iter=4, ddp_prefix=True)
    want_np, want_t = np.random.rand(3), torch.rand(3)
    ck = torch.load(str(path), weights_only=True)
    assert all(k.startswith("module.") for k in ck["model_nerf_fine_state_dict"])
    fresh = _models(5)
    opt2 = torch.optim.AdamW(_groups(fresh), lr=1e-4)
    sched2 = torch.optim.lr_scheduler.LambdaLR(opt2, lambda e: 0.5 ** e)
    extras = {}
    assert load_checkpoint(NS(load_checkpoint=str(path)), fresh, opt2, extras=extras) == 3
    np.random.seed(0)
    torch.manual_seed(0)
    assert resume_state(extras, sched2, 3) == 4
    assert sched2.last_epoch == 3
    assert np.array_equal(np.random.rand(3), want_np) and torch.equal(torch.rand(3), want_t)
    for name in models:
        for a, b in zip(models[name].state_dict().values(), fresh[name].state_dict().values()):
            assert torch.equal(a, b)
