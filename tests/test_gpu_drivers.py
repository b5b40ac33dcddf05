"""The build's driver loops (train.py:19-142, eval.py:41-79 + 82-205) composed from the package's pieces,
on a synthetic SRN tree (tests/golden/srn_tree.py):

* ``codenerf.train.train``: seeds, loaders, models, optimiser, checkpoint cadence -- and an exact resume:
  4 iterations, a checkpoint, a resume and 1 more iteration end bit-identical to 5 uninterrupted ones
  (the fp32 step is deterministic, the checkpoint carries the RNG streams and the scheduler);
* a reference-format checkpoint (the reference's keys only) still loads and resumes;
* ``codenerf.evaluate.eval_loop``: the validation loop (sixth-batch selection, test-time optimisation,
  full-view render) returns a finite PSNR per validation.
"""
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import srn_tree  # noqa: E402

pytestmark = pytest.mark.gpu


def _cfg(base, logdir, **exp):
    from codenerf.config import Cfg
    e = dict(id="drv", logdir=logdir, randomseed=55, iterations=5, val_iterations=3, validate_every=1000,
             save_every=4, print_every=1, val_print_every=100, regularizer_lambda=1e-5)
    e.update(exp)
    return Cfg(gpus=1, is_distributed=False, load_checkpoint="",
               experiment=e,
               dataset=dict(type="SRNDataset", basedir=base, train_batch_size=1, val_batch_size=1),
               models=dict(nerf_coarse=dict(type="CodeNeRFModel", hidden_size=256),
                           nerf_fine=dict(type="CodeNeRFModel", hidden_size=256),
                           embedding=dict(shape_code_size=256, texture_code_size=256)),
               optimizer=dict(type="AdamW", lr=1e-4, embedding_lr=1e-3, val_type="AdamW", val_lr=5e-3,
                              angle_lr=1e-2, radius_lr=1e-2, scheduler_gamma=0.1, scheduler_step_size=7),
               nerf=dict(ray_sampler=dict(num_random_rays=128),
                         point_sampler=dict(num_coarse=16, num_fine=16, near_limit=0.8, far_limit=1.8,
                                            spacing_mode="lindepth", perturb=True),
                         embedder=dict(num_encoding_fn_xyz=10, include_input_xyz=True, log_sampling_xyz=True,
                                       use_viewdirs=True, num_encoding_fn_dir=4, include_input_dir=True,
                                       log_sampling_dir=True),
                         train=dict(chunksize=128), validation=dict(chunksize=512)))


def _params(out):
    return {f"{k}.{n}": p.detach().clone() for k, m in out["models"].items() for n, p in m.named_parameters()}


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    return srn_tree.write_tree(str(tmp_path_factory.mktemp("srn")), channels=4)


def test_train_resume_is_exact(tree, tmp_path):
    from codenerf.train import train
    dev = torch.device("cuda", 0)
    full = train(0, _cfg(tree, str(tmp_path / "full")), device=dev, verbose=False)
    assert len(full["logs"]) == 5 and all(torch.isfinite(torch.tensor(lg["total_loss"])) for lg in full["logs"])
    part = train(0, _cfg(tree, str(tmp_path / "part")), device=dev, stop_after=4, verbose=False)
    assert part["checkpoints"] == []                      # i = 4 (save_every 4) is past the stop
    # so save at the stop with the driver's own save_checkpoint (train.py:129-138's dict + resume keys)
    from codenerf.checkpoint import save_checkpoint
    ck = tmp_path / "part" / "stop.ckpt"
    save_checkpoint(ck, 3, part["models"], part["optimizer"], scheduler=part["scheduler"], next_iter=4)
    resumed = train(0, _cfg(tree, str(tmp_path / "res")) | {"load_checkpoint": str(ck)}, device=dev,
                    verbose=False)
    assert len(resumed["logs"]) == 1                      # iteration 4 only
    assert resumed["logs"][0] == full["logs"][4]          # the same loss, bit for bit
    a, b = _params(full), _params(resumed)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    assert full["scheduler"].last_epoch == resumed["scheduler"].last_epoch == 5


def test_train_resume_mid_iteration_with_validation(tree, tmp_path):
    """A periodic save inside an iteration (2 chunks per iteration, the save after chunk 0) that
    coincides with a validation step, and one at an iteration's end: resuming from
    either continues the uninterrupted run bit for bit -- the cursor replays the iteration's ray
    draw, the generators are those after the save step's validation."""
    from codenerf.train import train
    dev = torch.device("cuda", 0)
    # iterations >= 6: validate picks the val loader's SIXTH batch (eval.py:103-109), and the loader
    # yields ``iterations`` of them (util.py:59-90)
    kw = dict(iterations=6, save_every=4, validate_every=4, val_iterations=2)

    def cfg(name, **extra):
        c = _cfg(tree, str(tmp_path / name), **kw)
        c.nerf.train.chunksize = 64                            # 128 rays per image -> 2 chunks
        return c | extra

    full = train(0, cfg("full"), device=dev, verbose=False)
    assert full["num_logs"] == 12 and [v["iteration"] for v in full["validation"]] == [4, 8]
    assert set(full["validation"][0]) >= {"iteration", "loss", "psnr", "pose_error"}
    names = [os.path.basename(p) for p in full["checkpoints"]]
    # i % save_every == 0 and i == iterations - 1 (train.py:129, i counts chunks)
    assert names == ["checkpoint    4.ckpt", "checkpoint    5.ckpt", "checkpoint    8.ckpt"], names
    ck4, ck5 = (torch.load(p, weights_only=True) for p in full["checkpoints"][:2])
    assert ck4["cn_cursor"].tolist() == [2, 1] and "cn_next_iter" not in ck4 and ck4["iter"] == 2
    assert ck5["cn_cursor"].tolist() == [3, 0] and ck5["cn_next_iter"] == 3
    a = _params(full)
    # after chunk 0 of iteration 2 (with that step's validation), after an iteration's last chunk
    for path, first in ((full["checkpoints"][0], 5), (full["checkpoints"][1], 6)):
        res = train(0, cfg("res" + str(first), load_checkpoint=path), device=dev, verbose=False)
        assert res["logs"] == full["logs"][first:], first
        b = _params(res)
        for k in a:
            assert torch.equal(a[k], b[k]), (first, k)
        assert res["scheduler"].last_epoch == full["scheduler"].last_epoch == 12


def test_train_checkpoint_cadence_and_reference_format(tree, tmp_path):
    """save_every / the last iteration (train.py:129) write checkpoint{i:5d}.ckpt with the reference's
    keys; one holding ONLY those keys (as the reference writes it) loads and resumes the reference's
    way (util.py:175-213: iteration ``iter`` again)."""
    from codenerf.train import train
    dev = torch.device("cuda", 0)
    out = train(0, _cfg(tree, str(tmp_path / "a"), iterations=5, save_every=2), device=dev, verbose=False)
    names = [os.path.basename(p) for p in out["checkpoints"]]
    assert names == ["checkpoint    2.ckpt", "checkpoint    4.ckpt"], names
    ck = torch.load(out["checkpoints"][-1], weights_only=True)
    for key in ("iter", "model_nerf_coarse_state_dict", "model_nerf_fine_state_dict", "model_embedding_state_dict",
                "optimizer_state_dict"):
        assert key in ck
    assert ck["iter"] == 4 and ck["cn_next_iter"] == 5
    ref_only = {k: v for k, v in ck.items() if not k.startswith("cn_")}
    path = tmp_path / "ref.ckpt"
    torch.save(ref_only, str(path))
    res = train(0, _cfg(tree, str(tmp_path / "b"), iterations=5) | {"load_checkpoint": str(path)}, device=dev,
                verbose=False)
    assert len(res["logs"]) == 1                         # iteration 4 again (the reference's resume)


def test_eval_loop_psnr(tree, tmp_path):
    from codenerf.evaluate import eval_loop
    dev = torch.device("cuda", 0)
    res = eval_loop(0, _cfg(tree, str(tmp_path / "e"), iterations=6, val_iterations=3), device=dev, verbose=False)
    assert len(res) == 6
    for r in res:
        assert torch.isfinite(torch.tensor(r["psnr"])) and r["rgb"].shape == (48 * 48, 3)
        assert len(r["history"]) == 3
