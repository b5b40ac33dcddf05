"""Checkpoint interop with the reference.

``save_checkpoint`` writes train.py:129-138's dict -- ``iter``,
``model_{nerf_coarse,nerf_fine,embedding}_state_dict`` and ``optimizer_state_dict`` --
so the reference can load what this build trains.  ``load_checkpoint`` is
utils/util.py:175-213: only an existing ``.ckpt`` file is read, tensors saved on
cuda:0 map to this rank's device, all ranks meet at a barrier before anyone could save,
the ``module.`` prefix DDP adds is stripped, the optimiser state is restored and the
start iteration returned.

Differences by design:
* the ``module.`` prefix is stripped in every mode and the state loaded into the bare module
  (``m.module`` of a DDP wrapper): the reference strips it only when not distributed, because
  its distributed modules are DDP wrappers that expect it.  ``save_checkpoint(ddp_prefix=True)``
  writes it the way the reference's distributed training does, for the reference to load;
* the file is read with ``torch.load(weights_only=True)``: the reference's checkpoints
  hold only tensors, numbers, lists and dicts, so nothing executes from the file;
* the optimiser may be this build's flat AdamW (codenerf.optim), whose state_dict format
  is torch.optim.AdamW's, or any torch optimiser;
* extra keys for an exact resume (the reference's loader reads only its own keys, so it still
  loads these files): ``cn_next_iter`` (the iteration after the one saved, when the save came after
  its last chunk), ``cn_scheduler_state_dict`` (the reference does not save the LambdaLR),
  ``cn_rng`` (the numpy, torch CPU and torch CUDA generator states, as tensors) and, from the
  driver (codenerf.train.train):
  - ``cn_cursor`` = (iteration, next chunk): where the uninterrupted run goes on -- a save after
    chunk j of an iteration with more chunks resumes at chunk j + 1 of the SAME iteration, with
    that iteration's ray draw;
  - ``cn_rng_ranks``: every rank's generator states (all_gather at the save), each as ``now``
    (after the save step's own validation, i.e. what the next chunk draws from) and
    ``iter_start`` (before the iteration's batch / ray draw, replayed for a mid-iteration resume).
    The reference seeds every rank differently (``(rank + 1) + randomseed``, train.py:28-31) so
    the ranks sample different rays; each rank restores its OWN state.  A checkpoint without
    per-rank states (one written by ``save_checkpoint`` alone, or by another world size) restores
    ``cn_rng`` only at world size 1; other ranks keep their own seeds.
"""
from __future__ import annotations

from collections import OrderedDict
from pathlib import Path
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch
import torch.distributed as dist


def _strip_module_prefix(state_dict) -> "OrderedDict[str, torch.Tensor]":
    sd = OrderedDict(state_dict)
    torch.nn.modules.utils.consume_prefix_in_state_dict_if_present(sd, "module.")
    return sd


def _device_of(models) -> torch.device:
    for m in models.values():
        for p in m.parameters():
            return p.device
    return torch.device("cpu")


def _rng_state(device) -> Dict[str, torch.Tensor]:
    import numpy as np
    kind, keys, pos, has_gauss, cached = np.random.get_state()
    out = {"numpy_keys": torch.from_numpy(keys.astype(np.int64)),
           "numpy_meta": torch.tensor([pos, has_gauss], dtype=torch.int64),
           "numpy_gauss": torch.tensor([cached], dtype=torch.float64),
           "torch": torch.get_rng_state()}
    if device is not None and device.type == "cuda":
        out["cuda"] = torch.cuda.get_rng_state(device)
    return out


def rng_state(device=None, ray_sampler=None) -> Dict[str, torch.Tensor]:
    """The generator states a resume restores: numpy, torch CPU, torch CUDA of ``device`` and, with a
    ``ray_sampler`` (rng="device"), its Philox draw counter.  Host copies only (no device sync)."""
    st = _rng_state(device)
    if ray_sampler is not None:
        st["ray_draws"] = torch.tensor([int(ray_sampler._draws)], dtype=torch.int64)
    return st


def set_rng_state(st: Dict[str, torch.Tensor], device=None, ray_sampler=None) -> None:
    _set_rng_state(st, device)
    if ray_sampler is not None and "ray_draws" in st:
        ray_sampler._draws = int(st["ray_draws"][0])


def gather_rng_states(state: Dict[str, Dict[str, torch.Tensor]]) -> List[Dict[str, Dict[str, torch.Tensor]]]:
    """Every rank's ``state`` (a dict of generator-state dicts, host tensors), rank-ordered; a
    collective when torch.distributed is initialised, else ``[state]``."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [state]
    out: List[Optional[dict]] = [None] * dist.get_world_size()
    dist.all_gather_object(out, state)
    return out


def _set_rng_state(st: Dict[str, torch.Tensor], device) -> None:
    import numpy as np
    meta = st["numpy_meta"].tolist()
    np.random.set_state(("MT19937", st["numpy_keys"].numpy().astype(np.uint32), int(meta[0]), int(meta[1]),
                         float(st["numpy_gauss"][0])))
    torch.set_rng_state(st["torch"].cpu())
    if "cuda" in st and device is not None and device.type == "cuda":
        torch.cuda.set_rng_state(st["cuda"].cpu(), device)


def load_checkpoint(cfg, models: Dict[str, torch.nn.Module], optimizer, extras: Optional[dict] = None) -> int:
    """utils/util.py:175-213 -> the start iteration (0 when ``cfg.load_checkpoint`` is not an
    existing ``.ckpt`` file).  ``extras``: receives this build's resume keys when the file has them
    (apply them with ``resume_state``)."""
    start_iter = 0
    is_distributed = bool(getattr(cfg, "is_distributed", False))
    rank = dist.get_rank() if is_distributed else 0
    path = getattr(cfg, "load_checkpoint", None)
    if not path:
        return start_iter
    checkpoint_file = Path(path)
    if checkpoint_file.exists() and checkpoint_file.is_file() and checkpoint_file.suffix == ".ckpt":
        dev = _device_of(models)
        if dev.type == "cuda":
            map_location = {"cuda:0": f"cuda:{rank if dev.index is None else dev.index}"}
        else:
            map_location = "cpu"
        checkpoint = torch.load(str(checkpoint_file), map_location=map_location, weights_only=True)
        # every rank has read the file before any rank could overwrite it (util.py:198-200)
        if is_distributed:
            dist.barrier()
        for model_name, model in models.items():
            getattr(model, "module", model).load_state_dict(
                _strip_module_prefix(checkpoint[f"model_{model_name}_state_dict"]))
        if optimizer is not None:
            optimizer.load_state_dict(checkpoint["optimizer_state_dict"])
        start_iter = checkpoint["iter"]
        if extras is not None:
            extras.update({k: v for k, v in checkpoint.items() if k.startswith("cn_")})
            extras["device"] = dev
    return start_iter


@dataclass
class ResumePoint:
    """Where a resumed run continues: ``iteration``, its first chunk ``chunk``, and this rank's
    generator states -- ``rng`` at that point, ``iter_rng`` at the start of ``iteration`` (needed
    when ``chunk`` > 0: the iteration's batch and ray draw are replayed from it, then ``rng`` is
    set before chunk ``chunk``).  Both None: keep this process's own seeding."""
    iteration: int
    chunk: int = 0
    rng: Optional[Dict[str, torch.Tensor]] = None
    iter_rng: Optional[Dict[str, torch.Tensor]] = None


def resume_point(extras: dict, scheduler, start_iter: int, rank: int = 0, world_size: int = 1) -> ResumePoint:
    """Apply a checkpoint's scheduler state (load_checkpoint's ``extras``) and pick this rank's resume
    point: ``cn_cursor`` (iteration, next chunk) when present, else ``cn_next_iter``, else
    ``start_iter`` (the reference's semantics: iteration ``iter`` again).  RNG: this rank's entry
    of ``cn_rng_ranks`` when the checkpoint holds one per rank of this world size; otherwise
    ``cn_rng`` at world size 1 only (a single-rank state handed to every rank would make them all
    draw the same rays)."""
    if not extras:
        return ResumePoint(start_iter)
    if scheduler is not None and "cn_scheduler_state_dict" in extras:
        scheduler.load_state_dict(extras["cn_scheduler_state_dict"])
    ranks = extras.get("cn_rng_ranks")
    rng = iter_rng = None
    if ranks is not None and len(ranks) == world_size:
        rng, iter_rng = ranks[rank].get("now"), ranks[rank].get("iter_start")
    elif world_size == 1 and "cn_rng" in extras:
        rng = extras["cn_rng"]
    if "cn_cursor" in extras:
        it, chunk = (int(v) for v in extras["cn_cursor"].tolist())
        if chunk > 0 and iter_rng is None:
            # no replayable draw for this rank: redo the whole iteration (the reference's way)
            return ResumePoint(it, 0, None, None)
        return ResumePoint(it, chunk, rng, iter_rng if chunk > 0 else None)
    return ResumePoint(int(extras.get("cn_next_iter", start_iter)), 0, rng, None)


def resume_state(extras: dict, scheduler, start_iter: int) -> int:
    """Apply a checkpoint's resume keys (load_checkpoint's ``extras``) at world size 1: the scheduler
    state, the RNG streams -> the iteration to continue from (``cn_next_iter``, else ``start_iter``).
    A mid-iteration cursor needs the driver (``resume_point``); here it redoes that iteration."""
    p = resume_point(extras, scheduler, start_iter)
    if p.chunk > 0:
        p = ResumePoint(p.iteration, 0, p.iter_rng)
    if p.rng is not None:
        _set_rng_state(p.rng, extras.get("device"))
    return p.iteration


def save_checkpoint(path, iteration: int, models: Dict[str, torch.nn.Module], optimizer, scheduler=None,
                    next_iter: Optional[int] = None, ddp_prefix: bool = False, rng: bool = True,
                    cursor: Optional[tuple] = None, rng_ranks: Optional[list] = None) -> None:
    """train.py:129-138's checkpoint dict, written with torch.save (+ the resume keys, see the module
    docstring).  ``ddp_prefix``: write the model keys with DDP's ``module.`` prefix, as the
    reference's distributed training does (its distributed load expects them).  ``cursor``
    (iteration, next chunk) and ``rng_ranks`` (gather_rng_states of {"now", "iter_start"}): the
    driver's exact-resume keys; ``cn_rng`` is then rank 0's ``now``."""
    checkpoint_dict = {"iter": iteration}
    for name in ("nerf_coarse", "nerf_fine", "embedding"):
        if name in models:
            sd = models[name].state_dict()
            if ddp_prefix and not hasattr(models[name], "module"):
                sd = OrderedDict((f"module.{k}", v) for k, v in sd.items())
            checkpoint_dict[f"model_{name}_state_dict"] = sd
    checkpoint_dict["optimizer_state_dict"] = optimizer.state_dict()
    if cursor is not None and next_iter is None and int(cursor[1]) == 0:
        next_iter = int(cursor[0])
    if next_iter is not None:
        checkpoint_dict["cn_next_iter"] = int(next_iter)
    if cursor is not None:
        checkpoint_dict["cn_cursor"] = torch.tensor([int(cursor[0]), int(cursor[1])], dtype=torch.int64)
    if scheduler is not None:
        checkpoint_dict["cn_scheduler_state_dict"] = scheduler.state_dict()
    if rng_ranks is not None:
        checkpoint_dict["cn_rng_ranks"] = list(rng_ranks)
        if rng:
            checkpoint_dict["cn_rng"] = rng_ranks[0]["now"]
    elif rng:
        checkpoint_dict["cn_rng"] = _rng_state(_device_of(models))
    torch.save(checkpoint_dict, str(path))
