"""Checkpoint interop with the reference.

``save_checkpoint`` writes train.py:129-138's dict -- ``iter``,
``model_{nerf_coarse,nerf_fine,embedding}_state_dict`` and ``optimizer_state_dict`` --
so the reference can load what this build trains.  ``load_checkpoint`` is
utils/util.py:175-213: only an existing ``.ckpt`` file is read, tensors saved on
cuda:0 map to this rank's device, all ranks meet at a barrier before anyone could save,
the ``module.`` prefix DDP adds is stripped, the optimiser state is restored and the
start iteration returned.

Differences by design:
* the build never wraps its modules in DDP (codenerf.train), so the ``module.`` prefix
  is stripped in every mode (the reference strips it only when not distributed, because
  its distributed modules expect it);
* the file is read with ``torch.load(weights_only=True)``: the reference's checkpoints
  hold only tensors, numbers, lists and dicts, so nothing executes from the file;
* the optimiser may be this build's flat AdamW (codenerf.optim), whose state_dict format
  is torch.optim.AdamW's, or any torch optimiser.
"""
from __future__ import annotations

from collections import OrderedDict
from pathlib import Path
from typing import Dict

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


def load_checkpoint(cfg, models: Dict[str, torch.nn.Module], optimizer) -> int:
    """utils/util.py:175-213 -> the start iteration (0 when ``cfg.load_checkpoint`` is not an
    existing ``.ckpt`` file)."""
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
            model.load_state_dict(_strip_module_prefix(checkpoint[f"model_{model_name}_state_dict"]))
        if optimizer is not None:
            optimizer.load_state_dict(checkpoint["optimizer_state_dict"])
        start_iter = checkpoint["iter"]
    return start_iter


def save_checkpoint(path, iteration: int, models: Dict[str, torch.nn.Module], optimizer) -> None:
    """train.py:129-138's checkpoint dict, written with torch.save."""
    checkpoint_dict = {"iter": iteration}
    for name in ("nerf_coarse", "nerf_fine", "embedding"):
        if name in models:
            checkpoint_dict[f"model_{name}_state_dict"] = models[name].state_dict()
    checkpoint_dict["optimizer_state_dict"] = optimizer.state_dict()
    torch.save(checkpoint_dict, str(path))
