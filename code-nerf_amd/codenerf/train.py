"""The training step of train.py on the gfx950 kernels.

``prepare_models`` / ``prepare_optimizer`` mirror utils/util.py:93-144 and :147-172;
``train_iteration`` is train.py:64-114 for one loaded batch (ray sampling and the
target-pixel gather :76-80, chunking :82-90, then per chunk ``train_minibatch``:
embedding lookup, hierarchical render, losses, backward, optimiser and scheduler
steps, :92-114).

By design:
* the three modules are not wrapped in DDP.  The gradient average DDP performs is
  ONE all-reduce of the optimiser's flat gradient buffer
  (``codenerf.optim.AdamW.allreduce_grads``) between ``loss.backward()`` and
  ``optimizer.step()``; DDP's construction-time broadcast is one broadcast of the
  flat parameter buffer (``prepare_optimizer``);
* ``cfg.optimizer.type == "AdamW"`` (every CodeNeRF config) selects the flat
  one-launch AdamW; any other type is built from ``torch.optim`` as the reference
  builds it (its update then runs in torch);
* the embedding lookup folds each chunk's distinct objects
  (``ShapeTextureEmbedding``), so the code layers run once per object.
The loss terms keep the reference's definitions, including the regulariser on
``.data`` (train.py:106-107 through model.py:113-120: a constant, no gradient).
"""
from __future__ import annotations

from collections import OrderedDict
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np
import torch
import torch.distributed as dist

from . import nerf
from .models import CodeNeRFModel, ShapeTextureEmbedding, get_params_tensor
from .optim import AdamW
from .autograd import backward_from, paired_fields, render_loss_autograd
from .utils import get_minibatches


def prepare_models(cfg, num_objects: int, device) -> "OrderedDict[str, torch.nn.Module]":
    """utils/util.py:93-144 without the DDP wrappers (see the module docstring)."""
    emb_cfg, e = cfg.models.embedding, cfg.nerf.embedder
    models = OrderedDict()
    models["embedding"] = ShapeTextureEmbedding(num_embeddings=num_objects, shape_code_size=emb_cfg.shape_code_size,
                                                texture_code_size=emb_cfg.texture_code_size).to(device)
    for key in ("nerf_coarse", "nerf_fine"):
        models[key] = CodeNeRFModel(hidden_size=getattr(cfg.models, key).hidden_size, num_embeddings=num_objects,
                                    shape_code_size=emb_cfg.shape_code_size,
                                    texture_code_size=emb_cfg.texture_code_size,
                                    num_encoding_fn_xyz=e.num_encoding_fn_xyz, include_input_xyz=e.include_input_xyz,
                                    num_encoding_fn_dir=e.num_encoding_fn_dir,
                                    include_input_dir=e.include_input_dir).to(device)
    return models


def prepare_optimizer(cfg, models):
    """utils/util.py:147-172: one optimiser over nerf_coarse, nerf_fine and the embedding
    (at ``embedding_lr``) and LambdaLR(gamma ** (epoch / step_size))."""
    groups = [{"params": list(models["nerf_coarse"].parameters())},
              {"params": list(models["nerf_fine"].parameters())},
              {"params": list(models["embedding"].parameters()), "lr": cfg.optimizer.embedding_lr}]
    if cfg.optimizer.type == "AdamW":
        optimizer = AdamW(groups, lr=cfg.optimizer.lr)
        if getattr(cfg, "is_distributed", False):
            optimizer.broadcast_params(0)
    else:
        optimizer = getattr(torch.optim, cfg.optimizer.type)(groups, lr=cfg.optimizer.lr)
        if getattr(cfg, "is_distributed", False):
            broadcast_parameters(models)
    gamma, step_size = cfg.optimizer.scheduler_gamma, cfg.optimizer.scheduler_step_size
    scheduler = torch.optim.lr_scheduler.LambdaLR(optimizer, lr_lambda=lambda epoch: gamma ** (epoch / step_size))
    return optimizer, scheduler


def broadcast_parameters(models, src: int = 0) -> None:
    """DDP's construction-time broadcast (utils/util.py:139-142) for any optimiser: every replica
    starts from rank ``src``'s parameters (one coalesced broadcast)."""
    params = [p for m in models.values() for p in m.parameters()]
    flat = torch.cat([p.detach().reshape(-1) for p in params])
    dist.broadcast(flat, src=src)
    o = 0
    with torch.no_grad():
        for p in params:
            p.copy_(flat[o:o + p.numel()].view_as(p))
            o += p.numel()


def _average_gradients(optimizer, models) -> None:
    if hasattr(optimizer, "allreduce_grads"):
        optimizer.allreduce_grads()
        return
    # a torch optimiser: one coalesced all-reduce over EVERY parameter (missing gradients as
    # zeros, so every rank reduces the same size) plus a has-grad flag per parameter
    params = [p for m in models.values() for p in m.parameters()]
    dev = params[0].device
    flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in params])
    flags = torch.tensor([int(p.grad is not None) for p in params], dtype=torch.int32, device=dev)
    dist.all_reduce(flags)
    dist.all_reduce(flat)
    flat.div_(dist.get_world_size())
    o = 0
    for p, cnt in zip(params, flags.cpu().tolist()):
        if cnt > 0:
            g = flat[o:o + p.numel()].view_as(p)
            if p.grad is None:
                p.grad = g.clone()
            else:
                p.grad.copy_(g)
        o += p.numel()


def _ddp_wrapped(models) -> bool:
    return any(isinstance(m, torch.nn.parallel.DistributedDataParallel) for m in models.values())


def train_minibatch(models, optimizer, scheduler, point_sampler, embedders, ro, rd, object_ids, target_pixels,
                    regularizer_lambda: float, is_distributed: bool = False, uniforms=None) -> Dict[str, object]:
    """train.py:92-114 for one chunk -> the losses train.py logs (tensors) and its psnr (float,
    read back every chunk as train.py:105 does).  ``uniforms``: (t_rand, u), the stratified / fine
    draws of point_sampler.py:64,93 injected (parity tests) instead of drawn on the device."""
    target_object_embedding = models["embedding"](object_ids)
    # both fields' training backwards in shared launches (autograd.FieldPair: the loss below reaches both);
    # data parallel with the flat AdamW, the two MLPs' gradients (param groups 0, 1: util.py:151-156) start
    # their all-reduce as soon as that shared backward has enqueued them (allreduce_begin), beside the rest
    # of the backward, as DDP's bucketed reduction overlaps its backward
    early = None
    if is_distributed and not _ddp_wrapped(models) and hasattr(optimizer, "allreduce_begin"):
        early = lambda: optimizer.allreduce_begin(2)  # noqa: E731
    with paired_fields(on_grads=early):
        if uniforms is None:
            rgb_coarse, rgb_fine = nerf.predict_radiance_and_render((ro, rd), point_sampler, embedders,
                                                                    models["nerf_coarse"], models["nerf_fine"],
                                                                    target_object_embedding)
        else:
            out = nerf.render_rays(ro, rd, *target_object_embedding, point_sampler, embedders, models["nerf_coarse"],
                                   models["nerf_fine"], t_rand=uniforms[0], u=uniforms[1])
            rgb_coarse, rgb_fine = out["rgb_coarse"], out["rgb_fine"]
    # mse coarse + mse fine + lambda (||shape table|| + ||texture table||) on .data (a constant):
    # one cn_render_loss launch forward, one backward into the two rgb tensors
    shape_params, texture_params = get_params_tensor(models["embedding"], is_distributed)
    # train.py:105's psnr of this chunk, written on the device by the loss launch itself (mse2psnr's
    # arithmetic in float64): the reference's .item() read-back every chunk made the host wait for
    # the GPU and the GPU then wait for the host's next launches; float() it when it is logged
    psnr = torch.empty((), dtype=torch.float64, device=target_pixels.device)
    loss, stats = render_loss_autograd(rgb_coarse, rgb_fine, target_pixels, shape_params, texture_params, 1,
                                       regularizer_lambda, psnr=psnr)
    loss_coarse, loss_fine, regularization = stats[0], stats[1], stats[2]
    optimizer.zero_grad()
    backward_from(loss)
    if is_distributed and not _ddp_wrapped(models):
        _average_gradients(optimizer, models)     # (DDP-wrapped modules averaged in the backward)
    optimizer.step()
    scheduler.step()
    return {"nerf_loss_coarse": loss_coarse, "nerf_loss_fine": loss_fine, "embedding_loss": regularization,
            "total_loss": loss.detach(), "psnr": psnr}


def psnr_tensor(mse: torch.Tensor) -> torch.Tensor:
    """utils/util.py:216-227 (mse2psnr) on a device scalar: -10 log10(mse), mse 0 -> 1e-5, float64."""
    m = mse.detach().double()
    return -10.0 * torch.log10(torch.where(m == 0, torch.full_like(m, 1e-5), m))


def train_iteration(cfg, train_data: Dict[str, torch.Tensor], models, optimizer, scheduler, samplers,
                    embedders, on_chunk=None, start_chunk: int = 0, after_draw=None) -> List[Dict[str, object]]:
    """train.py:64-114 for one loaded batch (``color`` (B,H,W,C), ``pose`` (B,4,4), ``object_id``
    (B,) on the device) -> the per-chunk logs.  ``on_chunk(j, num_batches, logs)``: called after
    chunk j's optimiser step (train.py:116-142's logging / checkpoint / validation slot).
    ``start_chunk`` / ``after_draw()``: a mid-iteration resume -- the batch's ray draw is made as
    usual, ``after_draw`` then restores the generators saved after chunk ``start_chunk - 1`` and
    the chunks before ``start_chunk`` are skipped."""
    ray_sampler, point_sampler = samplers
    is_distributed = bool(getattr(cfg, "is_distributed", False))
    for m in models.values():
        m.train()
    # sample + the per-image target gather (train.py:76-80) in one cn_pose_rays launch
    ro_batch, rd_batch, select_inds, target = ray_sampler.sample_pixels(train_data["pose"], train_data["color"])
    if after_draw is not None:
        after_draw()
    n_rays = ray_sampler.sample_size
    color = train_data["color"]
    object_ids = train_data["object_id"][:, None].expand(-1, n_rays).reshape(-1)
    # the per-image ids on the host (the resident loader hands them over; else one read per
    # iteration): the chunks' embedding lookups then need no device sync (ShapeTextureEmbedding)
    host_ids = train_data.get("object_id_host")
    if host_ids is None:
        host_ids = train_data["object_id"].cpu().numpy()
    host_ids = np.repeat(np.asarray(host_ids, dtype=np.int64), n_rays)
    chunk = cfg.nerf.train.chunksize
    assert chunk <= n_rays * color.shape[0], \
        "Chunksize needs to atleast be less than to the number of rays sampled from a single image"
    logs = []
    batches = list(zip(get_minibatches(ro_batch, chunk), get_minibatches(rd_batch, chunk),
                       get_minibatches(object_ids, chunk), get_minibatches(target, chunk)))
    for j, (ro, rd, ids, tp) in enumerate(batches):
        if j < start_chunk:
            continue
        ids._cn_host_ids = host_ids[j * chunk:j * chunk + ids.shape[0]]
        logs.append(train_minibatch(models, optimizer, scheduler, point_sampler, embedders, ro, rd, ids, tp,
                                    cfg.experiment.regularizer_lambda, is_distributed))
        if on_chunk is not None:
            on_chunk(j, len(batches), logs[-1])
    return logs


# ---------------------------------------------------------------- the driver loop (train.py:19-142)

def log_losses(mode: str, i: int, time_taken: float, losses: Dict[str, float],
               learning_rate: Optional[float] = None) -> str:
    """utils/util.py:238-264's console string (TensorBoard is not rebuilt)."""
    tag = {"train": "[TRAIN ]", "val": "[VAL   ]"}.get(mode, "[VALOPT]")
    out = f"{tag} Iter: {i:>8} Time taken: {time_taken:>4.4f} "
    if learning_rate:
        out += f"Learning rate: {learning_rate:0.8f} "
    for key, val in losses.items():
        out += f"{key}: {float(val):>4.4f} "
    return out


def prepare_experiment(cfg) -> Path:
    """utils/util.py:44-55: ``experiment.logdir / experiment.id``, with the config written beside."""
    import yaml
    logdir_path = Path(cfg.experiment.logdir) / str(cfg.experiment.id)
    logdir_path.mkdir(parents=True, exist_ok=True)
    with open(logdir_path / "config.yml", "w") as f:
        yaml.safe_dump(cfg.to_dict() if hasattr(cfg, "to_dict") else dict(cfg), f)
    return logdir_path


def _main(cfg) -> bool:
    return (not getattr(cfg, "is_distributed", False)) or dist.get_rank() == 0


def seed_rank(rank: int, cfg) -> int:
    """train.py:28-31 / eval.py:44-47: numpy and torch seeded with ``(rank + 1) + randomseed``, so
    every process samples different rays -> the seed."""
    seed = (rank + 1) + int(cfg.experiment.randomseed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    return seed


def next_train_batch(cfg, train_loader, iteration: int):
    """train.py:67-70: ``set_epoch(iteration)`` when distributed, then the first batch of a fresh
    iterator over the train loader."""
    if getattr(cfg, "is_distributed", False):
        train_loader.sampler.set_epoch(iteration)
    return next(iter(train_loader))


class LogBook:
    """The driver's per-chunk logs without holding the run: entries arrive as device scalars (no
    read-back per chunk), are read back together when printed or every ``flush_every`` chunks (one
    copy for the lot), and only the last ``keep`` host-float entries are retained (None: all)."""

    def __init__(self, keep: Optional[int] = 1000, flush_every: int = 64):
        from collections import deque
        self.keep, self.flush_every = keep, flush_every
        self.pending: List[Dict[str, object]] = []
        self.entries = deque(maxlen=keep)
        self.count = 0

    def add(self, lg: Dict[str, object]) -> None:
        self.pending.append(lg)
        self.count += 1
        if len(self.pending) >= self.flush_every:
            self.flush()

    def flush(self) -> None:
        if not self.pending:
            return
        keys = [list(lg) for lg in self.pending]
        vals = [v for lg in self.pending for v in lg.values()]
        dev = [v.detach().reshape(()).double() for v in vals if torch.is_tensor(v)]
        host = iter(torch.stack(dev).cpu().tolist()) if dev else iter(())
        flat = [next(host) if torch.is_tensor(v) else float(v) for v in vals]
        o = 0
        for ks in keys:
            self.entries.append(dict(zip(ks, flat[o:o + len(ks)])))
            o += len(ks)
        self.pending = []

    def last(self) -> Dict[str, float]:
        self.flush()
        return self.entries[-1]

    def as_list(self) -> List[Dict[str, float]]:
        self.flush()
        return list(self.entries)


def _validation_summary(res: Dict[str, object], iteration: int) -> Dict[str, object]:
    """What the driver keeps of a validation (host scalars): the reference logs loss / psnr and writes
    the images to TensorBoard, keeping nothing."""
    out = {"iteration": iteration, "pose": res.get("pose")}
    for k in ("loss", "psnr", "pose_error"):
        if k in res:
            out[k] = float(res[k])
    return out


def train(rank: int, cfg, device=None, resident: bool = True, stop_after: Optional[int] = None,
          verbose: bool = True, keep_logs: Optional[int] = None, keep_validation: bool = False) -> Dict[str, object]:
    """train.py:19-142 on the gfx950 path, with the reference's seeds, data order and cadence.

    * seed ``(rank + 1) + experiment.randomseed`` for numpy and torch (train.py:29-31);
    * the train / val loaders of utils/util.py:59-90 (``resident``: the split decoded once into HBM,
      codenerf.datasets.ResidentLoader: the same sampler, the same index order), the models, the
      optimiser + LambdaLR and the checkpoint (util.py:93-213), the samplers and embedders from the
      first batch (train.py:51-58);
    * per iteration: ``set_epoch`` when distributed (train.py:67-68), one batch from a fresh
      iterator (train.py:70), ``train_iteration``; after each chunk step i = iteration *
      num_batches + j: the log line every ``print_every`` (rank 0), ``validate`` every
      ``validate_every`` (every rank; eval.py:82-205), a checkpoint every ``save_every`` and at the
      last iteration (rank 0, ``checkpoint{i:5d}.ckpt``).
    ``stop_after``: leave the loop after this many iterations (an interrupted run, for resume tests).

    Exact resume: a checkpoint carries the scheduler, a cursor (iteration, next chunk) and EVERY
    rank's generator states (gathered at the save): the states after the save step -- taken after
    that step's validation, so the file is written once the validation has run (the reference
    writes it just before) -- and the states at the start of the iteration.  A resume from a save
    after chunk j < last replays the iteration's batch and ray draw from the latter, restores the
    former and continues at chunk j + 1; one at an iteration's end continues with the next.  Each
    rank restores its own states.  The continuation is bit-identical to the uninterrupted run
    where the step itself is deterministic: one object per chunk (every runnable config:
    chunksize <= num_random_rays), see DESIGN.md section 4.  A reference checkpoint resumes with
    the reference's semantics (``iter`` again, fresh RNG and scheduler).

    Memory: the per-chunk logs are read back in batches; ``keep_logs`` (None, the library default:
    all) caps how many of the last ones are kept (LogBook; the command line keeps 1000); a validation
    keeps its host scalars (``keep_validation``: also its history, codes and image).  Returns {"logs":
    host-float dicts, "num_logs", "first_log_index" (the chunk index of logs[0]: 0 unless capped),
    "checkpoints": paths, "validation": summaries, "models", "optimizer", "scheduler"}."""
    import time
    from . import checkpoint as C
    from .datasets import prepare_dataloader
    from .evaluate import validate, validation_batch
    seed_rank(rank, cfg)
    main = _main(cfg)
    is_distributed = bool(getattr(cfg, "is_distributed", False))
    world = dist.get_world_size() if is_distributed else 1
    logdir_path = prepare_experiment(cfg) if main else None
    device = torch.device("cuda", rank) if device is None else torch.device(device)
    torch.cuda.set_device(device)
    train_loader, train_dataset = prepare_dataloader("train", cfg, device if resident else None)
    val_loader, _ = prepare_dataloader("val", cfg, device if resident else None)
    models = prepare_models(cfg, train_dataset.num_objects, device)
    optimizer, scheduler = prepare_optimizer(cfg, models)
    extras: Dict[str, object] = {}
    start_iter = C.load_checkpoint(cfg, models, optimizer, extras=extras)
    first = next(iter(train_loader))
    (height, width), intrinsic = first["color"][0].shape[:2], first["intrinsic"][0]
    samplers = nerf.prepare_samplers(cfg, height, width, intrinsic.cpu(), torch.float32, device)
    embedders = nerf.prepare_embedders(cfg, torch.float32, device)
    ray_sampler = samplers[0]
    # after the first-batch draw, as saved
    point = C.resume_point(extras, scheduler, start_iter, rank=dist.get_rank() if is_distributed else 0,
                           world_size=world)
    if point.chunk == 0 and point.rng is not None:
        C.set_rng_state(point.rng, device, ray_sampler)
    book = LogBook(keep_logs)
    out = {"logs": [], "checkpoints": [], "validation": [], "models": models, "optimizer": optimizer,
           "scheduler": scheduler}
    total = int(cfg.experiment.iterations) // int(cfg.dataset.train_batch_size)
    e = cfg.experiment
    for iteration in range(point.iteration, total):
        if stop_after is not None and iteration - point.iteration >= stop_after:
            break
        resume_chunk = point.chunk if iteration == point.iteration else 0
        if resume_chunk:
            C.set_rng_state(point.iter_rng, device, ray_sampler)
        iter_rng = C.rng_state(device, ray_sampler)     # replayed by a resume from inside this iteration
        train_data = next_train_batch(cfg, train_loader, iteration)
        train_data = {k: (v.to(device, non_blocking=True) if torch.is_tensor(v) else v) for k, v in train_data.items()}
        then = time.time()

        def on_chunk(j, num_batches, lg):
            i = iteration * num_batches + j
            book.add(lg)                           # device scalars: read in batches (LogBook)
            if main and i > 0 and i % e.print_every == 0 and verbose:
                print(log_losses("train", i, time.time() - then, book.last(), scheduler.get_last_lr()[0]))
            if i > 0 and i % e.validate_every == 0:
                val_data = validation_batch(cfg, val_loader, i)
                res = validate(cfg, val_data, models, samplers, embedders, device,
                               log_every=e.val_print_every if verbose else None)
                out["validation"].append(res if keep_validation else _validation_summary(res, i))
            if i > 0 and (i % e.save_every == 0 or i == e.iterations - 1):
                # every rank's generators after this step (and its validation), and at the iteration's start
                states = C.gather_rng_states({"now": C.rng_state(device, ray_sampler), "iter_start": iter_rng})
                if main:
                    cursor = (iteration + 1, 0) if j == num_batches - 1 else (iteration, j + 1)
                    path = logdir_path / f"checkpoint{i:5d}.ckpt"
                    C.save_checkpoint(path, iteration, models, optimizer, scheduler=scheduler, cursor=cursor,
                                      rng_ranks=states)
                    out["checkpoints"].append(str(path))
                    if verbose:
                        print("================== Saved Checkpoint =================")

        after_draw = (lambda: C.set_rng_state(point.rng, device, ray_sampler)) if resume_chunk else None
        train_iteration(cfg, train_data, models, optimizer, scheduler, samplers, embedders, on_chunk=on_chunk,
                        start_chunk=resume_chunk, after_draw=after_draw)
    out["logs"] = book.as_list()
    out["num_logs"] = book.count
    out["first_log_index"] = book.count - len(out["logs"])
    return out


# ---------------------------------------------------------------- process launch (train.py:145-179)

def init_process(rank: int, fn, cfg, backend: str = "gloo", port: int = 29500, init_method: Optional[str] = None):
    """train.py:145-156 / eval.py:208-219: rendezvous at 127.0.0.1:``port`` (the reference's 29500),
    ``init_process_group(backend, rank, world_size=cfg.gpus)`` -- on "nccl" (RCCL) bound to
    ``cuda:rank`` -- then ``fn(rank, cfg)`` and ``destroy_process_group``.  This runs in a freshly
    spawned process: nothing has touched the GPU before it."""
    import os
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    kw = {}
    if backend == "nccl":
        torch.cuda.set_device(rank)
        kw["device_id"] = torch.device("cuda", rank)
    if init_method is not None:
        kw["init_method"] = init_method
    dist.init_process_group(backend, rank=rank, world_size=int(cfg.gpus), **kw)
    try:
        fn(rank, cfg)
    finally:
        dist.destroy_process_group()


def launch(fn, cfg, backend: Optional[str] = None, port: int = 29500, init_method: Optional[str] = None) -> None:
    """train.py:159-179's dispatch: with ``cfg.is_distributed`` and ``cfg.gpus`` > 1, one process per
    rank (``start_method="spawn"``: started before this process makes any GPU call, so each child
    initialises HIP itself) running ``init_process`` over ``backend`` (default "nccl", i.e. RCCL);
    otherwise ``fn(0, cfg)`` in this process."""
    gpus = int(getattr(cfg, "gpus", 1))
    if gpus > 1 and getattr(cfg, "is_distributed", False):
        import torch.multiprocessing as mp
        mp.start_processes(init_process, args=(fn, cfg, backend or "nccl", port, init_method), nprocs=gpus,
                           join=True, start_method="spawn")
    else:
        fn(0, cfg)


def _train_rank(rank: int, cfg) -> None:
    train(rank, cfg, keep_logs=1000)     # the command line: a long run keeps the last 1000 chunk logs


def main(cfg, backend: Optional[str] = None, port: int = 29500) -> None:
    """train.py:159-179: ``train`` on ``cfg.gpus`` ranks (one process per GPU over RCCL) or on one."""
    launch(_train_rank, cfg, backend=backend, port=port)


if __name__ == "__main__":
    import argparse
    from .config import load_config
    parser = argparse.ArgumentParser()
    parser.add_argument("-c", "--config", type=str, required=True, help="Path to (.yml) config file.")
    parser.add_argument("--load-checkpoint", type=str, default="", help="Path to load saved checkpoint from.")
    parser.add_argument("-g", "--gpus", default=1, type=int, help="Number of gpus per node")
    parser.add_argument("--distributed", action="store_true", dest="is_distributed",
                        help="Run the models in DataDistributedParallel")
    a = parser.parse_args()
    main(load_config(a.config, gpus=a.gpus, is_distributed=a.is_distributed, load_checkpoint=a.load_checkpoint))
