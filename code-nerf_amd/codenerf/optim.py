"""The training step's optimiser on the gfx950 kernels.

``AdamW`` is a drop-in for ``torch.optim.AdamW`` as the reference builds and drives
it (utils/util.py:159-170: param groups nerf_coarse, nerf_fine and the embedding
tables at ``embedding_lr`` under a LambdaLR; train.py:111-114: zero_grad, backward,
step, scheduler.step): the same constructor, ``param_groups``, per-parameter state
(``step``, ``exp_avg``, ``exp_avg_sq``) and state_dict format, so checkpoints move
between the two.

MI355X layout: every parameter of every group lives in ONE flat fp32 HBM buffer
(each tensor 256-B aligned) with matching flat buffers for the gradient and both
moments; the parameters (and the moments in ``state``) are views into them.
``step()`` is then one kernel launch (cn_adamw_step) for both MLPs and both code
tables, HBM-bound at 28 B per parameter, instead of torch's per-tensor kernel
chain; the data-parallel gradient average the reference gets from DDP
(util.py:139-142) is ONE collective over the flat gradient (``allreduce_grads``:
RCCL over xGMI with the nccl backend, gloo on CPU), and DDP's construction-time
parameter broadcast is one broadcast of the flat parameter buffer
(``broadcast_params``).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.distributed as dist

from . import ops

ALIGN = 64  # floats: every tensor starts on a 256-B boundary


def _round_up(n: int) -> int:
    return (n + ALIGN - 1) // ALIGN * ALIGN


class AdamW(torch.optim.Optimizer):
    """torch.optim.AdamW (decoupled weight decay; amsgrad / maximize off) on flat buffers."""

    # process-group backends on which allreduce_begin starts its bucket asynchronously: RCCL ("nccl"),
    # whose collective stream waits for the enqueued work without a host wait (gloo stages device tensors
    # through the host; the two-rank gloo tests add it to check the bucketed sums)
    bucket_backends = ("nccl",)

    def __init__(self, params, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8,
                 weight_decay: float = 1e-2, amsgrad: bool = False, *, maximize: bool = False,
                 foreach=None, capturable: bool = False, differentiable: bool = False, fused=None):
        if not 0.0 <= lr:
            raise ValueError(f"Invalid learning rate: {lr}")
        if not 0.0 <= eps:
            raise ValueError(f"Invalid epsilon value: {eps}")
        if not 0.0 <= betas[0] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 0: {betas[0]}")
        if not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"Invalid beta parameter at index 1: {betas[1]}")
        if not 0.0 <= weight_decay:
            raise ValueError(f"Invalid weight_decay value: {weight_decay}")
        if amsgrad or maximize or capturable or differentiable:
            raise NotImplementedError("codenerf.optim.AdamW implements amsgrad=False, maximize=False "
                                      "(the reference's AdamW)")
        defaults = dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay, amsgrad=False,
                        maximize=False, foreach=foreach, capturable=False, differentiable=False, fused=fused,
                        decoupled_weight_decay=True)
        self._flat: Optional[Dict[str, torch.Tensor]] = None
        super().__init__(params, defaults)
        self._build()

    # ---- flat buffers -------------------------------------------------
    def add_param_group(self, param_group) -> None:
        super().add_param_group(param_group)
        if self._flat is not None:
            self._build()

    def _build(self) -> None:
        params = [p for g in self.param_groups for p in g["params"]]
        dev = params[0].device
        for p in params:
            if p.dtype != torch.float32 or p.device != dev:
                raise TypeError("codenerf.optim.AdamW needs fp32 parameters on one device")
        offs, starts, o = {}, [0], 0
        for g in self.param_groups:
            for p in g["params"]:
                offs[p] = o
                o += _round_up(p.numel())
            starts.append(o)
        n = max(o, ALIGN)
        flat = {k: torch.zeros(n, device=dev, dtype=torch.float32)
                for k in ("param", "grad", "exp_avg", "exp_avg_sq")}
        with torch.no_grad():
            for p, off in offs.items():
                k = p.numel()
                flat["param"][off:off + k].copy_(p.detach().reshape(-1))
                grad = p.grad
                p.data = flat["param"][off:off + k].view_as(p)
                if grad is not None:
                    flat["grad"][off:off + k].copy_(grad.reshape(-1))
                    p.grad = flat["grad"][off:off + k].view_as(p)
        # the gradient buffer carries one has-grad flag per parameter after its end (allreduce_grads:
        # one collective for both); flat["grad"] is the gradient part
        n_flags = _round_up(len(offs))
        self._grad_ext = torch.zeros(n + n_flags, device=dev, dtype=torch.float32)
        self._grad_ext[:n].copy_(flat["grad"])
        flat["grad"] = self._grad_ext[:n]
        with torch.no_grad():
            for p, off in offs.items():
                if p.grad is not None:
                    p.grad = flat["grad"][off:off + p.numel()].view_as(p)
        self._flag_cache = {}
        self._flat, self._offs, self._starts = flat, offs, starts
        self._adopt_state()

    def _view(self, key: str, p: torch.Tensor) -> torch.Tensor:
        off = self._offs[p]
        return self._flat[key][off:off + p.numel()].view_as(p)

    def _adopt_state(self) -> None:
        """Point every parameter's moments at the flat buffers (after a build or a load)."""
        with torch.no_grad():
            for p in self._offs:
                st = self.state.get(p)
                if not st:
                    continue
                for key in ("exp_avg", "exp_avg_sq"):
                    view = self._view(key, p)
                    t = st.get(key)
                    if t is not None and t.data_ptr() != view.data_ptr():
                        view.copy_(t.reshape(p.shape))
                    st[key] = view
                step = st.get("step", 0.0)
                st["step"] = step if torch.is_tensor(step) else torch.tensor(float(step), dtype=torch.float32)

    def flat_buffers(self) -> Dict[str, torch.Tensor]:
        """The flat fp32 buffers: param, grad, exp_avg, exp_avg_sq (group g spans
        ``group_starts[g]:group_starts[g + 1]``)."""
        return self._flat

    @property
    def group_starts(self) -> List[int]:
        return list(self._starts)

    def _sync_grads(self) -> List[torch.Tensor]:
        """Move every gradient into the flat buffer (autograd may have installed a new
        tensor) and point ``.grad`` at it; returns the parameters without a gradient."""
        missing, dst, src, moved = [], [], [], []
        with torch.no_grad():
            for p in self._offs:
                if p.grad is None:
                    missing.append(p)
                    continue
                view = self._view("grad", p)
                if p.grad.data_ptr() != view.data_ptr():
                    dst.append(view)
                    src.append(p.grad)
                    moved.append((p, view))
            if dst:
                # one multi-tensor launch for all of them (the eval loop's five leaf gradients --
                # codes and pose -- were five copy launches per iteration)
                torch._foreach_copy_(dst, src)
                for p, view in moved:
                    p.grad = view
        return missing

    # ---- reference API ------------------------------------------------
    def zero_grad(self, set_to_none: bool = True) -> None:
        """train.py:111.  ``set_to_none`` (torch's default) drops the gradients as torch does;
        otherwise the flat gradient is cleared in one memset and stays attached.

        Either way the flat gradient is cleared, and each parameter carries its slice as
        ``p._cn_grad_slot``: a fused backward that finds ``p.grad is None`` accumulates straight
        into that (zeroed) slice and returns it, so autograd installs it as ``p.grad`` with no
        per-parameter fill or copy (autograd.RadianceField)."""
        self._flat["grad"].zero_()
        for p in self._offs:
            p._cn_grad_slot = self._view("grad", p)
        if set_to_none:
            for p in self._offs:
                p.grad = None
        else:
            for p in self._offs:
                p.grad = self._view("grad", p)

    @torch.no_grad()
    def step(self, closure=None):
        """One AdamW update of every parameter that has a gradient: ONE cn_adamw_step launch.
        Parameters without a gradient keep their values and state, as in torch."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        self._sync_grads()
        betas, eps = self._hyper()
        segments = self._plan(advance=True)
        if not segments:
            return loss
        f = self._flat
        ops.adamw_step(f["param"], f["grad"], f["exp_avg"], f["exp_avg_sq"], segments, betas[0], betas[1], eps)
        # the kernel wrote through raw pointers: tell autograd and the packed-weight caches
        torch.autograd.graph.increment_version(list(self._offs))
        return loss

    def _hyper(self):
        g0 = self.param_groups[0]
        betas, eps = tuple(g0["betas"]), float(g0["eps"])
        for g in self.param_groups:
            if g.get("amsgrad") or g.get("maximize"):
                raise NotImplementedError("codenerf.optim.AdamW: amsgrad / maximize")
            if tuple(g["betas"]) != betas or float(g["eps"]) != eps:
                raise NotImplementedError("codenerf.optim.AdamW: betas and eps must be shared by all groups")
        return betas, eps

    def _plan(self, advance: bool):
        """The step's segments [begin, end, lr, wd, step] over the parameters holding a gradient
        (state created on first use); ``advance``: count the step, as step() does."""
        segments = []
        for g in self.param_groups:
            lr, wd = float(g["lr"]), float(g["weight_decay"])
            for p in g["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0, dtype=torch.float32)
                    st["exp_avg"] = self._view("exp_avg", p)
                    st["exp_avg_sq"] = self._view("exp_avg_sq", p)
                if advance:
                    st["step"] += 1
                t = max(1, int(st["step"].item()))
                off = self._offs[p]
                end = off + _round_up(p.numel())
                if segments and segments[-1][1] == off and segments[-1][2:] == [lr, wd, t]:
                    segments[-1][1] = end
                else:
                    segments.append([off, end, lr, wd, t])
        return segments

    # ---- the captured form (codenerf.evaluate.GraphedEvalStep) ---------------------------
    def graph_step(self, scalars: torch.Tensor):
        """Enqueue a graph-capturable step (cn_adamw_step_dev): the same update as step(), its
        per-segment scalars read from ``scalars`` (device float32, 3 per segment) that
        graph_scalars() fills before each replay.  Every parameter must hold its flat gradient
        slice (zero_grad(set_to_none=False)).  Returns the segment count."""
        betas, eps = self._hyper()
        segments = self._plan(advance=False)
        assert segments and scalars.numel() >= 3 * len(segments), "graph_step: scalars too small"
        # the bounds are baked into the captured launch: graph_scalars() checks every later plan
        # has exactly these (a changed lr / wd / step pattern can merge or split segments)
        self._graph_bounds = [(b, e) for b, e, *_ in segments]
        f = self._flat
        ops.adamw_step_dev(f["param"], f["grad"], f["exp_avg"], f["exp_avg_sq"], segments, scalars, betas[0],
                           betas[1], eps)
        return len(segments)

    def graph_scalars(self, out) -> None:
        """Count one step (as step() does) and write its per-segment scalars into ``out`` (a float32
        numpy view of the pinned buffer a captured graph copies from)."""
        betas, _ = self._hyper()
        segments = self._plan(advance=True)
        bounds = getattr(self, "_graph_bounds", None)
        if bounds is not None and [(b, e) for b, e, *_ in segments] != bounds:
            raise RuntimeError("graph_scalars: the step's segments differ from the captured graph_step's "
                               f"({len(segments)} vs {len(bounds)}); per-group lr / weight_decay / step changes "
                               "that merge or split segments need a new capture")
        ops.adamw_scalars(segments, betas[0], betas[1], out)
        torch.autograd.graph.increment_version(list(self._offs))

    def state_dict(self):
        """torch.optim.AdamW's format; the moments are copied out of the flat buffers."""
        sd = super().state_dict()
        sd["state"] = {k: {n: (t.clone() if torch.is_tensor(t) else t) for n, t in v.items()}
                       for k, v in sd["state"].items()}
        return sd

    def load_state_dict(self, state_dict) -> None:
        super().load_state_dict(state_dict)
        self._adopt_state()

    # ---- data parallel ------------------------------------------------
    def allreduce_begin(self, n_groups: int, group=None) -> bool:
        """Start the all-reduce of the first ``n_groups`` parameter groups' gradients now, asynchronously
        (the first bucket of DDP's overlap, util.py:139-142): called from inside the backward once those
        gradients are final -- train_minibatch hands it to the render's FieldPair, which calls it right
        after both fields' weight gradients are enqueued -- so the collective runs while the rest of the
        backward (the code tables' dz, the pose / ray tail) does; allreduce_grads() then reduces the rest
        and waits for both.  On RCCL the collective's stream waits for the work enqueued so far and runs
        beside what follows.  Only when every parameter of those groups holds its gradient (else nothing
        starts and allreduce_grads() reduces everything at once).  -> whether it started."""
        if not (dist.is_available() and dist.is_initialized()) or getattr(self, "_pending_bucket", None):
            return False
        if dist.get_backend(group) not in self.bucket_backends:
            return False
        params = [p for g in self.param_groups[:n_groups] for p in g["params"]]
        if any(p.grad is None for p in params):
            return False
        with torch.no_grad():
            for p in params:
                view = self._view("grad", p)
                if p.grad.data_ptr() != view.data_ptr():
                    return False
        split = self._starts[n_groups]
        work = dist.all_reduce(self._grad_ext[:split], op=dist.ReduceOp.SUM, group=group, async_op=True)
        self._pending_bucket = (split, work, group)
        return True

    def allreduce_grads(self, group=None, average: bool = True) -> None:
        """Average the gradients over the process group (the reference's DDP, util.py:139-142):
        ONE all-reduce (SUM, then a division by the world size -- the same arithmetic on RCCL and
        gloo) of the flat gradient buffer with a per-parameter has-grad flag appended to it
        (``average=False``: the plain sum, for losses the ranks already weighted -- the ray-sharded
        eval step, codenerf.evaluate.sharded_eval_step).  A
        gradient missing on this rank counts as zero; a parameter without a gradient on every rank
        keeps ``grad = None``.

        No host synchronisation when every parameter holds a gradient here (every training step
        of the reference: each chunk runs both models and both code tables): the flags are a
        cached device tensor per has-grad pattern, copied into the buffer's tail, and only a rank
        that lacks some gradient reads the reduced flags back (to know whether another rank has
        it).  Every rank always issues the same single collective, whatever its pattern."""
        if not (dist.is_available() and dist.is_initialized()):
            return
        world = dist.get_world_size(group)
        # (world 1 runs the collective too, as DDP does: the same code path at every size)
        missing = set(self._sync_grads())
        params = list(self._offs)
        n = self._flat["grad"].numel()
        ext = self._grad_ext
        pattern = tuple(p not in missing for p in params)
        flags = self._flag_cache.get(pattern)
        if flags is None:
            flags = torch.tensor([1.0 if f else 0.0 for f in pattern], dtype=torch.float32).to(ext.device)
            self._flag_cache[pattern] = flags
        ext[n:n + len(params)].copy_(flags)
        for p in missing:
            self._view("grad", p).zero_()
        pending, self._pending_bucket = getattr(self, "_pending_bucket", None), None
        if pending is not None:
            # the first bucket went out during the backward (allreduce_begin): the rest now, then both done
            split, work, group0 = pending
            assert group0 is group, "allreduce_begin / allreduce_grads on different groups"
            dist.all_reduce(ext[split:], op=dist.ReduceOp.SUM, group=group)
            work.wait()
        else:
            dist.all_reduce(ext, op=dist.ReduceOp.SUM, group=group)
        if average:
            ext.div_(world)
        if missing:
            # which of this rank's missing parameters hold a gradient on SOME rank (DDP reduces
            # those; a parameter no rank touched keeps grad None, so step() skips it as torch does)
            anywhere = ext[n:n + len(params)].cpu().tolist()
            for i, p in enumerate(params):
                if p in missing and anywhere[i] > 0:
                    p.grad = self._view("grad", p)

    def broadcast_params(self, src: int = 0, group=None) -> None:
        """Start every replica from rank ``src``'s parameters (DDP's construction-time
        broadcast): one broadcast of the flat parameter buffer."""
        if dist.is_available() and dist.is_initialized():
            dist.broadcast(self._flat["param"], src=src, group=group)
