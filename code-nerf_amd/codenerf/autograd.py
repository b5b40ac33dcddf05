"""torch.autograd.Function wrappers of the HIP ops.

The gradients ``loss.backward()`` takes through the reference's eval step
(test-time optimisation of pose + codes, view_synthesis/eval.py) and training
step: get_bundle -> sample gather -> point sampling (depths detached,
point_sampler.py:115) -> forward_pass / CodeNeRFModel.forward -> volume_render.
Every forward and backward runs on the gfx950 kernels through the C ABI;
torch only allocates buffers and routes gradients.

When no input requires grad each wrapper returns the plain op result and
records nothing.  The differentiable field runs, for frozen weights and a
bf16x3 model (the eval step), the 3xbf16 kernel with ReLU masks and the fused
backward kernel; otherwise the fp32 kernel (``cn_radiance_field_train``) that
stores the activations the layer-wise backward reads.
"""
from __future__ import annotations

import weakref
from typing import Sequence

import torch

from . import _lib, ops

# packed weights per model and format: repacked only when a parameter's storage or version changed
# (an optimiser step bumps the versions; see optim.AdamW).  Keyed by id() of the model's first
# parameter (tensors compare elementwise, so no WeakKeyDictionary); the entry leaves with it.
_PACKS = {}


def _pack_cache(owner, params):
    """(the owner's cache dict, the weights' signature): packs stay valid while ``params`` are unchanged."""
    sig = tuple((p.data_ptr(), p._version) for p in params)
    key = id(owner)
    ent = _PACKS.get(key)
    if ent is None or ent[0]() is not owner:
        ent = (weakref.ref(owner), {})
        _PACKS[key] = ent
        weakref.finalize(owner, _PACKS.pop, key, None)
    return ent[1], sig


def _packed(owner, params, fmt: str):
    """ops.mlp_pack(params, fmt), cached while ``params`` are unchanged (frozen weights of the eval
    loop pack once instead of twice per iteration)."""
    cache, sig = _pack_cache(owner, params)
    hit = cache.get(fmt)
    if hit is not None and hit[0] == sig:
        return hit[1]
    packed = ops.mlp_pack(params, fmt)
    cache[fmt] = (sig, packed)
    return packed


def _prepare_w16(owner, params, z_s, z_t, n_zero: int):
    """The fp32 training step's per-model preparation in ONE launch (ops.field_prepare): the code terms,
    the forward and backward packs where the cache lacks them (after every optimiser step), and a
    zeroed g_code accumulator for the fused backward -> (cb, packed "f32_w16", zero, code-layer activations)."""
    cache, sig = _pack_cache(owner, params)
    have = {f: (cache.get(f) is not None and cache[f][0] == sig) for f in ("f32_w16", "f32_w16_t")}
    ((cb, pk, pkt, zero, act),) = ops.field_prepare_models(
        [(params, not have["f32_w16"], not have["f32_w16_t"], n_zero)], z_s, z_t, want_act=True)
    if pk is not None:
        cache["f32_w16"] = (sig, pk)
    if pkt is not None:
        cache["f32_w16_t"] = (sig, pkt)
    return cb, cache["f32_w16"][1], zero, act


def _zkey(z_s, z_t):
    return (z_s.data_ptr(), z_s._version, tuple(z_s.shape), z_t.data_ptr(), z_t._version, tuple(z_t.shape))


def _prep_plan(meta, n_codes: int, n_rays: int, needs):
    """The pre-field launch RadianceField.forward makes -> (mode, n_zero): "train_w16" (code terms, the
    fp32 packs where missing, a zeroed g_code), "fused" (the eval step: code terms and the fused
    backward's zeroed accumulators) or (None, 0) (code_bias alone).  ``needs``: its needs_input_grad."""
    if n_rays == 0 or n_codes == 0:
        return None, 0
    if (meta.precision in ("bf16x3", "f32") and not any(needs[7:])
            and ops.fused_backward_supported(n_codes, meta.n_samples, meta.code_index, meta.precision)):
        return "fused", ops.field_backward_x3_acc_floats(n_codes, n_rays, needs[3], needs[1])
    if (meta.precision == meta.train_precision == "f32"
            and ops.fused_backward_supported(n_codes, meta.n_samples, meta.code_index, "f32")):
        return "train_w16", n_codes * _lib.CN_CODE_BIAS_STRIDE
    return None, 0


def prefetch_prepares(fields, z_s, z_t) -> bool:
    """The pre-field launches of a render's two fields (coarse and fine, on the same code rows) as ONE
    cn_field_prepare_models launch before the coarse field; each field's RadianceField.forward then
    takes its part (_take_prepared) instead of launching its own.  ``fields``: [(model, meta, n_rays,
    needs)] as RadianceField.apply will see them.  -> [(mode, zeroed buffer)] per field, or False
    (nothing launched) unless both plan one."""
    entries = []
    for model, meta, n_rays, needs in fields:
        mode, n_zero = _prep_plan(meta, z_s.shape[0], n_rays, needs)
        if mode is None:
            return False
        orig = model.param_list()
        params = [p.detach() for p in orig]
        cache, sig = _pack_cache(orig[0], params)
        have = {f: (cache.get(f) is not None and cache[f][0] == sig) for f in ("f32_w16", "f32_w16_t")}
        pack = mode == "train_w16" and not have["f32_w16"]
        pack_t = mode == "train_w16" and not have["f32_w16_t"]
        entries.append((cache, sig, mode, n_zero, params, pack, pack_t))
    outs = ops.field_prepare_models([(e[4], e[5], e[6], e[3]) for e in entries], z_s, z_t, want_act=True)
    key = _zkey(z_s, z_t)
    for (cache, sig, mode, n_zero, _, _, _), (cb, pk, pkt, zero, act) in zip(entries, outs):
        if pk is not None:
            cache["f32_w16"] = (sig, pk)
        if pkt is not None:
            cache["f32_w16_t"] = (sig, pkt)
        cache["prep"] = ((sig, mode, n_zero, key), (cb, zero, act))
    return [(e[2], o[3]) for e, o in zip(entries, outs)]


def _take_prepared(owner, params, z_s, z_t, mode, n_zero):
    """This field's part of a prefetch_prepares launch -> (cb, zero, act), or None (none, or stale)."""
    cache, sig = _pack_cache(owner, params)
    ent = cache.pop("prep", None)
    if ent is None or ent[0] != (sig, mode, n_zero, _zkey(z_s, z_t)):
        return None
    return ent[1]


_ONES = {}


def backward_from(loss) -> None:
    """loss.backward() for a scalar loss with a cached device 1.0 as its seed gradient: torch's
    ones_like seed is a fill launch per step (train.py:111, eval.py:160)."""
    key = (loss.device, loss.dtype)
    one = _ONES.get(key)
    if one is None:
        one = _ONES[key] = torch.ones((), device=loss.device, dtype=loss.dtype)
    loss.backward(one if loss.dim() == 0 else one.expand_as(loss))


class RaySink:
    """The ray gradients of a pose's rays (PoseRays) added up in place: ``buf`` = (d ro, d rd) (R, 3)
    zeroed buffers -- set by render_rays' prefetch (the fine field's zeroed accumulators) -- into which
    both volume renders and both fused field backwards add, returning no gradient; PoseRays.backward
    reads the sum.  Replaces four (R, 3) autograd adds per eval step (eval.py:145-163)."""

    __slots__ = ("buf", "hold")

    def __init__(self):
        self.buf = None
        self.hold = None     # a FieldPair whose first field waits: ray gradients arriving meanwhile go to it


_RAY_SINKS = [False]


class eval_ray_sinks:
    """Context in which pose_rays_autograd attaches a RaySink to the rays of leaf (theta, phi, rho):
    the eval step (evaluate.eval_step_loss) only.  Outside it the rays' consumers return their
    gradients through autograd as usual, so torch.autograd.grad / hooks on the rays see them."""

    def __enter__(self):
        self.prev = _RAY_SINKS[0]
        _RAY_SINKS[0] = True
        return self

    def __exit__(self, *exc):
        _RAY_SINKS[0] = self.prev
        return False


def _ray_sink(rd, ro=None):
    s = getattr(rd, "_cn_ray_sink", None)
    if s is None or (ro is not None and getattr(ro, "_cn_ray_sink", None) is not s):
        return None
    return s


def _needs_grad(*ts) -> bool:
    return torch.is_grad_enabled() and any(isinstance(t, torch.Tensor) and t.requires_grad for t in ts)


def _d(t):
    return None if t is None else t.detach()


# ------------------------------------------------------------------ rays


class RayBundle(torch.autograd.Function):
    """get_bundle (ray_sampler.py:84-99) -> ro, rd; gradient w.r.t. tform_cam2world."""

    @staticmethod
    def forward(ctx, dirs, c2w):
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(dirs)
        ctx.batch = c2w.shape[0]
        return ops.ray_bundle(dirs, c2w)

    @staticmethod
    def backward(ctx, g_ro, g_rd):
        if not ctx.needs_input_grad[1] or (g_ro is None and g_rd is None):
            return None, None
        (dirs,) = ctx.saved_tensors
        return None, ops.ray_bundle_backward(dirs, ctx.batch, _c(g_ro), _c(g_rd))


class GatherRays(torch.autograd.Function):
    """RaySampler.sample gather (ray_sampler.py:77-80); scatter-add backward."""

    @staticmethod
    def forward(ctx, ro, rd, sel):
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(sel)
        ctx.shape = ro.shape
        return ops.gather_rays(ro, rd, sel)

    @staticmethod
    def backward(ctx, g_o, g_d):
        if g_o is None and g_d is None:
            return None, None, None
        (sel,) = ctx.saved_tensors
        b = sel.shape[0]
        hw = ctx.shape.numel() // (3 * b)
        d_ro, d_rd = ops.gather_rays_backward(_c(g_o), _c(g_d), b, hw, sel)
        return d_ro.view(ctx.shape), d_rd.view(ctx.shape), None


class PoseRays(torch.autograd.Function):
    """pose_spherical (eval.py:22-38) + sample (ray_sampler.py:53-99) + target gather (eval.py:147-148),
    one launch each way.  The pose is (theta, phi, rho) -- gradients through the analytic d c2w --
    or a c2w (B, 4, 4) -- gradient d c2w, as get_bundle + gather's autograd."""

    @staticmethod
    def forward(ctx, dirs, theta, phi, rho, c2w, sel, target, sink=None):
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(dirs, theta, phi, rho, sel)
        ctx.sink = sink
        ctx.leaves = (theta, phi, rho)
        ctx.angles = theta is not None
        ctx.shapes = (theta.shape, phi.shape, rho.shape) if ctx.angles else None
        ctx.batch = theta.numel() if ctx.angles else c2w.shape[0]
        ro, rd, c2w_out, tgt = ops.pose_rays(dirs, theta, phi, rho, c2w=c2w, select_inds=sel, target=target)
        ctx.mark_non_differentiable(c2w_out)
        if tgt is not None:
            ctx.mark_non_differentiable(tgt)
        return ro, rd, c2w_out, tgt

    @staticmethod
    def backward(ctx, g_ro, g_rd, _g_c2w, _g_tgt):
        none = [None] * 8
        sink, ctx.sink = ctx.sink, None
        if sink is not None and sink.buf is not None:
            # the consumers that added their ray gradients in place (RaySink), plus any that did not
            s_ro, s_rd = sink.buf
            g_ro = s_ro if g_ro is None else s_ro + g_ro
            g_rd = s_rd if g_rd is None else s_rd + g_rd
        if g_ro is None and g_rd is None:
            return tuple(none)
        dirs, theta, phi, rho, sel = ctx.saved_tensors
        want_c2w = ctx.needs_input_grad[4]
        if ctx.angles and not any(ctx.needs_input_grad[1:4]):
            return tuple(none)
        if not ctx.angles and not want_c2w:
            return tuple(none)
        # the angle gradients straight into the optimiser's zeroed slots (autograd installs them as .grad)
        out = None
        if ctx.angles and all(ctx.needs_input_grad[1:4]):
            slots = [getattr(t, "_cn_grad_slot", None) if (t.is_leaf and t.grad is None) else None
                     for t in ctx.leaves]
            if all(sl is not None and sl.is_contiguous() for sl in slots):
                for t in ctx.leaves:
                    t._cn_grad_slot = None
                out = [sl.view(-1) for sl in slots]
        (dt, dp, dr), d_c2w = ops.pose_rays_backward(dirs, ctx.batch, _c(g_ro), _c(g_rd), theta, phi, rho,
                                                     select_inds=sel, want_c2w=want_c2w, out=out)
        if ctx.angles:
            for i, (g, sh) in enumerate(zip((dt, dp, dr), ctx.shapes)):
                none[1 + i] = g.view(sh) if ctx.needs_input_grad[1 + i] else None
        none[4] = d_c2w
        return tuple(none)


class SamplePoints(torch.autograd.Function):
    """pts = ro + rd * z with z detached (point_sampler.py:70, :115-118)."""

    @staticmethod
    def forward(ctx, ro, rd, z):
        ctx.save_for_backward(z)
        return ops.ray_points(ro, rd, z)

    @staticmethod
    def backward(ctx, g):
        (z,) = ctx.saved_tensors
        d_ro, d_rd = ops.ray_points_backward(g.contiguous(), z, ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        return d_ro, d_rd, None


class Posenc(torch.autograd.Function):
    """PositionalEmbedder.embed (position_embed.py:35-53)."""

    @staticmethod
    def forward(ctx, x, freqs, include_input):
        ctx.save_for_backward(x)
        ctx.freqs, ctx.include_input = list(freqs), bool(include_input)
        return ops.posenc(x, freqs, include_input)

    @staticmethod
    def backward(ctx, g):
        (x,) = ctx.saved_tensors
        return ops.posenc_backward(x, ctx.freqs, ctx.include_input, g.contiguous()), None, None


class VolumeRender(torch.autograd.Function):
    """volume_render (volumetric_render.py:36-66) -> rgb, disp, acc, weights, depth."""

    @staticmethod
    def forward(ctx, raw, z, rd):
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(raw, z, rd)
        ctx.ray_sink = _ray_sink(rd)
        return ops.volume_render(raw, z, rd)

    @staticmethod
    def backward(ctx, g_rgb, g_disp, g_acc, g_w, g_depth):
        if all(g is None for g in (g_rgb, g_disp, g_acc, g_w, g_depth)):
            return None, None, None
        raw, z, rd = ctx.saved_tensors
        sink, ctx.ray_sink = ctx.ray_sink, None
        if sink is not None and sink.hold is not None and sink.buf is not None and ctx.needs_input_grad[2]:
            # a paired field backward is waiting (FieldPair): this d rd is added in its place by the shared launch
            d_raw, d_rd = ops.volume_render_backward(raw, z, rd, _c(g_rgb), _c(g_disp), _c(g_acc), _c(g_w),
                                                     _c(g_depth), want_rd=True)
            pair = sink.hold
            pair.between = d_rd if pair.between is None else pair.between + d_rd
            return d_raw, None, None
        into = sink.buf[1] if (sink is not None and sink.buf is not None and ctx.needs_input_grad[2]) else None
        d_raw, d_rd = ops.volume_render_backward(raw, z, rd, _c(g_rgb), _c(g_disp), _c(g_acc), _c(g_w), _c(g_depth),
                                                 want_rd=ctx.needs_input_grad[2], d_rd_into=into)
        return d_raw, None, (None if into is not None else d_rd)


def _c(t):
    return None if t is None else t.contiguous()


# ------------------------------------------------------------------ field


class _FieldMeta:
    """Non-tensor arguments of the field Functions."""

    def __init__(self, n_samples, chunk_rows, fx, fd, code_index=None, precision="f32", train_precision="f32",
                 sink=None, ray_sink=None, pair=None):
        self.pair = pair       # FieldPair of a train step's render, or None
        self.n_samples, self.chunk_rows = n_samples, chunk_rows
        self.precision = precision
        self.train_precision = train_precision
        self.fx, self.fd = list(fx) if fx is not None else None, list(fd) if fd is not None else None
        self.code_index = code_index
        self.sink = sink       # models.model.CodeGradSink of the code rows, or None
        self.ray_sink = ray_sink   # RaySink of the rays, or None


def _code_grads(meta, params, z_s, z_t, g_code, pg, want_z, act=None):
    """The code backward -> (dz_s, dz_t); (None, None) when they go in place into the code tables'
    gradient rows (meta.sink: the coarse and fine fields of a one-object chunk add up there).  With the
    forward's code-layer activations (act, from the preparation launch): cn_code_bias_backward_act now
    and cn_code_dz -- for a sink deferred, so both fields' dz are one launch (CodeGradSink.flush);
    otherwise the recomputing two-launch form (cn_code_bias_backward_ws)."""
    if act is not None:
        ws = ops.code_ds_outer(params, z_s, z_t, act, g_code, pg)
        if not want_z:
            return None, None
        if meta.sink is not None and meta.sink.defer(params, g_code, ws):
            return None, None
        return ops.code_dz([(params, g_code, ws)], z_s.shape[0])
    rows = meta.sink.rows() if (want_z and meta.sink is not None) else None
    if rows is not None:
        ops.code_bias_backward(params, z_s, z_t, g_code, pg, dz_into=rows)
        return None, None
    return ops.code_bias_backward(params, z_s, z_t, g_code, pg, want_z=want_z)


class _Slots(list):
    """The optimiser's flat gradient slots handed to a backward (_param_grad_buffers)."""


def _param_grad_buffers(params, needs, orig=None):
    """Zeroed gradient buffers the backward kernels accumulate into: the optimizer's flat-buffer
    slices when every parameter still has no .grad this step (optim.AdamW.zero_grad), else fresh
    zeros."""
    if not any(needs):
        return None
    if orig is not None:
        slots = [getattr(p, "_cn_grad_slot", None) for p in orig]
        if all(s is not None and p.grad is None for s, p in zip(slots, orig)):
            for p in orig:
                p._cn_grad_slot = None       # one use per zero_grad
            # (no other reference to a slot may survive the backward: AccumulateGrad adopts a returned
            # gradient as .grad only when nothing else holds it -- else it clones, one copy per tensor)
            return _Slots(slots)
    return [torch.zeros_like(p) for p in params]


class FieldPair:
    """A step's two fields (predict_radiance_and_render's coarse and fine, nerf/__init__.py:81-89): their
    backwards are independent (the fine depths are detached, point_sampler.py:115), so the first one
    autograd reaches waits and the second runs both -- training: ONE cn_field_backward_train_multi call
    (one dX launch, one batched dW launch with layer_xyz1's dW among its jobs, one DIRS-pass launch and
    one reduction launch for the two); eval: ONE cn_field_backward_fused_multi call (one dX launch, one
    ray / g_code launch).  Every gradient is bitwise that of the per-field calls.  Armed by train_minibatch
    and eval_step_loss (paired_fields()): the waiting field hands its gradients over in place -- the
    optimiser's flat slots installed as .grad at once, the code rows' dz through the CodeGradSink, the
    rays' gradient into the pose's RaySink -- so it returns none through autograd."""

    __slots__ = ("pending", "kinds", "between", "sink", "on_grads")

    def __init__(self, on_grads=None):
        self.on_grads = on_grads    # training: called once both fields' weight gradients are enqueued
        self.pending = None
        self.kinds = []         # per field forward: "train" (fp32 training) or "fused" (fp32 eval); else None
        self.between = None     # eval: the rays' d rd that arrived while the first field waited
        self.sink = None        # eval: the RaySink held meanwhile

    def ready(self, kind) -> bool:
        return len(self.kinds) == 2 and self.kinds[0] == self.kinds[1] == kind


_PAIRING = [None]


class paired_fields:
    """Context in which render_rays pairs its two fields' backwards (FieldPair).  ``on_grads``: a callable
    the training pair calls (once) right after both fields' weight gradients are enqueued -- the data-
    parallel step starts its first gradient bucket there (optim.AdamW.allreduce_begin)."""

    def __init__(self, on_grads=None):
        self.on_grads = on_grads

    def __enter__(self):
        self.prev = _PAIRING[0]
        _PAIRING[0] = self
        return self

    def __exit__(self, *exc):
        _PAIRING[0] = self.prev
        return False


def new_field_pair():
    """render_rays: a FieldPair for its two fields inside paired_fields(), else None."""
    ctx = _PAIRING[0]
    return FieldPair(ctx.on_grads) if (ctx is not None and torch.is_grad_enabled()) else None


def _pair_flush(pair):
    """End of the backward pass (queued by the waiting field): a field whose partner never ran its
    backward runs alone.  Its code gradient must still reach the code rows' sink."""
    if pair.pending is None:
        return
    job, post = pair.pending
    pair.pending = None
    meta, params, z_s, z_t, pg, want_z, act = post
    if want_z and (meta.sink is None or meta.sink.rows() is None):
        raise RuntimeError("paired field backward: the partner field never ran and the code rows' gradient "
                           "buffers were already handed out")
    if pair.kinds[0] == "fused":
        sink, pair.sink = pair.sink, None
        sink.hold = None
        r = ops.field_backward_x3(**job)
        if pair.between is not None:
            r["d_rd"].add_(pair.between)
            pair.between = None
    else:
        r = ops.field_backward_train_multi([job], meta.precision)[0]
    _code_grads(meta, params, z_s, z_t, r["g_code"], pg, want_z, act)


def _code_grads_pair(first, second):
    """_code_grads of a FieldPair's two fields (first: the one that waited) with their first halves in one
    launch (cn_code_bias_backward_act_multi); their dz queued in that order.  Each item: (meta, params, z_s,
    z_t, g_code, pg, want_z, act) with act given.  -> (dz_s, dz_t) of the second."""
    items = (first, second)
    wss = ops.code_ds_outer_multi([(it[1], it[7], it[4], it[5]) for it in items], first[2], first[3])
    out = None
    for (meta, params, z_s, z_t, g_code, pg, want_z, act), ws in zip(items, wss):
        out = (None, None)
        if not want_z:
            continue
        if meta.sink is not None and meta.sink.defer(params, g_code, ws):
            continue
        out = ops.code_dz([(params, g_code, ws)], z_s.shape[0])
    return out


class RadianceField(torch.autograd.Function):
    """forward_pass (nerf/__init__.py:94-134) + CodeNeRFModel.forward (model.py:160-194), fused.

    Inputs: rd (R,3), pts (R,S,3) or (ro (R,3), z (R,S)), code rows z_s/z_t (n_codes, 256),
    then the 18 parameters in state_dict order.  Output raw (R, S, 4).

    With frozen weights (the eval step) the forward is the field kernel of the model's
    precision writing ReLU masks and the backward ONE fused kernel (cn_field_backward_fused:
    fp32 16x16x4 for "f32", 3xbf16 for "bf16x3"); with weight gradients the same kernel pair
    also keeps the activations and the layer-input gradients for the dW GEMMs
    (cn_field_backward_train_fmt) when precision == train_precision.
    """

    @staticmethod
    def forward(ctx, meta, rd, pts, ro, z, z_s, z_t, *params):
        ctx.orig_params = params
        ctx.owner = params[0]
        params = [p.detach() for p in params]
        n_rays = rd.shape[0]
        ctx.empty = n_rays == 0 or z_s.shape[0] == 0
        if ctx.empty:      # a zero-ray batch: empty raw, and no gradient flows back (backward)
            return torch.empty(n_rays, meta.n_samples, 4, device=rd.device, dtype=torch.float32)
        mode, n_zero = _prep_plan(meta, z_s.shape[0], n_rays, ctx.needs_input_grad)
        fused = ctx.fused = mode == "fused"
        train_w16 = mode == "train_w16"
        ctx.g_code = None
        ctx.acc = None
        ctx.code_act = None        # the code layers' activations (the code backward's operand)
        # a render's two fields may have been prepared together (prefetch_prepares)
        pre = _take_prepared(ctx.owner, params, z_s, z_t, mode, n_zero) if mode else None
        if train_w16:
            # the fp32 training step: code terms, both packs and the backward's zeroed g_code, one launch
            nc = z_s.shape[0]
            if pre is not None:
                (cb, zero, ctx.code_act), packed_w16 = pre, _packed(ctx.owner, params, "f32_w16")
            else:
                cb, packed_w16, zero, ctx.code_act = _prepare_w16(ctx.owner, params, z_s, z_t, n_zero)
            ctx.g_code = zero.view(nc, _lib.CN_CODE_BIAS_STRIDE)
        elif fused:
            # the eval step (frozen weights, packs cached): the code terms and the fused backward's zeroed
            # accumulators (g_code, d ro, d rd) in one launch
            if pre is None:
                pre = ops.field_prepare_models([(params, False, False, n_zero)], z_s, z_t, want_act=True)[0]
                pre = (pre[0], pre[3], pre[4])
            cb, ctx.acc, ctx.code_act = pre
        else:
            cb = ops.code_bias(params, z_s, z_t)
        if fused:
            if meta.pair is not None:
                meta.pair.kinds.append("fused" if meta.precision == "f32" else None)
            pack = "bf16x3" if meta.precision == "bf16x3" else "f32_w16"
            raw, masks = ops.radiance_field_masks(_packed(ctx.owner, params, pack), cb, rd, meta.n_samples,
                                                  meta.chunk_rows, meta.fx, meta.fd, pts=pts, ro=ro, z=z,
                                                  code_index=meta.code_index, precision=meta.precision)
            ctx.masks = masks
            ctx.meta = meta
            ctx.save_for_backward(rd, pts, ro, z, z_s, z_t, *params)
            return raw
        # weights trained: the training forward keeps the activations.  precision == train_precision
        # ("f32": the 16x16x4 kernel, "bf16x3": the 3xbf16 kernel) with one code row per wave: that
        # kernel + the fused training backward; otherwise the fp32 32x32x2 kernel + the layer-wise
        # backward
        ctx.train_fused = (meta.precision == meta.train_precision and meta.precision in ("f32", "bf16x3")
                           and ops.fused_backward_supported(z_s.shape[0], meta.n_samples, meta.code_index,
                                                            meta.precision))
        ctx.masks = None
        if meta.pair is not None:
            meta.pair.kinds.append("train" if (ctx.train_fused and meta.precision == "f32") else None)
        if ctx.train_fused:
            x3 = meta.precision == "bf16x3"
            raw, saved, ctx.masks = ops.radiance_field_train_w16(
                packed_w16 if train_w16 else _packed(ctx.owner, params, "bf16x3"), cb, rd, meta.n_samples, meta.chunk_rows,
                meta.fx, meta.fd, pts=pts, ro=ro, z=z, code_index=meta.code_index, precision=meta.precision)
        else:
            raw, saved = ops.radiance_field_train(ops.mlp_pack(params, "f32"), cb, rd, meta.n_samples,
                                                  meta.chunk_rows, meta.fx, meta.fd, pts=pts, ro=ro, z=z,
                                                  code_index=meta.code_index)
        # the fused training backward generates the encodings inside its dW kernels
        ctx.x_enc = None if ctx.train_fused else ops.encode_inputs(rd, meta.n_samples, meta.chunk_rows, meta.fx,
                                                                   meta.fd, pts=pts, ro=ro, z=z)
        ctx.meta, ctx.acts = meta, saved
        ctx.save_for_backward(rd, pts, ro, z, z_s, z_t, *params)
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        if ctx.empty:
            return (None,) * len(ctx.needs_input_grad)
        rd, pts, ro, z, z_s, z_t, *params = ctx.saved_tensors
        needs = ctx.needs_input_grad
        meta = ctx.meta
        if ctx.fused:
            want_z = needs[5] or needs[6]
            pack_t = "bf16x3_t" if meta.precision == "bf16x3" else "f32_w16_t"
            # the rays' gradients added in place into the pose's RaySink (no autograd sums)
            rs = meta.ray_sink
            ray_into = rs.buf if (rs is not None and rs.buf is not None and needs[1] and needs[3]) else None
            job = dict(packed_t=_packed(ctx.owner, params, pack_t), masks=ctx.masks, d_raw=g_raw.contiguous(),
                       n_rays=rd.shape[0], n_samples=meta.n_samples, chunk_rows=meta.chunk_rows, n_codes=z_s.shape[0],
                       freqs_xyz=meta.fx, freqs_dir=meta.fd, rd=rd, pts=pts, ro=ro, z=z, code_index=meta.code_index,
                       want_pts=needs[2], want_ro=needs[3], want_rd=needs[1], precision=meta.precision, acc=ctx.acc,
                       ray_into=ray_into)
            act = ctx.code_act
            ctx.acc = ctx.code_act = ctx.masks = None
            post = (meta, params, z_s, z_t, None, want_z, act)
            pair = meta.pair
            if pair is not None and pair.ready("fused"):
                # a field pairs when everything it returns goes in place -- the rays' gradient into the pose's
                # RaySink, the codes' through the code rows' sink -- and the shared launch takes its shape
                pairable = (ray_into is not None and act is not None and not needs[2] and z_s.shape[0] == 1
                            and meta.n_samples % 16 == 0 and pts is None
                            and (not want_z or (meta.sink is not None and meta.sink.rows() is not None)))
                if pair.pending is None:
                    if pairable:         # the first of the pair waits for the other
                        pair.pending = (job, post)
                        pair.sink, rs.hold = rs, pair
                        torch.autograd.Variable._execution_engine.queue_callback(lambda: _pair_flush(pair))
                        return (None,) * len(needs)
                elif not pairable:
                    _pair_flush(pair)    # the waiting one alone (its sums, then the held d rd), then this one
                else:
                    other_job, other_post = pair.pending
                    pair.pending = None
                    pair.sink.hold, pair.sink = None, None
                    between, pair.between = pair.between, None
                    r_other, r = ops.field_backward_x3_multi([other_job, job], d_rd_between=between)
                    dz_s, dz_t = _code_grads_pair(other_post[:4] + (r_other["g_code"],) + other_post[4:],
                                                  post[:4] + (r["g_code"],) + post[4:])
                    return (None, None, r["d_pts"], None, None, dz_s, dz_t, *([None] * len(params)))
            r = ops.field_backward_x3(**job)
            dz_s = dz_t = None
            if want_z:
                dz_s, dz_t = _code_grads(meta, params, z_s, z_t, r["g_code"], None, True, act)
            d_ro, d_rd = (None, None) if ray_into is not None else (r["d_ro"], r["d_rd"])
            return (None, d_rd, r["d_pts"], d_ro, None, dz_s, dz_t, *([None] * len(params)))
        orig = ctx.orig_params
        pg = _param_grad_buffers(params, needs[7:], orig)
        slots = isinstance(pg, _Slots)
        ctx.orig_params = None
        want_z = needs[5] or needs[6]
        if ctx.train_fused:
            x3 = meta.precision == "bf16x3"
            job = dict(packed_t=_packed(ctx.owner, params, "bf16x3_t" if x3 else "f32_w16_t"), params=params,
                       masks=ctx.masks, saved=ctx.acts, x_enc=ctx.x_enc, d_raw=g_raw.contiguous(), n_rays=rd.shape[0],
                       n_samples=meta.n_samples, chunk_rows=meta.chunk_rows, n_codes=z_s.shape[0], freqs_xyz=meta.fx,
                       freqs_dir=meta.fd, rd=rd, pts=pts, ro=ro, z=z, code_index=meta.code_index, param_grads=pg,
                       want_pts=needs[2], want_ro=needs[3], want_rd=needs[1], g_code=ctx.g_code)
            act, ctx.acts, ctx.x_enc, ctx.masks, ctx.g_code, ctx.code_act = ctx.code_act, None, None, None, None, None
            post = (meta, params, z_s, z_t, pg, want_z, act)
            pair = meta.pair
            if pair is not None and pair.ready("train") and not x3:
                if pair.pending is None:
                    # the first of the pair waits for the other: only when everything it returns goes in place
                    # (the flat slots as .grad now, the code rows through the sink) and no ray gradient is wanted
                    if (slots and act is not None and not any(needs[1:4])
                            and (not want_z or (meta.sink is not None and meta.sink.rows() is not None))):
                        pair.pending = (job, post)
                        for p, g in zip(orig, pg):
                            p.grad = g                  # filled by the shared launch, on the stream
                        torch.autograd.Variable._execution_engine.queue_callback(lambda: _pair_flush(pair))
                        return (None,) * len(needs)
                else:
                    other_job, other_post = pair.pending
                    pair.pending = None
                    r_other, r = ops.field_backward_train_multi([other_job, job], meta.precision)
                    if act is not None and other_post[6] is not None:
                        dz_s, dz_t = _code_grads_pair(other_post[:4] + (r_other["g_code"],) + other_post[4:],
                                                      post[:4] + (r["g_code"],) + post[4:])
                    else:
                        _code_grads(*other_post[:4], r_other["g_code"], *other_post[4:])
                        dz_s, dz_t = _code_grads(meta, params, z_s, z_t, r["g_code"], pg, want_z, act)
                    if pair.on_grads is not None and slots:
                        for p, g in zip(orig, pg):
                            p.grad = g               # (autograd then finds .grad set and adds nothing: None below)
                        on_grads, pair.on_grads = pair.on_grads, None
                        on_grads()
                        return (None, None, None, None, None, dz_s, dz_t, *([None] * len(params)))
                    grads = pg if pg is not None else [None] * len(params)
                    return (None, r["d_rd"], r["d_pts"], r["d_ro"], None, dz_s, dz_t, *grads)
            r = ops.field_backward_train(precision=meta.precision, **job)
            dz_s, dz_t = _code_grads(meta, params, z_s, z_t, r["g_code"], pg, want_z, act)
            grads = pg if pg is not None else [None] * len(params)
            return (None, r["d_rd"], r["d_pts"], r["d_ro"], None, dz_s, dz_t, *grads)
        r = ops.field_backward(params, ctx.acts, ctx.x_enc, g_raw.contiguous(), rd.shape[0], meta.n_samples,
                               meta.chunk_rows, z_s.shape[0], meta.fx, meta.fd, rd=rd, pts=pts, ro=ro, z=z,
                               code_index=meta.code_index, param_grads=pg, want_code=want_z or pg is not None,
                               want_pts=needs[2], want_ro=needs[3], want_rd=needs[1],
                               precision=meta.train_precision)
        dz_s = dz_t = None
        if r["g_code"] is not None:
            dz_s, dz_t = _code_grads(meta, params, z_s, z_t, r["g_code"], pg, want_z)
        ctx.acts = ctx.x_enc = None
        grads = pg if pg is not None else [None] * len(params)
        return (None, r["d_rd"], r["d_pts"], r["d_ro"], None, dz_s, dz_t, *grads)


class MLPForward(torch.autograd.Function):
    """CodeNeRFModel.forward(z_s, z_t, x) on encoded rows (model.py:160-194)."""

    @staticmethod
    def forward(ctx, train_precision, x, z_s, z_t, *params):
        ctx.train_precision = train_precision
        params = [p.detach() for p in params]
        cb = ops.code_bias(params, z_s, z_t)
        packed = ops.mlp_pack(params, "f32")
        raw, saved = ops.mlp_forward_train(packed, cb, x)
        ctx.acts = saved
        ctx.save_for_backward(x, z_s, z_t, *params)
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        x, z_s, z_t, *params = ctx.saved_tensors
        needs = ctx.needs_input_grad[1:]
        pg = _param_grad_buffers(params, needs[3:])
        want_z = needs[1] or needs[2]
        m = x.shape[0]
        r = ops.field_backward(params, ctx.acts, x, g_raw.contiguous(), m, 1, m, z_s.shape[0], param_grads=pg,
                               want_code=want_z or pg is not None, want_x=needs[0], precision=ctx.train_precision)
        dz_s = dz_t = None
        if r["g_code"] is not None:
            dz_s, dz_t = ops.code_bias_backward(params, z_s, z_t, r["g_code"], pg, want_z=want_z)
        ctx.acts = None
        grads = pg if pg is not None else [None] * len(params)
        return (None, r.get("d_x"), dz_s, dz_t, *grads)


# ------------------------------------------------------------------ loss


class RenderLoss(torch.autograd.Function):
    """The step's loss (train.py:103-108, eval.py:157-163) -> total (scalar) and the (6,) stats
    [coarse, fine, regulariser, total, ||z_s||, ||z_t||] (not differentiable)."""

    @staticmethod
    def forward(ctx, rgb_c, rgb_f, target, z_s, z_t, expand, lam, psnr=None):
        ctx.set_materialize_grads(False)
        stats = ops.render_loss(rgb_c, rgb_f, target, z_s, z_t, expand, lam, psnr=psnr)
        ctx.save_for_backward(rgb_c, rgb_f, target, z_s, z_t, stats)
        ctx.expand, ctx.lam = expand, lam
        sink = getattr(z_s, "_cn_sink", None) if z_s is not None else None
        ctx.code_sink = sink if (sink is not None and getattr(z_t, "_cn_sink", None) is sink) else None
        ctx.mark_non_differentiable(stats)
        return stats[3], stats

    @staticmethod
    def backward(ctx, g_total, _g_stats):
        sink, ctx.code_sink = ctx.code_sink, None
        if g_total is None:
            return (None,) * 8
        rgb_c, rgb_f, target, z_s, z_t, stats = ctx.saved_tensors
        want = ctx.needs_input_grad[:2] + ctx.needs_input_grad[3:5]
        # the code rows' gradient added in place into their CodeGradSink (the eval step's codes): the field
        # backwards add theirs there too, no autograd sums
        rows = sink.rows() if (sink is not None and want[2] and want[3]) else None
        d = ops.render_loss_backward(rgb_c, rgb_f, target, z_s, z_t, ctx.expand, ctx.lam, stats,
                                     g_total.reshape(1).contiguous(), want,
                                     dz_into=None if rows is None else tuple(r.reshape(-1) for r in rows))
        if rows is not None:
            return d[0], d[1], None, None, None, None, None, None
        return d[0], d[1], None, d[2], d[3], None, None, None


def render_loss_autograd(rgb_c, rgb_f, target, z_s=None, z_t=None, expand: int = 1, lam: float = 0.0,
                         psnr=None):
    """-> (total loss, stats (6,)).  The regulariser is differentiated only where z_s / z_t require grad.
    ``psnr`` (float64 device scalar, optional): mse2psnr of the fine loss, written by the same launch."""
    tgt = target.detach()
    if not _needs_grad(rgb_c, rgb_f, z_s, z_t):
        stats = ops.render_loss(_d(rgb_c), _d(rgb_f), tgt, _d(z_s), _d(z_t), expand, lam, psnr=psnr)
        return stats[3], stats
    return RenderLoss.apply(rgb_c, rgb_f, tgt, z_s, z_t, expand, lam, psnr)


# ------------------------------------------------------------------ entry points used by the package


def ray_bundle_autograd(dirs, c2w):
    if not _needs_grad(c2w):
        return ops.ray_bundle(dirs, c2w.detach())
    return RayBundle.apply(dirs.detach(), c2w)


def pose_rays_autograd(dirs, theta=None, phi=None, rho=None, c2w=None, sel=None, target=None):
    """(theta, phi, rho) or c2w -> ro, rd (B*S, 3), c2w (B, 4, 4), target rows (B*S, C) | None."""
    tgt = None if target is None else target.detach()
    if not _needs_grad(theta, phi, rho, c2w):
        return ops.pose_rays(dirs, _d(theta), _d(phi), _d(rho), c2w=_d(c2w), select_inds=sel, target=tgt)
    # the eval step (pose leaves optimised by eval.py:145-167, inside eval_ray_sinks()): the rays' consumers
    # sum their gradients in place (RaySink; torch.autograd.grad w.r.t. these rays themselves then sees
    # none -- w.r.t. the pose leaves it is exact).  Elsewhere the rays' gradients flow through autograd.
    leaves = theta is not None and all(t is not None and t.is_leaf and t.requires_grad for t in (theta, phi, rho))
    sink = RaySink() if (leaves and _RAY_SINKS[0]) else None
    ro, rd, c2w_out, tgt_out = PoseRays.apply(dirs.detach(), theta, phi, rho, c2w, sel, tgt, sink)
    if sink is not None:
        ro._cn_ray_sink = rd._cn_ray_sink = sink
    return ro, rd, c2w_out, tgt_out


def gather_rays_autograd(ro, rd, sel):
    if not _needs_grad(ro, rd):
        return ops.gather_rays(ro.detach(), rd.detach(), sel)
    return GatherRays.apply(ro, rd, sel)


def sample_points_autograd(ro, rd, z):
    """pts = ro + rd * z for sorted depths z (detached, point_sampler.py:70,115-118)."""
    if not _needs_grad(ro, rd):
        return ops.ray_points(ro.detach(), rd.detach(), z.detach())
    return SamplePoints.apply(ro, rd, z.detach())


def posenc_autograd(x, freqs: Sequence[float], include_input: bool):
    if not _needs_grad(x):
        return ops.posenc(x.detach(), freqs, include_input)
    return Posenc.apply(x, list(freqs), include_input)


def volume_render_autograd(raw, z, rd):
    if not _needs_grad(raw, rd):
        return ops.volume_render(raw.detach(), z.detach(), rd.detach())
    return VolumeRender.apply(raw, z.detach(), rd)


def _code_rows(z_s, z_t):
    """One code row when the per-row codes are an expand() of one row, else one per row."""
    if z_s.dim() == 2 and z_s.stride(0) == 0 and z_t.stride(0) == 0:
        from .nerf import _expand_base
        return _expand_base(z_s), _expand_base(z_t)
    return z_s, z_t


def mlp_forward_autograd(model, z_s, z_t, x):
    cs, ct = _code_rows(z_s, z_t)
    return MLPForward.apply(getattr(model, "train_precision", "f32"), x, cs, ct, *model.param_list())


def _field_meta(model, cs, ct, n_samples, chunk_rows, fx, fd, code_index, rd=None, ro=None, pair=None):
    sink = getattr(cs, "_cn_sink", None)
    return _FieldMeta(n_samples, chunk_rows, fx, fd, code_index=code_index,
                      precision=getattr(model, "precision", "f32"),
                      train_precision=getattr(model, "train_precision", "f32"),
                      sink=sink if sink is not None and getattr(ct, "_cn_sink", None) is sink else None,
                      ray_sink=_ray_sink(rd, ro) if (rd is not None and ro is not None) else None, pair=pair)


def radiance_field_autograd(model, rd, z_s, z_t, chunk_rows, fx, fd, pts=None, ro=None, z=None, code_index=None,
                            pair=None):
    cs, ct = (z_s, z_t) if code_index is not None else _code_rows(z_s, z_t)
    n_samples = pts.shape[1] if pts is not None else z.shape[1]
    meta = _field_meta(model, cs, ct, n_samples, chunk_rows, fx, fd, code_index, rd, ro, pair)
    return RadianceField.apply(meta, rd, pts, ro, _d(z), cs, ct, *model.param_list())


def prefetch_render_prepares(coarse, fine, rd, ro, cs, ct, n_coarse, n_fine, chunk_rows, fx, fd,
                             code_index=None) -> bool:
    """render_rays' hook: both fields' pre-field launches in one (prefetch_prepares) when both run the
    differentiable field on the rays-and-depths form (coarse n_coarse, fine n_fine samples per ray)."""
    if not torch.is_grad_enabled():
        return False
    fields = []
    for model, n_s in ((coarse, n_coarse), (fine, n_fine)):
        params = model.param_list()
        needs = (False, rd.requires_grad, False, ro.requires_grad, False, cs.requires_grad, ct.requires_grad,
                 *[p.requires_grad for p in params])
        if not any(needs):
            return False                  # _field_op takes the no-grad path
        fields.append((model, _field_meta(model, cs, ct, n_s, chunk_rows, fx, fd, code_index), rd.shape[0], needs))
    done = prefetch_prepares(fields, cs, ct)
    sink = _ray_sink(rd, ro)
    if done and sink is not None and rd.requires_grad and ro.requires_grad and all(m == "fused" for m, _ in done):
        # the rays' gradient sums live in the fine field's zeroed d ro / d rd accumulators
        # (field_backward_x3's layout: g_code, d ro, d rd)
        acc, n = done[1][1], rd.shape[0]
        sink.buf = (acc[acc.numel() - 6 * n:acc.numel() - 3 * n].view(n, 3), acc[acc.numel() - 3 * n:].view(n, 3))
    return bool(done)
