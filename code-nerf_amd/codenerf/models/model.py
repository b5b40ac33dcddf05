"""CodeNeRFModel / ShapeTextureEmbedding with the reference's parameter contract.

view_synthesis/models/model.py:87-194.  The nn.Linear submodules keep the
reference's names and shapes (state_dicts load unchanged, including
checkpoints written by train.py:129-138), but ``forward`` runs the fused gfx950
field kernel (cn_mlp_forward) instead of nine addmm/cat/relu chains.

Only the configuration every runnable reference config instantiates is
implemented on the GPU: hidden 256, shape/texture codes 256, 10 xyz and 4 dir
frequencies with the inputs included.  Other shapes construct (so checkpoints
can be inspected) but raise on forward.
"""
from __future__ import annotations

import os
from typing import List, Tuple

import numpy as np
import torch

from .. import ops

PARAM_ORDER = ("layer_xyz1", "layer_xyz2", "fc_out", "shape_code_layer1", "shape_code_layer2",
               "texture_code_layer1", "layer_dir1", "layer_dir2", "fc_rgb")


class CodeNeRFModel(torch.nn.Module):
    """model.py:123-194."""

    def __init__(self, hidden_size=128, num_embeddings=1, shape_code_size=128, texture_code_size=128,
                 num_encoding_fn_xyz=6, num_encoding_fn_dir=4, include_input_xyz=True, include_input_dir=True):
        super().__init__()
        self.hidden_size = hidden_size
        self.shape_code_size = shape_code_size
        self.texture_code_size = texture_code_size
        self.dim_xyz = (3 if include_input_xyz else 0) + 6 * num_encoding_fn_xyz
        self.dim_dir = (3 if include_input_dir else 0) + 6 * num_encoding_fn_dir
        h, c = hidden_size, shape_code_size
        self.layer_xyz1 = torch.nn.Linear(self.dim_xyz, h)
        self.layer_xyz2 = torch.nn.Linear(h + c, h)
        self.fc_out = torch.nn.Linear(h + c, c + 1)
        self.shape_code_layer1 = torch.nn.Linear(c, c)
        self.shape_code_layer2 = torch.nn.Linear(c, c)
        self.texture_code_layer1 = torch.nn.Linear(c, c)
        self.layer_dir1 = torch.nn.Linear(self.dim_dir + c, h)
        self.layer_dir2 = torch.nn.Linear(h, h)
        self.fc_rgb = torch.nn.Linear(h + texture_code_size, 3)
        # field-kernel arithmetic: "f32" (exact-product fp32 MFMA, the reference's precision;
        # default) or "bf16x3" (opt-in: 3-product bf16 split, fp32 accumulate, ~2^-17 relative
        # per product; parity-tested at the same tolerances incl. trained-magnitude weights)
        self.precision = os.environ.get("CODENERF_PRECISION", "f32")
        # arithmetic of the training backward's weight-gradient / dX GEMMs, independent of the
        # inference format: the reference trains fully in fp32
        self.train_precision = os.environ.get("CODENERF_TRAIN_PRECISION", "f32")
        self._packed = None
        self._packed_key = None

    # --- kernel plumbing -------------------------------------------------
    def supported(self) -> bool:
        return (self.hidden_size == 256 and self.shape_code_size == 256 and self.texture_code_size == 256
                and self.dim_xyz == 63 and self.dim_dir == 27)

    def _require_supported(self):
        if not self.supported():
            raise NotImplementedError(
                "the gfx950 field kernel implements CodeNeRFModel(hidden 256, codes 256, L_xyz 10, L_dir 4, "
                f"inputs included); got hidden {self.hidden_size}, codes {self.shape_code_size}/"
                f"{self.texture_code_size}, dims {self.dim_xyz}/{self.dim_dir}")

    def param_list(self) -> List[torch.Tensor]:
        out = []
        for name in PARAM_ORDER:
            lin = getattr(self, name)
            out += [lin.weight, lin.bias]
        return out

    def kernel_format(self) -> str:
        """The packed format (= field kernel) of this model's inference precision."""
        from .._lib import kernel_format
        return kernel_format(self.precision)

    def packed(self) -> torch.Tensor:
        """MFMA-fragment layout of the weights, repacked whenever a parameter changed."""
        self._require_supported()
        params = self.param_list()
        fmt = self.kernel_format()
        key = (fmt,) + tuple((p.data_ptr(), p._version) for p in params)
        if self._packed is None or self._packed_key != key:
            self._packed = ops.mlp_pack(params, fmt)
            self._packed_key = key
        return self._packed

    def code_bias(self, z_s: torch.Tensor, z_t: torch.Tensor) -> torch.Tensor:
        return ops.code_bias(self.param_list(), z_s, z_t)

    # --- reference API ---------------------------------------------------
    def forward(self, z_s: torch.Tensor, z_t: torch.Tensor, x: torch.Tensor = None, *, field=None) -> torch.Tensor:
        """model.py:160-194: per-row codes (M, 256) x2 and encoded rows (M, 90) -> (M, 4).

        ``field`` (the renderer's fused path, codenerf.nerf._field): keyword arguments of the fused
        encode + MLP field op over rays / depths instead of encoded rows; ``z_s`` / ``z_t`` are then
        the distinct code rows.  Routing it through ``forward`` lets a DistributedDataParallel
        wrapper (util.py:139-142) see the forward it synchronises the gradients of."""
        if field is not None:
            return _field_op(self, z_s, z_t, **field)
        self._require_supported()
        if torch.is_grad_enabled() and any(t.requires_grad for t in [z_s, z_t, x] + self.param_list()):
            from ..autograd import mlp_forward_autograd
            return mlp_forward_autograd(self, z_s, z_t, x)
        codes_s, codes_t, index = _dedupe_codes(z_s, z_t)
        cb = ops.code_bias(self.param_list(), codes_s, codes_t)
        return ops.mlp_forward(self.packed(), cb, x, index, precision=self.kernel_format())


def _field_op(m: CodeNeRFModel, cs, ct, rd, chunk_rows, fx, fd, pts=None, ro=None, z=None, code_index=None,
              pair=None):
    """The fused radiance field (encode + MLP) of ``m`` on distinct code rows cs / ct (``pair``: the render's
    autograd.FieldPair, or None)."""
    needs_grad = torch.is_grad_enabled() and (
        any(t is not None and t.requires_grad for t in (rd, cs, ct, pts, ro)) or
        any(p.requires_grad for p in m.param_list()))
    if needs_grad:
        from ..autograd import radiance_field_autograd
        return radiance_field_autograd(m, rd, cs, ct, chunk_rows, fx, fd, pts=pts, ro=ro, z=z,
                                       code_index=code_index, pair=pair)
    cb = m.code_bias(cs, ct)
    n_samples = pts.shape[1] if pts is not None else z.shape[1]
    return ops.radiance_field(m.packed(), cb, rd, n_samples, chunk_rows, fx, fd, pts=pts, ro=ro, z=z,
                              code_index=code_index, precision=m.kernel_format())


def _dedupe_codes(z_s: torch.Tensor, z_t: torch.Tensor):
    """Rows of an ``expand``-ed code tensor share storage: fold them to one code row."""
    if z_s.dim() == 2 and z_s.stride(0) == 0 and z_t.stride(0) == 0:
        return z_s[:1], z_t[:1], None
    return z_s, z_t, None


class CodeGradSink:
    """The code-table gradient rows the field backwards add into in place (cn_code_bias_backward_ws with
    accumulate_dz): row k of the shape and of the texture table's zeroed flat gradient slice
    (optim.AdamW.zero_grad), claimed by the first field backward that asks and handed to the tables as
    their .grad by _TableRow.backward.  Per model and step this replaces an add of the coarse and fine
    code gradients and one into the table row (nn.Embedding's backward, model.py:102-105)."""

    __slots__ = ("tables", "k", "bufs", "pending")

    def __init__(self, tables, k: int):
        self.tables, self.k, self.bufs, self.pending = tables, k, None, []

    def rows(self):
        """-> (shape row, texture row) views (1, code size) of the claimed gradient buffers, or None when a
        table is frozen, already has a .grad or has no zeroed slot (the gradients then flow through
        autograd as usual)."""
        if self.bufs is None:
            slots = [getattr(w, "_cn_grad_slot", None) for w in self.tables]
            if not all(s is not None and w.requires_grad and w.grad is None and s.is_contiguous()
                       for s, w in zip(slots, self.tables)):
                return None
            for w in self.tables:
                w._cn_grad_slot = None            # one use per zero_grad
            self.bufs = slots
        return tuple(b[self.k:self.k + 1] for b in self.bufs)

    def defer(self, params, g_code, workspace) -> bool:
        """Queue a field's dz (cn_code_dz job: its parameters, g_code and cn_code_bias_backward_act's
        workspace) for flush(); False (nothing queued) when rows() has no buffers to give."""
        if self.rows() is None:
            return False
        self.pending.append((params, g_code, workspace))
        return True

    def flush(self) -> None:
        """The queued fields' dz added into the claimed rows: ONE cn_code_dz launch for a render's two
        fields (in the order they were queued)."""
        from .. import ops
        while self.pending:
            jobs, self.pending = self.pending[:2], self.pending[2:]
            ops.code_dz(jobs, 1, dz_into=self.rows())

    def take(self):
        """-> the claimed buffers or None (after flush()), dropping the sink's references to them
        (AccumulateGrad then adopts them as .grad without a copy)."""
        self.flush()
        b, self.bufs = self.bufs, None
        return b


class _TableRow(torch.autograd.Function):
    """Row k of the shape and texture tables (nn.Embedding's lookup of one id) whose backward adds the
    row gradients into the tables' gradient buffers directly: the optimiser's zeroed flat-buffer slice
    when the table has no .grad yet this step (optim.AdamW.zero_grad), else a fresh zero table -- one
    small add per table instead of torch's dense zero fill + scatter + copy into .grad.  With a
    CodeGradSink the field backwards have already added theirs in place: the claimed buffers are
    returned as they are (plus any gradient that still came through autograd)."""

    @staticmethod
    def forward(ctx, w_s, w_t, k, sink=None):
        ctx.set_materialize_grads(False)
        ctx.k = k
        ctx.tables = (w_s, w_t)
        ctx.sink = sink
        return w_s.detach().narrow(0, k, 1), w_t.detach().narrow(0, k, 1)   # views: no copy

    @staticmethod
    def backward(ctx, g_s, g_t):
        sunk = ctx.sink.take() if ctx.sink is not None else None
        out = []
        for i, (w, g, need) in enumerate(zip(ctx.tables, (g_s, g_t), ctx.needs_input_grad[:2])):
            if not need:
                out.append(None)
                continue
            if sunk is not None:
                buf = sunk[i]
            elif g is None:
                out.append(None)
                continue
            elif w.shape[0] == 1:
                out.append(g)                     # a one-row "table" (the eval step's code leaf): g is its grad
                continue
            else:
                slot = getattr(w, "_cn_grad_slot", None)
                if slot is not None and w.grad is None:
                    w._cn_grad_slot = None            # one use per zero_grad
                    buf = slot
                else:
                    buf = torch.zeros_like(w)
            if g is not None:
                buf[ctx.k:ctx.k + 1].add_(g)
            out.append(buf)
        sunk = buf = None
        return out[0], out[1], None, None


def code_rows_with_sink(z_s: torch.Tensor, z_t: torch.Tensor):
    """One code row each (1, C) -- the eval step's optimised leaf codes -- as _TableRow views carrying a
    CodeGradSink (eval.py:145-163): the loss and both fields add their code gradients in place into the
    leaves' zeroed optimiser slots, handed back to autograd as the leaves' gradients.  The rows are
    returned unchanged when they do not need it (no gradient, more than one row)."""
    if not (torch.is_grad_enabled() and z_s.requires_grad and z_t.requires_grad and z_s.is_leaf and z_t.is_leaf
            and z_s.dim() == 2 and z_t.dim() == 2 and z_s.shape[0] == 1 and z_t.shape[0] == 1):
        return z_s, z_t
    sink = CodeGradSink((z_s, z_t), 0)
    rows_s, rows_t = _TableRow.apply(z_s, z_t, 0, sink)
    rows_s._cn_sink = rows_t._cn_sink = sink
    return rows_s, rows_t


class CodeRows:
    """The distinct code rows behind per-ray codes: z_s = shape_rows[index], z_t = texture_rows[index]."""

    __slots__ = ("shape_rows", "texture_rows", "index")

    def __init__(self, shape_rows: torch.Tensor, texture_rows: torch.Tensor, index: torch.Tensor):
        self.shape_rows, self.texture_rows, self.index = shape_rows, texture_rows, index


class ShapeTextureEmbedding(torch.nn.Module):
    """model.py:87-120: per-object shape / texture code tables."""

    def __init__(self, num_embeddings, shape_code_size=128, texture_code_size=128):
        super().__init__()
        self.num_embeddings = num_embeddings
        self.shape_code_size = shape_code_size
        self.texture_code_size = texture_code_size
        self.shape_embedding = torch.nn.Embedding(num_embeddings, shape_code_size)
        self.texture_embedding = torch.nn.Embedding(num_embeddings, texture_code_size)

    def forward(self, object_ids: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """model.py:102-105.  On the device the distinct ids are looked up once and the per-ray
        rows gathered from them; both returned tensors carry that factorisation
        (``_cn_code_rows``), so the field kernels run the per-object code layers once per
        object (one per 4096-ray chunk in train.py) instead of once per ray."""
        if object_ids.device.type != "cuda" or object_ids.dim() != 1:
            return self.shape_embedding(object_ids), self.texture_embedding(object_ids)
        host = getattr(object_ids, "_cn_host_ids", None)
        if host is not None and len(host) == object_ids.shape[0]:
            uniq_h = np.unique(np.asarray(host, dtype=np.int64))
            if uniq_h.shape[0] == 1:
                # one object (every train.py chunk of one image): its table rows as views and the
                # per-ray codes as their expand -- no id upload, no index search, no gathers; the
                # field kernels take the one code row (nerf._codes)
                k = int(uniq_h[0])
                tables = (self.shape_embedding.weight, self.texture_embedding.weight)
                sink = CodeGradSink(tables, k)
                rows_s, rows_t = _TableRow.apply(*tables, k, sink)
                rows_s._cn_sink = rows_t._cn_sink = sink
                n = object_ids.shape[0]
                z_s, z_t = rows_s.expand(n, -1), rows_t.expand(n, -1)
                tag = CodeRows(rows_s, rows_t, None)
                z_s._cn_code_rows = tag
                z_t._cn_code_rows = tag
                return z_s, z_t
            # the caller knows the ids on the host (codenerf.train: the batch's per-image ids): the
            # distinct ids go up as a pinned copy and the per-ray index is a device searchsorted --
            # torch.unique on the device would wait for the GPU (its output size) every chunk
            uniq_h = np.unique(np.asarray(host, dtype=np.int64))
            uniq = torch.from_numpy(uniq_h).pin_memory().to(object_ids.device, non_blocking=True)
            index = torch.searchsorted(uniq, object_ids.contiguous())
        else:
            uniq, index = torch.unique(object_ids, return_inverse=True)
        rows_s, rows_t = self.shape_embedding(uniq), self.texture_embedding(uniq)
        z_s, z_t = rows_s[index], rows_t[index]
        tag = CodeRows(rows_s, rows_t, index)
        z_s._cn_code_rows = tag
        z_t._cn_code_rows = tag
        return z_s, z_t

    def get_all_embeddings(self, device) -> Tuple[torch.Tensor, torch.Tensor]:
        idx = torch.arange(0, self.num_embeddings, dtype=torch.int64, device=device)
        return self.shape_embedding(idx), self.texture_embedding(idx)

    def get_params_tensor(self) -> Tuple[torch.Tensor, torch.Tensor]:
        shape, texture = None, None
        for name, p in self.named_parameters():
            if "shape" in name:
                shape = p.data.reshape(-1)
            if "texture" in name:
                texture = p.data.reshape(-1)
        return shape, texture


def get_params_tensor(model, is_distributed):
    """model.py:79-84 (a DDP wrapper or the bare module: both work, whatever ``is_distributed`` says)."""
    m = getattr(model, "module", model)
    return m.get_params_tensor()
