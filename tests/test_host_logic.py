"""Host-side logic of the product path: rank split (Q5), chunking, Q1 index map, packing layout."""
import numpy as np
import pytest
import torch

from codenerf.utils import get_minibatches, mse2psnr, split_sizes
from oracle import codenerf_oracle as O


@pytest.mark.parametrize("n,k", [(16384, 1), (16384, 2), (16384, 3), (16384, 8), (1024, 3), (100, 7), (192, 3)])
def test_split_matches_reference_rule(n, k):
    assert split_sizes(n, k) == O.split_sizes(n, k)


def test_minibatches():
    x = torch.arange(10)
    assert [t.tolist() for t in get_minibatches(x, 4)] == [[0, 1, 2, 3], [4, 5, 6, 7], [8, 9]]


def test_mse2psnr():
    assert mse2psnr(0) == pytest.approx(50.0)
    assert mse2psnr(0.01) == pytest.approx(20.0)


def q1_dir_ray(ray, s, S, n_rays, chunk):
    """The field kernel's view-direction row map (mlp.hip), restated in Python."""
    base = (ray // chunk) * chunk
    rc = min(chunk, n_rays - base)
    return base + ((ray - base) * S + s) % rc


@pytest.mark.parametrize("n_rays,S,chunk", [(192, 8, 50), (100, 64, 4096), (37, 3, 10), (16384, 64, 4096)])
def test_q1_index_map_matches_repeat_semantics(n_rays, S, chunk):
    """row k = r*S+s of a chunk takes the view dir of ray k mod R (viewdirs.repeat([1,S,1]), nerf/__init__.py:127)."""
    for c0 in range(0, n_rays, chunk):
        r = min(chunk, n_rays - c0)
        ids = torch.arange(c0, c0 + r)[:, None].float()
        tiled = ids.repeat([1, S, 1]).reshape(-1)          # exactly the reference op on a (R,1) tensor
        got = [q1_dir_ray(c0 + k // S, k % S, S, n_rays, chunk) for k in range(r * S)]
        assert got == tiled.long().tolist()


def test_encoding_permutation_is_a_permutation():
    """mlp_layout.h k_from_enc: every encoded feature used exactly once across both lane halves."""
    def k_from_enc(t, h, P):
        if t < 2 * P:
            q = t if t < P else t - P
            p = 2 * q + h
            k, d = divmod(p, 3)
            return (3 if t < P else 6) + 6 * k + d
        raw = 2 * (t - 2 * P) + h
        return {0: 0, 1: 2, 2: 1}.get(raw, -1)
    for P, steps, dim in [(15, 32, 63), (6, 14, 27)]:
        got = sorted(k_from_enc(t, h, P) for t in range(steps) for h in (0, 1))
        assert got == [-1] + list(range(dim))


def test_acc_layout_is_a_permutation():
    rows = sorted(32 * (t >> 4) + (t & 3) + 8 * ((t >> 2) & 3) + 4 * h for t in range(128) for h in (0, 1))
    assert rows == list(range(256))


def test_synthetic_weights_are_deterministic():
    from codenerf import synthetic
    a, b = synthetic.codenerf_params(0), synthetic.codenerf_params(0)
    assert all(torch.equal(a[k], b[k]) for k in a)
    assert a["fc_out.bias"][0] > 4.0
    assert list(a) == [f"{n}.{p}" for n in ["layer_xyz1", "layer_xyz2", "fc_out", "shape_code_layer1",
                                            "shape_code_layer2", "texture_code_layer1", "layer_dir1", "layer_dir2",
                                            "fc_rgb"] for p in ["weight", "bias"]]


from test_gpu_grad import MASK_BAND, check_mask_agreement  # noqa: E402  (helpers only; no GPU needed)


def test_mask_checker_catches_a_flipped_bit():
    """A deliberately flipped ReLU decision at a large pre-activation fails check_mask_agreement
    (the guard that keeps the recorded-decision comparison from being self-fulfilling)."""
    g = torch.Generator().manual_seed(5)
    pre = {k: torch.randn(300, 256, generator=g) for k in ("h1", "h2", "v1", "v2")}
    masks = {k: (v > 0).float() for k, v in pre.items()}
    assert check_mask_agreement(masks, pre, MASK_BAND["bf16x3"]) == 0
    near = dict(masks)
    i = int(pre["h2"].abs().argmin())           # a kink-adjacent flip is allowed
    near["h2"] = masks["h2"].clone().view(-1)
    near["h2"][i] = 1.0 - near["h2"][i]
    near["h2"] = near["h2"].view(300, 256)
    if pre["h2"].view(-1)[i].abs() < MASK_BAND["bf16x3"] * pre["h2"].abs().max():
        assert check_mask_agreement(near, pre, MASK_BAND["bf16x3"]) == 1
    bad = dict(masks)
    j = int(pre["v1"].abs().argmax())
    bad["v1"] = masks["v1"].clone().view(-1)
    bad["v1"][j] = 1.0 - bad["v1"][j]
    bad["v1"] = bad["v1"].view(300, 256)
    with pytest.raises(AssertionError):
        check_mask_agreement(bad, pre, MASK_BAND["bf16x3"])


def test_bench_refuses_more_gpus_than_visible():
    """bench.py --gpus N with fewer than N visible GPUs fails loudly instead of reporting 1 rank."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, HIP_VISIBLE_DEVICES="0")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "64", "--steps", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode != 0
    assert "needs 64 visible GPUs" in (r.stderr + r.stdout)


def test_code_grad_sink_claims_zeroed_slots_once():
    """CodeGradSink (the in-place code-gradient rows): it claims the tables' zeroed optimiser slots only
    when every table is trainable, has no .grad yet and carries a slot; it hands out row k of each;
    queued dz jobs need those rows; take() drops its references; a second sink after the claim gets
    none (one use per zero_grad).  Host logic only (no launch)."""
    from codenerf.models.model import CodeGradSink
    ws = [torch.nn.Parameter(torch.randn(5, 4)) for _ in range(2)]
    assert CodeGradSink(ws, 2).rows() is None                  # no slots handed out
    for w in ws:
        w._cn_grad_slot = torch.zeros(5, 4)
    frozen = [torch.randn(5, 4), ws[1]]
    frozen[0]._cn_grad_slot = torch.zeros(5, 4)
    assert CodeGradSink(frozen, 2).rows() is None              # a table without requires_grad
    ws[1].grad = torch.zeros(5, 4)
    assert CodeGradSink(ws, 2).rows() is None                  # a table that already has a gradient
    assert ws[0]._cn_grad_slot is not None                     # nothing claimed on the way
    ws[1].grad = None
    slots = [w._cn_grad_slot for w in ws]
    sink = CodeGradSink(ws, 2)
    rows = sink.rows()
    assert rows is not None and all(r.shape == (1, 4) for r in rows)
    for r, s in zip(rows, slots):
        assert r.data_ptr() == s[2:3].data_ptr()
    assert all(w._cn_grad_slot is None for w in ws)            # claimed: one use per zero_grad
    assert sink.rows()[0].data_ptr() == rows[0].data_ptr()     # the same rows on every ask
    assert CodeGradSink(ws, 1).rows() is None                  # another sink finds no slot
    b = sink.take()                                            # nothing queued: no launch
    assert b is not None and b[0] is slots[0] and sink.bufs is None and sink.pending == []


def test_prep_plan_modes():
    """The pre-field launch RadianceField.forward plans (autograd._prep_plan): the eval step's fused
    mode with its accumulators (g_code, then d ro / d rd as wanted), the fp32 training mode with a
    zeroed g_code, none for an empty batch or a format the fused kernels do not take."""
    from codenerf import _lib, autograd as A
    meta = A._FieldMeta(64, 4096, [1.0] * 10, [1.0] * 4, precision="f32", train_precision="f32")
    frozen = (False, True, False, True, False, True, True) + (False,) * 18
    train = (False, False, False, False, False, True, True) + (True,) * 18
    stride = _lib.CN_CODE_BIAS_STRIDE
    assert A._prep_plan(meta, 1, 2048, frozen) == ("fused", stride + 6 * 2048)
    assert A._prep_plan(meta, 1, 2048, frozen[:3] + (False,) + frozen[4:]) == ("fused", stride + 3 * 2048)
    assert A._prep_plan(meta, 1, 4096, train) == ("train_w16", stride)
    assert A._prep_plan(meta, 0, 4096, train) == (None, 0)
    assert A._prep_plan(meta, 1, 0, train) == (None, 0)
    meta_v1 = A._FieldMeta(64, 4096, [1.0] * 10, [1.0] * 4, precision="f32_v1", train_precision="f32")
    assert A._prep_plan(meta_v1, 1, 4096, train) == (None, 0)
