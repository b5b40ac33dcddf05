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
