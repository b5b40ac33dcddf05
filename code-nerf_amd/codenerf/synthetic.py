"""Deterministic synthetic inputs for tests and benchmarks (no datasets offline).

Weights follow torch's default ``nn.Linear`` bounds (U(-1/sqrt(fan_in),
1/sqrt(fan_in)) for weight and bias) but are drawn from a counter-based hash
(splitmix64), so the same tensors are regenerated anywhere without storing
2.47 MB per model in fixtures.  ``fc_out.bias[0] += sigma_bias`` keeps the
field from being transparent.

Parameter names and shapes are the reference's state_dict contract
(view_synthesis/models/model.py:145-156).
"""
from __future__ import annotations

from collections import OrderedDict
from typing import Dict

import numpy as np
import torch

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
        z = x
        z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
        z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
        return z ^ (z >> np.uint64(31))


def hash_uniform(seed: int, stream: int, n: int) -> np.ndarray:
    """n float32 values in [-1, 1) from (seed, stream, index)."""
    idx = np.arange(n, dtype=np.uint64)
    base = np.uint64((seed * 1000003 + stream * 7919) & 0xFFFFFFFF) << np.uint64(32)
    h = _splitmix64(idx | base)
    u = (h >> np.uint64(40)).astype(np.float64) / float(1 << 24)
    return (2.0 * u - 1.0).astype(np.float32)


def layer_shapes(hidden: int = 256, code: int = 256, num_xyz: int = 10, num_dir: int = 4,
                 include_xyz: bool = True, include_dir: bool = True) -> "OrderedDict[str, tuple]":
    """(out, in) of every Linear in CodeNeRFModel, in the reference's order."""
    dx = (3 if include_xyz else 0) + 6 * num_xyz
    dd = (3 if include_dir else 0) + 6 * num_dir
    return OrderedDict([
        ("layer_xyz1", (hidden, dx)),
        ("layer_xyz2", (hidden, hidden + code)),
        ("fc_out", (code + 1, hidden + code)),
        ("shape_code_layer1", (code, code)),
        ("shape_code_layer2", (code, code)),
        ("texture_code_layer1", (code, code)),
        ("layer_dir1", (hidden, dd + code)),
        ("layer_dir2", (hidden, hidden)),
        ("fc_rgb", (3, hidden + code)),
    ])


def codenerf_params(seed: int = 0, hidden: int = 256, code: int = 256, num_xyz: int = 10,
                    num_dir: int = 4, sigma_bias: float = 5.0, weight_scale: float = 1.0) -> Dict[str, torch.Tensor]:
    """A CodeNeRFModel state_dict (CPU fp32) from the counter hash.

    ``weight_scale`` multiplies every weight (not the biases): 1 is torch's init scale;
    3-5 gives trained-net magnitudes (raw rgb |.| up to ~80, see ``trained_params``).
    """
    out: Dict[str, torch.Tensor] = OrderedDict()
    for li, (name, (o, i)) in enumerate(layer_shapes(hidden, code, num_xyz, num_dir).items()):
        bound = 1.0 / np.sqrt(i)
        w = hash_uniform(seed, 2 * li, o * i).reshape(o, i) * np.float32(bound)
        if weight_scale != 1.0:
            w = w * np.float32(weight_scale)
        b = hash_uniform(seed, 2 * li + 1, o) * np.float32(bound)
        if name == "fc_out":
            b[0] += np.float32(sigma_bias)
        out[name + ".weight"] = torch.from_numpy(w.astype(np.float32))
        out[name + ".bias"] = torch.from_numpy(b.astype(np.float32))
    return out


# Trained-magnitude cases (VERDICT r1 "What's weak" 2): weights x scale, unit-variance codes and
# an fc_out sigma bias that puts sigma_raw in the 10-50 range a trained density field reaches.
TRAINED_CASES = {"t4": {"weight_scale": 4.0, "sigma_bias": 20.0, "code_std": 1.0},
                 "t3": {"weight_scale": 3.0, "sigma_bias": 12.0, "code_std": 1.0}}


def trained_params(seed: int, case: str = "t4") -> Dict[str, torch.Tensor]:
    c = TRAINED_CASES[case]
    return codenerf_params(seed, sigma_bias=c["sigma_bias"], weight_scale=c["weight_scale"])


def trained_codes(seed: int, n: int, case: str = "t4") -> torch.Tensor:
    return latent_codes(seed, n, std=TRAINED_CASES[case]["code_std"])


def latent_codes(seed: int, n: int, size: int = 256, std: float = 0.3) -> torch.Tensor:
    """(n, size) codes ~ std * U(-sqrt3, sqrt3) (unit-variance hash noise)."""
    return torch.from_numpy(hash_uniform(seed, 99, n * size).reshape(n, size) * np.float32(std * np.sqrt(3.0)))


def uniforms01(seed: int, stream: int, shape) -> torch.Tensor:
    """Injected U[0,1) draws (t_rand / u of point_sampler.py:64,93)."""
    n = int(np.prod(shape))
    return torch.from_numpy(((hash_uniform(seed, stream, n) + 1.0) * 0.5).astype(np.float32).reshape(shape))


def srn_intrinsics(size: int = 128, focal: float = 131.25) -> torch.Tensor:
    """4x4 intrinsics of the uncropped SRN grid."""
    k = torch.eye(4, dtype=torch.float32)
    k[0, 0] = k[1, 1] = focal
    k[0, 2] = k[1, 2] = size / 2.0
    return k
