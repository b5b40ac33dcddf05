"""Host-side helpers the hot path depends on (view_synthesis/utils/util.py)."""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch


def get_minibatches(inputs: torch.Tensor, chunksize: Optional[int] = 1024 * 8) -> List[torch.Tensor]:
    """util.py:230-235."""
    return [inputs[i: i + chunksize] for i in range(0, inputs.shape[0], chunksize)]


def split_sizes(num_rays: int, n: int) -> Tuple[List[int], List[int]]:
    """Per-rank ray counts and pads of parallel_image_render (nerf/__init__.py:179-187, quirk Q5).

    Every rank but the last gets int(num_rays / n) (float division, truncated);
    the last takes the remainder; the others are padded up to it.
    """
    assert n >= 1, "need at least one rank"
    base = int(num_rays / n)
    per = [base] * n
    per[-1] = num_rays - base * (n - 1)
    padding = num_rays - base * n
    pad = [padding] * (n - 1) + [0] if padding > 0 else [0] * n
    assert sum(per) == num_rays, "Mismatch in batchsize per process and total number of rays"
    assert pad[0] + per[0] == per[-1], "Incorrect calculation of padding"
    return per, pad


def mse2psnr(mse_val: float) -> float:
    """util.py:216-227."""
    if mse_val == 0:
        mse_val = 1e-5
    return -10.0 * math.log10(mse_val)
