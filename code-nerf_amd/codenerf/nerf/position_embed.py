"""PositionalEmbedder on the gfx950 kernel (view_synthesis/nerf/position_embed.py:5-53)."""
from __future__ import annotations

import torch

from .. import ops


class PositionalEmbedder(object):

    def __init__(self, num_freq: int, log_sampling: bool, include_input: bool, dtype, device) -> None:
        assert num_freq > 0, "Number of frequency samples should be a positive integer"
        self.num_freq = num_freq
        self.log_sampling = log_sampling
        self.include_input = include_input
        self.dtype = torch.float32
        self.device = torch.device(device)
        if log_sampling:
            bands = 2.0 ** torch.linspace(0.0, num_freq - 1, num_freq, dtype=torch.float32)
        else:
            bands = torch.linspace(2.0 ** 0.0, 2.0 ** (num_freq - 1), num_freq, dtype=torch.float32)
        self.frequency_bands = bands.to(self.device)
        self.freqs = [float(f) for f in bands]   # host copy for kernel arguments

    @property
    def out_dim_per_input(self) -> int:
        return int(self.include_input) + 2 * self.num_freq

    def embed(self, tensor: torch.Tensor) -> torch.Tensor:
        """position_embed.py:35-53: (N, D) -> (N, D * (include_input + 2 * num_freq))."""
        from ..autograd import posenc_autograd
        return posenc_autograd(tensor, self.freqs, self.include_input)
