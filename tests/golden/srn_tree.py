"""Write a tiny synthetic SRN-layout dataset tree (no dataset download offline).

    srn_<name>/<name>_<stage>/<object>/{rgb/NNNNNN.png, pose/NNNNNN.txt, intrinsics.txt}

The layout and file formats are the ones view_synthesis/datasets/dataset.py:23-94 reads:
intrinsics.txt line 0 = "focal cx cy 0.", last line = "height width"; pose files = 16 numbers
(a 4x4 c2w, OpenCV convention); rgb = 8-bit PNG, white (255) background.  Objects alternate
RGB and RGBA PNGs so both decode paths are covered.  Deterministic: the same call writes the
same bytes (used by make_golden.py to pin the reference's loader, and by the tests).
"""
from __future__ import annotations

import math
import os

import numpy as np

STAGES = {"train": 3, "val": 2}   # objects per stage
VIEWS = 2
SIZE = 64


def _pose(i: int, j: int) -> np.ndarray:
    th, ph, rho = 0.3 + 0.4 * i, 0.7 * j - 0.2, 1.2 + 0.1 * j
    st, ct, sp, cp = math.sin(th), math.cos(th), math.sin(ph), math.cos(ph)
    m = np.eye(4)
    m[0, 0], m[1, 0] = -sp, cp
    m[0, 1], m[1, 1], m[2, 1] = -st * cp, -st * sp, ct
    m[0, 2], m[1, 2], m[2, 2] = ct * cp, ct * sp, st
    m[0, 3], m[1, 3], m[2, 3] = rho * ct * cp, rho * ct * sp, rho * st
    return m @ np.diag([1, -1, -1, 1])


def _image(seed: int, channels: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    img = np.full((SIZE, SIZE, channels), 255, np.uint8)
    yy, xx = np.mgrid[0:SIZE, 0:SIZE]
    cy, cx, r = rng.integers(20, 44), rng.integers(20, 44), rng.integers(10, 18)
    blob = (yy - cy) ** 2 + (xx - cx) ** 2 < r * r
    img[..., :3][blob] = rng.integers(0, 250, size=(int(blob.sum()), 3), dtype=np.uint8)
    img[5, 7, :3] = (255, 255, 0)   # a pixel with one channel below 255: not masked
    if channels == 4:
        img[..., 3] = np.where(blob, 255, 0)
        img[1, 1, 3] = 128
    return img


def write_tree(root: str, name: str = "cars", channels=None) -> str:
    """Write the tree under root; returns the dataset basedir (root/srn_<name>).  ``channels``: 3 or 4
    for every PNG (one image shape per split, as the real SRN release), None: alternating."""
    from PIL import Image
    base = os.path.join(root, f"srn_{name}")
    for stage, n_obj in STAGES.items():
        for i in range(n_obj):
            obj = os.path.join(base, f"{name}_{stage}", f"{stage}_obj{i:03d}")
            os.makedirs(os.path.join(obj, "rgb"), exist_ok=True)
            os.makedirs(os.path.join(obj, "pose"), exist_ok=True)
            focal = 70.0 + 3.0 * i
            with open(os.path.join(obj, "intrinsics.txt"), "w") as f:
                f.write(f"{focal} {SIZE // 2}. {SIZE // 2 + 1}. 0.\n0. 0. 0.\n1.\n{SIZE} {SIZE}\n")
            for j in range(VIEWS):
                ch = channels or (4 if (i + j) % 2 else 3)
                Image.fromarray(_image(1000 * i + j + (17 if stage == "val" else 0), ch)).save(
                    os.path.join(obj, "rgb", f"{j:06d}.png"))
                np.savetxt(os.path.join(obj, "pose", f"{j:06d}.txt"), _pose(i, j).reshape(1, 16), fmt="%.10f")
    return base
