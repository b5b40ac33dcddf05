"""SRN on-disk format: view_synthesis/datasets/dataset.py and the
dataloader of utils/util.py:59-90.

``SRNDataset(path, stage)`` is the reference's dataset: the same directory discovery
(``srn_<name>/<name>_<stage>/<object>/{rgb,pose,intrinsics.txt}``, the chairs_2.0_train
redirect, sorted objects and files), and ``__getitem__`` returns the same dict -- color /255,
mask where every channel != 255, the crop of size//8 per side (rows by the width's crop,
columns by the height's, as dataset.py:82-84), ``pose @ diag(1,-1,-1,1)`` and the principal
point shifted by the crops.  PNG decoding is Pillow (imageio's PNG backend; imageio itself is
not installed).

MI355X layout (``resident=True`` / ``load_resident(device)``): every view of the split is
decoded once -- on a thread pool, Pillow decodes without the GIL -- cropped, and kept as ONE
uint8 (n_views, h, w, c) tensor in HBM with the poses and intrinsics beside it (SRN cars
train: 4.5 GB of the 288 GB).  A batch is then an index tensor: ``batch(idx)`` unpacks the
views on the device (cn_srn_unpack: /255 and the mask in one launch) instead of reading and
decoding PNGs per iteration.  ``prepare_dataloader`` draws indices exactly as the
reference's DataLoader does (RandomSampler with replacement over ``experiment.iterations``
samples, or DistributedSampler), so the resident loader yields the same views in the same
order.
"""
from __future__ import annotations

import os
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path
from typing import Dict, Iterator, Optional

import numpy as np
import torch

from . import ops


def _decode(path) -> np.ndarray:
    """imageio.imread of an 8-bit PNG (dataset.py:71): RGB / RGBA / L / LA as stored; a palette
    image expanded to RGBA when it has transparency, else RGB (imageio's Pillow plugin does the
    same); anything else (16-bit, float) is refused rather than misread."""
    from PIL import Image
    with Image.open(path) as im:
        if im.mode == "P":
            im = im.convert("RGBA" if "transparency" in im.info else "RGB")
        if im.mode not in ("RGB", "RGBA", "L", "LA"):
            raise ValueError(f"{path}: PNG mode {im.mode} is not an 8-bit image the SRN loader reads")
        return np.asarray(im)


def _read_intrinsics(path):
    with Path(path).open() as f:
        lines = f.readlines()
    focal, cx, cy, _ = map(float, lines[0].split())
    height, width = map(int, lines[-1].split())
    return focal, cx, cy, height, width


class SRNDataset(torch.utils.data.Dataset):
    """dataset.py:10-94 (+ the HBM-resident store, see the module docstring)."""

    def __init__(self, path: str, stage: str = "train", device=None, threads: Optional[int] = None):
        super().__init__()
        self.base_path = Path(path)
        self.dataset_name = self.base_path.stem.split("_")[-1]
        self.base_path = self.base_path / f"{self.dataset_name}_{stage}"
        self.stage = stage
        assert self.base_path.exists(), f"{self.base_path} does not exist"
        if "chair" in self.dataset_name and stage == "train":
            tmp = self.base_path / "chairs_2.0_train"
            if tmp.exists():
                self.base_path = tmp
        self.intrinsic = sorted(self.base_path.glob("*/intrinsics.txt"))
        self.num_objects = len(self.intrinsic)
        self.rgb_all_filenames, self.pose_all_filenames = [], []
        for index, intrinsic_path in enumerate(self.intrinsic):
            rgb_directory = intrinsic_path.parent / "rgb"
            pose_directory = intrinsic_path.parent / "pose"
            self.rgb_all_filenames.extend(sorted([(index, p) for p in rgb_directory.iterdir()]))
            self.pose_all_filenames.extend(sorted([(index, p) for p in pose_directory.iterdir()]))
        assert len(self.rgb_all_filenames) == len(self.pose_all_filenames)
        self.num_views = len(self.rgb_all_filenames) // max(1, self.num_objects)
        self.resident: Optional[Dict[str, torch.Tensor]] = None
        if device is not None:
            self.load_resident(device, threads)

    def __len__(self):
        return len(self.rgb_all_filenames)

    # ---- one view, as the reference -------------------------------------------------
    def _geometry(self, index):
        object_index, _ = self.rgb_all_filenames[index]
        _, pose_filename = self.pose_all_filenames[index]
        focal, cx, cy, height, width = _read_intrinsics(self.intrinsic[object_index])
        crop_h, crop_w = height // 8, width // 8
        pose = np.loadtxt(pose_filename).reshape(4, 4) @ np.diag([1, -1, -1, 1])
        k = np.eye(4)
        k[0, 0], k[1, 1] = focal, focal
        k[0, 2], k[1, 2] = cx - crop_w, cy - crop_h
        return object_index, pose.astype(np.float32), k.astype(np.float32), (height, width, crop_h, crop_w)

    def _cropped_u8(self, index, geo=None) -> np.ndarray:
        _, rgb_filename = self.rgb_all_filenames[index]
        _, _, _, (height, width, crop_h, crop_w) = geo if geo is not None else self._geometry(index)
        rgb = _decode(rgb_filename)
        return np.ascontiguousarray(rgb[crop_w:width - crop_w, crop_h:height - crop_h, ...])

    def __getitem__(self, index):
        """dataset.py:60-94."""
        object_index, pose, k, _ = self._geometry(index)
        rgb = self._cropped_u8(index)
        mask = (rgb != 255).all(axis=-1)[..., None].astype(np.uint8) * 255
        return {"object_id": object_index, "intrinsic": k, "color": (rgb / 255.0).astype(np.float32),
                "mask": (mask / 255.0).astype(np.float32), "pose": pose}

    # ---- HBM-resident store ----------------------------------------------------------
    def load_resident(self, device, threads: Optional[int] = None, chunk_views: int = 256) -> Dict[str, torch.Tensor]:
        """Decode every view once (thread pool; each view's geometry read once) and upload ONE uint8
        (n_views, h, w, c) tensor + poses / intrinsics / object ids to ``device``.  The pixels go
        up in slices of ``chunk_views`` views through two small pinned staging buffers (decode of
        one slice overlaps the upload of the previous), which are released afterwards: no
        split-sized pinned host block stays cached for the run."""
        n = len(self)
        assert n > 0, "empty split"
        dev = torch.device(device)
        pinned = dev.type == "cuda"
        threads = threads or min(16, os.cpu_count() or 1)
        with ThreadPoolExecutor(max_workers=threads) as pool:
            geo = list(pool.map(self._geometry, range(n)))
            first = self._cropped_u8(0, geo[0])
            h, w = first.shape[:2]
            c = first.shape[2] if first.ndim == 3 else 1
            images = torch.empty((n, h, w, c), dtype=torch.uint8, device=dev)
            per = max(1, min(chunk_views, n))
            stage = [torch.empty((per, h, w, c), dtype=torch.uint8, pin_memory=pinned) for _ in range(2)]
            done = [None, None]
            for k, s0 in enumerate(range(0, n, per)):
                s1 = min(n, s0 + per)
                buf = stage[k % 2]
                if done[k % 2] is not None:
                    done[k % 2].synchronize()      # the upload that last read this buffer finished

                def fill(i, buf=buf, s0=s0):
                    a = first if i == 0 else self._cropped_u8(i, geo[i])
                    if a.shape[:2] != (h, w) or (a.shape[2] if a.ndim == 3 else 1) != c:
                        raise ValueError(f"view {i} is {a.shape}, the split's first view is {(h, w, c)}: the "
                                         "resident store needs one image shape per split")
                    buf[i - s0].copy_(torch.from_numpy(a.reshape(h, w, c)))

                list(pool.map(fill, range(s0, s1)))
                images[s0:s1].copy_(buf[: s1 - s0], non_blocking=pinned)
                if pinned:
                    done[k % 2] = torch.cuda.Event()
                    done[k % 2].record()
            if pinned:
                torch.cuda.current_stream(dev).synchronize()
        del stage, done
        if pinned and hasattr(torch._C, "_host_emptyCache"):
            torch._C._host_emptyCache()            # hand the staging buffers back to the OS
        self.resident = {
            "images": images,
            "pose": torch.from_numpy(np.stack([g[1] for g in geo])).to(dev),
            "intrinsic": torch.from_numpy(np.stack([g[2] for g in geo])).to(dev),
            "object_id": torch.tensor([g[0] for g in geo], dtype=torch.int64, device=dev),
        }
        return self.resident

    def batch(self, index) -> Dict[str, torch.Tensor]:
        """The collated batch of views ``index`` from the resident store, on the device:
        color (B, h, w, c), mask (B, h, w, 1), pose (B, 4, 4), intrinsic (B, 4, 4), object_id (B,)."""
        assert self.resident is not None, "call load_resident(device) first"
        r = self.resident
        idx = torch.as_tensor(index, dtype=torch.int64).reshape(-1).to(r["images"].device, non_blocking=True)
        color, mask = ops.srn_unpack(r["images"], idx)
        host_idx = np.asarray(index, dtype=np.int64).reshape(-1)
        return {"object_id": r["object_id"][idx], "intrinsic": r["intrinsic"][idx], "color": color, "mask": mask,
                "pose": r["pose"][idx],
                "object_id_host": np.asarray([self.rgb_all_filenames[i][0] for i in host_idx], dtype=np.int64)}


class ResidentLoader:
    """The reference's DataLoader (util.py:87-88: batch_size, sampler, no shuffle) over a resident
    SRNDataset: the same sampler draws the same indices; each batch is unpacked on the device."""

    def __init__(self, dataset: SRNDataset, sampler, batch_size: int):
        self.dataset, self.sampler, self.batch_size = dataset, sampler, batch_size

    def __iter__(self) -> Iterator[Dict[str, torch.Tensor]]:
        # a DataLoader iterator draws its base seed from the global RNG before the sampler runs
        torch.empty((), dtype=torch.int64).random_()
        for idx in torch.utils.data.BatchSampler(self.sampler, self.batch_size, drop_last=False):
            yield self.dataset.batch(idx)

    def __len__(self):
        return len(torch.utils.data.BatchSampler(self.sampler, self.batch_size, drop_last=False))


def prepare_dataloader(stage: str, cfg, device=None):
    """utils/util.py:59-90 -> (dataloader, dataset).  ``device``: keep the split resident in HBM and
    return a ResidentLoader (same sampler, same index order) instead of a torch DataLoader."""
    import torch.distributed as dist
    is_distributed = bool(getattr(cfg, "is_distributed", False))
    dataset = SRNDataset(cfg.dataset.basedir, stage=stage, device=device)
    sampler = torch.utils.data.RandomSampler(dataset, replacement=True, num_samples=cfg.experiment.iterations)
    if is_distributed:
        sampler = torch.utils.data.DistributedSampler(dataset, num_replicas=dist.get_world_size(),
                                                      rank=dist.get_rank(), drop_last=False)
    batch_size = cfg.dataset.train_batch_size if stage == "train" else cfg.dataset.val_batch_size
    if device is not None:
        return ResidentLoader(dataset, sampler, batch_size), dataset
    loader = torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=False, num_workers=0,
                                         sampler=sampler, pin_memory=torch.cuda.is_available())
    return loader, dataset
