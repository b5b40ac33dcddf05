"""SRN on-disk format on the CPU: codenerf.datasets.SRNDataset
reproduces the reference's SRNDataset (dataset.py:10-94) bit for bit on a synthetic SRN tree
(tests/golden/srn_tree.py; the reference's own outputs in srn_tiny.npz from make_golden.py), and
the resident loader draws the reference DataLoader's indices in the same order
(utils/util.py:59-90)."""
import os
import sys

import numpy as np
import pytest
import torch

from conftest import GOLDEN

sys.path.insert(0, GOLDEN)
import srn_tree  # noqa: E402


@pytest.fixture(scope="module")
def tree(tmp_path_factory):
    return srn_tree.write_tree(str(tmp_path_factory.mktemp("srn")))


@pytest.mark.parametrize("stage", ["train", "val"])
def test_items_match_reference(tree, stage):
    from codenerf.datasets import SRNDataset
    g = np.load(os.path.join(GOLDEN, "srn_tiny.npz"))
    ds = SRNDataset(tree, stage)
    assert ds.num_objects == int(g[f"{stage}_num_objects"]) and ds.num_views == int(g[f"{stage}_num_views"])
    assert [os.path.relpath(str(p), tree) for _, p in ds.rgb_all_filenames] == list(g[f"{stage}_files"])
    for i in range(len(ds)):
        item = ds[i]
        for k in ("color", "mask", "pose", "intrinsic", "object_id"):
            ref = g[f"{stage}_{i}_{k}"]
            got = np.asarray(item[k])
            assert got.dtype == ref.dtype and np.array_equal(got, ref), (stage, i, k)


def test_missing_split_asserts(tmp_path):
    from codenerf.datasets import SRNDataset
    with pytest.raises(AssertionError, match="does not exist"):
        SRNDataset(str(tmp_path / "srn_cars"), "train")


class _IndexDataset:
    """Stands in for the resident store: a batch is its index list."""

    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n

    def __getitem__(self, i):
        return i

    def batch(self, idx):
        return torch.as_tensor(idx)


@pytest.mark.parametrize("batch_size", [1, 4])
def test_resident_loader_draws_dataloader_order(batch_size):
    """train.py:70 takes next(iter(loader)) every iteration: a fresh iterator each time.  The
    resident loader must consume the global RNG exactly like torch's DataLoader does."""
    from codenerf.datasets import ResidentLoader
    ds = _IndexDataset(37)
    sampler = torch.utils.data.RandomSampler(ds, replacement=True, num_samples=50)
    torch.manual_seed(5)
    dl = torch.utils.data.DataLoader(ds, batch_size=batch_size, shuffle=False, num_workers=0, sampler=sampler)
    ref = [next(iter(dl)).tolist() for _ in range(6)]
    torch.manual_seed(5)
    rl = ResidentLoader(ds, sampler, batch_size)
    got = [next(iter(rl)).tolist() for _ in range(6)]
    assert got == ref
    assert len(rl) == len(dl)


@pytest.mark.parametrize("chunk_views", [1, 3, 1000])
def test_load_resident_cpu_slices(tmp_path, chunk_views):
    """load_resident's sliced upload (two staging buffers, chunk_views views each) fills every view
    with the crop __getitem__ decodes, whatever the slice size; geometry tensors match item order."""
    from codenerf.datasets import SRNDataset
    root = srn_tree.write_tree(str(tmp_path), channels=4)
    ds = SRNDataset(root, "train")
    r = ds.load_resident("cpu", threads=2, chunk_views=chunk_views)
    assert r["images"].shape[0] == len(ds)
    for i in range(len(ds)):
        item = ds[i]
        rgb = r["images"][i].numpy()
        assert np.array_equal((rgb / 255.0).astype(np.float32), item["color"]), i
        assert np.array_equal(r["pose"][i].numpy(), item["pose"]) and int(r["object_id"][i]) == item["object_id"]
