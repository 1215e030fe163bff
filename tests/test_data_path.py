"""On-disk dataset path: the mirror's PDE2DDataset / MemMapDataset / DataCreator /
DeviceLoader vs the REFERENCE's own outputs on the same files (tests/golden/data_twophase.pt, written by
tests/golden/make_golden_data.py from the dataset of tests/data_fixture.py).  Bit-exact: pure data movement.
"""
import os

import pytest
import torch

from conftest import load_golden
from data_fixture import write_twophase_dataset, DATASET_KW


@pytest.fixture(scope="module")
def root(tmp_path_factory):
    r = str(tmp_path_factory.mktemp("ds"))
    write_twophase_dataset(r)
    write_twophase_dataset(os.path.join(r, "nosplit"), with_split=False)
    return r


def test_pde2d_dataset_matches_reference(root):
    from data import PDE2DDataset
    g = load_golden("data_twophase")
    ds = PDE2DDataset(base_path=root, **DATASET_KW)
    for k, v in g["pde"].items():
        assert float(getattr(ds.pde, k)) == v, k
    assert torch.equal(ds.pde.x, g["x"])
    for split in ("train", "valid", "test"):
        sub = getattr(ds, split)
        assert torch.equal(torch.tensor([int(i) for i in sub.indices]), g[f"{split}_indices"])
        items = [sub[i] for i in range(len(sub))]
        for j, name in enumerate(("u_base", "u", "x", "cond", "t_cond", "sc")):
            assert torch.equal(torch.stack([it[j] for it in items]), g[f"{split}_{name}"]), (split, name)


def test_default_split_matches_reference(root):
    from data import PDE2DDataset
    g = load_golden("data_twophase")
    ds = PDE2DDataset(base_path=os.path.join(root, "nosplit"),
                      **dict(DATASET_KW, split_file=None, split_val=0.2, split_test=0.15))
    for split in ("train", "valid", "test"):
        assert torch.equal(torch.tensor([int(i) for i in getattr(ds, split).indices]), g[f"nosplit_{split}_indices"])


def test_load_batch_is_the_collated_batch(root):
    """MemMapDataset.load_batch == default_collate of the items (the reference DataLoader's batch)."""
    from data import PDE2DDataset
    from torch.utils.data import default_collate
    ds = PDE2DDataset(base_path=root, **DATASET_KW)
    idx = [5, 0, 3]
    ref = default_collate([ds.dataset[i] for i in idx])
    got = ds.dataset.load_batch(idx)
    for a, b in zip(got, ref):
        assert a.shape == b.shape and torch.equal(a, b)


def test_device_loader_cpu_epoch_covers_split(root):
    from data import PDE2DDataset, DeviceLoader
    ds = PDE2DDataset(base_path=root, **DATASET_KW)
    ld = DeviceLoader(ds.train, batch_size=3, shuffle=True, device="cpu", generator=torch.Generator().manual_seed(0))
    seen = torch.cat([b[1] for b in ld])
    ref = torch.stack([ds.train[i][1] for i in range(len(ds.train))])
    assert len(ld) == 2 and seen.shape == ref.shape
    # same multiset of trajectories (shuffled order)
    key = lambda t: sorted(t.flatten(1).sum(1).tolist())  # noqa: E731
    assert key(seen) == key(ref)


def test_create_data_host_matches_reference():
    from trainers.autoregressivepushforwardtrainer import DataCreator
    g = load_golden("data_twophase")
    dc = DataCreator(pde=None, neighbors=3, time_window=3, t_resolution=11, x_resolution=(8, 6))
    d, l = dc.create_data(g["train_u"], g["cd_steps"].tolist())
    assert torch.equal(d, g["cd_data"]) and torch.equal(l, g["cd_labels"])


@pytest.mark.parametrize("batch_size", [3, 2, 7])
def test_device_loader_order_matches_dataloader_over_epochs(root, batch_size):
    """Sample order per epoch == torch DataLoader(shuffle=True, generator=g) over three epochs (the
    RandomSampler's trailing randperm keeps the two generators in step), and with generator=None from the
    same global RNG state."""
    from data import PDE2DDataset, DeviceLoader
    from torch.utils.data import DataLoader
    ds = PDE2DDataset(base_path=root, **DATASET_KW)
    key = lambda b: b[1].flatten(1).sum(1).tolist()  # noqa: E731  (one id per trajectory)
    for explicit in (True, False):
        g1 = torch.Generator().manual_seed(7) if explicit else None
        g2 = torch.Generator().manual_seed(7) if explicit else None
        ref = DataLoader(ds.train, batch_size=batch_size, shuffle=True, generator=g1)
        ld = DeviceLoader(ds.train, batch_size=batch_size, shuffle=True, device="cpu", generator=g2)
        for _ in range(3):
            torch.manual_seed(11)
            want = [key(b) for b in ref]
            torch.manual_seed(11)
            got = [key(b) for b in ld]
            assert got == want


def test_device_loader_unpadded_shards_cover_split_once(root):
    """pad=False (evaluation loaders under a process group): rank shards are disjoint, differ in length by
    at most one, and together hold every sample of the split exactly once (no wrap-around duplicates)."""
    from data import PDE2DDataset, DeviceLoader
    ds = PDE2DDataset(base_path=root, **DATASET_KW)
    n = len(ds.train)
    for R in (2, 3, 4):
        ids = []
        for r in range(R):
            ld = DeviceLoader(ds.train, batch_size=2, shuffle=True, device="cpu", num_replicas=R, rank=r, pad=False)
            pos = ld.shard_positions().tolist()
            assert len(pos) == len(range(r, n, R)) and len(ld) == (len(pos) + 1) // 2
            ids += pos
        assert sorted(ids) == list(range(n))
