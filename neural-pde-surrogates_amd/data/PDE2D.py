"""PDE2DDataset: the twophase cfgs' dataset object (reference data/PDE2D.py:12-110).

One MemMapDataset over <base_path>/<experiment>, split into train / valid / test Subsets (from a split
yaml, else a trailing val / test fraction), plus the PDE2D metadata the model builder reads (time axis,
grid lengths and sizes, conditioning channel counts).  `c_filter` keeps a subset of the trajectory
channels (cfg_twophase_*: c_filter=[6])."""
import os
from typing import Optional, Sequence, Tuple

import numpy as np
import torch

from common.interfaces import D
from data import transforms
from data.base import DatasetInterface
from data.memmap_dataset import MemMapDataset
from pdes import PDE2D
from utils.load_yaml import load_yaml


class ChannelFilter:
    """Per-item transform u (C, T, ...) -> u[channels]."""

    def __init__(self, channels: Sequence[int]):
        self.channels = np.asarray(channels)

    def __call__(self, u):
        return u[self.channels]


def split_indices(n: int, split_path: Optional[str], split_val: float,
                  split_test: float) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(train, valid, test) sample indices: the lists of a split yaml when given, else the last
    int(split_test * n) samples for test, the int(split_val * n) before them for validation and the rest
    for training (an empty valid / test fraction gives an empty split)."""
    if split_path is not None:
        s = load_yaml(split_path)
        return tuple(np.array(s[k]) for k in ("train", "valid", "test"))
    idx = np.arange(n)
    n_val, n_test = int(split_val * n), int(split_test * n)
    # negative-start slicing as the reference (idx[:-(v+t)], idx[-(v+t):-t], idx[-t:]): an empty valid
    # or test fraction therefore selects nothing for training / everything for test
    tr = idx[:-(n_val + n_test)]
    va = idx[-(n_val + n_test):-n_test]
    te = idx[-n_test:]
    print(f"Warning: no split file given; splitting {n} samples by fraction "
          f"(valid {split_val:g}, test {split_test:g}): train {tr.shape[0]} / valid {va.shape[0]} / "
          f"test {te.shape[0]}")
    return tr, va, te


class PDE2DDataset(DatasetInterface):
    data_interface = D.sim2d

    def __init__(self, base_path: str, experiment: str, data_format: str, data_file: str, conditioning: str = None,
                 t_conditioning: str = None, spatial_conditioning: str = None, c_filter: list = None,
                 split_file: str = None, split_val: float = .05, split_test: float = .05, name: str = "PDE2D",
                 preprocess: bool = False, preprocess_path: str = None):
        self.experiment = experiment
        root = os.path.join(base_path, experiment)
        self.dataset = MemMapDataset(
            root, data_file, data_format=data_format, conditioning=conditioning, t_conditioning=t_conditioning,
            spatial_conditioning=spatial_conditioning,
            data_transform=ChannelFilter(c_filter) if c_filter is not None else None,
            preprocess=preprocess, preprocess_path=preprocess_path)
        split_path = None
        if split_file is not None:
            split_path = os.path.join(root, split_file if split_file.lower().endswith(".yaml") else split_file + ".yaml")
        parts = split_indices(len(self.dataset), split_path, split_val, split_test)
        self.train_dataset, self.valid_dataset, self.test_dataset = (torch.utils.data.Subset(self.dataset, p)
                                                                     for p in parts)
        self._pde = self._make_pde(name, conditioning, t_conditioning, spatial_conditioning)

    def _make_pde(self, name, conditioning, t_conditioning, spatial_conditioning) -> PDE2D:
        """PDE2D metadata (PDE2D.py:73-89): the full time axis of the files (nt = tmax / dt + 1), the grid
        extents x[-1,0,0] - x[0,0,0] and x[0,-1,1] - x[0,0,1], and the channel count of each
        conditioning array that is in use (read from item 0)."""
        ds = self.dataset
        nt = int(ds.tmax / ds.dt) + 1
        tmin, tmax = transforms.get_t_downsample(ds.tmin, ds.tmax, nt, ratio_nt=1)
        x = ds.x
        item = ds[0]
        counts = [item[i].shape[0] if used is not None else 0
                  for i, used in ((3, conditioning), (4, t_conditioning), (5, spatial_conditioning))]
        return PDE2D(tmin=tmin, tmax=tmax, nt=nt, L1=x[-1, 0, 0] - x[0, 0, 0], L2=x[0, -1, 1] - x[0, 0, 1],
                     nx1=x.shape[0], nx2=x.shape[1], x=x, name=name, n_cond_static=counts[0],
                     n_cond_dynamic=counts[1], n_cond_spatial=counts[2])

    @property
    def pde(self):
        return self._pde

    def __repr__(self):
        return f"{self.pde}_{self.experiment}"

    @property
    def train(self):
        return self.train_dataset

    @property
    def valid(self):
        return self.valid_dataset

    @property
    def test(self):
        return self.test_dataset
