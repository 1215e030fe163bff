"""MemMapDataset (reference data/memmap_dataset.py:78-305), memmap format.

Same constructor, on-disk layout and item tuple as the reference:
  <path>/<data_file>.npy              (N, C, T, X1, X2) float trajectories (numpy .npy, memory-mapped)
  <path>/<data_file>.yaml             grid x1, x2 (or x), tmin, tmax, dt
  <path>/<conditioning>.npy           (N, K) static conditioning            [optional]
  <path>/<t_conditioning>.npy         (N, K_t, T) time-varying conditioning  [optional]
  <path>/<spatial_conditioning>.npy   (N, S, X1, X2) spatial conditioning    [optional]
  __getitem__ -> (u_base, u, x, conditioning, t_conditioning, spatial_conditioning)
The 'raggedmemmap' format (variable-length 1-D trajectories through mmap_ninja) is not on the 2-D grid
path and raises.  `load_batch` reads a whole batch with one fancy-indexed read per array, the entry point
of the device-resident loader (data/device_loader.py).
"""
import os
import weakref
from typing import Sequence, Tuple

import numpy as np
import torch
from numpy.lib.format import open_memmap
from torch.utils.data import Dataset

from utils.load_yaml import load_yaml


def load_data(data_format, data_dir, load_name):
    """utils/load_memmap.py:8-15 (memmap only)."""
    if data_format == "memmap":
        return open_memmap(os.path.join(data_dir, load_name + ".npy"), mode="r")
    if data_format == "raggedmemmap":
        raise NotImplementedError("raggedmemmap (variable-length 1-D data via mmap_ninja) is not on the 2-D grid path")
    raise ValueError(f"data format {data_format} not supported")


def precompute_and_save_memmap(memmap_in, filename, transform, dtype):
    """memmap_dataset.py:18-26."""
    N = memmap_in.shape[0]
    element_shape = transform(torch.tensor(memmap_in[0], dtype=dtype)).shape
    memmap_out = open_memmap(filename, mode="w+", dtype=memmap_in.dtype, shape=(N, *element_shape))
    for i in range(N):
        memmap_out[i] = transform(torch.tensor(memmap_in[i], dtype=dtype)).numpy()
    memmap_out.flush()
    return open_memmap(filename, mode="r")




# the optional arrays of a dataset directory: (key in self.data, position in the item tuple)
_OPTIONAL = (("baseline", 0), ("conditioning", 3), ("t_conditioning", 4), ("spatial_conditioning", 5))


def read_grid(config: dict, dtype) -> Tuple[torch.Tensor, list]:
    """Grid of a <data_file>.yaml: a 1-D `x` list, or axes x1, x2, ... (each key present exactly once,
    numbered from 1) combined into an (n1, n2, ..., ndim) coordinate tensor (meshgrid 'ij').
    Returns (x, [per-axis coordinate tensors])."""
    if "x" in config:
        x = torch.tensor(config["x"], dtype=dtype)
        return x, [x]
    axes = sorted(int(k[1:]) for k in config if k.startswith("x") and k[1:].isdigit())
    if axes != list(range(1, len(axes) + 1)):
        raise ValueError(f"grid axes {['x' + str(a) for a in axes]} are not numbered 1..{len(axes)}")
    if not axes:
        raise ValueError("no grid (x or x1, x2, ...) in the dataset yaml")
    coords = [torch.tensor(config[f"x{a}"], dtype=dtype) for a in axes]
    if len(coords) == 1:
        return coords[0], coords
    return torch.stack(torch.meshgrid(*coords, indexing="ij"), dim=-1), coords


class MemMapDataset(Dataset):
    """memmap_dataset.py:78-305: trajectories + optional baseline / conditioning arrays of one directory,
    items (u_base, u, x, conditioning, t_conditioning, spatial_conditioning) with per-item transforms
    (applied on access, or once up front into temporary memmaps with preprocess=True)."""

    def __init__(self, path: str, data_file: str, baseline_file: str = None, conditioning: str = None,
                 t_conditioning: str = None, spatial_conditioning: str = None, data_transform=None,
                 grid_transform=None, baseline_transform=None, conditioning_transform=None,
                 t_conditioning_transform=None, spatial_conditioning_transform=None, data_format: str = "memmap",
                 raggedmemmap_batch_size: int = 128, dtype: torch.dtype = torch.float32, preprocess: bool = False,
                 preprocess_path: str = None, load_all: bool = False) -> None:
        super().__init__()
        if data_format not in ("memmap", "raggedmemmap"):
            raise AssertionError("data format must be memmap (numpy) or raggedmemmap (numpy+mmap_ninja)")
        self.dtype = dtype
        self.data_format = data_format
        files = dict(baseline=baseline_file, conditioning=conditioning, t_conditioning=t_conditioning,
                     spatial_conditioning=spatial_conditioning)
        given = dict(data=data_transform, baseline=baseline_transform, conditioning=conditioning_transform,
                     t_conditioning=t_conditioning_transform, spatial_conditioning=spatial_conditioning_transform)
        # a transform only counts for an array that is in use
        self.transforms = {k: (t if k == "data" or files[k] is not None else None) for k, t in given.items()}
        self.return_baseline = baseline_file is not None
        self.return_conditioning = conditioning is not None
        self.return_t_conditioning = t_conditioning is not None
        self.return_spatial_conditioning = spatial_conditioning is not None
        self.data_transform = self.transforms["data"]
        self.baseline_transform = self.transforms["baseline"]
        self.conditioning_transform = self.transforms["conditioning"]
        self.t_conditioning_transform = self.transforms["t_conditioning"]
        self.spatial_conditioning_transform = self.transforms["spatial_conditioning"]
        self.grid_transform = grid_transform

        # preprocessing only pays when one of the trajectory / conditioning transforms exists (:152-156;
        # a spatial-conditioning transform alone does not enable it)
        if preprocess and all(self.transforms[k] is None for k in ("data", "baseline", "conditioning",
                                                                    "t_conditioning")):
            print("preprocess=True ignored: no transform to precompute")
            preprocess = False
        self.preprocess = preprocess
        self.preprocess_dir = (preprocess_path or os.path.join(path, "tmp")) if preprocess else None
        if preprocess:
            os.makedirs(self.preprocess_dir, exist_ok=True)

        self.data = {"data": load_data(data_format, path, data_file)}
        self.data.update({k: load_data(data_format, path, f) for k, f in files.items() if f is not None})

        self.config = load_yaml(os.path.join(path, data_file + ".yaml"))
        self.x, self.x_all = read_grid(self.config, self.dtype)
        self.tmin, self.tmax, self.dt = self.config["tmin"], self.config["tmax"], self.config["dt"]
        if grid_transform is not None:  # the grid is shared by every item: transformed once
            self.x = grid_transform(self.x)

        if preprocess:
            self.preprocess_output = {}
            for key, t in self.transforms.items():
                if t is None or key not in self.data:
                    continue
                fname = os.path.join(self.preprocess_dir, f"{key}_{os.getpid()}_{id(self)}.npy")
                self.data[key] = precompute_and_save_memmap(self.data[key], fname, t, self.dtype)
                self.preprocess_output[key] = fname
            self._finalizer = weakref.finalize(self, MemMapDataset._delete_files, dict(self.preprocess_output))

        if load_all:
            self.data = {k: np.asarray(v[:]) for k, v in self.data.items()}

    @staticmethod
    def _delete_files(paths):
        for p in paths.values():
            if os.path.exists(p):
                os.remove(p)

    def cleanup(self):
        if hasattr(self, "_finalizer"):
            self._finalizer()

    def __len__(self):
        return self.data["data"].shape[0]

    def _transforms(self):
        if self.preprocess:
            return (None,) * 5
        return (self.data_transform, self.baseline_transform, self.conditioning_transform,
                self.t_conditioning_transform, self.spatial_conditioning_transform)

    def __getitem__(self, idx: int) -> Tuple[torch.Tensor, ...]:
        """memmap_dataset.py:262-305."""
        u = torch.tensor(self.data["data"][idx], dtype=self.dtype)
        u_base = torch.tensor(self.data["baseline"][idx], dtype=self.dtype) if self.return_baseline else torch.empty(0)
        cond = torch.tensor(self.data["conditioning"][idx], dtype=self.dtype) if self.return_conditioning \
            else torch.empty(0)
        t_cond = torch.tensor(self.data["t_conditioning"][idx], dtype=self.dtype) if self.return_t_conditioning \
            else torch.empty(0)
        sc = torch.tensor(self.data["spatial_conditioning"][idx], dtype=self.dtype) \
            if self.return_spatial_conditioning else torch.empty(0)
        tu, tb, tc, tt, ts = self._transforms()
        if tu is not None:
            u = tu(u)
        if tb is not None:
            u_base = tb(u_base)
        if tc is not None:
            cond = tc(cond)
        if tt is not None:
            t_cond = tt(t_cond)
        if ts is not None:
            sc = ts(sc)
        return u_base, u, self.x, cond, t_cond, sc

    def load_batch(self, indices: Sequence[int]) -> Tuple[torch.Tensor, ...]:
        """The default-collated batch of `indices` (torch.utils.data default_collate of __getitem__ items),
        read with one sorted fancy-indexed memmap read per array and returned as CPU tensors."""
        idx = np.asarray(indices, dtype=np.int64)
        order = np.argsort(idx, kind="stable")
        inv = np.empty_like(order)
        inv[order] = np.arange(len(order))

        def read(key):
            a = np.asarray(self.data[key][idx[order]])  # ascending offsets: sequential I/O on the memmap
            return torch.from_numpy(np.ascontiguousarray(a[inv])).to(self.dtype)

        tu, tb, tc, tt, ts = self._transforms()

        def apply(t, batch):
            return batch if t is None else torch.stack([t(b) for b in batch])

        u = apply(tu, read("data"))
        B = u.shape[0]
        u_base = apply(tb, read("baseline")) if self.return_baseline else torch.empty(B, 0)
        cond = apply(tc, read("conditioning")) if self.return_conditioning else torch.empty(B, 0)
        t_cond = apply(tt, read("t_conditioning")) if self.return_t_conditioning else torch.empty(B, 0)
        sc = apply(ts, read("spatial_conditioning")) if self.return_spatial_conditioning else torch.empty(B, 0)
        x = self.x.unsqueeze(0).expand(B, *self.x.shape).contiguous()
        return u_base, u, x, cond, t_cond, sc
