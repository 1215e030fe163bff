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




class MemMapDataset(Dataset):
    """memmap_dataset.py:78-305."""

    def __init__(self, path: str, data_file: str, baseline_file: str = None, conditioning: str = None,
                 t_conditioning: str = None, spatial_conditioning: str = None, data_transform=None,
                 grid_transform=None, baseline_transform=None, conditioning_transform=None,
                 t_conditioning_transform=None, spatial_conditioning_transform=None, data_format: str = "memmap",
                 raggedmemmap_batch_size: int = 128, dtype: torch.dtype = torch.float32, preprocess: bool = False,
                 preprocess_path: str = None, load_all: bool = False) -> None:
        super().__init__()
        self.dtype = dtype
        assert data_format in ["memmap", "raggedmemmap"], \
            "data format must be memmap (numpy) or raggedmemmap (numpy+mmap_ninja)"
        self.data_format = data_format
        self.return_baseline = baseline_file is not None
        self.return_conditioning = conditioning is not None
        self.return_t_conditioning = t_conditioning is not None
        self.return_spatial_conditioning = spatial_conditioning is not None
        self.data_transform = data_transform
        self.grid_transform = grid_transform
        self.baseline_transform = baseline_transform if self.return_baseline else None
        self.conditioning_transform = conditioning_transform if self.return_conditioning else None
        self.t_conditioning_transform = t_conditioning_transform if self.return_t_conditioning else None
        self.spatial_conditioning_transform = spatial_conditioning_transform if self.return_spatial_conditioning \
            else None
        self.preprocess = preprocess
        if all(v is None for v in [self.data_transform, self.baseline_transform, self.conditioning_transform,
                                   self.t_conditioning_transform]):  # :152-156
            if self.preprocess:
                print("Overriding preprocess to False, since no transforms were specified")
                self.preprocess = False
        if self.preprocess:
            self.preprocess_dir = preprocess_path if preprocess_path is not None else os.path.join(path, "tmp")
            os.makedirs(self.preprocess_dir, exist_ok=True)
        else:
            self.preprocess_dir = None

        self.data = {"data": load_data(self.data_format, path, data_file)}
        for key, name, on in (("baseline", baseline_file, self.return_baseline),
                              ("conditioning", conditioning, self.return_conditioning),
                              ("t_conditioning", t_conditioning, self.return_t_conditioning),
                              ("spatial_conditioning", spatial_conditioning, self.return_spatial_conditioning)):
            if on:
                self.data[key] = load_data(self.data_format, path, name)

        self.config = load_yaml(os.path.join(path, data_file + ".yaml"))  # :178-200
        if "x" in self.config:
            self.x = torch.tensor(self.config["x"], dtype=self.dtype)
            self.x_all = [self.x]
        else:
            x_keys = [k for k in self.config if k.startswith("x")]
            x_keys = [int(k[1:]) for k in x_keys if str.isdigit(k[1:])]
            if set(range(1, len(x_keys) + 1)) != set(x_keys):
                raise ValueError(f"Found grid keys {['x' + str(k) for k in x_keys]}, "
                                 f"expected keys {['x' + str(k) for k in range(1, len(x_keys) + 1)]}")
            if len(x_keys) == 0:
                raise ValueError(f"Could not find a grid in {data_file}.yaml")
            x_keys = sorted("x" + str(k) for k in x_keys)
            self.x_all = [torch.tensor(self.config[k], dtype=self.dtype) for k in x_keys]
            if len(self.x_all) == 1:
                self.x = self.x_all[0]
            else:
                self.x = torch.movedim(torch.stack(torch.meshgrid(*self.x_all, indexing="ij")), 0, -1)
        self.tmin = self.config["tmin"]
        self.tmax = self.config["tmax"]
        self.dt = self.config["dt"]
        if self.grid_transform is not None:
            self.x = self.grid_transform(self.x)

        if self.preprocess:  # :205-226 (memmap)
            self.preprocess_output = {}
            for data_name, on, transform in (("data", True, self.data_transform),
                                             ("baseline", self.return_baseline, self.baseline_transform),
                                             ("conditioning", self.return_conditioning, self.conditioning_transform),
                                             ("t_conditioning", self.return_t_conditioning,
                                              self.t_conditioning_transform),
                                             ("spatial_conditioning", self.return_spatial_conditioning,
                                              self.spatial_conditioning_transform)):
                if not on or transform is None:
                    continue
                fname = os.path.join(self.preprocess_dir, f"{data_name}_{os.getpid()}_{id(self)}.npy")
                self.data[data_name] = precompute_and_save_memmap(self.data[data_name], fname, transform, self.dtype)
                self.preprocess_output[data_name] = fname
            self._finalizer = weakref.finalize(self, MemMapDataset._delete_files, dict(self.preprocess_output))

        if load_all:  # :228-231
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
