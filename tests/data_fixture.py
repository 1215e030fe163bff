"""Deterministic on-disk twophase-format dataset (reference data/PDE2D.py + data/memmap_dataset.py layout)
shared by the golden generator (tests/golden/make_golden_data.py) and the data-path tests."""
import os

import numpy as np
import yaml

N, C, T, X1, X2, K = 7, 8, 11, 8, 6, 3


def write_twophase_dataset(root, experiment="twophase", with_split=True, seed=2024, shape=None):
    """<root>/<experiment>/{snapshots.npy,.yaml, conditioning.npy, spatial_conditioning.npy, split.yaml};
    shape = (N, C, T, X1, X2) overrides the default sizes."""
    N, C, T, X1, X2 = shape if shape is not None else (globals()["N"], globals()["C"], globals()["T"],
                                                       globals()["X1"], globals()["X2"])
    rng = np.random.default_rng(seed)
    d = os.path.join(root, experiment)
    os.makedirs(d, exist_ok=True)
    u = rng.random((N, C, T, X1, X2), dtype=np.float32)
    np.save(os.path.join(d, "snapshots.npy"), u)
    cfg = dict(x1=[float(v) for v in np.linspace(0.0, 0.7, X1)], x2=[float(v) for v in np.linspace(0.0, 0.5, X2)],
               tmin=0.0, tmax=1.0, dt=0.1)
    with open(os.path.join(d, "snapshots.yaml"), "w") as f:
        yaml.safe_dump(cfg, f)
    np.save(os.path.join(d, "conditioning.npy"), rng.random((N, K), dtype=np.float32))
    np.save(os.path.join(d, "spatial_conditioning.npy"), (rng.random((N, 1, X1, X2)) > 0.8).astype(np.float32))
    if with_split:
        with open(os.path.join(d, "split.yaml"), "w") as f:
            yaml.safe_dump(dict(train=[i for i in range(N) if i % 7 in (0, 2, 3, 5)],
                                valid=[i for i in range(N) if i % 7 in (1, 6)],
                                test=[i for i in range(N) if i % 7 == 4]), f)
    return d


DATASET_KW = dict(experiment="twophase", split_file="split", data_format="memmap", data_file="snapshots",
                  conditioning="conditioning", spatial_conditioning="spatial_conditioning", name="twophase",
                  preprocess=False, c_filter=[6])  # configs/train/cfg_twophase_ufno.py:14-26
