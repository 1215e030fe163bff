"""GPU side of the on-disk data path: nps_gather_windows vs the reference's create_data semantics, the
device-resident loader vs the host batches, and one pushforward training epoch fed from memmapped files
through AutoregressivePushforwardTrainer.get_dataloaders()."""
import math
import os

import pytest
import torch

from conftest import load_golden
from data_fixture import write_twophase_dataset, DATASET_KW

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_gather_windows_matches_reference_create_data():
    from trainers.autoregressivepushforwardtrainer import DataCreator
    g = load_golden("data_twophase")
    dc = DataCreator(pde=None, neighbors=3, time_window=3, t_resolution=11, x_resolution=(8, 6))
    d, l = dc.create_data(g["train_u"].to(DEV), g["cd_steps"].tolist())
    assert torch.equal(d.cpu(), g["cd_data"]) and torch.equal(l.cpu(), g["cd_labels"])
    # odd plane size (scalar path) and labels-only mode
    u = torch.randn(3, 2, 20, 5, 7, device=DEV)
    steps = [4, 9, 12]
    lab = dc.create_data(u, steps, mode="labels")
    ref = torch.stack([u[b, :, s:s + 3] for b, s in enumerate(steps)])
    assert torch.equal(lab, ref)
    with pytest.raises(AssertionError):
        dc.create_data(u, [1, 2, 3])


def test_device_loader_batches_equal_host_batches(tmp_path):
    from data import PDE2DDataset, DeviceLoader
    write_twophase_dataset(str(tmp_path))
    ds = PDE2DDataset(base_path=str(tmp_path), **DATASET_KW)
    host = list(DeviceLoader(ds.train, 3, shuffle=True, device="cpu", generator=torch.Generator().manual_seed(5)))
    dev = list(DeviceLoader(ds.train, 3, shuffle=True, device=DEV, generator=torch.Generator().manual_seed(5)))
    assert len(host) == len(dev) == 2
    for hb, db in zip(host, dev):
        for h, d in zip(hb, db):
            assert d.is_cuda and torch.equal(d.cpu(), h)


def test_train_epoch_from_disk(tmp_path):
    """UNet-free tiny U-FNO (the smoke model) trained for one epoch on a 32x32 memmapped dataset."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__ as ge
    from data import PDE2DDataset
    from trainers.autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer
    write_twophase_dataset(str(tmp_path), shape=(8, 8, 80, 32, 32))
    ds = PDE2DDataset(base_path=str(tmp_path), **DATASET_KW)
    model, _, _ = ge._tiny_ufno(DEV, num_c=1)
    assert ds.pde.nx1 == 32 and ds.pde.n_cond_static == 3 and ds.pde.n_cond_spatial == 1
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    tr = AutoregressivePushforwardTrainer(model, ds, torch.nn.MSELoss(reduction="sum"), optimizer=opt,
                                          time_window=25, base_resolution=(80, 32, 32), batch_size=2,
                                          device=DEV, lr_step_interval=1, unrolling=1)
    train_loader, valid_loader, _ = tr.get_dataloaders()
    loss = tr.train_one_epoch(train_loader, epoch=1)
    assert math.isfinite(float(loss))
