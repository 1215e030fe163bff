"""Host logic of the train.py surface (CPU, no GPU): the DeviceLoader reproduces torch DataLoader's sample
order from the same RNG state (the basis of the value-for-value train.py replay in test_gpu_trainer.py),
shards like DistributedSampler, and TrainInterface.train / test / save_model follow the reference's
loop (trainers/base.py:219-470) on a torch-only toy trainer."""
import argparse
import os

import pytest
import torch
from torch.utils.data import DataLoader, Subset
from torch.utils.data.distributed import DistributedSampler

from data_fixture import write_twophase_dataset, DATASET_KW


@pytest.fixture(scope="module")
def ds(tmp_path_factory):
    from data import PDE2DDataset
    root = str(tmp_path_factory.mktemp("ds"))
    write_twophase_dataset(root, shape=(13, 8, 11, 8, 6), with_split=False)
    return PDE2DDataset(base_path=root, **dict(DATASET_KW, split_file=None, split_val=0.0, split_test=0.0))


def _ids(batches):
    return [round(float(b[1][i].sum()), 4) for b in batches for i in range(b[1].shape[0])]


@pytest.mark.parametrize("shuffle", [True, False])
def test_device_loader_order_is_dataloaders(ds, shuffle):
    from data import DeviceLoader
    sub = Subset(ds.dataset, list(range(1, 12)))
    torch.manual_seed(5)
    ref_first = _ids([next(iter(DataLoader(sub, batch_size=3, shuffle=shuffle)))])
    ref = [_ids(list(DataLoader(sub, batch_size=3, shuffle=shuffle))) for _ in range(3)]
    after_ref = torch.rand(3)
    torch.manual_seed(5)
    dl = DeviceLoader(sub, batch_size=3, shuffle=shuffle, device="cpu")
    got_first = _ids([next(iter(dl))])
    got = [_ids(list(dl)) for _ in range(3)]
    assert got_first == ref_first and got == ref
    assert torch.equal(torch.rand(3), after_ref)  # the global RNG advanced exactly as the DataLoader's did
    assert len(dl) == len(DataLoader(sub, batch_size=3))


def test_device_loader_generator(ds):
    from data import DeviceLoader
    ref = _ids(list(DataLoader(ds.dataset, batch_size=4, shuffle=True, generator=torch.Generator().manual_seed(3))))
    got = _ids(list(DeviceLoader(ds.dataset, batch_size=4, shuffle=True, device="cpu",
                                 generator=torch.Generator().manual_seed(3))))
    assert got == ref


@pytest.mark.parametrize("n,world,drop_last", [(13, 2, False), (13, 3, True), (12, 4, False), (5, 8, False)])
def test_device_loader_shards_are_distributed_samplers(ds, n, world, drop_last):
    from data import DeviceLoader
    sub = Subset(ds.dataset, list(range(n)))
    for epoch in (0, 3):
        seen = []
        for rank in range(world):
            ref = DistributedSampler(sub, num_replicas=world, rank=rank, shuffle=True, seed=0, drop_last=drop_last)
            ref.set_epoch(epoch)
            dl = DeviceLoader(sub, batch_size=2, shuffle=True, device="cpu", num_replicas=world, rank=rank,
                              drop_last=drop_last)
            dl.set_epoch(epoch)
            pos = dl.shard_positions().tolist()
            assert pos == list(ref)
            assert len(dl) == (len(ref) + 1) // 2
            seen += pos
        if n % world == 0:
            assert sorted(seen) == list(range(n))  # disjoint shards covering the split exactly once
        else:
            assert set(seen) <= set(range(n)) and (drop_last or set(seen) == set(range(n)))


# --------------------------------------------------------------------------- TrainInterface loop
class _Toy(torch.nn.Module):
    from common.interfaces import M
    model_interface = M.AR_TB

    def __init__(self):
        super().__init__()
        from common.interfaces import D
        self.data_interface = [D.sim2d]
        self.lin = torch.nn.Linear(4, 1)


def _toy_trainer(tmp_path, **cfg):
    from common.interfaces import D, M
    from trainers.base import TrainInterface

    class ToyTrainer(TrainInterface):
        model_interface = [M.AR_TB]
        data_interface = [D.sim2d]

        def train_step(self, batch, epoch, batch_idx, loader=None):
            x, y = batch
            pred = self.model.lin(x).squeeze(-1)
            return torch.sqrt(self.criterion(pred, y)), pred

    g = torch.Generator().manual_seed(0)
    xs, ys = torch.randn(10, 4, generator=g), torch.randn(10, generator=g)
    split = torch.utils.data.TensorDataset(xs, ys)
    data = argparse.Namespace(data_interface=D.sim2d, train=split, valid=split, test=split, pde=None)
    config = argparse.Namespace(device="cpu", batch_size=3, num_epochs=4, print_interval=2, test_interval=2,
                                lr_step_interval=2, nw=0, **cfg)
    torch.manual_seed(0)
    model = _Toy()
    tr = ToyTrainer(model=model, data=data, criterion=torch.nn.MSELoss(reduction="sum"), config=config,
                    save_path=str(tmp_path / "ck"))
    opt = torch.optim.SGD(tr.get_parameters(), lr=0.01)
    tr.set_optimizer(opt)
    tr.set_lr_scheduler(torch.optim.lr_scheduler.StepLR(opt, 1, gamma=0.5))
    return tr, opt


def test_train_interface_loop(tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    os.makedirs("models")
    tr, opt = _toy_trainer(tmp_path)
    with pytest.warns(UserWarning, match="Falling back"):
        train_losses, val_losses, val_stats = tr.train()
    assert len(train_losses) == 4 and len(val_losses["default"]) == 2 and val_stats["default"] == [{}, {}]
    assert os.path.exists(tmp_path / "ck_final.pt") and os.path.exists(tmp_path / "ck_default.pt")
    assert os.path.isdir("experiments/log") and os.path.isdir("models/output")
    assert opt.param_groups[0]["lr"] == pytest.approx(0.01 * 0.5 ** 2)  # stepped every lr_step_interval epochs
    sd = torch.load(tmp_path / "ck_final.pt", weights_only=True)
    assert set(sd) == {"lin.weight", "lin.bias"}


def test_train_one_epoch_divides_by_len_loader(tmp_path):
    """trainers/base.py:500: the epoch loss is the per-sample batch losses summed over len(loader)
    batches, also when max_train_batches stops the epoch early."""
    tr, _ = _toy_trainer(tmp_path)
    tr.max_train_batches = 0  # one batch, then stop
    loader = DataLoader(tr.data.train, batch_size=3)
    x, y = next(iter(loader))
    with torch.no_grad():
        want = torch.sqrt(((tr.model.lin(x).squeeze(-1) - y) ** 2).sum()) / 3 / len(loader)
    got = tr.train_one_epoch(loader, epoch=0)
    assert float(got) == pytest.approx(float(want), rel=1e-6)
