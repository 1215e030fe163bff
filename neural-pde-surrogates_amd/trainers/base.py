"""TrainInterface: the epoch / validation / checkpoint driver of the reference (trainers/base.py:24-507),
the surface `train.py` binds (train.py:128-165: get_dataloaders, test, get_parameters, set_optimizer,
set_lr_scheduler, train).

The loop structure, return values and model-selection rule are the reference's; what differs is where
the data lives: on a GPU device the loaders are `data.DeviceLoader`s (batches already in HBM, the
sample order of torch's DataLoader from the same RNG state), and under one process per GPU
(torch.distributed initialised) every loader takes its rank's shard and losses / metrics are averaged
over the ranks, so every rank makes the same model-selection decision and rank 0 alone writes
checkpoints.  A `grad_sync` (trainers.distributed.GradAllReducer) all-reduces gradients between
backward and the optimizer step.
"""
import argparse
import os
import timeit
import warnings
from typing import Callable, Dict, List, Tuple

import torch

from common.interfaces import D
from utils import misc as util

try:  # optional, as in the reference (trainers/base.py:17-21)
    import wandb
    WANDB_AVAILABLE = True
except ModuleNotFoundError:
    wandb = None
    WANDB_AVAILABLE = False


def _dist():
    """(world_size, rank) of the default process group, (1, 0) without one."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


class _UnpaddedShardSampler(torch.utils.data.Sampler):
    """Evaluation shard of a CPU DataLoader under a process group: positions rank, rank + R, ... of a
    per-epoch permutation (DistributedSampler's seed + epoch), without wrap-around duplicates."""

    def __init__(self, n, num_replicas, rank, shuffle=True, seed=0):
        self.n, self.R, self.rank, self.shuffle, self.seed, self.epoch = n, num_replicas, rank, shuffle, seed, 0

    def set_epoch(self, epoch):
        self.epoch = epoch

    def __iter__(self):
        g = torch.Generator()
        g.manual_seed(self.seed + self.epoch)
        order = torch.randperm(self.n, generator=g) if self.shuffle else torch.arange(self.n)
        return iter(order[self.rank::self.R].tolist())

    def __len__(self):
        return len(range(self.rank, self.n, self.R))


class TrainInterface:
    """Base trainer; subclasses define train_step / test_step / simulate and the supported interfaces."""
    model_interface: list = []
    data_interface: list = []

    def __init__(self, model, data, criterion: Callable, optimizer=None, lr_scheduler=None,
                 config: argparse.Namespace = None, save_path: str = "models/model.pt",
                 max_train_batches=float("inf"), max_test_batches=float("inf"), epoch_callback: Callable = None,
                 use_wandb=False, wandb_kwargs=None, wandb_config_dict=None, grad_sync=None, **kwargs):
        self.model = model
        self.data = data
        self.config = config if config is not None else argparse.Namespace(**kwargs)
        self.config.save_path = save_path
        if self.data.data_interface == D.sim1d_var_t:
            self.config.variable_time = True
        elif not hasattr(self.config, "variable_time"):
            self.config.variable_time = False
        self.optimizer = optimizer
        self.criterion = criterion
        self.lr_scheduler = lr_scheduler
        self.max_train_batches = max_train_batches
        self.max_test_batches = max_test_batches
        self.epoch_callback = epoch_callback
        self.world, self.rank = _dist()
        # the per-rank training loss is the rank's share of the global-batch loss (distributed.global_sqrt_loss);
        # its gradients are right when the ranks SUM them.  A reducer that averages — GradAllReducer(average=True),
        # or grad_sync=False with the caller's own torch DDP wrapper (which averages) — gets the share's gradient
        # scaled by the world size, so every documented option trains the 1-process model.
        self.grad_world_scale = 1.0
        if self.world > 1:
            # data parallelism wired here, so an unchanged train.py under torchrun trains one model
            from trainers.distributed import GradAllReducer, check_rank_device, sync_python_random
            check_rank_device(self.model.parameters())  # every rank's model on its own card
            sync_python_random()  # every rank draws rank 0's unroll depths / start steps, whatever the reducer
            if grad_sync is None:
                grad_sync = GradAllReducer(self.model.parameters())
                grad_sync.broadcast_parameters(0)
            if grad_sync is False or getattr(grad_sync, "average", False):
                self.grad_world_scale = float(self.world)
        self.grad_sync = grad_sync if grad_sync is not False else None
        self.print_setting = getattr(self.config, "print_setting", dict(print_per_step=False))
        self.use_wandb = bool(use_wandb) and WANDB_AVAILABLE
        if use_wandb and not WANDB_AVAILABLE:
            warnings.warn("Could not import WandB -- WandB not used!")
        self.wandb_kwargs = wandb_kwargs
        self.wand_config_dict = wandb_config_dict
        self.test_kwargs_list = getattr(self.config, "test_kwargs_list", [("default", {})])

    def __repr__(self):
        return type(self).__name__

    def __call__(self):
        self.train()

    # ------------------------------------------------------------------ wiring (train.py:128-145)
    def get_parameters(self):
        return self.model.parameters()

    def set_optimizer(self, optimizer):
        self.optimizer = optimizer

    def set_lr_scheduler(self, lr_scheduler):
        self.lr_scheduler = lr_scheduler

    def get_dataloaders(self):
        """(train, valid, test) loaders (trainers/base.py:157-179, fixed-length time; batch_size, shuffle).
        GPU device: data.DeviceLoader; CPU: torch DataLoader.  Under torch.distributed `batch_size` is per
        rank; the training split is sharded like DistributedSampler (padded so every rank takes the same
        number of steps), the validation / test splits without padding (each sample counted once)."""
        if self.config.variable_time:
            raise NotImplementedError("variable-length time (sim1d_var_t) is not on the grid path")
        device = torch.device(self.config.device)
        bs = self.config.batch_size
        world, rank = _dist()
        splits = (self.data.train, self.data.valid, self.data.test)
        if device.type == "cuda":
            from data.device_loader import DeviceLoader
            return tuple(DeviceLoader(d, bs, shuffle=True, device=device, num_replicas=world, rank=rank,
                                      pad=(i == 0)) for i, d in enumerate(splits))
        from torch.utils.data import DataLoader
        nw = getattr(self.config, "nw", 0)
        if world > 1:
            from torch.utils.data.distributed import DistributedSampler
            samplers = [DistributedSampler(splits[0], num_replicas=world, rank=rank, shuffle=True)]
            samplers += [_UnpaddedShardSampler(len(d), world, rank) for d in splits[1:]]
            return tuple(DataLoader(d, batch_size=bs, num_workers=nw, sampler=sm) for d, sm in zip(splits, samplers))
        return tuple(DataLoader(d, batch_size=bs, shuffle=True, num_workers=nw, persistent_workers=nw > 0,
                                pin_memory=True) for d in splits)

    # ------------------------------------------------------------------ steps (subclass)
    def train_step(self, batch, epoch, batch_idx, loader=None):
        raise NotImplementedError("The method train_step should be implemented!")

    def test_step(self, batch, batch_idx, use_train_loss_calc=False, include_data=False, **kwargs):
        """trainers/base.py:130-152: without an override, validation falls back to the training loss."""
        if include_data:
            raise ValueError("include_data is only supported when implemented in test_step")
        if not use_train_loss_calc:
            raise NotImplementedError("The test_step method is not implemented!")
        loss, _ = self.train_step(batch, epoch=0, batch_idx=batch_idx)
        return loss, {}

    def simulate(self, u, *args, compute_loss=True, include_data=True, nr_gt_steps=1, t_res=100, **kwargs):
        raise NotImplementedError("The method simulate is not implemented!")

    # ------------------------------------------------------------------ loops
    @staticmethod
    def _to_device(batch, device):
        return tuple(t.to(device) if isinstance(t, torch.Tensor) else t for t in batch)

    @staticmethod
    def _set_epoch(loader, epoch):
        for obj in (loader, getattr(loader, "sampler", None)):
            if obj is not None and hasattr(obj, "set_epoch"):
                obj.set_epoch(epoch)

    def _reduce(self, value, mean: bool):
        """Sum (or average) a scalar / tensor over the ranks in fp64; identity in a single process."""
        world, _ = _dist()
        if world == 1:
            return value
        import torch.distributed as dist
        dev = torch.device(self.config.device)
        t = (value.detach().to(dev, torch.float64).clone() if isinstance(value, torch.Tensor)
             else torch.tensor(float(value), dtype=torch.float64, device=dev))
        dist.all_reduce(t)
        if mean:
            t = t / world
        return t.to(value.dtype) if isinstance(value, torch.Tensor) else t.item()

    def _reduce_mean(self, value):
        return self._reduce(value, True)

    def _global_batch_size(self, batch) -> int:
        """Samples of this step over all ranks (the padded training shards give every rank the same
        batch sizes, step by step)."""
        return util.get_batch_size(batch) * self.world

    def train_one_epoch(self, loader, epoch) -> torch.Tensor:
        """trainers/base.py:472-507: zero_grad -> train_step -> backward -> [RCCL all-reduce] -> step;
        returns the sum of per-sample batch losses divided by len(loader), as the reference does (also
        when max_train_batches stops the epoch early).  Under a process group the loss is the global
        batch's, divided by the global batch size — the value the 1-process run logs."""
        self.model.train()
        device = self.config.device
        self._set_epoch(loader, epoch)
        total_loss = 0
        for batch_idx, batch in enumerate(loader):
            batch_on_device = self._to_device(batch, device)
            self.optimizer.zero_grad()
            loss, _ = self.train_step(batch_on_device, epoch, batch_idx, loader=loader)
            loss.backward()
            if self.grad_sync is not None:
                self.grad_sync.finish()
            self.optimizer.step()
            total_loss += loss.detach() / self._global_batch_size(batch)
            if batch_idx >= self.max_train_batches:
                break
        total_loss = total_loss / len(loader)
        if self.epoch_callback is not None:
            self.epoch_callback(self, loader, epoch)
        if self.lr_scheduler is not None and (epoch + 1) % self.config.lr_step_interval == 0:
            self.lr_scheduler.step()
        return total_loss

    def test(self, loader, use_train_loss_calc=False, include_data=False, test_kwargs=None):
        """trainers/base.py:378-470: batch-size-weighted mean of test_step's loss and metrics over the
        loader, without gradients.  Returns (loss, metrics) or, with include_data, also
        (stack([gt, pred]), per-sample info) (this rank's samples).  Under a process group the weighted
        sums and sample counts are summed over the ranks (unpadded shards: each sample once)."""
        test_kwargs = {} if test_kwargs is None else test_kwargs
        if getattr(loader, "batch_size", self.config.batch_size) != self.config.batch_size:
            print("Alert: batch_size in the supplied dataloader is not equal to that in the config.")
        device = self.config.device
        self.model.eval()
        loss, n_total, metrics = 0, 0, {}
        gt, pred, other = [], [], []
        with torch.no_grad():
            for batch_idx, batch in enumerate(loader):
                out = self.test_step(self._to_device(batch, device), batch_idx, use_train_loss_calc, include_data,
                                     **test_kwargs)
                batch_loss, batch_metrics = out[0], out[1]
                bs = util.get_batch_size(batch)
                loss += batch_loss * bs
                n_total += bs
                for k, v in batch_metrics.items():
                    metrics[k] = metrics[k] + v * bs if k in metrics else v * bs
                if include_data:
                    gt.append(out[2][0])
                    pred.append(out[2][1])
                    other.extend(out[2][2])
                if batch_idx >= self.max_test_batches - 1:
                    break
        if self.world > 1:
            import torch.distributed as dist
            keys = [sorted(metrics)]
            allkeys = [None] * self.world
            dist.all_gather_object(allkeys, keys[0])  # a rank with an empty shard has no metric keys
            for k in sorted(set().union(*map(set, allkeys))):
                if k not in metrics:
                    metrics[k] = 0.0
            n_total = self._reduce(n_total, False)
            loss = self._reduce(loss, False)
            metrics = {k: self._reduce(metrics[k], False) for k in sorted(metrics)}
        loss = loss / n_total
        metrics = {k: v / n_total for k, v in metrics.items()}
        if not include_data:
            return loss, metrics
        if self.data.data_interface == D.sim1d_var_t:
            raise NotImplementedError("variable-length time (sim1d_var_t) is not on the grid path")
        data = torch.stack([torch.cat([x.cpu() for x in gt]), torch.cat([x.cpu() for x in pred])])
        return loss, metrics, (data, other)

    def _evaluate(self, loader, test_kwargs, fallback):
        """One validation / test pass with the reference's test_step -> train-loss fallback rule."""
        if callable(test_kwargs):
            with torch.no_grad():
                return test_kwargs(loader, self), fallback
        try:
            return self.test(loader, fallback, test_kwargs=test_kwargs), fallback
        except NotImplementedError:
            warnings.warn("test_step method not implemented."
                          "Falling back to training loss calculation for validation set performance!")
            return self.test(loader, True, test_kwargs=test_kwargs), True

    def _print_stats(self, stats):
        if not self.print_setting.get("print_per_step", False):
            stats = {k: v for k, v in stats.items() if "step" not in k.lower()}
        floats = util.to_floatdict(stats)
        print(util.dict_str(floats, prefix="-"))
        print()
        return stats, floats

    def train(self) -> Tuple[List, Dict[str, List], Dict[str, List]]:
        """trainers/base.py:219-347: num_epochs of train_one_epoch; every test_interval epochs a validation
        pass per test setting, the checkpoint and a test-set pass whenever a setting's validation loss
        improves; final checkpoint.  Returns (train_losses, val_losses, val_stats) per setting."""
        assert self.model.model_interface in self.model_interface, f"{self} does not support model {self.model}."
        assert self.data.data_interface in self.model.data_interface, \
            f"{self.model} does not support data from {self.data}."
        assert self.data.data_interface in self.data_interface, f"{self} does not support data from {self.data}."
        _, rank = _dist()
        if rank == 0:
            util.check_directory()
        train_loader, valid_loader, test_loader = self.get_dataloaders()
        if self.use_wandb:
            wandb.init(config=self.wand_config_dict, **(self.wandb_kwargs or {}))
        fallback = False
        names = [name for name, _ in self.test_kwargs_list]
        train_losses = []
        best = {n: float("inf") for n in names}
        val_losses = {n: [] for n in names}
        val_stats_list = {n: [] for n in names}
        t_start = timeit.default_timer()
        for epoch in range(self.config.num_epochs):
            train_loss = self._reduce_mean(self.train_one_epoch(train_loader, epoch))
            train_losses.append(train_loss)
            if (epoch + 1) % self.config.print_interval == 0:
                ti = self.config.test_interval
                progress = 1.0 if (epoch + 1) % ti == 0 else ((epoch + 1) % ti) / ti
                print(f"Epoch {epoch} (progress: {progress:.2f}, {timeit.default_timer() - t_start:.4f}s), "
                      f"Loss {train_loss}")
                t_start = timeit.default_timer()
            log = {"train_loss": train_loss}
            if (epoch + 1) % self.config.test_interval == 0:
                for name, test_kwargs in self.test_kwargs_list:
                    print(f"Evaluation on validation dataset for setting [{name}]:")
                    (val_loss, val_stats), fallback = self._evaluate(valid_loader, test_kwargs, fallback)
                    print(f"Evaluation metric: {util.to_float(val_loss)}")
                    val_stats, floats = self._print_stats(val_stats)
                    log[name + " - val loss"] = val_loss
                    log.update({f"{name}-{k}": v for k, v in floats.items()})
                    val_losses[name].append(val_loss)
                    val_stats_list[name].append(val_stats)
                    if val_loss < best[name]:
                        self.save_model(self.config.save_path + f"_{name}.pt")
                        best[name] = val_loss
                        print("Found new best model, evaluation on test dataset:")
                        (test_loss, test_stats), fallback = self._evaluate(test_loader, test_kwargs, fallback)
                        print(f"Test metric: {util.to_float(test_loss)}")
                        self._print_stats(test_stats)
            if self.use_wandb:
                wandb.log(log)
        self.save_model(self.config.save_path + "_final.pt")
        if self.use_wandb:
            wandb.finish()
        return train_losses, val_losses, val_stats_list

    def save_model(self, save_name):
        """state_dict checkpoint (trainers/base.py:349-355; '.pt' when the name has no extension).  The
        keys / dtypes are the reference's, so the file loads into either implementation.  Under
        torch.distributed only rank 0 writes."""
        root, ext = os.path.splitext(save_name)
        save_name = root + (ext or ".pt")
        if _dist()[1] == 0:
            torch.save(self.model.state_dict(), save_name)
            print(f"Saved model at {save_name}")
        return save_name
