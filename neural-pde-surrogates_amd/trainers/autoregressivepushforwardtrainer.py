"""Autoregressive rollout driver (reference trainers/autoregressivepushforwardtrainer.py) on TrainInterface
(trainers/base.py: train / test / checkpointing, the train.py surface).

`simulate` keeps the reference's signature, loop bounds (:354-358), loss
normalisation (:422, :433-434) and return conventions, with the trajectory
resident on the device (windows are views, no per-step host copies) and the
MSE_sum criterion computed by a HIP fp64 reduction.  `train_step` /
`train_one_epoch` are the pushforward training loop (:43-163,
trainers/base.py:472-507) whose backward runs the HIP backward kernels
(nps_hip.autograd).  Under a process group each rank draws the global batch's
random steps, takes its slice, and backpropagates its share of the global
sqrt(MSE_sum) (trainers.distributed.global_sqrt_loss); the summed RCCL
all-reduce between backward and optimizer step then gives the 1-process
gradient of the concatenated batch.  Grid models only.
"""
import argparse
import math
import random
from typing import Tuple

import torch
from torch import nn

from common.interfaces import D, M
from nps_hip import ops
from nps_hip import autograd as ad
from trainers.base import TrainInterface


class DataCreator:
    """common/data_creator.py:48-78 (windowing only; the GNN graph builders are not built).  Windows of
    device-resident batches are cut on the device (one view when every sample shares the step, else one
    HIP gather); the per-sample slicing + torch.cat of the reference remains for host tensors."""

    def __init__(self, pde=None, neighbors: int = 2, time_window: int = 5, t_resolution: int = 250,
                 x_resolution=100):
        self.pde = pde
        self.n = neighbors
        self.tw = time_window
        self.t_res = t_resolution
        self.x_res = x_resolution
        assert isinstance(self.n, int)
        assert isinstance(self.tw, int)

    def to(self, device):
        return self

    def create_data(self, datapoints: torch.Tensor, steps: list, mode="both"):
        assert mode in ["data", "labels", "both"]
        steps = list(steps)[:datapoints.shape[0]]  # zip(datapoints, steps) semantics (a short last batch)
        T = datapoints.shape[2]
        for step in steps:
            assert step - self.tw >= 0 and step + self.tw <= T, 'this step - time window combination is not valid'
        if len(set(steps)) == 1:  # the rollout case: one slice of the whole batch, no per-sample cat
            s = steps[0]
            data = datapoints[:, :, s - self.tw:s]
            labels = datapoints[:, :, s:s + self.tw]
        elif datapoints.is_cuda and datapoints.dtype == torch.float32:
            # per-sample windows of a device-resident batch: one HIP gather each (nps_gather_windows)
            data = ops.gather_windows(datapoints, steps, self.tw, -self.tw) if mode != "labels" else None
            labels = ops.gather_windows(datapoints, steps, self.tw, 0) if mode != "data" else None
        else:
            data = torch.stack([dp[:, s - self.tw:s] for dp, s in zip(datapoints, steps)])
            labels = torch.stack([dp[:, s:s + self.tw] for dp, s in zip(datapoints, steps)])
        if mode == "data":
            return data
        if mode == "labels":
            return labels
        return data, labels


class AutoregressivePushforwardTrainer(TrainInterface):
    data_interface = [D.sim1d, D.sim2d, D.sim1d_var_t]
    model_interface = [M.AR_TB, M.AR_TB_GNN]

    def __init__(self, model, data, criterion, optimizer=None, lr_scheduler=None, config: argparse.Namespace = None,
                 save_path: str = "models/model.pt", **kwargs):
        super().__init__(model=model, data=data, criterion=criterion, optimizer=optimizer, lr_scheduler=lr_scheduler,
                         config=config, save_path=save_path, **kwargs)
        if not hasattr(self.config, "process_settings"):
            self.config.process_settings = {}
        self.data_creator = DataCreator(pde=self.data.pde, neighbors=getattr(self.config, "neighbors", 3),
                                        time_window=self.config.time_window,
                                        t_resolution=self.config.base_resolution[0],
                                        x_resolution=self.config.base_resolution[1])

    def _loss(self, pred, labels):
        c = self.criterion
        if isinstance(c, nn.MSELoss) and c.reduction == "sum" and pred.is_cuda:
            return ops.sq_err_sum(pred, labels)
        return c(pred, labels)

    def _train_loss(self, pred, labels):
        """torch.sqrt(criterion(pred, labels)) (:158-162); MSELoss(sum) runs as a HIP fp64 reduction with a
        HIP backward.  Under a process group the loss is that of the global batch: S_r all-reduced before
        backward, gradient ∇S_r / (2·sqrt(S)) (distributed.global_sqrt_loss)."""
        c = self.criterion
        mse = isinstance(c, nn.MSELoss) and c.reduction in ("sum", "mean")
        if self.world > 1:
            if not mse:
                raise NotImplementedError("data-parallel training reproduces the global-batch loss for "
                                          "nn.MSELoss(reduction='sum' | 'mean') criteria only")
            from trainers.distributed import global_sqrt_loss
            s_local = ad.mse_sum(pred, labels) if pred.is_cuda else torch.sum((pred - labels) ** 2)
            return global_sqrt_loss(s_local, pred.numel() if c.reduction == "mean" else None,
                                    grad_scale=self.grad_world_scale)
        if isinstance(c, nn.MSELoss) and c.reduction == "sum" and pred.is_cuda:
            return ad.sqrt_mse_sum(pred, labels)
        return torch.sqrt(c(pred, labels))

    def _random_steps(self, steps, batch_size):
        """random.choices(steps, k=batch_size) (:95); under a process group the draw is for the global
        batch (every rank holds rank 0's Python RNG state) and this rank takes its slice."""
        if self.world == 1:
            return random.choices(steps, k=batch_size)
        allsteps = random.choices(steps, k=batch_size * self.world)
        return allsteps[self.rank * batch_size:(self.rank + 1) * batch_size]

    def train_step(self, batch: Tuple, epoch, batch_idx, loader=None):
        """Pushforward training step, autoregressivepushforwardtrainer.py:43-163 (grid models, static time):
        a random unroll depth (<= min(epoch // lr_step_interval, unrolling)) of no-grad model calls from
        random start steps per sample, then one model call with grad; loss = sqrt(MSE_sum)."""
        batch_size = self.config.batch_size
        device = self.config.device
        if self.data.data_interface == D.sim1d_var_t:
            raise NotImplementedError("variable-length time (sim1d_var_t) is not on the grid path")
        if self.model.model_interface != M.AR_TB:
            raise NotImplementedError("graph (GNN) models are not on the MI355X path")
        u_base, u_super, x, conditioning, t_conditioning, spatial_conditioning = batch
        t_res = self.data_creator.t_res
        use_t_conditioning = torch.numel(t_conditioning) != 0
        if torch.numel(spatial_conditioning) == 0:
            spatial_conditioning = None
        unrolling_epoch = epoch // self.config.lr_step_interval                       # :78-82
        max_unrolling = min(unrolling_epoch, self.config.unrolling)
        unrolled_graphs = random.choice(list(range(max_unrolling + 1)))
        steps = [t for t in range(self.data_creator.tw,
                                  t_res - self.data_creator.tw - (self.data_creator.tw * unrolled_graphs) + 1)]
        random_steps = self._random_steps(steps, batch_size)                           # :95
        data, labels = self.data_creator.create_data(u_super, random_steps)
        data, labels = data.to(device), labels.to(device)
        t_cond = self.data_creator.create_data(t_conditioning, random_steps, mode="labels") \
            if use_t_conditioning else None
        with torch.no_grad():                                                          # :115-144
            for _ in range(unrolled_graphs):
                data = self.model(data, cond=conditioning, bc=None, pos=x, t_cond=t_cond,
                                  spatial_cond=spatial_conditioning)
                random_steps = [rs + self.data_creator.tw for rs in random_steps]
                _, labels = self.data_creator.create_data(u_super, random_steps)
                labels = labels.to(device)
                t_cond = self.data_creator.create_data(t_conditioning, random_steps, mode="labels") \
                    if use_t_conditioning else None
        pred = self.model(data, cond=conditioning, bc=None, pos=x, t_cond=t_cond,     # :150
                          spatial_cond=spatial_conditioning)
        loss = self._train_loss(pred, labels)
        return loss, pred

    def simulate(self, u, conditioning, x, compute_loss, include_data, nr_gt_steps, t_res,
                 t_conditioning=torch.empty(0), spatial_conditioning=torch.empty(0), clip_min=True, use_bc=True,
                 u_bc=None, u_mask=None, divide_by_t=True):
        """autoregressivepushforwardtrainer.py:288-440 (grid models; process_step is a no-op for twophase)."""
        use_mask = u_mask is not None
        if compute_loss is False and use_mask:
            raise ValueError("Mask supplied for computing the loss, but 'compute_loss'=False!")
        if compute_loss is True and u.shape[2] < t_res:
            raise ValueError("Cannot compute loss if no ground-truth simulation is provided for the full rollout")
        if u_bc is None:
            u_bc = u
        if use_bc and u_bc.shape[2] < t_res:
            raise ValueError("Cannot set BCs if the provided BC information is <= the unrolling time")
        if u.shape[2] < nr_gt_steps * self.data_creator.tw:
            raise ValueError("The training data is shorter than the specified number of unrolling steps")
        if self.model.model_interface != M.AR_TB:
            raise NotImplementedError("graph (GNN) models are not on the MI355X path")
        if str(getattr(self.data.pde, "name", "")) == "DIV1D":
            raise NotImplementedError("DIV1D boundary processing is not on the grid path")
        use_t_conditioning = torch.numel(t_conditioning) != 0
        use_spatial_conditioning = torch.numel(spatial_conditioning) != 0
        batch_size = u.shape[0]
        device = self.config.device
        tw = self.data_creator.tw
        pred = self.data_creator.create_data(u, [tw * nr_gt_steps] * batch_size, mode="data").to(device)
        if include_data:
            data_gt = [pred] if compute_loss else None
            data_pred = [pred]
        losses = []
        n_t = 0
        for step in range(tw * nr_gt_steps, t_res - tw + 1, tw):
            same_steps = [step] * batch_size
            if compute_loss:
                labels = self.data_creator.create_data(u, same_steps, mode="labels").to(device)
            if use_mask:
                labels_mask = self.data_creator.create_data(u_mask, same_steps, mode="labels").to(device)
            t_cond = self.data_creator.create_data(t_conditioning, same_steps, mode="labels") \
                if use_t_conditioning else None
            spatial_cond = spatial_conditioning if use_spatial_conditioning else None
            pred = self.model(pred, cond=conditioning, bc=None, pos=x, t_cond=t_cond, spatial_cond=spatial_cond)
            if compute_loss and use_mask:
                pred = pred * labels_mask
                labels = labels * labels_mask
            if compute_loss:
                loss = self._loss(pred, labels) / math.prod(self.config.base_resolution[1:])
                losses.append(loss / batch_size)
            if include_data:
                if compute_loss:
                    data_gt.append(labels)
                data_pred.append(pred)
            n_t += tw
        if divide_by_t:
            losses = [v / n_t for v in losses]
        losses = [v.float() for v in losses]
        if compute_loss and not include_data:
            return losses
        elif not compute_loss and include_data:
            return data_pred
        else:
            return losses, (data_gt, data_pred)

    def test_step(self, batch: Tuple, batch_idx: int, use_train_loss_calc=False, include_data=False,
                  max_test_len=None):
        """autoregressivepushforwardtrainer.py:165-286 (grid models, fixed-length time): one-step losses of
        every window (ground-truth input), then the full rollout.  Returns (mean unrolled loss, metrics
        {'Unrolled base losses', 'Unrolled forward losses', 'Mean per-step loss', 'Step s, mean loss'...}
        [, (gt, pred, per-sample info)])."""
        if use_train_loss_calc:
            raise RuntimeError("We should probably not have use_train_loss=True when having implemented the "
                               "test_step method...")
        if self.data.data_interface == D.sim1d_var_t:
            raise NotImplementedError("variable-length time (sim1d_var_t) is not on the grid path")
        if self.model.model_interface != M.AR_TB:
            raise NotImplementedError("graph (GNN) models are not on the MI355X path")
        u_base, u_super, x, conditioning, t_conditioning, spatial_conditioning = batch
        t_res = self.data_creator.t_res
        tw = self.data_creator.tw
        device = self.config.device
        B = u_super.shape[0]
        use_t = torch.numel(t_conditioning) != 0
        per_step, per_step_named = [], {}
        for step in range(tw, t_res - tw + 1, tw):
            same = [step] * B
            data, labels = self.data_creator.create_data(u_super, same)
            t_cond = self.data_creator.create_data(t_conditioning, same, mode="labels") if use_t else None
            pred = self.model(data.to(device), cond=conditioning, bc=None, pos=x, t_cond=t_cond,
                              spatial_cond=spatial_conditioning)
            loss = self._loss(pred, labels.to(device)).float() / B
            per_step.append(loss)
            per_step_named[f"Step {step}, mean loss"] = loss
        per_step = torch.stack(per_step)
        out = self._test_unrolled_losses(batch, include_data, max_test_len, divide_by_t=True)
        metrics = {"Unrolled base losses": out[1], "Unrolled forward losses": out[0],
                   "Mean per-step loss": torch.mean(per_step), **per_step_named}
        if include_data:
            return torch.mean(out[0]), metrics, out[2]
        return torch.mean(out[0]), metrics

    def _test_unrolled_losses(self, batch, include_data=False, max_test_len=None, divide_by_t=True):
        """autoregressivepushforwardtrainer.py:442-514: the summed per-window rollout loss of `simulate`
        (from nr_gt_steps ground-truth windows) and the numerical baseline's loss against the
        high-resolution solution (0 when the dataset has no baseline)."""
        if self.data.data_interface == D.sim1d_var_t:
            raise NotImplementedError("variable-length time (sim1d_var_t) is not on the grid path")
        u_base, u_super, x, conditioning, t_conditioning, spatial_conditioning = batch
        t_res = self.data_creator.t_res
        tw = self.data_creator.tw
        nr_gt = self.config.nr_gt_steps
        res = self.simulate(u_super, conditioning, x, t_conditioning=t_conditioning,
                            spatial_conditioning=spatial_conditioning, compute_loss=True, include_data=include_data,
                            nr_gt_steps=nr_gt, t_res=t_res, u_mask=None, divide_by_t=divide_by_t)
        losses, sims = (res[0], res[1]) if include_data else (res, None)
        B = u_super.shape[0]
        spatial = math.prod(self.config.base_resolution[1:])
        base, n_t = [], 0
        for step in range(tw * nr_gt, t_res - tw + 1, tw):
            if torch.numel(u_base) == 0:
                base.append(torch.zeros(0))  # no baseline solver data: contributes nothing
                continue
            same = [step] * B
            _, lab_super = self.data_creator.create_data(u_super, same)
            _, lab_base = self.data_creator.create_data(u_base, same)
            base.append(self._loss(lab_super, lab_base).float() / spatial / B)
            n_t += tw
        base_loss = torch.sum(torch.cat([b.reshape(-1).cpu() for b in base]))
        if divide_by_t:
            base_loss = base_loss / (n_t if n_t > 0 else 1)
        unrolled = torch.sum(torch.stack(losses))  # divide_by_t already applied by simulate
        if not include_data:
            return unrolled, base_loss
        gt, pred = torch.cat(sims[0], dim=2), torch.cat(sims[1], dim=2)
        return unrolled, base_loss, [gt, pred, [{} for _ in range(B)]]
