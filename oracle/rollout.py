"""Oracle restatement of the autoregressive rollout (test infrastructure only).

AutoregressivePushforwardTrainer.simulate, trainers/autoregressivepushforwardtrainer.py:288-440,
with DataCreator.create_data (common/data_creator.py:48-78) as plain slicing.
Grid models only (model_interface AR_TB), no BC processing (process_step is a
no-op for twophase, utils/process_output.py:53-54), no mask.
"""
import math

import torch


def simulate(model, u, cond, pos, spatial_cond, tw, t_res, nr_gt_steps=1, compute_loss=True, include_data=True,
             divide_by_t=True):
    B = u.shape[0]
    pred = u[:, :, tw * nr_gt_steps - tw: tw * nr_gt_steps]          # :332-334
    preds, losses = [pred], []
    n_t = 0
    for step in range(tw * nr_gt_steps, t_res - tw + 1, tw):       # :354-358
        pred = model(pred, cond=cond, pos=pos, spatial_cond=spatial_cond)  # :401
        if compute_loss:
            labels = u[:, :, step: step + tw]                       # :363-364
            loss = torch.sum((pred - labels) ** 2) / math.prod(u.shape[3:])  # nn.MSELoss(sum), :422
            losses.append(loss / B)
        if include_data:
            preds.append(pred)
        n_t += tw
    if divide_by_t:
        losses = [v / n_t for v in losses]
    return losses, preds
