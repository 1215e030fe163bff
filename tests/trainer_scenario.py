"""The train.py call sequence (reference src/train.py:102-165, `get_config_static` :22-99 included) on a small
synthetic twophase dataset, parameterised by the `models` / `trainers` / `data` packages it resolves names
against.  tests/golden/make_golden_trainer.py runs it against the REFERENCE's packages on the CPU and
stores the returned numbers; tests/test_gpu_trainer.py runs the same function against the MI355X mirror
on the GPU and compares.  Only plain numbers / tensors leave this function.
"""
import os
import random

import numpy as np
import torch
from torch import nn

from data_fixture import write_twophase_dataset

# N, C, T, X1, X2: 9 trajectories of 8 channels, 101 timesteps (3 windows of tw = 25 per rollout), 32x32
SHAPE = (9, 8, 101, 32, 32)
SPLIT = dict(train=[0, 2, 3, 5, 7], valid=[1, 6], test=[4, 8])
SEED = 42  # configs/train/defaults/base.py:4, applied by configs/parse.py:318

DATASET = dict(object="PDE2DDataset", experiment="twophase", split_file="split", data_format="memmap",
               data_file="snapshots", conditioning="conditioning", spatial_conditioning="spatial_conditioning",
               name="twophase", preprocess=False, c_filter=[2, 4, 6])
TRAINER = dict(object="AutoregressivePushforwardTrainer", neighbors=3, time_window=25, base_resolution=(101, 32, 32),
               super_resolution=(101, 32, 32), batch_size=2, nr_gt_steps=1, nw=0, num_epochs=3,
               lr_step_interval=1, unrolling=2, print_interval=1, test_interval=1,
               max_train_batches=float("inf"), max_test_batches=float("inf"),
               print_setting=dict(print_per_step=True), process_settings={})
# cfg_twophase_ufno.py's model dict at reduced width (hidden 16, 4 modes, 2 blocks) and 3 fields
MODEL = dict(object="activation_wrapper", activation_final=nn.Tanh(), enforce_spatial_cond=True,
             spatial_cond_channel=0, approx_volume_preserve=True, approx_volume_preserve_mode="individual_static",
             max_pct_dif=1 / 25, model_class="EncProcDec", num_c=3, num_spatial_dims=2, time_window=25,
             data_structure="grid", processor_residual=False, encoder="enc_grid.ElementWise", activation=nn.GELU(),
             processor="UFNO", fno_modes=4, hidden_blocks=2, hidden_features=16, fno_kernel_size=1,
             fno_conv_mode="single", padding_mode="circular", ch_mults=[1, 1], is_attn=[False, False],
             mid_attn=False, norm=True, use1x1=True, decoder="dec_grid.TimeConvDense", dec_delta_mode="per_step")
OPTIMIZER = dict(lr=1e-4)                                   # defaults/optimizer.py Adam
LR_SCHEDULER = dict(milestones=[1, 5, 10, 15], gamma=0.4)   # defaults/lr_scheduler.py MultiStepLR


def write_dataset(root):
    d = write_twophase_dataset(root, shape=SHAPE, with_split=False, seed=77)
    import yaml
    with open(os.path.join(d, "split.yaml"), "w") as f:
        yaml.safe_dump(SPLIT, f)
    cfg_path = os.path.join(d, "snapshots.yaml")
    with open(cfg_path) as f:
        cfg = yaml.safe_load(f)
    cfg.update(x1=[float(v) for v in np.linspace(0.0, 1.0, SHAPE[3])],
               x2=[float(v) for v in np.linspace(0.0, 1.0, SHAPE[4])], tmin=0.0, tmax=1.0, dt=0.01)
    with open(cfg_path, "w") as f:
        yaml.safe_dump(cfg, f)
    return root


def _f(x):
    return float(x.item()) if isinstance(x, torch.Tensor) else float(x)


def run(models, trainers, data, device, root, save_dir):
    """train.py:102-165 with the cfg above; returns every number train.py prints or pickles."""
    random.seed(SEED)
    np.random.seed(SEED)
    torch.manual_seed(SEED)
    dataset_kw = {k: v for k, v in DATASET.items() if k != "object"}
    dataset = getattr(data, DATASET["object"])(base_path=root, **dataset_kw)
    model_kw = {k: v for k, v in MODEL.items() if k != "object"}
    model = getattr(models, MODEL["object"])(**model_kw, pde=dataset.pde).to(device)
    criterion = nn.MSELoss(reduction="sum")
    config = type("Config", (), {})()
    for k, v in TRAINER.items():
        if k != "object":
            setattr(config, k, v)
    config.device = device
    import argparse
    config = argparse.Namespace(**vars(config))
    trainer = getattr(trainers, TRAINER["object"])(
        model=model, data=dataset, config=config, criterion=criterion, optimizer=None, lr_scheduler=None,
        save_path=os.path.join(save_dir, "run"), epoch_callback=None, use_wandb=False, wandb_kwargs=None,
        wandb_config_dict={})
    _, valid_loader, test_loader = trainer.get_dataloaders()                               # train.py:128
    shape = list(next(iter(valid_loader))[1].size())                                       # :129
    valid_loss, valid_summary = trainer.test(valid_loader)                                 # :130
    optimizer = torch.optim.Adam(trainer.get_parameters(), **OPTIMIZER)                    # :135-137
    lr_scheduler = torch.optim.lr_scheduler.MultiStepLR(optimizer, **LR_SCHEDULER)         # :138-141
    trainer.set_optimizer(optimizer)                                                        # :144
    trainer.set_lr_scheduler(lr_scheduler)                                                  # :145
    n_params = sum(p.numel() for p in trainer.get_parameters() if p.requires_grad)         # :152
    train_losses, val_losses, val_stats = trainer.train()                                  # :154
    test_loss, test_summary = trainer.test(test_loader)                                    # :162
    state = {k: v.detach().cpu().clone() for k, v in model.state_dict().items()}
    return dict(
        shape=shape, n_params=n_params,
        valid_loss=_f(valid_loss), valid_summary={k: _f(v) for k, v in valid_summary.items()},
        train_losses=[_f(v) for v in train_losses],
        val_losses={k: [_f(v) for v in vs] for k, vs in val_losses.items()},
        val_stats={k: [{kk: _f(vv) for kk, vv in s.items()} for s in vs] for k, vs in val_stats.items()},
        test_loss=_f(test_loss), test_summary={k: _f(v) for k, v in test_summary.items()},
        lr=float(optimizer.param_groups[0]["lr"]),
        checkpoints=sorted(os.listdir(save_dir)),
        final_state=state,
    )
