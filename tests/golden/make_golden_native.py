"""Generate the native-geometry fixtures (the twophase cfgs' own base_resolution) from the reference.

CONTAINER-ONLY TOOL (imports /root/reference, like make_golden.py; see its header for the stubbed imports).
Every twophase cfg sets base_resolution = (501, 96, 64) (reference src/configs/train/cfg_twophase_ufno.py:6-7,
cfg_twophase_unet.py, cfg_twophase_drn.py), so that is the geometry an unchanged train.py feeds the models.
For each of the three cfg models at full width — U-FNO (hidden 192, 3 blocks, modes 10), UNetModern (hidden 32,
ch_mults [2, 2, 1, 2]), DilatedResnet (hidden 128, k 5, 2 blocks) — with num_c = 1, twophase with the disc
obstacle, B = 2, t_res = 110: the reference's own `simulate` (autoregressivepushforwardtrainer.py:288-440) makes
3 model calls (windows 25, 50, 75; range(25, t_res - tw + 1, tw) at :354-358) and skips the partial last window
[100, 110).

Like make_golden_c1.py the fixture stores no weights and no trajectory (both regenerated from seeds by the mirror
and pinned by fp64 checksums), only the outputs of every window and the per-window losses.

Usage: python tests/golden/make_golden_native.py
"""
import argparse
import os
import sys
import tempfile
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _install_stubs, REF_SRC  # noqa: E402
from make_golden_c1 import _load_synthetic, checksums  # noqa: E402

SEED_DATA = 4242
B, NUM_C, T, H, W, TW = 2, 1, 110, 96, 64, 25

WRAP = dict(enforce_spatial_cond=True, spatial_cond_channel=0, approx_volume_preserve=True,
            approx_volume_preserve_mode="individual_static", max_pct_dif=1 / 25, model_class="EncProcDec",
            num_c=NUM_C, num_spatial_dims=2, time_window=TW, data_structure="grid", processor_residual=False,
            encoder="enc_grid.ElementWise", decoder="dec_grid.TimeConvDense", dec_delta_mode="per_step")
CFGS = {  # the processor sections of cfg_twophase_{ufno,unet,drn}.py
    "ufno": dict(processor="UFNO", fno_modes=10, hidden_blocks=3, hidden_features=192, fno_kernel_size=1,
                 fno_conv_mode="single", padding_mode="circular", ch_mults=[1, 1], is_attn=[False, False],
                 mid_attn=False, norm=True, use1x1=True),
    "unet": dict(processor="UNetModern", ch_mults=[2, 2, 1, 2], is_attn=[False] * 4, mid_attn=False,
                 hidden_features=32, norm=True, use1x1=True, cond_mode="concat", padding_mode="circular",
                 dec_kernel_size=5, dec_padding_mode="circular"),
    "drn": dict(processor="DilatedResnet", kernel_size=5, hidden_blocks=2, hidden_features=128,
                padding_mode="circular", dec_kernel_size=5, dec_padding_mode="circular"),
}


def main():
    syn = _load_synthetic()
    _install_stubs()
    os.chdir(tempfile.mkdtemp())
    sys.path.insert(0, REF_SRC)
    import torch
    from torch import nn
    torch.set_num_threads(8)
    import models
    from pdes import PDE2D
    from common.interfaces import D
    from trainers.autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer

    pde_kw = dict(tmin=0.0, tmax=1.0, nt=501, nx1=H, nx2=W, n_cond_static=3, n_cond_spatial=1)
    u, cond, pos, sc = syn.twophase_batch(B, NUM_C, T, H, W, seed=SEED_DATA, obstacle="disc")
    for name, proc in CFGS.items():
        cfg = dict(WRAP, **proc, activation=nn.GELU(), activation_final=nn.Tanh())
        pde = PDE2D(L1=1.0, L2=1.0, x=None, name="twophase", **pde_kw)
        torch.manual_seed(42)
        model = models.activation_wrapper(**cfg, pde=pde).eval()
        config = argparse.Namespace(time_window=TW, base_resolution=(T, H, W), device="cpu", nr_gt_steps=1)
        trainer = AutoregressivePushforwardTrainer(model=model, data=types.SimpleNamespace(pde=pde,
                                                                                           data_interface=D.sim2d),
                                                   criterion=nn.MSELoss(reduction="sum"), optimizer=None,
                                                   lr_scheduler=None, config=config)
        with torch.no_grad():
            losses, (gt, preds) = trainer.simulate(u, cond, pos, compute_loss=True, include_data=True,
                                                   nr_gt_steps=1, t_res=T, spatial_conditioning=sc)
        assert len(preds) == 4, len(preds)  # the ground-truth window + 3 calls; [100, 110) skipped
        payload = dict(
            cfg={k: v for k, v in cfg.items() if k not in ("activation", "activation_final")},
            pde=pde_kw,
            data=dict(B=B, num_c=NUM_C, T=T, H=H, W=W, seed=SEED_DATA, obstacle="disc"),
            state_checksums=checksums(model.state_dict()),
            input_checksums=checksums(dict(u=u, cond=cond, pos=pos, sc=sc)),
            sim_losses=torch.stack([l.reshape(()) for l in losses]),
            sim_pred=torch.cat(preds[1:], dim=2))
        path = os.path.join(HERE, f"native_{name}_96x64.pt")
        torch.save(payload, path)
        print(f"wrote {path} ({os.path.getsize(path) / 1024:.1f} KiB)", flush=True)


if __name__ == "__main__":
    main()
