"""Generate the golden parity fixtures from the reference implementation.

CONTAINER-ONLY TOOL.  This script imports the upstream reference
(yoeripoels/neural-pde-surrogates, mounted read-only at /root/reference) to
produce small input/output vectors that pin `oracle/` (the CPU restatement).
Nothing on the GPU box or in the product path runs it; only its outputs
(`tests/golden/*.pt`, plain tensors loaded with `weights_only=True`) travel.

The reference has no tests of its own, so these vectors are the
parity anchor.  Each fixture stores: the module kwargs, the seeded reference
`state_dict`, the inputs and the reference outputs (and grads where useful).

Two import-time dependencies of the reference are absent from the image and
unused on the grid path (`torch_geometric`, `mmap_ninja`); they
are replaced by empty stub modules before import.

Usage (from any cwd; run it outside /root/reference so nothing is written there):
    python tests/golden/make_golden.py
"""
import os
import sys
import types
import tempfile
import argparse

sys.dont_write_bytecode = True
REF_SRC = "/root/reference/src"
OUT_DIR = os.path.dirname(os.path.abspath(__file__))


def _install_stubs():
    tg = types.ModuleType("torch_geometric")
    tgd = types.ModuleType("torch_geometric.data")

    class Data:  # never instantiated on the grid path
        pass

    tgd.Data = Data
    tg.data = tgd
    sys.modules["torch_geometric"] = tg
    sys.modules["torch_geometric.data"] = tgd
    mn = types.ModuleType("mmap_ninja")
    mnr = types.ModuleType("mmap_ninja.ragged")

    class RaggedMmap:  # only used by the ragged (1D variable-time) loader
        pass

    mnr.RaggedMmap = RaggedMmap
    mn.ragged = mnr
    sys.modules["mmap_ninja"] = mn
    sys.modules["mmap_ninja.ragged"] = mnr


def main():
    _install_stubs()
    os.chdir(tempfile.mkdtemp())  # reference's utils.misc may mkdir relative to cwd
    sys.path.insert(0, REF_SRC)
    import torch
    from torch import nn
    torch.set_num_threads(8)
    import models
    from models.enc_proc_dec_components.proc_fno import SpectralConv2d, SpectralConv3d, FNO_Layer, FNO
    from models.enc_proc_dec_components.proc_unet_modern import UNetModern
    from models.enc_proc_dec_components.proc_dilatedresnet import DilatedResnet
    from models.enc_proc_dec_components.proc_ufno import UFNO
    from pdes import PDE2D
    from common.interfaces import D
    from trainers.autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer

    def save(name, **payload):
        path = os.path.join(OUT_DIR, f"{name}.pt")
        torch.save(payload, path)
        print(f"wrote {name}.pt  ({os.path.getsize(path) / 1024:.1f} KiB)")

    gen = torch.Generator().manual_seed(1234)

    def rnd(*shape, lo=-1.0, hi=1.0):
        return torch.rand(*shape, generator=gen) * (hi - lo) + lo

    # ---------------- SpectralConv2d (+ grads) ----------------
    cases = [
        ("spectral2d_a", dict(in_channels=6, out_channels=5, modes=(4, 3)), (2, 6, 16, 12)),
        # 2*m1 > H: the second corner write wins (proc_fno.py:266-269); odd W
        ("spectral2d_overlap", dict(in_channels=3, out_channels=4, modes=(4, 3)), (2, 3, 6, 7)),
        # m2 == W//2+1: Nyquist column kept (imag discarded by c2r)
        ("spectral2d_nyq", dict(in_channels=3, out_channels=2, modes=(3, 5)), (1, 3, 8, 8)),
    ]
    for name, kw, xs in cases:
        torch.manual_seed(42)
        m = SpectralConv2d(**kw)
        x = rnd(*xs).requires_grad_(True)
        y = m(x)
        g = rnd(*y.shape)
        y.backward(g)
        save(name, kwargs=dict(kw, modes=list(kw["modes"])), state_dict=m.state_dict(), x=x.detach(), y=y.detach(),
             g=g, dx=x.grad, dw1=m.weights1.grad, dw2=m.weights2.grad)

    # ---------------- SpectralConv3d ----------------
    torch.manual_seed(42)
    kw = dict(in_channels=3, out_channels=4, modes=(3, 3, 2))
    m = SpectralConv3d(**kw)
    x = rnd(2, 3, 8, 8, 6)
    with torch.no_grad():
        y = m(x)
    save("spectral3d", kwargs=dict(kw, modes=list(kw["modes"])), state_dict=m.state_dict(), x=x, y=y)

    # ---------------- FNO_Layer ----------------
    torch.manual_seed(42)
    kw = dict(hidden_dim=6, num_spatial_dims=2, modes=4, hidden_dim_out=5, padding_mode="circular")
    m = FNO_Layer(**kw)
    x = rnd(2, 6, 16, 16)
    with torch.no_grad():
        y = m(x)
    save("fno_layer", kwargs=kw, state_dict=m.state_dict(), x=x, y=y)

    # ---------------- processors ----------------
    def proc_case(name, cls, kw, hshape, n_cond):
        torch.manual_seed(42)
        m = cls(pde=None, **kw)
        h = rnd(*hshape)
        vb = rnd(hshape[0], n_cond, *hshape[2:], lo=0.0, hi=1.0)
        with torch.no_grad():
            y = m(h=h, variables_broadcast=vb, pos=None)
        save(name, kwargs={k: v for k, v in kw.items() if k != "activation"}, state_dict=m.state_dict(),
             h=h, vb=vb, y=y)

    gelu = nn.GELU()
    proc_case("unet_ufno_style", UNetModern,
              dict(num_spatial_dims=2, n_cond=2, hidden_features=8, activation=gelu, norm=True, ch_mults=[1, 1],
                   is_attn=[False, False], mid_attn=False, n_blocks=1, use1x1=True, padding_mode="circular"),
              (2, 8, 20, 20), 2)
    proc_case("unet_cfg", UNetModern,
              dict(num_spatial_dims=2, n_cond=2, hidden_features=8, activation=gelu, norm=True, ch_mults=[2, 2, 1, 2],
                   is_attn=[False] * 4, mid_attn=False, n_blocks=2, use1x1=True, padding_mode="circular"),
              (2, 8, 64, 64), 2)
    proc_case("unet_ones", UNetModern,
              dict(num_spatial_dims=2, n_cond=1, hidden_features=4, activation=gelu, norm=False, ch_mults=[1, 2],
                   is_attn=[False] * 2, mid_attn=False, n_blocks=1, use1x1=False, padding_mode="ones"),
              (2, 4, 16, 16), 1)
    proc_case("drn", DilatedResnet,
              dict(num_spatial_dims=2, n_cond=2, hidden_features=6, kernel_size=5, hidden_blocks=2, activation=gelu,
                   padding_mode="circular"),
              (2, 6, 20, 20), 2)
    proc_case("ufno", UFNO,
              dict(num_spatial_dims=2, n_cond=2, hidden_features=8, hidden_blocks=2, fno_modes=4, activation=gelu,
                   norm=True, ch_mults=[1, 1], is_attn=[False, False], mid_attn=False, n_blocks=1, use1x1=True,
                   padding_mode="circular"),
              (2, 8, 24, 24), 2)
    proc_case("fno", FNO,
              dict(num_spatial_dims=2, n_cond=2, hidden_features=8, hidden_blocks=2, fno_modes=4,
                   padding_mode="circular"),
              (2, 8, 16, 16), 2)

    # ---------------- full ActWrapper-EncProcDec models + simulate ----------------
    base_model = dict(
        object="activation_wrapper", activation_final=nn.Tanh(), enforce_spatial_cond=True, spatial_cond_channel=0,
        approx_volume_preserve=True, approx_volume_preserve_mode="individual_static", max_pct_dif=1 / 25,
        model_class="EncProcDec", num_spatial_dims=2, time_window=25, data_structure="grid",
        processor_residual=False, encoder="enc_grid.ElementWise", activation=gelu,
        decoder="dec_grid.TimeConvDense", dec_delta_mode="per_step")
    model_cfgs = {
        "model_ufno": (dict(num_c=3, processor="UFNO", fno_modes=4, hidden_blocks=2, hidden_features=16,
                            fno_kernel_size=1, fno_conv_mode="single", padding_mode="circular", ch_mults=[1, 1],
                            is_attn=[False, False], mid_attn=False, norm=True, use1x1=True), 16),
        # the full cfg_twophase_unet processor structure is pinned by `unet_cfg` above; here a smaller
        # UNet keeps the fixture small while covering the composition
        "model_unet": (dict(num_c=1, processor="UNetModern", ch_mults=[1, 2], is_attn=[False] * 2,
                            mid_attn=False, hidden_features=8, norm=True, use1x1=True, cond_mode="concat",
                            padding_mode="circular", dec_kernel_size=5, dec_padding_mode="circular"), 32),
        "model_drn": (dict(num_c=1, processor="DilatedResnet", kernel_size=5, hidden_blocks=2, hidden_features=8,
                           padding_mode="circular", dec_kernel_size=5, dec_padding_mode="circular"), 16),
        "model_ufno_fno": (dict(num_c=1, hidden_blocks=1, processor=[dict(object="FNO"), dict(object="UFNO")],
                                fno_modes=4, hidden_features=16, fno_kernel_size=1, fno_conv_mode="single",
                                padding_mode="circular", ch_mults=[1, 1], is_attn=[False, False], mid_attn=False,
                                norm=True, use1x1=True), 20),
    }
    for name, (extra, res) in model_cfgs.items():
        torch.manual_seed(42)
        cfg = dict(base_model, **extra)
        pde = PDE2D(tmin=0.0, tmax=1.0, nt=501, L1=1.0, L2=1.0, nx1=res, nx2=res, x=None, name="twophase",
                    n_cond_static=3, n_cond_spatial=1)
        kw = dict(cfg)
        kw.pop("object")
        model = models.activation_wrapper(**{k: (dict(v) if isinstance(v, dict) else
                                                 ([dict(p) for p in v] if isinstance(v, list) and v and isinstance(v[0], dict) else v))
                                             for k, v in kw.items()}, pde=pde)
        model.eval()
        B, c, tw = 2, cfg["num_c"], 25
        T = 100
        # smooth two-phase fronts in [0,1] plus a little noise
        xs = torch.linspace(0, 1, res)
        X, Y = torch.meshgrid(xs, xs, indexing="ij")
        ts = torch.linspace(0, 1, T)
        phase = torch.rand(B, c, 1, 1, 1, generator=gen) * 6.28
        u = 0.5 + 0.5 * torch.tanh((Y[None, None, None] - 0.3 - 0.4 * ts[None, None, :, None, None]
                                    - 0.1 * torch.sin(2 * 3.14159265 * X[None, None, None] + phase)) / 0.05)
        u = (u + 0.02 * torch.rand(B, c, T, res, res, generator=gen)).float()
        cond = torch.rand(B, 3, generator=gen)
        pos = torch.stack([X, Y], dim=-1)[None].repeat(B, 1, 1, 1)
        spatial_cond = (torch.rand(B, 1, res, res, generator=gen) > 0.9).float()
        x_in = u[:, :, :tw]
        with torch.no_grad():
            y = model(x_in, cond=cond, bc=None, pos=pos, t_cond=None, spatial_cond=spatial_cond)
        # autoregressive rollout through the reference's own simulate
        # (autoregressivepushforwardtrainer.py:288-440)
        config = argparse.Namespace(time_window=tw, base_resolution=(T, res, res), device="cpu", nr_gt_steps=1)
        data = types.SimpleNamespace(pde=pde, data_interface=D.sim2d)
        trainer = AutoregressivePushforwardTrainer(model=model, data=data, criterion=nn.MSELoss(reduction="sum"),
                                                   optimizer=None, lr_scheduler=None, config=config)
        with torch.no_grad():
            losses, (data_gt, data_pred) = trainer.simulate(u, cond, pos, compute_loss=True, include_data=True,
                                                            nr_gt_steps=1, t_res=T,
                                                            spatial_conditioning=spatial_cond)
        save(name, cfg={k: v for k, v in cfg.items() if k not in ("activation", "activation_final")},
             pde=dict(tmin=0.0, tmax=1.0, nt=501, nx1=res, nx2=res, n_cond_static=3, n_cond_spatial=1),
             state_dict=model.state_dict(), u=u, cond=cond, pos=pos, spatial_cond=spatial_cond,
             y=y, sim_losses=torch.stack([l.reshape(()) for l in losses]),
             sim_pred=torch.cat(data_pred[1:], dim=2))  # data_pred[0] is u[:, :, :tw]


if __name__ == "__main__":
    main()
