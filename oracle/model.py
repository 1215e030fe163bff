"""Oracle restatement of the full `activation_wrapper(EncProcDec)` grid model (test infrastructure only).

activation_wrapper.py:9-108, enc_proc_dec.py:41-183, models/base.py:24-73.
Supports the components the twophase cfgs use: encoder enc_grid.ElementWise,
processors UFNO / FNO / UNetModern / DilatedResnet (single or list), decoder
dec_grid.TimeConvDense with dec_delta_mode='per_step'.
"""
import torch

from . import functional as Fo


class OracleModel:
    def __init__(self, cfg, pde, state_dict):
        self.cfg = dict(cfg)
        self.pde = dict(pde)
        self.sd = {k: v.detach().to("cpu", copy=False) for k, v in state_dict.items()}
        self.dt = self.pde["tmax"] / (self.pde["nt"] - 1)  # pdes/base.py:43
        self.num_c = self.cfg.get("num_c", 1)
        self.tw = self.cfg.get("time_window", 25)
        self.n_cond = self.pde.get("n_cond_static", 0) + self.pde.get("n_cond_spatial", 0)  # enc_proc_dec.py:87
        proc = self.cfg["processor"]
        self.processors = proc if isinstance(proc, (list, tuple)) else [proc]

    def _proc_cfg(self, i):
        p = self.processors[i]
        base = {k: v for k, v in self.cfg.items() if k not in ("processor",)}
        base["n_cond"] = self.n_cond
        if isinstance(p, dict):
            base.update({k: v for k, v in p.items() if k != "object"})
            return p["object"], base
        return p, base

    def core_forward(self, x, cond, pos, spatial_cond):
        """EncProcDec.forward, enc_proc_dec.py:117-183 (grid branch, no bc encoder)."""
        u = x
        variables = None
        if cond is not None and cond.numel() > 0:
            variables = torch.stack([cond[:, i] for i in range(cond.shape[1])], dim=1)  # base.py:333-360
        H, W = u.shape[3:]
        if variables is not None:
            vb = variables[:, :, None, None].repeat(1, 1, H, W)  # utils/broadcast_to_grid.py:4-14
            vb = torch.cat([vb, spatial_cond], dim=1) if spatial_cond is not None else vb
        else:
            vb = spatial_cond
        h = Fo.enc_elementwise(self.sd, "encoder", u, pos, vb)
        for i in range(len(self.processors)):
            name, pcfg = self._proc_cfg(i)
            pre = f"processor.{i}"
            if name == "UFNO":
                h_next = Fo.ufno(self.sd, pre, pcfg, h, vb)
            elif name == "FNO":
                h_next = Fo.fno(self.sd, pre, pcfg, h, vb)
            elif name == "UNetModern":
                h_next = Fo.unet_modern(self.sd, pre, pcfg, h, vb)
            elif name == "DilatedResnet":
                h_next = Fo.dilated_resnet(self.sd, pre, pcfg, h, vb)
            else:
                raise ValueError(f"oracle: unsupported processor {name}")
            h = h_next + h if (self.cfg.get("processor_residual", False) and i > 0) else h_next
        return Fo.dec_timeconvdense(self.sd, "decoder", h, u, self.dt, self.num_c, self.tw)

    def __call__(self, x, cond=None, pos=None, spatial_cond=None):
        """activation_wrapper.new_forward, activation_wrapper.py:33-106 ('individual_static' mode)."""
        u = torch.tanh(self.core_forward(x, cond, pos, spatial_cond))
        enforce = self.cfg.get("enforce_spatial_cond", False)
        ch = self.cfg.get("spatial_cond_channel", 0)

        def apply_sc(v):  # :25-31
            m = spatial_cond[:, ch][:, None, None]
            return v - m * v

        if enforce:
            u = apply_sc(u)
        if self.cfg.get("approx_volume_preserve", False):
            mode = self.cfg.get("approx_volume_preserve_mode", "block")
            if mode != "individual_static":
                raise ValueError("oracle: only approx_volume_preserve_mode='individual_static' is restated")
            mpd = self.cfg.get("max_pct_dif", 1)
            new_tot = torch.sum(u, dim=(3, 4))                                     # :81
            prev = torch.sum(x[:, :, -1, ...], dim=(2, 3))[:, :, None].repeat(1, 1, u.shape[2])  # :84-86
            mpd_all = torch.cumsum(torch.ones_like(new_tot) * mpd, dim=2)          # :87-88
            dif = (1 - new_tot / prev) * 100
            dif = torch.tanh(dif / mpd_all) / 100 * mpd_all
            resc = 1 - dif
            u = (u / new_tot[..., None, None]) * (resc * prev)[..., None, None]    # :101
            if enforce:
                u = apply_sc(u)
        return u


def build_oracle_model(cfg, pde, state_dict):
    return OracleModel(cfg, pde, state_dict)
