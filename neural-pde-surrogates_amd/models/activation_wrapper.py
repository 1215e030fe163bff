"""activation_wrapper (reference models/activation_wrapper.py:9-108).

Returns an instance of a dynamic subclass `ActWrapper-<model_class>` exactly
like the reference.  On the MI355X path the final tanh and the spatial-cond
mask run inside the decoder kernel; 'individual_static' volume preservation
is two fp64 plane-sum reductions + one element-wise rescale/mask kernel.
"""
import numpy as np
import torch
from torch import nn

import models
from nps_hip import ops
from nps_hip import autograd as ad
from utils.attr import getattr_nested


def _mpd_cumsum(max_pct_dif, tw):
    """fp32 torch.cumsum(ones * max_pct_dif) (activation_wrapper.py:87-88)."""
    return np.cumsum(np.full(tw, np.float32(max_pct_dif), dtype=np.float32), dtype=np.float32)


def activation_wrapper(model_class: str, activation_final: nn.Module, enforce_spatial_cond=False,
                       spatial_cond_channel=0, approx_volume_preserve=False, approx_volume_preserve_mode='block',
                       max_pct_dif=1, *args, **kwargs):
    modeltype = None
    for module in [models.enc_proc_dec_components, models, models.common]:
        if (model_init := getattr_nested(module, model_class)) is not False:
            modeltype = model_init
            break
    if modeltype is None:
        raise ValueError(f"Model {model_class} not found")

    def new_forward(self, *a, **b):
        if not isinstance(self, models.EncProcDec) or not isinstance(activation_final, nn.Tanh):
            raise NotImplementedError("activation_wrapper: the fused MI355X path wraps EncProcDec with Tanh")
        x = b["x"] if "x" in b else a[0]
        fwd_kw = dict(b)
        fwd_kw.pop("x", None)
        names = ["cond", "bc", "pos", "t_cond", "spatial_cond"]
        for n, v in zip(names, a[1:]):
            fwd_kw[n] = v
        sc = fwd_kw.get("spatial_cond")
        if enforce_spatial_cond and (sc is None or torch.numel(sc) == 0):
            raise ValueError("enforce_spatial_cond needs spatial_cond")
        u = self.forward_fused(x, final_tanh=True,
                               mask_channel=spatial_cond_channel if enforce_spatial_cond else None, **fwd_kw)
        if approx_volume_preserve:
            if approx_volume_preserve_mode != 'individual_static':
                raise NotImplementedError(
                    f"approx_volume_preserve_mode '{approx_volume_preserve_mode}' is not on the MI355X path "
                    "(twophase cfgs use 'individual_static')")
            B, c, tw, H, W = u.shape
            key = (float(max_pct_dif), tw, str(u.device))
            if getattr(self, "_mpd_key", None) != key:
                self._mpd_tab = torch.from_numpy(_mpd_cumsum(max_pct_dif, tw)).to(u.device)
                self._mpd_key = key
            mask = sc.float().contiguous() if enforce_spatial_cond else None
            if u.requires_grad:
                return ad.VolumeRescaleFn.apply(spatial_cond_channel, u, x.detach(), self._mpd_tab, mask)
            xc = x.contiguous()
            new_tot = ops.plane_sums(u, 0, H * W, H * W, B * c * tw)                        # :81
            prev_tot = ops.plane_sums(xc, (xc.shape[2] - 1) * H * W, xc.shape[2] * H * W, H * W, B * c)  # :84
            ops.volume_rescale(u, new_tot, prev_tot, self._mpd_tab, mask, spatial_cond_channel)
        return u

    return type(f'ActWrapper-{model_class}', (modeltype,), {'forward': new_forward})(*args, **kwargs)
