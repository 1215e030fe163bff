"""Grid decoders (reference models/enc_proc_dec_components/dec_grid.py).

TimeConvDense: the pre_decoder 1x1 conv writes a planar (B, 3*c*tw, H, W)
buffer straight from its epilogue; one HIP kernel then runs the per-pixel
Conv1d(k=ceil(tw/2), s=2) -> GELU -> Conv1d chain, add_delta('per_step') and,
when called through activation_wrapper, the final tanh and obstacle mask.
"""
import math

import numpy as np
import torch
from torch import nn

from models.common import get_conv_with_right_spatial_dim, Swish, activation_code, use_autograd
from nps_hip import ops
from nps_hip import autograd as ad
from pdes import PDE


def add_delta(delta, u, pde_dt, time_window, num_spatial_dims, delta_mode='per_step', delta_dt=True):
    """dec_grid.py:8-31 — fused into nps_timeconv_decode on the MI355X path."""
    raise NotImplementedError("add_delta runs fused inside the TimeConvDense HIP kernel")


def dt_cumsum(pde_dt, time_window):
    """fp32 cumsum of (ones(tw) * dt), exactly as dec_grid.py:14-15 builds it."""
    return np.cumsum(np.full(time_window, np.float32(pde_dt), dtype=np.float32), dtype=np.float32)


class TimeConvDense(nn.Module):
    """dec_grid.py:97-146."""

    def __init__(self, pde: PDE, num_c, num_spatial_dims, time_window, hidden_features, activation,
                 dec_delta_mode='per_step', dec_delta_dt=True, **kwargs):
        super().__init__()
        self.pde = pde
        self.num_spatial_dims = num_spatial_dims
        self.time_window = time_window
        self.num_c = num_c
        self.dec_delta_mode = dec_delta_mode
        self.dec_delta_dt = dec_delta_dt
        decoder_input_dim = time_window * 3 * num_c
        self.pre_decoder = get_conv_with_right_spatial_dim(num_spatial_dims, in_channels=hidden_features,
                                                           out_channels=decoder_input_dim, kernel_size=1)
        kernel_size_a = math.ceil(time_window / 2)
        kernel_size_b = math.ceil(time_window / 4) + 1
        if time_window % 4 == 0:
            kernel_size_b += 1
        self.decoder = nn.Sequential(nn.Conv1d(num_c, num_c * 2, kernel_size_a, stride=2),
                                     activation,
                                     nn.Conv1d(num_c * 2, num_c, kernel_size_b, stride=1))

    def _dtcum(self, device):
        dt = self.pde.dt if self.dec_delta_dt else 1
        key = (float(dt), self.time_window, str(device))
        if getattr(self, "_dt_key", None) != key:
            self._dt_tab = torch.from_numpy(dt_cumsum(dt, self.time_window)).to(device)
            self._dt_key = key
        return self._dt_tab

    def run(self, h, u, final_tanh=False, mask=None, mask_ch=0):
        """h: (B,H,W,hidden) NHWC; u: model input (B,c,tw,H,W).  Returns (B,c,tw,H,W)."""
        if self.dec_delta_mode != 'per_step':
            raise NotImplementedError("TimeConvDense: dec_delta_mode='per_step' only on the MI355X path")
        if activation_code(self.decoder[1]) != ops.GELU:
            raise NotImplementedError("TimeConvDense: GELU activation only")
        H, W = h.shape[1:3]
        pre = self.pre_decoder.run([ops.Src(h)], (H, W), out_nchw=True)
        c1, c2 = self.decoder[0], self.decoder[2]
        return ops.timeconv_decode(pre, u.contiguous(), c1.weight.detach().contiguous(), c1.bias.detach(),
                                   c2.weight.detach().contiguous(), c2.bias.detach(), self._dtcum(h.device), mask,
                                   mask_ch, final_tanh, self.num_c, self.time_window)

    def run_ad(self, h, u, final_tanh=False, mask=None, mask_ch=0):
        """Differentiable form of run(): pre-decoder conv, planar transpose, fused conv1d-chain kernel."""
        if self.dec_delta_mode != 'per_step':
            raise NotImplementedError("TimeConvDense: dec_delta_mode='per_step' only on the MI355X path")
        if activation_code(self.decoder[1]) != ops.GELU:
            raise NotImplementedError("TimeConvDense: GELU activation only")
        pre = ad.to_nchw(ad.conv2d(self.pre_decoder, h))
        c1, c2 = self.decoder[0], self.decoder[2]
        return ad.TimeConvDecodeFn.apply((mask_ch, bool(final_tanh), self.num_c, self.time_window), pre,
                                         u.contiguous(), c1.weight, c1.bias, c2.weight, c2.bias,
                                         self._dtcum(h.device), mask)

    def forward(self, h: torch.Tensor, u: torch.Tensor, **kwargs):
        if use_autograd(self):
            return self.run_ad(ad.to_nhwc(h), u)
        return self.run(ops.nchw_to_nhwc(h), u)


class TimeConv(nn.Module):
    """dec_grid.py:34-94 — parameters only (not used by the twophase cfgs)."""

    def __init__(self, pde: PDE, num_c, num_spatial_dims, time_window, hidden_features, dec_delta_mode='per_step',
                 dec_delta_dt=True, **kwargs):
        super().__init__()
        var = time_window + 9
        stride = hidden_features // var
        assert stride > 0, "found stride 0 -- most likely, hidden_features is too small!"
        kernelsize = hidden_features - stride * var + 1
        self.decoder = nn.Sequential(nn.Conv1d(1, 8, kernelsize, stride=stride), Swish(), nn.Conv1d(8, num_c, 10))

    def forward(self, h, u, **kwargs):
        raise NotImplementedError("dec_grid.TimeConv is not on the MI355X path")


class LinearConv(nn.Module):
    """dec_grid.py:34-59 — parameters only."""

    def __init__(self, pde: PDE, num_c, num_spatial_dims, time_window, hidden_features, dec_kernel_size,
                 dec_padding_mode, dec_delta_mode='per_step', dec_delta_dt=True, **kwargs):
        super().__init__()
        self.decoder = get_conv_with_right_spatial_dim(num_spatial_dims, in_channels=hidden_features,
                                                       out_channels=num_c * time_window, kernel_size=dec_kernel_size,
                                                       padding="same", padding_mode=dec_padding_mode)

    def forward(self, h, u, **kwargs):
        raise NotImplementedError("dec_grid.LinearConv is not on the MI355X path")
