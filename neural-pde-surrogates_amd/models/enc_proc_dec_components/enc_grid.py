"""Grid encoders (reference models/enc_proc_dec_components/enc_grid.py)."""
import torch
from torch import nn

from models.common import get_conv_with_right_spatial_dim, Swish, activation_code, use_autograd
from nps_hip import ops
from nps_hip import autograd as ad
from pdes import PDE


class LinearConv(nn.Module):
    """enc_grid.py:7-21 — parameters only (not used by the twophase cfgs)."""

    def __init__(self, pde: PDE, num_c, num_spatial_dims, time_window, hidden_features, enc_kernel_size,
                 enc_padding_mode, **kwargs):
        super().__init__()
        self.encoder = get_conv_with_right_spatial_dim(num_spatial_dims, in_channels=num_c * time_window,
                                                       out_channels=hidden_features, kernel_size=enc_kernel_size,
                                                       padding="same", padding_mode=enc_padding_mode)

    def forward(self, u, **kwargs):
        raise NotImplementedError("enc_grid.LinearConv is not on the MI355X path")


class ElementWise(nn.Module):
    """enc_grid.py:24-50: cat(u, pos, vb) -> 1x1 -> act -> 1x1 -> act, two fused HIP launches."""

    def __init__(self, pde: PDE, num_c, num_spatial_dims, time_window, hidden_features, n_cond, activation=Swish(),
                 **kwargs):
        super().__init__()
        num_channels = num_c * time_window
        self.n_in = num_channels + num_spatial_dims + n_cond
        self.encoder = nn.Sequential(
            get_conv_with_right_spatial_dim(num_spatial_dims, in_channels=num_channels + num_spatial_dims + n_cond,
                                            out_channels=hidden_features, kernel_size=1),
            activation,
            get_conv_with_right_spatial_dim(num_spatial_dims, in_channels=hidden_features,
                                            out_channels=hidden_features, kernel_size=1),
            activation,
        )

    def run_packed(self, xin):
        """xin: (B,H,W,Cp) NHWC packed [u | pos | vb | 0-pad] (nps_pack_grid_input)."""
        act = activation_code(self.encoder[1])
        c1, c2 = self.encoder[0], self.encoder[2]
        H, W = xin.shape[1:3]
        # xin carries <= 3 zero channels of padding; the packed weight is zero-padded to
        # 16-channel chunks, so the same packed buffer serves (ceil16(Cp) == ceil16(n_in)).
        h = c1.run([ops.Src(xin)], (H, W), act=act)
        # the output carries its GroupNorm(1) moments (a U-Net processor's first norm reads it): no statistics pass
        st = ops.new_stats(h.shape[0], h)
        return ops.attach_stats(c2.run([ops.Src(h)], (H, W), act=act, out_stats=st), st)

    def run_packed_ad(self, xin):
        """Differentiable form of run_packed (the packed input is data: no gradient flows into it)."""
        act = activation_code(self.encoder[1])
        h = ad.act(ad.conv2d(self.encoder[0], xin), act)
        return ad.act(ad.conv2d(self.encoder[2], h), act)

    def forward(self, u: torch.Tensor, pos: torch.Tensor, variables_broadcast: torch.Tensor = None, **kwargs):
        if pos.dim() != 4:
            raise NotImplementedError("ElementWise: 2-D grids only on the MI355X path")
        B = u.shape[0]
        vb = variables_broadcast
        K = 0 if vb is None else vb.shape[1]
        Cp = ((self.n_in + 3) // 4) * 4
        # the broadcast conditioning is already a spatial field here: pass it as spatial channels
        xin, _ = ops.pack_grid_input(u.contiguous(), pos.contiguous(), None, vb.contiguous() if vb is not None else None, Cp)
        if use_autograd(self):
            return ad.to_nchw(self.run_packed_ad(xin))
        return ops.nhwc_to_nchw(self.run_packed(xin))
