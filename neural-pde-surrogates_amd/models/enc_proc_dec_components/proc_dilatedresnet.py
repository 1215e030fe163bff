"""Dilated ResNet processor (reference models/enc_proc_dec_components/proc_dilatedresnet.py).

7 dilated convs (d = 1,2,4,8,4,2,1) per block, GELU after each, residual add.
Each conv is one HIP launch; dilated convs are tiled on the dilation lattice,
circular 'same' padding is a wrap in the patch loader, the trailing GELU and
the residual `h + block(...)` are fused into the last conv's epilogue.
"""
import torch
from torch import nn

from common.interfaces import D, M
from models.common import get_conv_with_right_spatial_dim, activation_code, use_autograd
from nps_hip import ops
from nps_hip import autograd as ad
from pdes import PDE


class DilatedResnet(nn.Module):
    """proc_dilatedresnet.py:15-50."""
    model_interface = M.AR_TB
    data_interface = [D.sim1d, D.sim2d, D.sim1d_var_t]

    def __init__(self, pde: PDE, hidden_features: int = 128, kernel_size: int = 3, hidden_blocks: int = 4,
                 activation: nn.Module = nn.ReLU(), padding_mode: str = 'zeros', num_spatial_dims: int = 1,
                 n_cond: int = 0, **kwargs):
        super().__init__()
        dilation_rates = (1, 2, 4, 8, 4, 2, 1)
        self.num_spatial_dims = num_spatial_dims
        self.processor = nn.Sequential(*[
            DilatedResnetBlock(num_spatial_dims, hidden_features + n_cond, kernel_size, dilation_rates, activation,
                               padding_mode, hidden_features_out=hidden_features)
            for _ in range(hidden_blocks)])

    def __repr__(self):
        return f"DRN{self.num_spatial_dims}D"

    def run(self, h, vb):
        for block in self.processor.children():
            srcs = [ops.Src(h)] + ([ops.Src(vb)] if vb is not None else [])
            h = block.run(srcs, residual=h)
        return h

    def run_ad(self, h, vb):
        for block in self.processor.children():
            srcs = [ops.Src(h)] + ([ops.Src(vb)] if vb is not None else [])
            h = ad.add_at(h, block.run_ad(ad.frame(srcs, h.shape[1:3])))
        return h

    def forward(self, h: torch.Tensor, variables_broadcast: torch.Tensor = None, pos=None):
        if use_autograd(self):
            vb = ad.to_nhwc(variables_broadcast) if variables_broadcast is not None else None
            return ad.to_nchw(self.run_ad(ad.to_nhwc(h), vb))
        vb = ops.nchw_to_nhwc(variables_broadcast) if variables_broadcast is not None else None
        return ops.nhwc_to_nchw(self.run(ops.nchw_to_nhwc(h), vb))


class DilatedResnetBlock(nn.Module):
    """proc_dilatedresnet.py:53-84."""

    def __init__(self, num_spatial_dims=1, hidden_features_in=48, kernel_size=3, dilation_rates=(1, 2, 4, 8, 4, 2, 1),
                 activation: nn.Module = nn.ReLU(), padding_mode: str = 'zeros', hidden_features_out=None):
        super().__init__()
        self.num_spatial_dims = num_spatial_dims
        self.hidden_features_in = hidden_features_in
        self.hidden_features_out = hidden_features_out if hidden_features_out is not None else hidden_features_in
        self.dilation_rates = dilation_rates
        self.activation = activation
        self.padding_mode = padding_mode
        layer_list = []
        for l, dilrate in enumerate(dilation_rates):
            conv = get_conv_with_right_spatial_dim(
                num_spatial_dims, in_channels=self.hidden_features_in if l == 0 else self.hidden_features_out,
                out_channels=self.hidden_features_out, kernel_size=kernel_size, padding='same', dilation=dilrate,
                padding_mode=self.padding_mode)
            layer_list.append(conv)
            layer_list.append(self.activation)
        self.layers = nn.Sequential(*layer_list)

    def run(self, srcs, residual=None):
        """act(conv) x 7 on the virtual input; `residual` is added after the last activation."""
        act = activation_code(self.activation)
        convs = [m for m in self.layers if not isinstance(m, type(self.activation))]
        H, W = srcs[0].t.shape[1:3]
        x = srcs
        for i, conv in enumerate(convs):
            last = i == len(convs) - 1
            y = conv.run(x, (H, W), act=act, addends=[residual] if (last and residual is not None) else [],
                         add_after_act=True)
            x = [ops.Src(y)]
            H, W = y.shape[1:3]
        return y

    def run_ad(self, x):
        act = activation_code(self.activation)
        for conv in [m for m in self.layers if not isinstance(m, type(self.activation))]:
            x = ad.act(ad.conv2d(conv, x), act)
        return x

    def forward(self, x: torch.Tensor):
        if use_autograd(self):
            return ad.to_nchw(self.run_ad(ad.to_nhwc(x)))
        x = ops.nchw_to_nhwc(x)
        return ops.nhwc_to_nchw(self.run([ops.Src(x)]))
