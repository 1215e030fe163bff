"""U-FNO processor (reference models/enc_proc_dec_components/proc_ufno.py).

Per block h = GELU(FNO_Layer(cat(h, vb)) + UNetModern(h, vb)): the FNO branch
(1x1 conv + truncated-DFT spectral conv accumulated in one output pass) is
written once, and the U-Net's final conv epilogue adds it and applies GELU,
so the block output is produced by that single launch.
"""
from typing import List, Tuple, Union

import torch
from torch import nn

from common.interfaces import D, M
from models.common import activation_code, use_autograd, to_ndhwc, to_ncdhw
from models.enc_proc_dec_components.proc_fno import FNO_Layer
from models.enc_proc_dec_components.proc_unet_modern import UNetModern
from nps_hip import ops
from nps_hip import autograd as ad
from pdes import PDE


class UFNO(nn.Module):
    """proc_ufno.py:25-118."""
    model_interface = M.AR_TB
    data_interface = [D.sim1d, D.sim1d_var_t, D.sim2d]

    def __init__(self, pde: PDE, num_spatial_dims: int = 1, n_cond: int = 0, hidden_features: int = 128,
                 hidden_blocks: int = 4, cond_mode: str = "concat", padding_mode: str = "circular",
                 fno_modes: int = 48, fno_kernel_size: int = 1, fno_conv_mode: str = "single",
                 activation: nn.Module = nn.GELU(), norm: bool = False,
                 ch_mults: Union[Tuple[int, ...], List[int]] = (1, 1, 1),
                 is_attn: Union[Tuple[bool, ...], List[bool]] = (False, False, False), mid_attn: bool = False,
                 n_blocks: int = 1, use1x1: bool = True, **kwargs):
        super().__init__()
        self.pde = pde
        self.num_spatial_dims = num_spatial_dims
        self.cond_mode = cond_mode
        self.activation = activation
        assert self.cond_mode in ["film", "concat", None], "Incorrect conditioning mode supplied"
        if self.cond_mode == "film":
            feature_transform, feature_transform_dim, hidden_dim_in = n_cond > 0, n_cond, hidden_features
        elif self.cond_mode == "concat":
            feature_transform, feature_transform_dim, hidden_dim_in = False, 0, hidden_features + n_cond
        else:
            feature_transform, feature_transform_dim, hidden_dim_in = False, 0, hidden_features
        self.fno_layers = nn.ModuleList([FNO_Layer(
            hidden_dim=hidden_dim_in, hidden_dim_out=hidden_features, num_spatial_dims=num_spatial_dims,
            modes=fno_modes, feature_transform=feature_transform, feature_transform_dim=feature_transform_dim,
            kernel_size=fno_kernel_size, conv_mode=fno_conv_mode,
            padding_mode=padding_mode if padding_mode != "ones" else "zeros", activation=None,
        ) for _ in range(hidden_blocks)])
        self.unet_layers = nn.ModuleList([UNetModern(
            pde=pde, num_spatial_dims=num_spatial_dims, n_cond=n_cond, hidden_features=hidden_features,
            cond_mode=cond_mode, activation=activation, norm=norm, ch_mults=ch_mults, is_attn=is_attn,
            mid_attn=mid_attn, n_blocks=n_blocks, use1x1=use1x1, padding_mode=padding_mode,
        ) for _ in range(hidden_blocks)])

    def __repr__(self):
        return f'U-FNO{self.num_spatial_dims}D'

    def run(self, h, vb):
        if self.cond_mode != "concat":
            raise NotImplementedError("U-FNO: only cond_mode='concat' runs on the MI355X path")
        act = activation_code(self.activation)
        for fno, unet in zip(self.fno_layers, self.unet_layers):
            srcs = [ops.Src(h)] + ([ops.Src(vb)] if vb is not None else [])
            # the FNO layer and the U-Net read the same h: the FNO layer runs on a side stream (ops.Fork,
            # lane 1) beside the U-Net, whose final conv joins it and adds its output
            fork = ops.fno_fork(h, settle=[s.t for s in srcs])
            with fork:
                h_fno = fno.run(srcs)
            h = unet.run(h, vb, addend=h_fno, act_after=act, addend_fork=fork)
        return h

    def run3d(self, h, vb):
        """3-D U-FNO (BASELINE config C5) on NDHWC (B, D, H, W, C) activations, fp32 or bf16 storage: per
        block the FNO-3D layer on cat(h, vb) (the (B, D*H, W, C) view), then the 3-D U-Net whose final conv
        epilogue adds it and applies the activation (proc_ufno.py:105-118)."""
        if self.cond_mode != "concat":
            raise NotImplementedError("U-FNO: only cond_mode='concat' runs on the MI355X path")
        if self.num_spatial_dims != 3:
            raise NotImplementedError("UFNO.run3d: 3-D only")
        act = activation_code(self.activation)
        bf16 = h.dtype == torch.bfloat16
        B, D, H, W = h.shape[:4]
        flat = lambda t: t.view(t.shape[0], D * H, W, t.shape[4])  # noqa: E731
        for fno, unet in zip(self.fno_layers, self.unet_layers):
            srcs = [ops.Src(flat(h))] + ([ops.Src(flat(vb))] if vb is not None else [])
            # the FNO layer beside the U-Net (as run(); at every size: C5 at B = 8 +1 %,
            # profiles/r4/experiments/side_stream_forks_ab.txt)
            fork = ops.Fork(h, lane=1, on=ops.SIDE_FNO, settle=[s.t for s in srcs])
            with fork:
                h_fno = fno.run_bf16(srcs, D) if bf16 else fno.run(srcs, D=D)
            h = unet.run3d(h, vb, addend=h_fno.view(B, D, H, W, h_fno.shape[3]), act_after=act, addend_fork=fork)
        return h

    def run_ad(self, h, vb):
        """Differentiable form of run() (training)."""
        if self.cond_mode != "concat":
            raise NotImplementedError("U-FNO: only cond_mode='concat' runs on the MI355X path")
        act = activation_code(self.activation)
        for fno, unet in zip(self.fno_layers, self.unet_layers):
            srcs = [ops.Src(h)] + ([ops.Src(vb)] if vb is not None else [])
            h_fno = fno.run_ad(ad.frame(srcs, h.shape[1:3]))
            h = ad.act(ad.add_at(h_fno, unet.run_ad(h, vb)), act)
        return h

    def forward(self, h: torch.Tensor, variables: torch.Tensor = None, variables_broadcast: torch.Tensor = None,
                pos=None):
        if self.num_spatial_dims == 3:  # (B, C, D, H, W), fp32 or bf16 storage (C5)
            if use_autograd(self):
                raise NotImplementedError("the 3-D U-FNO is inference-only on the MI355X path (C5 rollout)")
            vb = to_ndhwc(variables_broadcast) if variables_broadcast is not None else None
            if vb is not None and vb.dtype != h.dtype:  # conditioning in the activations' storage dtype
                vb = ops.to_bf16(vb) if h.dtype == torch.bfloat16 else ops.to_f32(vb)
            return to_ncdhw(self.run3d(to_ndhwc(h), vb))
        if use_autograd(self):
            vb = ad.to_nhwc(variables_broadcast) if variables_broadcast is not None else None
            return ad.to_nchw(self.run_ad(ad.to_nhwc(h), vb))
        vb = ops.nchw_to_nhwc(variables_broadcast) if variables_broadcast is not None else None
        return ops.nhwc_to_nchw(self.run(ops.nchw_to_nhwc(h), vb))
