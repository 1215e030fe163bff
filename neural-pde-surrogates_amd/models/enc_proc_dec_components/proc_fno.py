"""FNO processor and spectral convolutions (reference models/enc_proc_dec_components/proc_fno.py).

Same classes, constructor kwargs and parameters (weights1/weights2 complex64
(Cin, Cout, m1, m2)) as the reference; forward runs the truncated-DFT HIP
pipeline (nps_hip.ops.spectral_conv2d).  Internal entry points `run(...)` take
NHWC tensors / virtual frames so composite models never transpose.
"""
import torch
from torch import nn

from common.interfaces import D, M
from models.common import get_conv_with_right_spatial_dim, activation_code, use_autograd
from nps_hip import ops
from nps_hip import autograd as ad
from pdes import PDE


class FNO(nn.Module):
    """proc_fno.py:22-83."""
    model_interface = M.AR_TB
    data_interface = [D.sim1d, D.sim1d_var_t, D.sim2d]

    def __init__(self, pde: PDE, num_spatial_dims: int = 1, n_cond: int = 0, hidden_features: int = 128,
                 fno_modes: int = 48, hidden_blocks: int = 4, cond_mode: str = "concat", fno_kernel_size: int = 1,
                 fno_conv_mode: str = "single", padding_mode: str = "circular", **kwargs):
        super().__init__()
        self.pde = pde
        self.num_spatial_dims = num_spatial_dims
        self.cond_mode = cond_mode
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
            padding_mode=padding_mode if padding_mode != "ones" else "zeros",
        ) for _ in range(hidden_blocks)])

    def __repr__(self):
        return f'FNO{self.num_spatial_dims}D'

    def run(self, h, vb, D=None):
        """NHWC: h (B,H,W,C), vb (B,H,W,K) or None (3-D: NDHWC viewed as (B, D*H, W, C), depth D)."""
        if self.cond_mode == "film":
            raise NotImplementedError("FiLM conditioning is not on the MI355X path (twophase cfgs use concat)")
        for layer in self.fno_layers:
            srcs = [ops.Src(h)] + ([ops.Src(vb)] if (vb is not None and self.cond_mode == "concat") else [])
            h = layer.run(srcs, D=D) if self.num_spatial_dims == 3 else layer.run(srcs)
        return h

    def run_ad(self, h, vb, D=None):
        if self.cond_mode == "film":
            raise NotImplementedError("FiLM conditioning is not on the MI355X path (twophase cfgs use concat)")
        for layer in self.fno_layers:
            srcs = [ops.Src(h)] + ([ops.Src(vb)] if (vb is not None and self.cond_mode == "concat") else [])
            x = ad.frame(srcs, h.shape[1:3])
            h = layer.run_ad(x, D) if self.num_spatial_dims == 3 else layer.run_ad(x)
        return h

    def run_bf16(self, h, vb, D):
        """bf16-storage forward of a 3-D FNO (BASELINE config C5): h (B, D*H, W, C), vb (B, D*H, W, K) bf16
        NDHWC views; every layer in bf16 storage with fp32 arithmetic (FNO_Layer.run_bf16)."""
        if self.num_spatial_dims != 3:
            raise NotImplementedError("the bf16 storage path is the 3-D FNO's (config C5)")
        if self.cond_mode == "film":
            raise NotImplementedError("FiLM conditioning is not on the MI355X path (twophase cfgs use concat)")
        for layer in self.fno_layers:
            srcs = [ops.Src(h)] + ([ops.Src(vb)] if (vb is not None and self.cond_mode == "concat") else [])
            h = layer.run_bf16(srcs, D)
        return h

    def forward(self, h: torch.Tensor, variables: torch.Tensor = None, variables_broadcast: torch.Tensor = None,
                pos=None):
        if self.num_spatial_dims == 3:  # (B, C, D, H, W): the layers run on the (B, D*H, W, C) view
            B, C, D, H, W = h.shape
            flat = lambda t: t.reshape(t.shape[0], t.shape[1], D * H, W)
            if h.dtype == torch.bfloat16:  # bf16 storage (C5); inference only
                if use_autograd(self):
                    raise NotImplementedError("the bf16 3-D FNO path is inference-only (fp32 for training)")
                # (an fp32 variables_broadcast next to bf16 h is converted as fp32)
                tob = lambda t: ops.to_bf16(ops.nchw_to_nhwc(ops.to_f32(flat(t)) if t.dtype == torch.bfloat16
                                                             else flat(t).float()))
                vb = tob(variables_broadcast) if variables_broadcast is not None else None
                y = ops.nhwc_to_nchw(ops.to_f32(self.run_bf16(tob(h), vb, D)))
                return ops.to_bf16(y).reshape(B, y.shape[1], D, H, W)
            if use_autograd(self):
                vb = ad.to_nhwc(flat(variables_broadcast)) if variables_broadcast is not None else None
                y = ad.to_nchw(self.run_ad(ad.to_nhwc(flat(h)), vb, D))
            else:
                vb = ops.nchw_to_nhwc(flat(variables_broadcast)) if variables_broadcast is not None else None
                y = ops.nhwc_to_nchw(self.run(ops.nchw_to_nhwc(flat(h)), vb, D))
            return y.reshape(B, y.shape[1], D, H, W)
        if use_autograd(self):
            vb = ad.to_nhwc(variables_broadcast) if variables_broadcast is not None else None
            return ad.to_nchw(self.run_ad(ad.to_nhwc(h), vb))
        vb = ops.nchw_to_nhwc(variables_broadcast) if variables_broadcast is not None else None
        return ops.nhwc_to_nchw(self.run(ops.nchw_to_nhwc(h), vb))


class FNO_Layer(nn.Module):
    """proc_fno.py:87-155: spectral conv + `w` conv (+ `w2`), then optional GELU — one fused output pass."""

    def __init__(self, hidden_dim, num_spatial_dims: int = 1, kernel_size=1, modes=16, activation=nn.GELU,
                 activation_params=None, feature_transform=False, feature_transform_dim=6, transform_mode=0,
                 hidden_dim_out=None, conv_mode="single", padding_mode="circular"):
        super().__init__()
        self.num_spatial_dims = num_spatial_dims
        assert conv_mode in ["single", "double"]
        self.conv_mode = conv_mode
        if isinstance(modes, int):
            modes = tuple([modes for _ in range(num_spatial_dims)])
        assert len(modes) == num_spatial_dims, 'modes should be int or tuple of ints with length equal to spatial dim!'
        self.modes = modes
        if hidden_dim_out is None:
            hidden_dim_out = hidden_dim
        self.conv = get_spectral_conv_with_right_spatial_dim(
            spatial_dim=num_spatial_dims, in_channels=hidden_dim, out_channels=hidden_dim_out, modes=modes,
            feature_transform=feature_transform, feature_transform_dim=feature_transform_dim,
            transform_mode=transform_mode)
        if conv_mode == "single":
            self.w = get_conv_with_right_spatial_dim(spatial_dim=num_spatial_dims, in_channels=hidden_dim,
                                                     out_channels=hidden_dim_out, kernel_size=kernel_size,
                                                     padding='same', padding_mode=padding_mode)
        else:
            self.w = get_conv_with_right_spatial_dim(spatial_dim=num_spatial_dims, in_channels=hidden_dim,
                                                     out_channels=hidden_dim_out, kernel_size=1, padding='same')
            self.w2 = get_conv_with_right_spatial_dim(spatial_dim=num_spatial_dims, in_channels=hidden_dim,
                                                      out_channels=hidden_dim_out, kernel_size=kernel_size,
                                                      padding='same', padding_mode=padding_mode)
        if activation is None:
            self.act = None
        else:
            self.act = activation(**(activation_params or {}))

    def _check_modes(self, spat_dim):
        for i, s in enumerate(spat_dim):  # proc_fno.py:134-139
            if i == len(spat_dim) - 1:
                assert self.modes[i] <= s // 2 + 1, \
                    'modes should be at most the spatial dim // 2 + 1 for the last spatial dimension!'
            else:
                assert self.modes[i] <= s, 'modes should be at most the spatial dim all but the last spatial dimensions!'

    def run(self, srcs, act_override=None, D=None):
        """srcs: virtual NHWC input frame (h, vb) — for 3-D layers NDHWC sources viewed as (B, D*H, W, C).
        Returns act(spectral(x) + w(x) [+ w2(x)])."""
        if self.num_spatial_dims == 3:
            DH, W = srcs[0].t.shape[1:3]
            self._check_modes((D, DH // D, W))
            if self.conv_mode != "single":
                raise NotImplementedError("FNO_Layer 3-D: conv_mode 'single' only on the MI355X path")
            act = activation_code(self.act) if act_override is None else act_override
            out = self.w.run(srcs, (DH, W))
            return self.conv.run(srcs, D, out=out, accumulate=True, act=act)
        if self.num_spatial_dims != 2:
            raise NotImplementedError("FNO_Layer: 2-D / 3-D only on the MI355X path")
        H, W = srcs[0].t.shape[1:3]
        self._check_modes((H, W))
        act = activation_code(self.act) if act_override is None else act_override
        if (self.conv_mode != "double" and not self.conv.feature_transform and
                ops.spectral_fusable(W, self.conv.modes2, self.conv.out_channels)):
            # conv(x) + w(x) in one output pass: the 1x1's epilogue synthesises the spectral conv's W pass
            # (nps_conv2d_t.spec_z; scale 1 / (H W) of irfft2's norm), then the activation
            Z = self.conv.run_z(srcs)
            return self.w.run(srcs, (H, W), spec=(Z, self.conv.modes2, 1.0 / (H * W)), act=act)
        out = self.w.run(srcs, (H, W))
        if self.conv_mode == "double":
            self.w2.run(srcs, (H, W), out=out, accumulate=True)
        return self.conv.run(srcs, out=out, accumulate=True, act=act)

    def run_bf16(self, srcs, D, act_override=None):
        """3-D layer in bf16 storage: act(spectral(x) + w(x)) with bf16 sources / output, fp32 sums."""
        if self.num_spatial_dims != 3 or self.conv_mode != "single":
            raise NotImplementedError("bf16 storage: 3-D FNO layers with conv_mode 'single' (config C5)")
        DH, W = srcs[0].t.shape[1:3]
        self._check_modes((D, DH // D, W))
        act = activation_code(self.act) if act_override is None else act_override
        out = self.w.run_bf16(srcs)
        return self.conv.run_bf16(srcs, D, out=out, accumulate=True, act=act)

    def run_ad(self, x, D=None):
        """Differentiable form: x (B,H,W,Cin) materialised frame ((B, D*H, W, Cin) for 3-D layers)."""
        if self.num_spatial_dims == 3:
            DH, W = x.shape[1:3]
            self._check_modes((D, DH // D, W))
            if self.conv_mode != "single":
                raise NotImplementedError("FNO_Layer 3-D: conv_mode 'single' only on the MI355X path")
            y = ad.add_at(ad.spectral_conv3d(self.conv, x, D), self.w.run_ad(x))
            return ad.act(y, activation_code(self.act))
        if self.num_spatial_dims != 2:
            raise NotImplementedError("FNO_Layer: 2-D / 3-D only on the MI355X path")
        self._check_modes(x.shape[1:3])
        y = ad.add_at(ad.spectral_conv2d(self.conv, x), ad.conv2d(self.w, x))
        if self.conv_mode == "double":
            y = ad.add_at(y, ad.conv2d(self.w2, x))
        return ad.act(y, activation_code(self.act))

    def forward(self, x, p=None):
        if self.num_spatial_dims == 3:
            B, C, D, H, W = x.shape
            x4 = x.reshape(B, C, D * H, W)
            if use_autograd(self):
                y = ad.to_nchw(self.run_ad(ad.to_nhwc(x4), D))
            else:
                y = ops.nhwc_to_nchw(self.run([ops.Src(ops.nchw_to_nhwc(x4))], D=D))
            return y.reshape(B, y.shape[1], D, H, W)
        if use_autograd(self):
            return ad.to_nchw(self.run_ad(ad.to_nhwc(x)))
        x = ops.nchw_to_nhwc(x)
        return ops.nhwc_to_nchw(self.run([ops.Src(x)]))


class SpectralConv2d(nn.Module):
    """proc_fno.py:225-288: rfft2 -> per-mode complex mixing of the 2 retained corners -> irfft2."""

    def __init__(self, in_channels, out_channels, modes: tuple, feature_transform=False, feature_transform_dim=6,
                 transform_mode=1):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.modes1 = modes[0]
        self.modes2 = modes[1]
        self.scale = (1 / (in_channels * out_channels))
        self.weights1 = nn.Parameter(
            self.scale * torch.rand(in_channels, out_channels, self.modes1, self.modes2, dtype=torch.cfloat))
        self.weights2 = nn.Parameter(
            self.scale * torch.rand(in_channels, out_channels, self.modes1, self.modes2, dtype=torch.cfloat))
        self.feature_transform = feature_transform
        self.feature_transform_dim = feature_transform_dim
        self.transform_mode = transform_mode
        if feature_transform:
            self.weights_feat = nn.Linear(feature_transform_dim, self.out_channels * 2 * self.modes1 * self.modes2)

    def packed(self, H):
        w1, w2 = self.weights1, self.weights2
        key = (H, w1.data_ptr(), w1._version, w2.data_ptr(), w2._version, str(w1.device))
        if getattr(self, "_pk_key", None) != key:
            self._pk = ops.pack_spectral_weight(w1, w2, H)
            self._pk_key = key
        return self._pk

    def run(self, srcs, out=None, accumulate=False, addend=None, act=0):
        if self.feature_transform:
            raise NotImplementedError("FiLM spectral conditioning is not on the MI355X path")
        H = srcs[0].t.shape[1]
        return ops.spectral_conv2d(srcs, self.packed(H), self.modes1, self.modes2, self.out_channels, out=out,
                                   accumulate=accumulate, addend=addend, act=act)

    def run_z(self, srcs):
        """The spectrum Z (B, H, m2, Cout) before the W-pass synthesis (ops.spectral_z): the FNO layer hands it to
        its 1x1 `w`, whose epilogue synthesises it (conv2d(spec=...))."""
        if self.feature_transform:
            raise NotImplementedError("FiLM spectral conditioning is not on the MI355X path")
        H = srcs[0].t.shape[1]
        return ops.spectral_z(srcs, self.packed(H), self.modes1, self.modes2, self.out_channels)

    def forward(self, x, p=None):
        if self.feature_transform:
            raise NotImplementedError("FiLM spectral conditioning is not on the MI355X path")
        if use_autograd(self):
            x = ad.to_nhwc(x)
            H, W = x.shape[1:3]
            if not (self.modes1 <= H and self.modes2 <= W // 2 + 1):
                raise AssertionError("modes should be at most the spatial dim (// 2 + 1 for the last spatial dimension)")
            return ad.to_nchw(ad.spectral_conv2d(self, x))
        x = ops.nchw_to_nhwc(x)
        return ops.nhwc_to_nchw(self.run([ops.Src(x)]))


class SpectralConv1d(nn.Module):
    """proc_fno.py:158-222 — parameters only; not on the 2-D MI355X path."""

    def __init__(self, in_channels, out_channels, modes: tuple, feature_transform=False, feature_transform_dim=6,
                 transform_mode=1):
        super().__init__()
        self.in_channels, self.out_channels, self.modes1 = in_channels, out_channels, modes[0]
        self.scale = (1 / (in_channels * out_channels))
        self.weights1 = nn.Parameter(self.scale * torch.rand(in_channels, out_channels, self.modes1,
                                                             dtype=torch.complex64))
        self.feature_transform = feature_transform
        self.feature_transform_dim = feature_transform_dim
        self.transform_mode = transform_mode
        if feature_transform:
            self.weights_feat = nn.Linear(feature_transform_dim, self.out_channels * self.modes1)

    def forward(self, x, p=None):
        raise NotImplementedError("SpectralConv1d is not on the MI355X hot path")


class SpectralConv3d(nn.Module):
    """proc_fno.py:291-376: rfftn over (D, H, W) -> per-mode complex mixing of the 4 retained corners ->
    irfftn, on the per-axis truncated-DFT HIP pipeline (include/nps.h, SpectralConv3d)."""

    def __init__(self, in_channels, out_channels, modes: tuple, feature_transform=False, feature_transform_dim=6,
                 transform_mode=1):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.modes1, self.modes2, self.modes3 = modes[0], modes[1], modes[2]
        self.scale = (1 / (in_channels * out_channels))
        for i in range(1, 5):
            setattr(self, f"weights{i}", nn.Parameter(self.scale * torch.rand(
                in_channels, out_channels, self.modes1, self.modes2, self.modes3, dtype=torch.cfloat)))
        self.feature_transform = feature_transform
        self.feature_transform_dim = feature_transform_dim
        self.transform_mode = transform_mode
        if feature_transform:
            self.weights_feat = nn.Linear(feature_transform_dim,
                                          self.out_channels * 2 * self.modes1 * 2 * self.modes2 * self.modes3)

    def _weights(self):
        return [self.weights1, self.weights2, self.weights3, self.weights4]

    def packed(self, D, H):
        ws = self._weights()
        key = (D, H, str(ws[0].device)) + tuple((w.data_ptr(), w._version) for w in ws)
        if getattr(self, "_pk_key", None) != key:
            self._pk = ops.pack_spectral3d_weight(ws, D, H)
            self._pk_key = key
        return self._pk

    def packed_bf16(self, D, H):
        wp = self.packed(D, H)
        if getattr(self, "_pkb_src", None) is not wp:
            self._pkb = ops.to_bf16(wp)
            self._pkb_src = wp
        return self._pkb

    def run_bf16(self, srcs, D, out=None, accumulate=False, addend=None, act=0):
        """bf16-storage form: bf16 NDHWC sources viewed as (B, D*H, W, C) -> bf16 (B, D*H, W, Cout)."""
        if self.feature_transform:
            raise NotImplementedError("FiLM spectral conditioning is not on the MI355X path")
        H = srcs[0].t.shape[1] // D
        return ops.spectral_conv3d_bf16(srcs, D, self.packed_bf16(D, H), self.modes1, self.modes2, self.modes3,
                                        self.out_channels, out=out, accumulate=accumulate, addend=addend, act=act)

    def run(self, srcs, D, out=None, accumulate=False, addend=None, act=0):
        """srcs: NDHWC sources viewed as (B, D*H, W, C).  Returns (B, D*H, W, Cout)."""
        if self.feature_transform:
            raise NotImplementedError("FiLM spectral conditioning is not on the MI355X path")
        H = srcs[0].t.shape[1] // D
        return ops.spectral_conv3d(srcs, D, self.packed(D, H), self.modes1, self.modes2, self.modes3,
                                   self.out_channels, out=out, accumulate=accumulate, addend=addend, act=act)

    def forward(self, x, p=None):
        if self.feature_transform:
            raise NotImplementedError("FiLM spectral conditioning is not on the MI355X path")
        B, C, D, H, W = x.shape
        ops.check_modes3d(D, H, W, self.modes1, self.modes2, self.modes3)
        x4 = x.reshape(B, C, D * H, W)
        if x.dtype == torch.bfloat16:  # bf16 storage (C5), inference only
            xb = ops.to_bf16(ops.nchw_to_nhwc(ops.to_f32(x4.contiguous())))
            y = ops.nhwc_to_nchw(ops.to_f32(self.run_bf16([ops.Src(xb)], D)))
            return ops.to_bf16(y).reshape(B, self.out_channels, D, H, W)
        if use_autograd(self):
            y = ad.to_nchw(ad.spectral_conv3d(self, ad.to_nhwc(x4), D))
        else:
            y = ops.nhwc_to_nchw(self.run([ops.Src(ops.nchw_to_nhwc(x4))], D))
        return y.reshape(B, self.out_channels, D, H, W)


def get_spectral_conv_with_right_spatial_dim(spatial_dim, **kwargs):
    """proc_fno.py:379-389."""
    if spatial_dim == 1:
        return SpectralConv1d(**kwargs)
    if spatial_dim == 2:
        return SpectralConv2d(**kwargs)
    if spatial_dim == 3:
        return SpectralConv3d(**kwargs)
    raise NotImplementedError(f'only 0<x<=3d convs implemented so far, but found spatial dim {spatial_dim}!')
