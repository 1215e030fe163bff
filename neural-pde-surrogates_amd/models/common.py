"""Conv building blocks of the grid models (reference models/common.py).

The parameter-holding classes subclass torch.nn's Conv2d / ConvTranspose2d /
GroupNorm so construction, initialisation and `state_dict` keys are identical
to the reference; their forward never calls aten convolution: it runs the
gfx950 implicit-GEMM kernel through nps_hip (fails loudly off-GPU).
"""
import copy

import torch
from torch import nn

from nps_hip import ops
from nps_hip import autograd as ad


def use_autograd(module) -> bool:
    """True when this forward must be differentiable (training): grad mode on and trainable parameters.
    The differentiable path runs the same HIP kernels unfused plus their backward kernels (nps_hip.autograd)."""
    return torch.is_grad_enabled() and any(p.requires_grad for p in module.parameters())


class Swish(nn.Module):
    """common.py:7-17 (unused by the twophase cfgs, which pass GELU)."""

    def __init__(self, beta=1):
        super().__init__()
        self.beta = beta

    def forward(self, x):
        raise NotImplementedError("Swish is not on the MI355X hot path (twophase cfgs use GELU)")


def activation_code(act):
    """Map an activation module to the fused-epilogue code of the HIP kernels."""
    if act is None or isinstance(act, nn.Identity):
        return 0
    if isinstance(act, nn.GELU) and getattr(act, "approximate", "none") == "none":
        return ops.GELU
    raise NotImplementedError(f"activation {act!r} is not fused on the MI355X path (GELU only)")


def crop_offsets(cur_hw, des_hw):
    """(top, left) placement of a cur-sized map inside a des-sized frame, crop_Nd semantics (common.py:20-34)."""
    return ops.crop_offset(cur_hw[0], des_hw[0]), ops.crop_offset(cur_hw[1], des_hw[1])


def crop_Nd(num_spatial_dims, enc_ftrs, shape):
    """common.py:20-34 on NCHW device tensors (module-boundary helper; the fused paths never call it)."""
    if num_spatial_dims != 2:
        raise NotImplementedError("crop_Nd: 2-D only on the MI355X path")
    if isinstance(shape, torch.Tensor):
        shape = shape.shape
    H, W = shape[-2], shape[-1]
    B, C, h, w = enc_ftrs.shape
    oy, ox = crop_offsets((h, w), (H, W))
    x = ops.nchw_to_nhwc(enc_ftrs)
    out = torch.zeros((B, H, W, C), dtype=torch.float32, device=x.device)
    y0, y1 = max(0, oy), min(H, oy + h)
    x0, x1 = max(0, ox), min(W, ox + w)
    out[:, y0:y1, x0:x1] = x[:, y0 - oy:y1 - oy, x0 - ox:x1 - ox]
    return ops.nhwc_to_nchw(out)


class _PackedMixin:
    """Caches the MFMA-packed copy of `weight`, re-packed when the parameter changes."""

    def _packed(self, fn, kind="conv"):
        return ops.cached_pack(self.weight, kind, fn)


class Conv2d(_PackedMixin, nn.Conv2d):
    """nn.Conv2d parameters; forward = fused HIP implicit-GEMM conv (NHWC internally)."""

    def geometry(self):
        """(KH, KW, stride, dil, pad_top_left, pad_bottom_right, circ) of this conv."""
        KH, KW = self.kernel_size
        if self.stride[0] != self.stride[1] or self.dilation[0] != self.dilation[1]:
            raise NotImplementedError("anisotropic stride/dilation")
        s, d = self.stride[0], self.dilation[0]
        if self.padding == "same":
            tot = (d * (KH - 1), d * (KW - 1))
            lo = (tot[0] // 2, tot[1] // 2)
            hi = (tot[0] - lo[0], tot[1] - lo[1])
        elif self.padding == "valid":
            lo = hi = (0, 0)
        else:
            lo = hi = tuple(self.padding)
        if self.padding_mode == "circular":
            if lo != hi or lo[0] != lo[1]:
                raise NotImplementedError("asymmetric circular padding")
            return KH, KW, s, d, (0, 0), (0, 0), lo[0]
        if self.padding_mode != "zeros":
            raise NotImplementedError(f"padding_mode {self.padding_mode}")
        return KH, KW, s, d, lo, hi, 0

    def run(self, srcs, frame_hw, **kw):
        KH, KW, s, d, lo, hi, circ = self.geometry()
        x = srcs[0].t
        if (s == 2 and KH == 3 and KW == 3 and d == 1 and circ == 0 and lo == hi and lo[0] == lo[1]
                and len(srcs) == 1 and srcs[0].off_y == 0 and srcs[0].off_x == 0
                and tuple(x.shape[1:3]) == tuple(frame_hw) and x.shape[3] % 4 == 0
                and "gn" not in kw and not kw.get("pre_act")):
            # U-Net Downsample: 3x3/s2 as a 2x2 stride-1 conv over the space-to-depth input
            p = lo[0]
            Ho = (frame_hw[0] + 2 * p - 3) // 2 + 1
            Wo = (frame_hw[1] + 2 * p - 3) // 2 + 1
            pk2 = self._packed(ops.pack_conv_weight_s2d, "s2d")
            if ops.S2D_VIEW and x.shape[3] % 16 == 0 and pk2.nps_precision == ops.PREC_X3F16:
                # the split-fp16 producers read the space-to-depth view straight from x (nps_conv2d_t.s2d)
                return ops.conv2d([ops.Src(x)], (Ho + 1, Wo + 1), pk2, self.bias, self.out_channels, 2, 2,
                                  out_hw=(Ho, Wo), s2d_pad=p, **kw)
            xq = ops.space_to_depth(x, p, Ho + 1, Wo + 1)
            return ops.conv2d([ops.Src(xq)], (Ho + 1, Wo + 1), pk2, self.bias, self.out_channels, 2, 2,
                              out_hw=(Ho, Wo), **kw)
        pk = self._packed(lambda w: ops.pack_conv_weight(w, s, d), ("conv", s, d))
        return ops.conv2d(srcs, frame_hw, pk, self.bias, self.out_channels, KH, KW,
                          stride=s, dil=d, pad=lo, pad_bottom=hi, circ=circ, **kw)

    def forward(self, x):
        if use_autograd(self):
            return ad.to_nchw(ad.conv2d(self, ad.to_nhwc(x)))
        x = ops.nchw_to_nhwc(x)
        y = self.run([ops.Src(x)], x.shape[1:3])
        return ops.nhwc_to_nchw(y)


class ConvTranspose2d(_PackedMixin, nn.ConvTranspose2d):
    """nn.ConvTranspose2d(k=4, s=2) parameters; forward = 4 phase convs on the HIP conv kernel.

    Output phase (py, px) of a stride-2 4x4 transposed conv is a 2x2 conv of the
    input with taps (py + 2(1-ty), px + 2(1-tx)), written to rows 2*qy+py."""
    pre_pad = 0  # circular pre-padding (ConvTranspose2d_padded)

    def run(self, x, act=0):
        if tuple(self.kernel_size) != (4, 4) or tuple(self.stride) != (2, 2) or tuple(self.dilation) != (1, 1) \
                or tuple(self.output_padding) != (0, 0) or self.groups != 1:
            raise NotImplementedError("only the U-Net Upsample transposed conv (k=4, s=2) runs on the MI355X path")
        p = self.padding[0]
        if self.padding[1] != p or p not in (0, 1):
            raise NotImplementedError("transposed conv padding must be 0 or 1")
        B, H, W, C = x.shape
        c = self.pre_pad
        Hp, Wp = H + 2 * c, W + 2 * c
        Ho, Wo = 2 * Hp + 2 - 2 * p, 2 * Wp + 2 - 2 * p
        out = ops.empty_nhwc(B, Ho, Wo, self.out_channels, x)
        phases = self._packed(ops.pack_convT_phases, "convT")
        st = ops.new_stats(B, x)  # the 4 phases store every output element once: GroupNorm(1) moments of out
        if getattr(phases[0], "nps_precision", None) == ops.PREC_X3F16 and ops.MERGE_CONVT_PHASES:
            # one launch: the phases' work-groups share each input patch (nps_conv2d_t.nphase)
            ops.conv2d([ops.Src(x)], (H, W), phases[0], self.bias, self.out_channels, 2, 2, pad=(1, 1), circ=c,
                       out_hw=(Hp + 1, Wp + 1), out=out, out_os=2, out_off=(-p, -p), act=act, out_stats=st, phases=4)
            return ops.attach_stats(out, st)
        for ph in range(4):
            py, px = ph >> 1, ph & 1
            ops.conv2d([ops.Src(x)], (H, W), phases[ph], self.bias, self.out_channels, 2, 2, pad=(1, 1), circ=c,
                       out_hw=(Hp + 1, Wp + 1), out=out, out_os=2, out_off=(py - p, px - p), act=act, out_stats=st)
        return ops.attach_stats(out, st)

    def forward(self, x):
        if use_autograd(self):
            return ad.to_nchw(ad.conv_transpose2d(self, ad.to_nhwc(x)))
        return ops.nhwc_to_nchw(self.run(ops.nchw_to_nhwc(x)))


class ConvTranspose2d_padded(ConvTranspose2d):
    """common.py:93-100: circular_pad_2d(x, pad) then the transposed conv (fused as circular frame extension)."""

    def __init__(self, pad, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.pad = pad
        self.pre_pad = pad


def crop_offsets3(cur, des):
    """(d, h, w) placement of a cur-sized volume inside a des-sized frame, crop_Nd semantics (common.py:20-34)."""
    return tuple(ops.crop_offset(c, d) for c, d in zip(cur, des))


def to_ndhwc(x):
    """(B, C, D, H, W) -> contiguous (B, D, H, W, C) on the HIP transpose (fp32; bf16 via fp32)."""
    B, C, D, H, W = x.shape
    bf = x.dtype == torch.bfloat16
    x4 = x.reshape(B, C, D * H, W)
    y = ops.nchw_to_nhwc(ops.to_f32(x4.contiguous()) if bf else x4)
    return (ops.to_bf16(y) if bf else y).view(B, D, H, W, C)


def to_ncdhw(y):
    """(B, D, H, W, C) -> (B, C, D, H, W) on the HIP transpose."""
    B, D, H, W, C = y.shape
    bf = y.dtype == torch.bfloat16
    y4 = y.reshape(B, D * H, W, C)
    x = ops.nhwc_to_nchw(ops.to_f32(y4) if bf else y4)
    return (ops.to_bf16(x) if bf else x).view(B, C, D, H, W)


class _Packed3Mixin:
    """Caches the nps_conv3d packing of `weight` per storage dtype, re-packed when the parameter changes."""

    def _packed3(self, bf16: bool, transposed: bool = False):
        w = self.weight
        key = (w.data_ptr(), w._version, str(w.device), bf16)
        cache = self.__dict__.setdefault("_pk3", {})
        if cache.get("key_" + str(bf16)) != key:
            cache[bf16] = ops.pack_conv3d_weight(w, transposed=transposed, bf16=bf16)
            cache["key_" + str(bf16)] = key
        return cache[bf16]


class Conv3d(_Packed3Mixin, _PackedMixin, nn.Conv3d):
    """nn.Conv3d parameters (common.py:37-47 with spatial_dim 3).  The FNO-3D pointwise `w` conv
    (fno_kernel_size 1) runs as a 1x1 conv over the (D*H, W) view of NDHWC activations on the 2-D HIP
    conv kernels (run / run_bf16); the 3-D U-Net's convs (k = 1 or 3, stride 1 or 2, valid / zero / circular
    padding) run on the NDHWC implicit-GEMM kernel nps_conv3d (run3d)."""

    def geometry3d(self):
        """(K, stride, circ, zpad) of a cubic, isotropic, undilated conv."""
        ks, st, dl = set(self.kernel_size), set(self.stride), set(self.dilation)
        if len(ks) != 1 or len(st) != 1 or dl != {1} or self.groups != 1:
            raise NotImplementedError("3-D convs: cubic kernel, isotropic stride, no dilation or groups")
        K, s = ks.pop(), st.pop()
        if self.padding == "same":
            if K % 2 == 0:
                raise NotImplementedError("3-D 'same' padding with an even kernel")
            p = (K - 1) // 2
        elif self.padding == "valid":
            p = 0
        else:
            pads = set(self.padding)
            if len(pads) != 1:
                raise NotImplementedError("anisotropic 3-D padding")
            p = pads.pop()
        if self.padding_mode == "circular":
            return K, s, p, 0
        if self.padding_mode != "zeros":
            raise NotImplementedError(f"padding_mode {self.padding_mode}")
        return K, s, 0, p

    def run3d(self, srcs, frame_dhw, **kw):
        """srcs: ops.Src3 NDHWC sources (fp32 or bf16) of a virtual frame -> (B, Do, Ho, Wo, Cout)."""
        K, s, circ, zpad = self.geometry3d()
        bf16 = srcs[0].t.dtype == torch.bfloat16
        return ops.conv3d(srcs, frame_dhw, self._packed3(bf16), self.bias, self.out_channels, K, stride=s, circ=circ,
                          zpad=zpad, **kw)

    def _check(self):
        if tuple(self.kernel_size) != (1, 1, 1) or tuple(self.stride) != (1, 1, 1) or self.groups != 1 \
                or tuple(self.dilation) != (1, 1, 1):
            raise NotImplementedError("only pointwise (kernel 1) 3-D convs run on the MI355X path")

    def geometry(self):
        return 1, 1, 1, 1, (0, 0), (0, 0), 0

    def run(self, srcs, frame_hw, **kw):
        """srcs: NDHWC sources viewed as (B, D*H, W, C); frame_hw = (D*H, W)."""
        self._check()
        pk = self._packed(lambda w: ops.pack_conv_weight(w.reshape(w.shape[0], w.shape[1], 1, 1)), "conv1d")
        return ops.conv2d(srcs, frame_hw, pk, self.bias, self.out_channels, 1, 1, **kw)

    def run_bf16(self, srcs, act=0, addend=None):
        """bf16-storage form (C5): bf16 NDHWC sources viewed as (B, D*H, W, C) -> bf16 (B, D*H, W, Cout)."""
        self._check()
        w = self.weight
        key = ("bf16", w.data_ptr(), w._version, str(w.device))
        if getattr(self, "_pkb_key", None) != key:
            self._pkb = ops.pack_1x1_bf16(w)
            self._pkb_key = key
        return ops.conv1x1_bf16(srcs, self._pkb, self.bias, self.out_channels, act=act, addend=addend)

    def run_ad(self, x):
        self._check()
        return ad.Conv2dFn.apply(self.geometry(), x, self.weight.reshape(self.out_channels, self.in_channels, 1, 1),
                                 self.bias)

    def forward(self, x):
        if tuple(self.kernel_size) != (1, 1, 1) or tuple(self.stride) != (1, 1, 1):
            if use_autograd(self):
                raise NotImplementedError("the 3-D U-Net is inference-only on the MI355X path (C5 rollout)")
            return to_ncdhw(self.run3d([ops.Src3(to_ndhwc(x))], x.shape[2:]))
        B, C, D, H, W = x.shape
        x4 = x.reshape(B, C, D * H, W)
        if use_autograd(self):
            y = ad.to_nchw(self.run_ad(ad.to_nhwc(x4)))
        else:
            x4 = ops.nchw_to_nhwc(x4)
            y = ops.nhwc_to_nchw(self.run([ops.Src(x4)], (D * H, W)))
        return y.reshape(B, self.out_channels, D, H, W)


def get_conv_with_right_spatial_dim(spatial_dim, **kwargs):
    """common.py:37-47."""
    if spatial_dim == 1:
        return nn.Conv1d(**kwargs)
    if spatial_dim == 2:
        return Conv2d(**kwargs)
    if spatial_dim == 3:
        return Conv3d(**kwargs)
    raise NotImplementedError(f"only 0<x<=3d convs implemented so far, but found spatial dim {spatial_dim}!")


class ConvTranspose3d_padded(_Packed3Mixin, nn.ConvTranspose3d):
    """The 3-D U-Net Upsample, DEFINED by this build (the reference raises NotImplementedError for 3-D,
    common.py:103-120): the 2-D rule of ConvTranspose2d_padded (common.py:93-100) applied per axis —
    circular pad `pad` on every spatial axis, then ConvTranspose3d(k=4, s=2, p=0).  Runs as the 8 phase
    convs of nps_conv3d (transposed)."""

    def __init__(self, pad, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.pad = pad

    def run3d(self, x, **kw):
        if (set(self.kernel_size) != {4} or set(self.stride) != {2} or set(self.padding) != {0}
                or set(self.output_padding) != {0} or set(self.dilation) != {1} or self.groups != 1):
            raise NotImplementedError("3-D Upsample: ConvTranspose3d(k=4, s=2, p=0) only")
        bf16 = x.dtype == torch.bfloat16
        return ops.conv3d([ops.Src3(x)], x.shape[1:4], self._packed3(bf16, transposed=True), self.bias,
                          self.out_channels, 2, transposed=True, circ=self.pad, zpad=1, **kw)

    def forward(self, x):
        if use_autograd(self):
            raise NotImplementedError("the 3-D U-Net is inference-only on the MI355X path (C5 rollout)")
        return to_ncdhw(self.run3d(to_ndhwc(x)))


def get_upconv_with_right_spatial_dim(spatial_dim, in_channels, out_channels, **kwargs):
    """common.py:103-120, plus a 3-D circular form the reference lacks (ConvTranspose3d_padded)."""
    if spatial_dim == 1:
        return nn.ConvTranspose1d(in_channels, out_channels, **kwargs)
    if spatial_dim == 2:
        if kwargs.get("padding_mode") == "circular":
            kernel_size = kwargs["kernel_size"]
            slice_size = (kernel_size - 1) // 2
            kw = copy.deepcopy(kwargs)
            del kw["padding_mode"]
            return ConvTranspose2d_padded(slice_size, in_channels, out_channels, **kw)
        return ConvTranspose2d(in_channels, out_channels, **kwargs)
    if spatial_dim == 3 and kwargs.get("padding_mode") == "circular":
        # DESIGN.md "3-D U-FNO": BASELINE config C5 needs a 3-D Upsample; defined as the 2-D rule per axis
        kw = copy.deepcopy(kwargs)
        del kw["padding_mode"]
        return ConvTranspose3d_padded((kw["kernel_size"] - 1) // 2, in_channels, out_channels, **kw)
    raise NotImplementedError(f"only 0<x<=2d convs implemented so far, but found spatial dim {spatial_dim}!")
