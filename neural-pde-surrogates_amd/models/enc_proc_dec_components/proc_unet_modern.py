"""Modern U-Net (reference models/enc_proc_dec_components/proc_unet_modern.py).

Same module tree / kwargs / state_dict as the reference.  The forward is a
chain of fused HIP launches on NHWC tensors:
  * a ResidualBlock = GN-stats(x) -> conv1 [GN+GELU prologue] -> GN-stats ->
    conv2 [GN+GELU prologue] accumulated at the crop_Nd offset into the
    shortcut (1x1 conv or x);
  * torch.cat((h, crop_Nd(skip), crop_Nd(vb))) never exists: the three tensors
    are sources of one virtual conv input frame with their crop offsets;
  * the final GN(8)+GELU+conv+crop is one conv launch whose epilogue can also
    fuse the U-FNO `GELU(h_fno + h_unet)` (proc_ufno.py:118).
"""
from typing import List, Tuple, Union

import torch
from torch import nn

from common.interfaces import D, M
from models.common import (get_conv_with_right_spatial_dim, get_upconv_with_right_spatial_dim, crop_offsets,
                           crop_offsets3, activation_code, use_autograd, to_ndhwc, to_ncdhw)
from nps_hip import ops
from nps_hip import autograd as ad
from pdes import PDE


def _gn_args(norm_mod, stats):
    return ops.GN(stats, norm_mod.weight, norm_mod.bias, norm_mod.num_groups, float(norm_mod.eps))


class UNetModern(nn.Module):
    """proc_unet_modern.py:24-196."""
    model_interface = M.AR_TB
    data_interface = [D.sim1d, D.sim2d, D.sim1d_var_t]

    def __init__(self, pde: PDE, num_spatial_dims: int = 1, n_cond: int = 0, hidden_features: int = 128,
                 cond_mode: str = "concat", activation: nn.Module = nn.GELU(), norm: bool = False,
                 ch_mults: Union[Tuple[int, ...], List[int]] = (1, 2, 2, 4),
                 is_attn: Union[Tuple[bool, ...], List[bool]] = (False, False, False, False), mid_attn: bool = False,
                 n_blocks: int = 2, use1x1: bool = False, padding_mode: str = "ones", **kwargs) -> None:
        super().__init__()
        self.hidden_features = hidden_features
        self.num_spatial_dims = num_spatial_dims
        assert cond_mode in ["concat", None], "Incorrect conditioning mode supplied"
        self.cond_mode = cond_mode
        self.n_cond = 0 if self.cond_mode is None else n_cond
        assert padding_mode in ["ones", "circular"]
        self.padding_mode = padding_mode
        padding_kwargs = dict(padding=1) if padding_mode == "ones" else dict(padding_mode="circular")
        self.activation: nn.Module = activation
        n_resolutions = len(ch_mults)
        n_channels = hidden_features
        down = []
        out_channels = in_channels = n_channels
        for i in range(n_resolutions):
            out_channels = in_channels * ch_mults[i]
            for _ in range(n_blocks):
                down.append(DownBlock(in_channels + n_cond, out_channels, has_attn=is_attn[i], activation=activation,
                                      norm=norm, num_spatial_dims=num_spatial_dims, padding_kwargs=padding_kwargs))
                in_channels = out_channels
            if i < n_resolutions - 1:
                down.append(Downsample(in_channels, num_spatial_dims=num_spatial_dims, n_cond=n_cond,
                                       padding_kwargs=padding_kwargs))
        self.down = nn.ModuleList(down)
        self.middle = MiddleBlock(in_channels=out_channels + n_cond, out_channels=out_channels, has_attn=mid_attn,
                                  activation=activation, norm=norm, num_spatial_dims=num_spatial_dims,
                                  padding_kwargs=padding_kwargs)
        up = []
        in_channels = out_channels
        for i in reversed(range(n_resolutions)):
            out_channels = in_channels
            for _ in range(n_blocks):
                up.append(UpBlock(in_channels + n_cond, out_channels, has_attn=is_attn[i], activation=activation,
                                  norm=norm, num_spatial_dims=num_spatial_dims, padding_kwargs=padding_kwargs))
            out_channels = in_channels // ch_mults[i]
            up.append(UpBlock(in_channels + n_cond, out_channels, has_attn=is_attn[i], activation=activation,
                              norm=norm, num_spatial_dims=num_spatial_dims, padding_kwargs=padding_kwargs))
            in_channels = out_channels
            if i > 0:
                up.append(Upsample(in_channels, num_spatial_dims=num_spatial_dims, padding_kwargs=padding_kwargs))
        self.up = nn.ModuleList(up)
        self.norm = nn.GroupNorm(8, n_channels) if norm else nn.Identity()
        if use1x1:
            self.final = get_conv_with_right_spatial_dim(num_spatial_dims, in_channels=hidden_features,
                                                         out_channels=hidden_features, kernel_size=1)
        else:
            self.final = get_conv_with_right_spatial_dim(num_spatial_dims, in_channels=hidden_features,
                                                         out_channels=hidden_features, kernel_size=3, **padding_kwargs)

    def run(self, h, vb, addend=None, act_after=0, addend_fork=None):
        """NHWC forward (proc_unet_modern.py:169-196).  Optional fused epilogue on the final conv:
        out = act_after(final(...) + addend) — the U-FNO block combination.  addend_fork: the ops.Fork whose
        side stream computes addend (joined just before the final conv)."""
        if self.num_spatial_dims != 2:
            raise NotImplementedError("UNetModern: 2-D only on the MI355X path")
        if self.n_cond > 0 and vb is None:
            # reference Downsample.forward returns a bare tensor here (proc_unet_modern.py:451-455) which
            # :175 then unpacks along the batch dimension; refuse instead of reproducing that bug
            raise ValueError("UNetModern with n_cond > 0 needs variables_broadcast")
        if self.n_cond == 0:
            vb = None
        h_shape = h.shape
        feats, vbs = [h], [vb]
        for m in self.down:
            if isinstance(m, Downsample):
                h, vb = m.run(h, vb)
            else:
                h = m.run(h, vb)
            feats.append(h)
            vbs.append(vb)
        h = self.middle.run(h, vb)
        for m in self.up:
            if isinstance(m, Upsample):
                h = m.conv.run(h)
            else:
                s = feats.pop()
                v = vbs.pop()
                H, W = h.shape[1:3]
                srcs = [ops.Src(h), ops.Src(s, *crop_offsets(s.shape[1:3], (H, W)))]
                if v is not None:
                    srcs.append(ops.Src(v, *crop_offsets(v.shape[1:3], (H, W))))
                h = m.res.run(srcs, (H, W))
        # final: conv(act(norm(h))) then crop_Nd to the input size, as one launch
        H, W = h.shape[1:3]
        gn = None
        if isinstance(self.norm, nn.GroupNorm):
            gn = _gn_args(self.norm, ops.group_norm_stats([ops.Src(h)], (H, W), self.norm.num_groups))
        oy, ox = crop_offsets(self.final_out_hw(H, W), h_shape[1:3])
        B, Ht, Wt = h_shape[0], h_shape[1], h_shape[2]
        if addend_fork is not None:
            addend_fork.join(addend)
        out = ops.empty_nhwc(B, Ht, Wt, self.final.out_channels, h)
        if oy > 0 or ox > 0:
            out.zero_()  # crop_Nd zero-pads when the output is smaller than the input
        # the output carries its GroupNorm(1) moments (the next U-FNO block's norm1 frame reads it): no statistics
        # pass over it (zero crop padding adds nothing to the sums)
        st = ops.new_stats(B, out)
        self.final.run([ops.Src(h)], (H, W), gn=gn, pre_act=activation_code(self.activation), out=out,
                       out_off=(oy, ox), addends=[addend] if addend is not None else [], act=act_after, out_stats=st)
        return ops.attach_stats(out, st)

    def run_ad(self, h, vb):
        """Differentiable NHWC forward (training): proc_unet_modern.py:169-196 as unfused HIP ops."""
        if self.num_spatial_dims != 2:
            raise NotImplementedError("UNetModern: 2-D only on the MI355X path")
        if self.n_cond > 0 and vb is None:
            raise ValueError("UNetModern with n_cond > 0 needs variables_broadcast")
        if self.n_cond == 0:
            vb = None
        h_shape = h.shape
        feats, vbs = [h], [vb]
        for m in self.down:
            if isinstance(m, Downsample):
                h, vb = m.run_ad(h, vb)
            else:
                h = m.run_ad(h, vb)
            feats.append(h)
            vbs.append(vb)
        h = self.middle.run_ad(h, vb)
        for m in self.up:
            if isinstance(m, Upsample):
                h = ad.conv_transpose2d(m.conv, h)
            else:
                _check_no_attn(m)
                s = feats.pop()
                v = vbs.pop()
                H, W = h.shape[1:3]
                srcs = [ops.Src(h), ops.Src(s, *crop_offsets(s.shape[1:3], (H, W)))]
                if v is not None:
                    srcs.append(ops.Src(v, *crop_offsets(v.shape[1:3], (H, W))))
                h = m.res.run_ad(srcs, (H, W))
        H, W = h.shape[1:3]
        norm = self.norm if isinstance(self.norm, nn.GroupNorm) else None
        y = ad.conv2d(self.final, ad.frame([ops.Src(h)], (H, W), norm, activation_code(self.activation)))
        return ad.crop(y, h_shape[1:3], crop_offsets(y.shape[1:3], h_shape[1:3]))

    def run3d(self, h, vb, addend=None, act_after=0, addend_fork=None):
        """NDHWC forward of the 3-D U-Net (proc_unet_modern.py:169-196 with num_spatial_dims=3; the 3-D
        Upsample is this build's ConvTranspose3d_padded), fp32 or bf16 storage.  Optional fused epilogue on
        the final conv: out = act_after(final(...) + addend) — the U-FNO block combination."""
        if self.num_spatial_dims != 3:
            raise NotImplementedError("UNetModern.run3d: 3-D U-Nets only")
        if self.n_cond > 0 and vb is None:
            raise ValueError("UNetModern with n_cond > 0 needs variables_broadcast")
        if self.n_cond == 0:
            vb = None
        h_shape = h.shape
        feats, vbs = [h], [vb]
        for m in self.down:
            if isinstance(m, Downsample):
                h, vb = m.run3d(h, vb)
            else:
                h = m.run3d(h, vb)
            feats.append(h)
            vbs.append(vb)
        h = self.middle.run3d(h, vb)
        for m in self.up:
            if isinstance(m, Upsample):
                st = ops.new_stats(h.shape[0], h) if ops.CARRY3D else None  # (moments of the 8 phases' outputs)
                h = m.conv.run3d(h, out_stats=st)
                if st is not None:
                    ops.attach_stats(h, st)
            else:
                _check_no_attn(m)
                s = feats.pop()
                v = vbs.pop()
                dhw = tuple(h.shape[1:4])
                srcs = [ops.Src3(h), ops.Src3(s, *crop_offsets3(s.shape[1:4], dhw))]
                if v is not None:
                    srcs.append(ops.Src3(v, *crop_offsets3(v.shape[1:4], dhw)))
                h = m.res.run3d(srcs, dhw)
        dhw = tuple(h.shape[1:4])
        gn = None
        if isinstance(self.norm, nn.GroupNorm):
            gn = _gn_args(self.norm, ops.gn_stats3d([ops.Src3(h)], dhw, self.norm.num_groups))
        K, s, circ, zpad = self.final.geometry3d()
        fo = tuple((n + 2 * (circ + zpad) - K) // s + 1 for n in dhw)
        off = crop_offsets3(fo, h_shape[1:4])
        if addend_fork is not None:
            addend_fork.join(addend)
        out = torch.empty(tuple(h_shape[:4]) + (self.final.out_channels,), dtype=h.dtype, device=h.device)
        if any(o > 0 for o in off):
            out.zero_()  # crop_Nd zero-pads when the output is smaller than the input
        # the output's moments (the next U-FNO block's first norm1): those of the values the final conv stores
        # (after the addend and act_after; the crop border stays zero)
        st = ops.new_stats(out.shape[0], out) if ops.CARRY3D else None
        self.final.run3d([ops.Src3(h)], dhw, gn=gn, pre_act=activation_code(self.activation), out=out, out_off=off,
                         addend=addend, act=act_after, out_stats=st)
        if st is not None:
            ops.attach_stats(out, st)
        return out

    def final_out_hw(self, H, W):
        KH, KW, s, d, lo, hi, circ = self.final.geometry()
        return ((H + 2 * circ + lo[0] + hi[0] - d * (KH - 1) - 1) // s + 1,
                (W + 2 * circ + lo[1] + hi[1] - d * (KW - 1) - 1) // s + 1)

    def forward(self, h: torch.Tensor, variables_broadcast: torch.Tensor = None, pos=None):
        assert h.dim() == 2 + self.num_spatial_dims
        if self.num_spatial_dims == 3:
            if use_autograd(self):
                raise NotImplementedError("the 3-D U-Net is inference-only on the MI355X path (C5 rollout)")
            vb = to_ndhwc(variables_broadcast) if variables_broadcast is not None else None
            return to_ncdhw(self.run3d(to_ndhwc(h), vb))
        if use_autograd(self):
            vb = ad.to_nhwc(variables_broadcast) if variables_broadcast is not None else None
            return ad.to_nchw(self.run_ad(ad.to_nhwc(h), vb))
        vb = ops.nchw_to_nhwc(variables_broadcast) if variables_broadcast is not None else None
        return ops.nhwc_to_nchw(self.run(ops.nchw_to_nhwc(h), vb))


class ResidualBlock(nn.Module):
    """proc_unet_modern.py:199-250."""

    def __init__(self, in_channels: int, out_channels: int, activation: nn.Module = torch.nn.GELU(),
                 norm: bool = False, n_groups: int = 1, num_spatial_dims: int = 1, padding_kwargs: dict = None):
        super().__init__()
        self.activation: nn.Module = activation
        padding_kwargs = padding_kwargs or dict()
        self.conv1 = get_conv_with_right_spatial_dim(num_spatial_dims, in_channels=in_channels,
                                                     out_channels=out_channels, kernel_size=3, **padding_kwargs)
        self.conv2 = get_conv_with_right_spatial_dim(num_spatial_dims, in_channels=out_channels,
                                                     out_channels=out_channels, kernel_size=3, **padding_kwargs)
        if in_channels != out_channels:
            self.shortcut = get_conv_with_right_spatial_dim(num_spatial_dims, in_channels=in_channels,
                                                            out_channels=out_channels, kernel_size=1)
        else:
            self.shortcut = nn.Identity()
        if norm:
            self.norm1 = nn.GroupNorm(n_groups, in_channels)
            self.norm2 = nn.GroupNorm(n_groups, out_channels)
        else:
            self.norm1 = nn.Identity()
            self.norm2 = nn.Identity()
        self.num_spatial_dims = num_spatial_dims

    def _shortcut_fork(self, srcs, H, W):
        """An ops.Fork for the shortcut when conv1's launch leaves >= SIDE_MIN_IDLE of the CUs idle in its
        last round (the 258^2 convs: 1122 tiles on 256 CUs at B = 2), else None (no fork: cross-stream waits
        cost more than an exact-round launch leaves idle)."""
        x0 = srcs[0].t
        if not (x0.is_cuda and ops.SIDE_STREAM):
            return None
        KH, KW, s, d, lo, hi, circ = self.conv1.geometry()
        Ho = (H + 2 * circ + lo[0] + hi[0] - d * (KH - 1) - 1) // s + 1
        Wo = (W + 2 * circ + lo[1] + hi[1] - d * (KW - 1) - 1) // s + 1
        idle = ops.last_round_idle(Ho, Wo, x0.shape[0], self.conv1.out_channels, x0.device,
                                   Cin=sum(s.t.shape[3] for s in srcs))
        return ops.Fork(x0, settle=[s.t for s in srcs]) if idle >= ops.SIDE_MIN_IDLE else None

    def run(self, srcs, frame_hw):
        """srcs: the virtual NHWC input x (concat of slices).  Returns crop_Nd(h, sc) + sc."""
        act = activation_code(self.activation)
        H, W = frame_hw
        gn1 = gn2 = None
        if isinstance(self.norm1, nn.GroupNorm):
            gn1 = _gn_args(self.norm1, ops.group_norm_stats(srcs, (H, W), self.norm1.num_groups))
        # The block output's moments (the next block's norm1): those of the shortcut output — x's own for
        # the identity, else added by the 1x1 conv — then conv2, accumulating at its crop offset, adds
        # the change it makes (nps_conv2d_t.out_stats)
        st2 = out = None
        fork = None
        if isinstance(self.shortcut, nn.Identity):
            if len(srcs) != 1 or srcs[0].off_y or srcs[0].off_x or tuple(srcs[0].t.shape[1:3]) != (H, W):
                raise RuntimeError("identity shortcut on a concatenated input")
            out = ops.share_tag(srcs[0].t.clone(), srcs[0].t)  # conv2 accumulates into it: same bound
            if isinstance(self.norm1, nn.GroupNorm):
                st2 = ops.copy_stats(ops.source_stats(srcs[0].t))
        else:
            # the 1x1 shortcut reads only x: it runs on a side stream beside conv1 (ops.Fork) when conv1's
            # persistent grid leaves many CUs idle in its last round (the 258^2 convs), its work-groups
            # taking them; its moments buffer is taken before the fork point (no fill on the side stream)
            st2 = ops.new_stats(srcs[0].t.shape[0], srcs[0].t) if isinstance(self.norm1, nn.GroupNorm) else None
            fork = self._shortcut_fork(srcs, H, W)
            if fork is None:
                out = self.shortcut.run(srcs, (H, W), out_stats=st2)
        # conv1 adds norm2's moments of h1 as it stores it (ops.conv2d out_stats): no statistics pass
        st1 = ops.new_stats(srcs[0].t.shape[0], srcs[0].t) if isinstance(self.norm2, nn.GroupNorm) else None
        h1 = self.conv1.run(srcs, (H, W), gn=gn1, pre_act=act, out_stats=st1)
        if st1 is not None:
            ops.attach_stats(h1, st1)
        if fork is not None:
            with fork:
                out = self.shortcut.run(srcs, (H, W), out_stats=st2)
        H1, W1 = h1.shape[1:3]
        if isinstance(self.norm2, nn.GroupNorm):
            gn2 = _gn_args(self.norm2, ops.group_norm_stats([ops.Src(h1)], (H1, W1), self.norm2.num_groups))
        if fork is not None:
            fork.join(out)  # conv2 accumulates into the shortcut output
        KH, KW, s, d, lo, hi, circ = self.conv2.geometry()
        H2 = (H1 + 2 * circ + lo[0] + hi[0] - d * (KH - 1) - 1) // s + 1
        W2 = (W1 + 2 * circ + lo[1] + hi[1] - d * (KW - 1) - 1) // s + 1
        oy, ox = crop_offsets((H2, W2), out.shape[1:3])
        self.conv2.run([ops.Src(h1)], (H1, W1), gn=gn2, pre_act=act, out=out, out_off=(oy, ox), accumulate=True,
                       out_stats=st2)
        if st2 is not None:
            ops.attach_stats(out, st2)
        return out

    def run3d(self, srcs, frame_dhw):
        """3-D form of run() on NDHWC Src3 sources: GN-stats -> conv1 [GN+GELU prologue] -> GN-stats ->
        conv2 [GN+GELU prologue] accumulated at the crop_Nd offset into the shortcut (1x1 conv or x)."""
        act = activation_code(self.activation)
        gn1 = gn2 = None
        if isinstance(self.norm1, nn.GroupNorm):
            # GroupNorm(1) of a frame of carried-moment sources: their sum, no pass (ops.group_norm_stats3d)
            gn1 = _gn_args(self.norm1, ops.group_norm_stats3d(srcs, frame_dhw, self.norm1.num_groups))
        # conv1 adds the moments of what it stores (nps_conv3d_t.out_stats): norm2's GroupNorm(1) statistics
        # without a pass over h1
        B = srcs[0].t.shape[0]
        carry = isinstance(self.norm2, nn.GroupNorm) and self.norm2.num_groups == 1
        st1 = ops.new_stats(B, srcs[0].t) if carry else None
        h1 = self.conv1.run3d(srcs, frame_dhw, gn=gn1, pre_act=act, out_stats=st1)
        # the block output's moments (the next block's norm1): the shortcut output's — x's own for the identity,
        # else added by the 1x1x1 conv — plus the change conv2 makes accumulating into it (as the 2-D run())
        carry_out = ops.CARRY3D and isinstance(self.norm1, nn.GroupNorm)
        st_out = None
        if isinstance(self.shortcut, nn.Identity):
            s0 = srcs[0]
            if len(srcs) != 1 or s0.off_d or s0.off_h or s0.off_w or tuple(s0.t.shape[1:4]) != tuple(frame_dhw):
                raise RuntimeError("identity shortcut on a concatenated input")
            out = s0.t.clone()
            if carry_out:
                st_out = ops.copy_stats(ops.source_stats3d(s0.t))
        else:
            st_out = ops.new_stats(B, srcs[0].t) if carry_out else None
            out = self.shortcut.run3d(srcs, frame_dhw, out_stats=st_out)
        d1 = tuple(h1.shape[1:4])
        if isinstance(self.norm2, nn.GroupNorm):
            st2 = (ops._stats_sum([st1], B, ops.new_stats(B, h1, 1)) if carry
                   else ops.gn_stats3d([ops.Src3(h1)], d1, self.norm2.num_groups))
            gn2 = _gn_args(self.norm2, st2)
        K, s, circ, zpad = self.conv2.geometry3d()
        d2 = tuple((n + 2 * (circ + zpad) - K) // s + 1 for n in d1)
        self.conv2.run3d([ops.Src3(h1)], d1, gn=gn2, pre_act=act, out=out,
                         out_off=crop_offsets3(d2, out.shape[1:4]), accumulate=True, out_stats=st_out)
        if st_out is not None:
            ops.attach_stats(out, st_out)
        return out

    def run_ad(self, srcs, frame_hw):
        """Differentiable form of run(): frame -> GN+GELU -> conv1 -> GN+GELU -> conv2, + shortcut."""
        act = activation_code(self.activation)
        H, W = frame_hw
        n1 = self.norm1 if isinstance(self.norm1, nn.GroupNorm) else None
        n2 = self.norm2 if isinstance(self.norm2, nn.GroupNorm) else None
        if isinstance(self.shortcut, nn.Identity):
            if len(srcs) != 1 or srcs[0].off_y or srcs[0].off_x or tuple(srcs[0].t.shape[1:3]) != (H, W):
                raise RuntimeError("identity shortcut on a concatenated input")
        # conv1's frame and the shortcut's input (x itself for the identity) from one node: the backward adds the
        # shortcut path's gradient inside the frame backward (ad.frame_pair), not as a separate accumulation
        f1, xin = ad.frame_pair(srcs, (H, W), n1, act) if ad.FRAME_PAIR else (ad.frame(srcs, (H, W), n1, act), None)
        h1 = ad.conv2d(self.conv1, f1)
        if isinstance(self.shortcut, nn.Identity):
            sc = xin if xin is not None else srcs[0].t
        else:
            sc = ad.conv2d(self.shortcut, xin if xin is not None else ad.frame(srcs, (H, W)))
        h2 = ad.conv2d(self.conv2, ad.frame([ops.Src(h1)], h1.shape[1:3], n2, act))
        return ad.add_at(sc, h2, crop_offsets(h2.shape[1:3], sc.shape[1:3]))

    def forward(self, x: torch.Tensor):
        if self.num_spatial_dims == 3:
            if use_autograd(self):
                raise NotImplementedError("the 3-D U-Net is inference-only on the MI355X path (C5 rollout)")
            x = to_ndhwc(x)
            return to_ncdhw(self.run3d([ops.Src3(x)], x.shape[1:4]))
        if use_autograd(self):
            x = ad.to_nhwc(x)
            return ad.to_nchw(self.run_ad([ops.Src(x)], x.shape[1:3]))
        x = ops.nchw_to_nhwc(x)
        return ops.nhwc_to_nchw(self.run([ops.Src(x)], x.shape[1:3]))


class AttentionBlock(nn.Module):
    """proc_unet_modern.py:253-317 — parameters only (is_attn / mid_attn are False in every cfg)."""

    def __init__(self, in_channels: int, out_channels: int = None, n_heads: int = 1, d_k=None, n_groups: int = 1,
                 num_spatial_dims: int = 1):
        super().__init__()
        out_channels = in_channels if out_channels is None else out_channels
        d_k = in_channels if d_k is None else d_k
        self.in_channels, self.out_channels = in_channels, out_channels
        self.norm = nn.GroupNorm(n_groups, in_channels)
        self.projection = nn.Linear(in_channels, n_heads * d_k * 3)
        self.output = nn.Linear(n_heads * d_k, out_channels)
        self.scale = d_k ** -0.5
        self.n_heads, self.d_k = n_heads, d_k
        if in_channels != out_channels:
            self.shortcut = get_conv_with_right_spatial_dim(num_spatial_dims, in_channels=in_channels,
                                                            out_channels=out_channels, kernel_size=1)
        else:
            self.shortcut = nn.Identity()

    def forward(self, x):
        raise NotImplementedError("U-Net attention is not on the MI355X path (is_attn=False in all cfgs)")


def _check_no_attn(m):
    if not isinstance(m.attn, nn.Identity):
        raise NotImplementedError("U-Net attention is not on the MI355X path (is_attn=False in all cfgs)")


class DownBlock(nn.Module):
    """proc_unet_modern.py:320-354."""

    def __init__(self, in_channels: int, out_channels: int, has_attn: bool = False, activation: nn.Module = nn.GELU(),
                 norm: bool = False, num_spatial_dims: int = 1, padding_kwargs: dict = None):
        super().__init__()
        self.res = ResidualBlock(in_channels, out_channels, activation=activation, norm=norm,
                                 num_spatial_dims=num_spatial_dims, padding_kwargs=padding_kwargs)
        self.attn = AttentionBlock(out_channels, num_spatial_dims=num_spatial_dims) if has_attn else nn.Identity()

    def run(self, x, vb):
        _check_no_attn(self)
        srcs = [ops.Src(x)] + ([ops.Src(vb)] if vb is not None else [])
        return self.res.run(srcs, x.shape[1:3])

    def run_ad(self, x, vb):
        _check_no_attn(self)
        srcs = [ops.Src(x)] + ([ops.Src(vb)] if vb is not None else [])
        return self.res.run_ad(srcs, x.shape[1:3])

    def run3d(self, x, vb):
        _check_no_attn(self)
        srcs = [ops.Src3(x)] + ([ops.Src3(vb)] if vb is not None else [])
        return self.res.run3d(srcs, x.shape[1:4])

    def forward(self, x: torch.Tensor, variables_broadcast: torch.Tensor = None):
        if self.res.num_spatial_dims == 3:
            vb = to_ndhwc(variables_broadcast) if variables_broadcast is not None else None
            return to_ncdhw(self.run3d(to_ndhwc(x), vb)), variables_broadcast
        if use_autograd(self):
            vb = ad.to_nhwc(variables_broadcast) if variables_broadcast is not None else None
            return ad.to_nchw(self.run_ad(ad.to_nhwc(x), vb)), variables_broadcast
        vb = ops.nchw_to_nhwc(variables_broadcast) if variables_broadcast is not None else None
        return ops.nhwc_to_nchw(self.run(ops.nchw_to_nhwc(x), vb)), variables_broadcast


class UpBlock(nn.Module):
    """proc_unet_modern.py:357-391."""

    def __init__(self, in_channels: int, out_channels: int, has_attn: bool = False, activation: nn.Module = nn.GELU(),
                 norm: bool = False, num_spatial_dims: int = 1, padding_kwargs: dict = None):
        super().__init__()
        self.res = ResidualBlock(in_channels + out_channels, out_channels, activation=activation, norm=norm,
                                 num_spatial_dims=num_spatial_dims, padding_kwargs=padding_kwargs)
        self.attn = AttentionBlock(out_channels, num_spatial_dims=num_spatial_dims) if has_attn else nn.Identity()

    def forward(self, x: torch.Tensor):
        _check_no_attn(self)
        if self.res.num_spatial_dims == 3:
            return self.res(x)
        if use_autograd(self):
            x = ad.to_nhwc(x)
            return ad.to_nchw(self.res.run_ad([ops.Src(x)], x.shape[1:3]))
        x = ops.nchw_to_nhwc(x)
        return ops.nhwc_to_nchw(self.res.run([ops.Src(x)], x.shape[1:3]))


class MiddleBlock(nn.Module):
    """proc_unet_modern.py:394-422."""

    def __init__(self, in_channels, out_channels: int, has_attn: bool = False, activation: nn.Module = nn.GELU(),
                 norm: bool = False, num_spatial_dims: int = 1, padding_kwargs: dict = None):
        super().__init__()
        self.res1 = ResidualBlock(in_channels, out_channels, activation=activation, norm=norm,
                                  num_spatial_dims=num_spatial_dims, padding_kwargs=padding_kwargs)
        self.attn = AttentionBlock(out_channels, num_spatial_dims=num_spatial_dims) if has_attn else nn.Identity()
        self.res2 = ResidualBlock(out_channels, out_channels, activation=activation, norm=norm,
                                  num_spatial_dims=num_spatial_dims, padding_kwargs=padding_kwargs)

    def run(self, x, vb):
        _check_no_attn(self)
        srcs = [ops.Src(x)] + ([ops.Src(vb)] if vb is not None else [])
        h = self.res1.run(srcs, x.shape[1:3])
        return self.res2.run([ops.Src(h)], h.shape[1:3])

    def run_ad(self, x, vb):
        _check_no_attn(self)
        srcs = [ops.Src(x)] + ([ops.Src(vb)] if vb is not None else [])
        h = self.res1.run_ad(srcs, x.shape[1:3])
        return self.res2.run_ad([ops.Src(h)], h.shape[1:3])

    def run3d(self, x, vb):
        _check_no_attn(self)
        srcs = [ops.Src3(x)] + ([ops.Src3(vb)] if vb is not None else [])
        h = self.res1.run3d(srcs, x.shape[1:4])
        return self.res2.run3d([ops.Src3(h)], h.shape[1:4])

    def forward(self, x: torch.Tensor, variables_broadcast: torch.Tensor = None):
        if self.res1.num_spatial_dims == 3:
            vb = to_ndhwc(variables_broadcast) if variables_broadcast is not None else None
            return to_ncdhw(self.run3d(to_ndhwc(x), vb)), variables_broadcast
        if use_autograd(self):
            vb = ad.to_nhwc(variables_broadcast) if variables_broadcast is not None else None
            return ad.to_nchw(self.run_ad(ad.to_nhwc(x), vb)), variables_broadcast
        vb = ops.nchw_to_nhwc(variables_broadcast) if variables_broadcast is not None else None
        return ops.nhwc_to_nchw(self.run(ops.nchw_to_nhwc(x), vb)), variables_broadcast


class Upsample(nn.Module):
    """proc_unet_modern.py:425-436 (ConvTranspose2d k=4 s=2, circularly pre-padded in 'circular' mode)."""

    def __init__(self, n_channels: int, num_spatial_dims: int, padding_kwargs: dict):
        super().__init__()
        self.conv = get_upconv_with_right_spatial_dim(num_spatial_dims, in_channels=n_channels,
                                                      out_channels=n_channels, kernel_size=4, stride=2,
                                                      **padding_kwargs)

    def forward(self, x: torch.Tensor):
        return self.conv(x)


class Downsample(nn.Module):
    """proc_unet_modern.py:439-455 (3x3 stride-2 conv on h and on the conditioning channels)."""

    def __init__(self, n_channels: int, num_spatial_dims: int, n_cond: int, padding_kwargs: dict):
        super().__init__()
        self.conv = get_conv_with_right_spatial_dim(num_spatial_dims, in_channels=n_channels, out_channels=n_channels,
                                                    kernel_size=3, stride=2, **padding_kwargs)
        if n_cond > 0:
            self.conv_variables_broadcast = get_conv_with_right_spatial_dim(
                num_spatial_dims, in_channels=n_cond, out_channels=n_cond, kernel_size=3, stride=2, **padding_kwargs)

    def run(self, x, vb):
        st = ops.new_stats(x.shape[0], x)  # the next ResidualBlock's norm1 moments of h
        h = ops.attach_stats(self.conv.run([ops.Src(x)], x.shape[1:3], out_stats=st), st)
        if vb is not None:
            vb = self.conv_variables_broadcast.run([ops.Src(vb)], vb.shape[1:3])
        return h, vb

    def run_ad(self, x, vb):
        h = ad.conv2d(self.conv, x)
        if vb is not None:
            vb = ad.conv2d(self.conv_variables_broadcast, vb)
        return h, vb

    def run3d(self, x, vb):
        st = ops.new_stats(x.shape[0], x) if ops.CARRY3D else None  # the next ResidualBlock's norm1 moments of h
        h = self.conv.run3d([ops.Src3(x)], x.shape[1:4], out_stats=st)
        if st is not None:
            ops.attach_stats(h, st)
        if vb is not None:
            vb = self.conv_variables_broadcast.run3d([ops.Src3(vb)], vb.shape[1:4])
        return h, vb

    def forward(self, x: torch.Tensor, variables_broadcast: torch.Tensor = None):
        if use_autograd(self):
            if variables_broadcast is not None:
                h, v = self.run_ad(ad.to_nhwc(x), ad.to_nhwc(variables_broadcast))
                return ad.to_nchw(h), ad.to_nchw(v)
            return self.conv(x)
        if variables_broadcast is not None and x.dim() == 5:
            h, v = self.run3d(to_ndhwc(x), to_ndhwc(variables_broadcast))
            return to_ncdhw(h), to_ncdhw(v)
        if variables_broadcast is not None:
            h, v = self.run(ops.nchw_to_nhwc(x), ops.nchw_to_nhwc(variables_broadcast))
            return ops.nhwc_to_nchw(h), ops.nhwc_to_nchw(v)
        return self.conv(x)
