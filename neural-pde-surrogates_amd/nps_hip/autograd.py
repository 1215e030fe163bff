"""Differentiable front end of the HIP kernels (the training / backward hot path).

Each `torch.autograd.Function` below runs its forward AND backward through
libnps_hip.so: convs (input gradients as forward convs of dy with re-packed
weights, weight gradients on the MFMA wgrad kernel), the GroupNorm+GELU frame
backward, SpectralConv2d backward, the TimeConvDense decoder and the
activation_wrapper volume rescale.  Tensors are NHWC fp32 on the MI355X; no op
falls back to a CPU or aten compute path.  PyTorch supplies autograd's graph,
memory (clone / zeros) and gradient accumulation only.

Reference semantics: trainers/base.py:492 `loss.backward()` over the modules of
models/ (see each Function's docstring for the op it differentiates).
"""
import ctypes
import os
from typing import List, Optional, Sequence

import torch

from . import Conv2dArgs, WgradArgs, check, lib, ptr, stream_ptr
from . import ops
from .ops import Src

GELU = ops.GELU


def _c(t):
    return t if t.is_contiguous() else t.contiguous()


# ------------------------------------------------------------------------- weight gradient
def wgrad(a: torch.Tensor, x: torch.Tensor, KH: int, KW: int, dil=1, pad=(0, 0), circ=0,
          g: Optional[torch.Tensor] = None, a_range: Optional[int] = None, x_range: Optional[int] = None,
          db: Optional[torch.Tensor] = None) -> torch.Tensor:
    """G[m][n][KH*KW] (+)= sum_pix a[pix][m] * Xext[pix + tap*dil - pad][n].

    Split-fp16 MFMA (nps_conv2d_wgrad_x3) under ops.CONV_PRECISION == PREC_X3F16 for undilated square
    kernels up to 3x3 over channel counts that are multiples of 4 — a and x range-scaled from their
    max |.| (a_range / x_range: a's / x's range-tag pointers when the caller already has them) — else exact fp32 MFMA
    (nps_conv2d_wgrad).  db ([M], with g is None): also db[m] = sum_pix a[pix][m] (the conv's bias gradient when
    a = dy) — from the split-fp16 kernels' own staging of a (nps_wgrad_t.db), else an nps_channel_sums pass."""
    a, x = _c(a), _c(x)
    B, Ha, Wa, M = a.shape
    _, Hx, Wx, N = x.shape
    x3 = ops.CONV_PRECISION == ops.PREC_X3F16 and KH == KW and KH <= 3 and dil == 1
    store = g is None and x3 and M % 4 == 0 and N % 4 == 0  # the split-fp16 fold stores g: no zero-fill
    if db is not None and not (store and FUSE_DB):
        db.zero_()
        check(lib.nps_channel_sums(ptr(a), a.numel() // M, M, ptr(db), stream_ptr()), "channel_sums")
        db = None
    if g is None:
        g = (torch.empty if store else torch.zeros)((M, N, KH, KW), dtype=torch.float32, device=a.device)
    if (ops.CONV_PRECISION == ops.PREC_X3F16 and KH == KW and KH <= 3 and dil == 1 and (M % 4 or N % 4)):
        # channel counts off the split-fp16 kernel's 4-channel quads (the encoder's 81-channel input): zero-pad
        # to a multiple of 4, run the split-fp16 weight gradient and add the real channels' block into g
        def pad4(t):
            c = t.shape[3]
            if c % 4 == 0:
                return t
            tp = torch.zeros(t.shape[:3] + (c + (-c) % 4,), dtype=t.dtype, device=t.device)
            tp[..., :c] = t
            return tp
        gp = wgrad(pad4(a), pad4(x), KH, KW, dil, pad, circ, None, None)
        g += gp[:M, :N]
        return g
    p = WgradArgs()
    p.a, p.B, p.Ha, p.Wa, p.M = ptr(a), B, Ha, Wa, M
    p.x, p.Hx, p.Wx, p.N = ptr(x), Hx, Wx, N
    p.KH, p.KW, p.dil, p.pad_y, p.pad_x, p.circ = KH, KW, dil, pad[0], pad[1], circ
    p.g = ptr(g)
    if ops.CONV_PRECISION == ops.PREC_X3F16 and KH == KW and KH <= 3 and dil == 1 and M % 4 == 0 and N % 4 == 0:
        # operand ranges: the tensors' live range tags (written by the kernels that produced them), an absmax
        # pass only for a tensor without one (ops.input_tag); a_range: a's tag pointer when the caller has it
        ops.reserve_tags(a.device, 2)
        ar = a_range if a_range is not None else _range_ptr(a)
        xr = x_range if x_range is not None else _range_ptr(x)
        ws = torch.empty(lib.nps_wgrad_x3_ws_floats(M, N, KH, KW), dtype=torch.float32, device=a.device)
        p.db = ptr(db)  # (None -> NULL)
        arith = "x3w"

        fn = lib.nps_conv2d_wgrad_x3_set if store else lib.nps_conv2d_wgrad_x3

        def launch():
            check(fn(ctypes.byref(p), ar, xr, ptr(ws), stream_ptr()), "conv2d_wgrad_x3")
    else:
        arith = "f32w"

        def launch():
            check(lib.nps_conv2d_wgrad(ctypes.byref(p), stream_ptr()), "conv2d_wgrad")
    if ops.conv_probe is not None:  # bench.py's live roofline probe (ops.conv_probe)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        launch()
        e1.record()
        ops.conv_probe.append((e0, e1, 2.0 * B * Ha * Wa * M * N * KH * KW, (arith, KH * KW, 0),
                               4.0 * (a.numel() + x.numel() + g.numel())))
        if ops.conv_shape_log is not None:  # (tools/call_shapes.py --train)
            ops.conv_shape_log.append(dict(cin=N, cout=M, k=(KH, KW), hw=(Hx, Wx), out=(Ha, Wa), B=B, nsrc=1,
                                           acc=not store, addends=0, act=0, gn=False, pre_act=0, stats=False))
    else:
        launch()
    return g


def _range_ptr(t: torch.Tensor) -> int:
    """Device pointer of an upper bound of |t| (a range tag, include/nps.h): t's live tag, else a fresh absmax."""
    if ops.USE_IN_TAGS:
        return ops.input_tag(t)
    return ptr(_keep(ops.absmax(t)))


_KEEP = []


def _keep(t):
    """Hold a one-off range tensor (NPS_RANGE_TAGS without input tags) for the launches that read its pointer.
    The invariant that makes this safe: those launches are enqueued on the stream the tensor was allocated on
    (or on a side stream that is joined before the caller returns, before 8 more _keep calls can drop it), so the
    caching allocator's stream-ordered reuse cannot hand its memory out before they ran."""
    _KEEP.append(t)
    del _KEEP[:-8]
    return t


# the bias gradient of a conv from its weight-gradient launch (wgrad(db=...)) instead of a channel_sums pass over dy
# (dev knob NPS_FUSE_DB=0: off)
FUSE_DB = os.environ.get("NPS_FUSE_DB", "1") != "0"


def channel_sums(x: torch.Tensor) -> torch.Tensor:
    x = _c(x)
    C = x.shape[-1]
    out = torch.zeros(C, dtype=torch.float32, device=x.device)
    check(lib.nps_channel_sums(ptr(x), x.numel() // C, C, ptr(out), stream_ptr()), "channel_sums")
    return out


# Training forward convs carry the GroupNorm(1) moments of their outputs (nps_conv2d_t.out_stats), so the
# differentiable frames' group_norm_stats sums them instead of a statistics pass (dev knob NPS_CARRY_TRAIN=0: off)
CARRY_TRAIN = os.environ.get("NPS_CARRY_TRAIN", "1") != "0"


# the residual add of the differentiable path in one pass (nps_add_at_copy) instead of clone + nps_add_at
# (dev knob NPS_ADD_AT_COPY=0: off)
ADD_AT_COPY = os.environ.get("NPS_ADD_AT_COPY", "1") != "0"
# ... which also carries the sum's GroupNorm(1) moments (dev knob NPS_CARRY_ADD=0: off)
CARRY_ADD = os.environ.get("NPS_CARRY_ADD", "1") != "0"


def _carry_buffer(x):
    return ops.new_stats(x.shape[0], x) if CARRY_TRAIN and x.is_cuda and ops.CONV_PRECISION == ops.PREC_X3F16 else None


def _carry(y, st):
    if st is not None:
        ops.attach_stats(y, st)  # (ignored when the conv's kernel could not take the moments: incomplete)


def _pack_plain(w, dil=1):
    """Pack a [Cout][Cin][KH][KW] stride-1 conv weight (any derived tensor)."""
    return ops.pack_conv_weight(w, 1, dil)


# ------------------------------------------------------------------------- frame (cat/crop/GN/GELU)
class FrameFn(torch.autograd.Function):
    """act(GroupNorm(cat(crop_Nd(src_i)))) — proc_unet_modern.py:245-247, :191, :351; common.py:20-34."""

    @staticmethod
    def forward(ctx, meta, gamma, beta, *srcs):
        offsets, frame_hw, groups, eps, act = meta
        ss = [Src(_c(t), *o) for t, o in zip(srcs, offsets)]
        gn = None
        if gamma is not None:
            stats = ops.group_norm_stats(ss, frame_hw, groups)
            gn = ops.GN(stats, gamma.detach(), beta.detach(), groups, eps)
        out = ops.frame_pack(ss, frame_hw, gn, act)
        ctx.meta = meta
        ctx.has_gn = gamma is not None
        ctx.save_for_backward(*( [gamma, beta, gn.stats] if gn is not None else []), *[s.t for s in ss])
        return out

    @staticmethod
    def backward(ctx, gout):
        return _frame_bwd(ctx, gout, None)


# ResidualBlock's two uses of its input in one autograd node (frame_pair; dev knob NPS_FRAME_PAIR=0: two FrameFns)
FRAME_PAIR = os.environ.get("NPS_FRAME_PAIR", "1") != "0"


def _frame_bwd(ctx, gout, gplain):
    """FrameFn / FramePairFn backward: the sources' gradients (and GroupNorm affine's) in one frame-backward pass,
    gplain (the plain concatenation's gradient, or None) added inside it (nps_frame_pack_bwd2)."""
    offsets, frame_hw, groups, eps, act = ctx.meta
    saved = ctx.saved_tensors
    if ctx.has_gn:
        gamma, beta, stats = saved[:3]
        srcs = saved[3:]
    else:
        gamma = beta = stats = None
        srcs = saved
    gout = _c(gout)
    B = srcs[0].shape[0]
    Cin = sum(t.shape[3] for t in srcs)
    a = Conv2dArgs()
    a.nsrc = len(srcs)
    a.src = ops._c_src([Src(t, *o) for t, o in zip(srcs, offsets)])
    a.B, a.Hin, a.Win, a.Cin = B, frame_hw[0], frame_hw[1], Cin
    dgamma = dbeta = work = None
    if ctx.has_gn:
        a.gn_stats, a.gn_gamma, a.gn_beta = ptr(stats), ptr(gamma), ptr(beta)
        a.gn_groups, a.gn_eps = groups, eps
        dgamma = torch.empty_like(gamma)
        dbeta = torch.empty_like(beta)
        work = ops.new_stats(B, gout, Cin)  # zero on entry (nps_frame_pack_bwd2): a slice of a zeroed chunk
    a.pre_act = act
    need = ctx.needs_input_grad[3:]
    dsrc = [torch.empty_like(t) if need[i] else None for i, t in enumerate(srcs)]
    arr = (ctypes.c_void_p * 3)(*[(d.data_ptr() if d is not None else None) for d in dsrc] +
                               [None] * (3 - len(dsrc)))
    # each source gradient leaves with a range tag: the conv backward reading it as dy needs no absmax pass
    tags = [None] * 3
    if ops.USE_OUT_TAGS:
        ops.reserve_tags(gout.device, len(dsrc))
        tags[:len(dsrc)] = [ops.new_tag(d) if d is not None else None for d in dsrc]
    tarr = (ctypes.c_void_p * 3)(*tags)
    gp = _c(gplain) if gplain is not None else None
    check(lib.nps_frame_pack_bwd2(ctypes.byref(a), ptr(gout), ptr(gp), arr, tarr, ptr(dgamma), ptr(dbeta),
                                  ptr(work), stream_ptr()), "frame_pack_bwd")
    return (None, dgamma, dbeta, *dsrc)


class FramePairFn(torch.autograd.Function):
    """(act(GroupNorm(cat(crop_Nd(src_i)))), cat(crop_Nd(src_i))) — a ResidualBlock's conv1 input and its shortcut's
    (or identity path's) input, proc_unet_modern.py:243-250 — from one node, so the backward adds the second
    output's gradient inside the frame backward (nps_frame_pack_bwd2) instead of autograd accumulating two
    gradients per source with a separate pass.  A single source covering the frame is returned as the plain
    output itself (a view: no copy)."""

    @staticmethod
    def forward(ctx, meta, gamma, beta, *srcs):
        offsets, frame_hw, groups, eps, act = meta
        ss = [Src(_c(t), *o) for t, o in zip(srcs, offsets)]
        gn = None
        if gamma is not None:
            stats = ops.group_norm_stats(ss, frame_hw, groups)
            gn = ops.GN(stats, gamma.detach(), beta.detach(), groups, eps)
        out = ops.frame_pack(ss, frame_hw, gn, act)
        ident = len(ss) == 1 and tuple(offsets[0]) == (0, 0) and tuple(srcs[0].shape[1:3]) == tuple(frame_hw)
        plain = srcs[0] if ident else ops.frame_pack(ss, frame_hw, None, 0)
        ctx.meta = meta
        ctx.has_gn = gamma is not None
        ctx.ident = ident
        ctx.save_for_backward(*([gamma, beta, gn.stats] if gn is not None else []), *[s.t for s in ss])
        return out, plain

    @staticmethod
    def backward(ctx, gout, gplain):
        if gout is None:  # (only the plain output was used)
            gout = torch.zeros((ctx.saved_tensors[-1].shape[0], *ctx.meta[1],
                                sum(t.shape[3] for t in ctx.saved_tensors[(3 if ctx.has_gn else 0):])),
                               dtype=torch.float32, device=gplain.device)
        return _frame_bwd(ctx, gout, gplain)


def frame_pair(srcs: Sequence[Src], frame_hw, norm=None, act=0):
    """(frame(srcs, norm, act), frame(srcs)) through FramePairFn: one frame backward for both consumers."""
    frame_hw = (int(frame_hw[0]), int(frame_hw[1]))
    meta = (tuple((int(s.off_y), int(s.off_x)) for s in srcs), frame_hw,
            norm.num_groups if norm is not None else 0, float(norm.eps) if norm is not None else 0.0, act)
    gamma = norm.weight if norm is not None else None
    beta = norm.bias if norm is not None else None
    f, p = FramePairFn.apply(meta, gamma, beta, *[s.t for s in srcs])
    t0 = srcs[0].t
    if p._base is t0:  # the identity view carries the source's live range tag and moments (same version counter)
        for attr in ("_nps_tag", "_nps_stats"):
            if getattr(t0, attr, None) is not None:
                setattr(p, attr, getattr(t0, attr))
    return f, p


def frame(srcs: Sequence[Src], frame_hw, norm=None, act=0) -> torch.Tensor:
    """Materialise the virtual conv input frame (differentiably).  `norm` is an nn.GroupNorm or None."""
    frame_hw = (int(frame_hw[0]), int(frame_hw[1]))
    if norm is None and act == 0 and len(srcs) == 1:
        s = srcs[0]
        if s.off_y == 0 and s.off_x == 0 and tuple(s.t.shape[1:3]) == frame_hw:
            return s.t
    meta = (tuple((int(s.off_y), int(s.off_x)) for s in srcs), frame_hw,
            norm.num_groups if norm is not None else 0, float(norm.eps) if norm is not None else 0.0, act)
    gamma = norm.weight if norm is not None else None
    beta = norm.bias if norm is not None else None
    return FrameFn.apply(meta, gamma, beta, *[s.t for s in srcs])


def crop(x: torch.Tensor, out_hw, off) -> torch.Tensor:
    """crop_Nd (common.py:20-34): place x at `off` inside a zero frame of size out_hw."""
    return frame([Src(x, off[0], off[1])], out_hw)


# ------------------------------------------------------------------------- conv
def _s2_phase_weight(w, ry, rx, p):
    """Input-gradient phase (ry, rx) of a stride-2 3x3 conv with top/left padding p in {0, 1}: dx[2q + r]
    sums dy[o] w[k] over 2o + k - p = 2q + r, i.e. o in {q - 1 + p, q + p}.  As a 2x2 conv of dy with top
    padding 1 - p, tap t reads dy[q - 1 + p + t] and uses kernel element k = r - p + 2 - 2t."""
    Cout, Cin, K, _ = w.shape
    out = torch.zeros((Cin, Cout, 2, 2), dtype=w.dtype, device=w.device)
    wt = w.detach().transpose(0, 1)
    for ty in range(2):
        ky = ry - p + 2 - 2 * ty
        if not 0 <= ky < K:
            continue
        for tx in range(2):
            kx = rx - p + 2 - 2 * tx
            if 0 <= kx < K:
                out[:, :, ty, tx] = wt[:, :, ky, kx]
    return out


class Conv2dFn(torch.autograd.Function):
    """nn.Conv2d forward/backward (models/common.py:37-47): stride 1 (valid / zero / circular 'same',
    dilated) or the 3x3 stride-2 Downsample (proc_unet_modern.py:445-455, space-to-depth form)."""

    @staticmethod
    def forward(ctx, geo, x, weight, bias):
        KH, KW, s, d, lo, hi, circ = geo
        x = _c(x)
        B, H, W, Cin = x.shape
        Cout = weight.shape[0]
        if s == 2:
            if not (KH == 3 and KW == 3 and d == 1 and circ == 0 and lo == hi and lo[0] == lo[1] and lo[0] in (0, 1)):
                raise NotImplementedError("stride-2 conv: only the 3x3 U-Net Downsample form (padding 0 or 1)")
            p = lo[0]
            Ho, Wo = (H + 2 * p - 3) // 2 + 1, (W + 2 * p - 3) // 2 + 1
            xq = ops.space_to_depth(x, p, Ho + 1, Wo + 1)
            st = _carry_buffer(x)
            y = ops.conv2d([Src(xq)], (Ho + 1, Wo + 1), ops.cached_pack(weight, "s2d", ops.pack_conv_weight_s2d),
                           bias, Cout, 2, 2,
                           out_hw=(Ho, Wo), out_stats=st)
            _carry(y, st)
            ctx.save_for_backward(xq, weight)
        elif s == 1:
            wp = ops.cached_pack(weight, ("conv", 1, d), lambda w: ops.pack_conv_weight(w, 1, d))
            st = _carry_buffer(x)
            y = ops.conv2d([Src(x)], (H, W), wp, bias, Cout, KH, KW, dil=d, pad=lo,
                           pad_bottom=hi, circ=circ, out_stats=st)
            _carry(y, st)
            ctx.save_for_backward(x, weight)
        else:
            raise NotImplementedError(f"conv stride {s}")
        ctx.geo, ctx.in_hw, ctx.has_bias = geo, (H, W), bias is not None
        ctx.param = weight  # the nn.Parameter itself: its input-gradient packing is cached on it (ops.cached_pack)
        return y

    @staticmethod
    def backward(ctx, gy):
        KH, KW, s, d, lo, hi, circ = ctx.geo
        xs, w = ctx.saved_tensors
        gy = _c(gy)
        H, W = ctx.in_hw
        B, Ho, Wo, Cout = gy.shape
        Cin = w.shape[1]
        dx = dw = db = rng = None
        if ops.CONV_PRECISION == ops.PREC_X3F16 and (ctx.needs_input_grad[1] or ctx.needs_input_grad[2]):
            # rng is a raw pointer into the tag arena, passed to every launch below: reserve the tags of the
            # WHOLE backward first (gy's tag; 2 per input-gradient conv — one, or four stride-2 phases; 2 for
            # the weight gradient), so no later reserve can wrap the arena (zeroing gy's tag) while rng is live
            ops.reserve_tags(gy.device, 1 + (2 if s == 1 else 8) + 2)
            rng = _range_ptr(gy)  # gradients: any magnitude (its tag, or one absmax pass shared by dx and dw)
        # the weight gradient reads only gy and x: it runs on a side stream beside the input-gradient conv(s)
        # (ops.Fork), each filling the CUs the other's last round leaves idle; joined before returning
        fork = ops.Fork(gy, on=ops.SIDE_WGRAD and ctx.needs_input_grad[1] and ctx.needs_input_grad[2])
        if ctx.needs_input_grad[1]:
            if s == 1:
                wd = ops.cached_pack(ctx.param, ("dgrad", d), lambda p: ops.pack_conv_weight_dgrad(p, d))
                if circ:
                    dx = ops.conv2d([Src(gy)], (Ho, Wo), wd, None, Cin, KH, KW, dil=d,
                                    circ=circ, out_hw=(H, W), in_scale=rng)
                else:
                    pt = (d * (KH - 1) - lo[0], d * (KW - 1) - lo[1])
                    dx = ops.conv2d([Src(gy)], (Ho, Wo), wd, None, Cin, KH, KW, dil=d,
                                    pad=pt, out_hw=(H, W), in_scale=rng)
            else:
                p = lo[0]
                dx = torch.empty((B, H, W, Cin), dtype=torch.float32, device=gy.device)
                for ry in range(2):
                    for rx in range(2):
                        hq, wq = (H - ry + 1) // 2, (W - rx + 1) // 2
                        if hq <= 0 or wq <= 0:
                            continue
                        ops.conv2d([Src(gy)], (Ho, Wo), _pack_plain(_s2_phase_weight(w, ry, rx, p)), None, Cin, 2, 2,
                                   pad=(1 - p, 1 - p), out_hw=(hq, wq), out=dx, out_os=2, out_off=(ry, rx),
                                   in_scale=rng)
        if ctx.needs_input_grad[2]:
            with fork:
                # the bias gradient from the weight-gradient launch's staging of gy (wgrad(db=...))
                db = (torch.empty(Cout, dtype=torch.float32, device=gy.device)
                      if ctx.has_bias and ctx.needs_input_grad[3] else None)
                if s == 1:
                    dw = wgrad(gy, xs, KH, KW, dil=d, pad=lo, circ=circ, a_range=rng, db=db)
                    if dw.shape[1] != Cin:      # input carried zero padding channels (packed encoder input)
                        dw = dw[:, :Cin].contiguous()
                else:
                    C = Cin
                    G = wgrad(gy, xs, 2, 2, a_range=rng, db=db)                # [Cout][4C][2][2]
                    G = G.view(Cout, 2, 2, C, 2, 2).permute(0, 3, 4, 1, 5, 2).reshape(Cout, C, 4, 4)
                    dw = G[:, :, :3, :3].contiguous()
            fork.join(dw, *([db] if db is not None else []))
        if ctx.has_bias and ctx.needs_input_grad[3] and db is None:
            db = channel_sums(gy)
        return None, dx, dw, db


class ConvTranspose2dFn(torch.autograd.Function):
    """nn.ConvTranspose2d(k=4, s=2) of the U-Net Upsample, optionally circularly pre-padded
    (ConvTranspose2d_padded, models/common.py:93-100; proc_unet_modern.py:425-436)."""

    @staticmethod
    def forward(ctx, geo, x, weight, bias):
        c, p = geo
        x = _c(x)
        B, H, W, Cin = x.shape
        Cout = weight.shape[1]
        Hp, Wp = H + 2 * c, W + 2 * c
        Ho, Wo = 2 * Hp + 2 - 2 * p, 2 * Wp + 2 - 2 * p
        out = ops.empty_nhwc(B, Ho, Wo, Cout, x)
        phases = ops.cached_pack(weight, "convT", ops.pack_convT_phases)
        st = _carry_buffer(x)  # (the 4 phases write disjoint elements: their moments add up to out's)
        for ph in range(4):
            py, px = ph >> 1, ph & 1
            ops.conv2d([Src(x)], (H, W), phases[ph], bias, Cout, 2, 2, pad=(1, 1), circ=c, out_hw=(Hp + 1, Wp + 1),
                       out=out, out_os=2, out_off=(py - p, px - p), out_stats=st)
        _carry(out, st)
        ctx.geo, ctx.has_bias = geo, bias is not None
        ctx.save_for_backward(x, weight)
        return out

    @staticmethod
    def backward(ctx, gout):
        c, p = ctx.geo
        x, w = ctx.saved_tensors
        gout = _c(gout)
        B, H, W, Cin = x.shape
        Cout = w.shape[1]
        Hp, Wp = H + 2 * c, W + 2 * c
        # the transposed conv's adjoint is a 4x4 stride-2 conv of gout: space-to-depth + 2x2 conv
        dq = ops.space_to_depth(gout, p, Hp + 1, Wp + 1)                    # [B][Hp+1][Wp+1][4 Cout]
        dx = dw = db = None
        forked = ops.SIDE_WGRAD and ctx.needs_input_grad[1] and ctx.needs_input_grad[2]
        # dq is read by both streams: its range tag is settled before the fork point (ops.Fork settle)
        fork = ops.Fork(gout, on=forked, settle=[dq])
        if ctx.needs_input_grad[1]:
            w2 = w.detach().view(Cin, Cout, 2, 2, 2, 2).permute(0, 3, 5, 1, 2, 4).reshape(Cin, 4 * Cout, 2, 2)
            dxp = ops.conv2d([Src(dq)], (Hp + 1, Wp + 1), _pack_plain(w2.contiguous()), None, Cin, 2, 2,
                             out_hw=(Hp, Wp))  # dq's range: its tag (ops.input_tag), shared from gout
            if c:
                dx = torch.empty_like(x)
                check(lib.nps_circular_fold(ptr(dxp), ptr(dx), B, H, W, Cin, c, stream_ptr()), "circular_fold")
            else:
                dx = dxp
        if ctx.needs_input_grad[2]:
            with fork:  # beside the input-gradient conv, as in Conv2dFn.backward
                if c:
                    xp = torch.empty((B, Hp, Wp, Cin), dtype=torch.float32, device=x.device)
                    check(lib.nps_circular_pad(ptr(x), ptr(xp), B, H, W, Cin, c, stream_ptr()), "circular_pad")
                else:
                    xp = x
                G = wgrad(xp, dq, 2, 2)                                            # [Cin][4 Cout][2][2]
                dw = G.view(Cin, 2, 2, Cout, 2, 2).permute(0, 3, 4, 1, 5, 2).reshape(Cin, Cout, 4, 4).contiguous()
            fork.join(dw)
        if ctx.has_bias and ctx.needs_input_grad[3]:
            db = channel_sums(gout)
        return None, dx, dw, db


def conv2d(conv, x: torch.Tensor) -> torch.Tensor:
    """Differentiable forward of a models.common.Conv2d on an NHWC tensor (no fused epilogue)."""
    return Conv2dFn.apply(conv.geometry(), x, conv.weight, conv.bias)


def conv_transpose2d(conv, x: torch.Tensor) -> torch.Tensor:
    if tuple(conv.kernel_size) != (4, 4) or tuple(conv.stride) != (2, 2) or tuple(conv.dilation) != (1, 1) \
            or tuple(conv.output_padding) != (0, 0) or conv.groups != 1 or conv.padding[0] != conv.padding[1] \
            or conv.padding[0] not in (0, 1):
        raise NotImplementedError("only the U-Net Upsample transposed conv (k=4, s=2) runs on the MI355X path")
    return ConvTranspose2dFn.apply((conv.pre_pad, conv.padding[0]), x, conv.weight, conv.bias)


# ------------------------------------------------------------------------- element-wise
class GeluFn(torch.autograd.Function):
    """nn.GELU() (erf form)."""

    @staticmethod
    def forward(ctx, x):
        x = _c(x)
        y = torch.empty_like(x)
        check(lib.nps_gelu(ptr(x), ptr(y), x.numel(), stream_ptr()), "gelu")
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, gy):
        (x,) = ctx.saved_tensors
        gy = _c(gy)
        gx = torch.empty_like(x)
        check(lib.nps_gelu_bwd(ptr(x), ptr(gy), ptr(gx), x.numel(), stream_ptr()), "gelu_bwd")
        return gx


def gelu(x):
    return GeluFn.apply(x)


def act(x, code):
    return gelu(x) if code == GELU else x


class AddAtFn(torch.autograd.Function):
    """base + crop_Nd(src) placed at `off` (the residual `crop_Nd(h) + shortcut`, proc_unet_modern.py:250;
    off = (0, 0) and equal sizes is a plain sum, e.g. proc_ufno.py:118, proc_dilatedresnet.py:49)."""

    @staticmethod
    def forward(ctx, off, base, src):
        base, src = _c(base), _c(src)
        B, Ho, Wo, C = base.shape
        Hs, Ws = src.shape[1:3]
        if C % 4 == 0 and ADD_AT_COPY:  # one pass: out = base + crop_Nd(src) (nps_add_at_copy)
            out = torch.empty_like(base)
            st = _carry_buffer(base) if CARRY_ADD else None  # out's GroupNorm(1) moments, for the next frame
            check(lib.nps_add_at_copy(ptr(out), ptr(base), ptr(src), B, Ho, Wo, Hs, Ws, C, off[0], off[1], ptr(st),
                                      stream_ptr()), "add_at_copy")
            _carry(out, st)
        else:
            out = base.clone()
            check(lib.nps_add_at(ptr(out), ptr(src), B, Ho, Wo, Hs, Ws, C, off[0], off[1], stream_ptr()), "add_at")
        ctx.off, ctx.src_hw = off, (Hs, Ws)
        return out

    @staticmethod
    def backward(ctx, g):
        g = _c(g)
        gs = None
        if ctx.needs_input_grad[2]:
            gs = ops.frame_pack([Src(g, -ctx.off[0], -ctx.off[1])], ctx.src_hw)
        return None, g, gs


def add_at(base, src, off=(0, 0)):
    return AddAtFn.apply((int(off[0]), int(off[1])), base, src)


class NchwToNhwcFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return ops.nchw_to_nhwc(x)

    @staticmethod
    def backward(ctx, g):
        return ops.nhwc_to_nchw(_c(g))


class NhwcToNchwFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return ops.nhwc_to_nchw(_c(x))

    @staticmethod
    def backward(ctx, g):
        return ops.nchw_to_nhwc(_c(g))


def to_nhwc(x):
    return NchwToNhwcFn.apply(x)


def to_nchw(x):
    return NhwcToNchwFn.apply(x)


# ------------------------------------------------------------------------- spectral conv
class SpectralConv2dFn(torch.autograd.Function):
    """SpectralConv2d.forward (proc_fno.py:257-288) and its torch.fft / complex-einsum backward."""

    @staticmethod
    def forward(ctx, meta, x, w1, w2, wpack):
        m1, m2, Cout = meta
        x = _c(x)
        B, H, W, Cin = x.shape
        R = min(H, 2 * m1)
        dev = x.device
        X1 = torch.empty((B, H, m2, Cin), dtype=torch.complex64, device=dev)
        X2 = torch.empty((B, R, m2, Cin), dtype=torch.complex64, device=dev)
        Y = torch.empty((B, R, m2, Cout), dtype=torch.complex64, device=dev)
        Z = torch.empty((B, H, m2, Cout), dtype=torch.complex64, device=dev)
        y = ops.empty_nhwc(B, H, W, Cout, x)
        s = stream_ptr()
        check(lib.nps_spectral_dft_w(ops._c_src([Src(x)]), 1, B, H, W, Cin, m2, ptr(X1), s), "spectral_dft_w")
        check(lib.nps_spectral_dft_h(ptr(X1), ptr(X2), B, H, m1, m2, Cin, s), "spectral_dft_h")
        check(lib.nps_spectral_mix(ptr(X2), ptr(wpack), ptr(Y), B, R, m2, Cin, Cout, s), "spectral_mix")
        check(lib.nps_spectral_idft_h(ptr(Y), ptr(Z), B, H, m1, m2, Cout, s), "spectral_idft_h")
        check(lib.nps_spectral_idft_w(ptr(Z), ptr(y), B, H, W, m2, Cout, 0, None, 0, ops.new_tag(y), s),
              "spectral_idft_w")
        ctx.meta, ctx.shape = meta, (B, H, W, Cin)
        ctx.save_for_backward(X2, wpack)
        return y

    @staticmethod
    def backward(ctx, gy):
        m1, m2, Cout = ctx.meta
        B, H, W, Cin = ctx.shape
        X2, wpack = ctx.saved_tensors
        R = X2.shape[1]
        gy = _c(gy)
        dev = gy.device
        s = stream_ptr()
        gZ = torch.empty((B, H, m2, Cout), dtype=torch.complex64, device=dev)
        gY = torch.empty((B, R, m2, Cout), dtype=torch.complex64, device=dev)
        gX2 = torch.empty((B, R, m2, Cin), dtype=torch.complex64, device=dev)
        gwp = torch.empty((R, m2, Cin, Cout), dtype=torch.complex64, device=dev)
        check(lib.nps_spectral_idft_w_bwd(ptr(gy), ptr(gZ), B, H, W, m2, Cout, s), "spectral_idft_w_bwd")
        check(lib.nps_spectral_dft_h(ptr(gZ), ptr(gY), B, H, m1, m2, Cout, s), "spectral_dft_h (bwd)")
        check(lib.nps_spectral_mix_bwd(ptr(X2), ptr(wpack), ptr(gY), ptr(gX2), ptr(gwp), B, R, m2, Cin, Cout, s),
              "spectral_mix_bwd")
        dx = dw1 = dw2 = None
        if ctx.needs_input_grad[1]:
            gX1 = torch.empty((B, H, m2, Cin), dtype=torch.complex64, device=dev)
            check(lib.nps_spectral_idft_h(ptr(gX2), ptr(gX1), B, H, m1, m2, Cin, s), "spectral_idft_h (bwd)")
            dx = torch.empty((B, H, W, Cin), dtype=torch.float32, device=dev)
            check(lib.nps_spectral_dft_w_bwd(ptr(gX1), ptr(dx), B, H, W, m2, Cin, s), "spectral_dft_w_bwd")
        if ctx.needs_input_grad[2] or ctx.needs_input_grad[3]:
            dw1 = torch.empty((Cin, Cout, m1, m2), dtype=torch.complex64, device=dev)
            dw2 = torch.empty((Cin, Cout, m1, m2), dtype=torch.complex64, device=dev)
            check(lib.nps_spectral_unpack_grad(ptr(gwp), ptr(dw1), ptr(dw2), Cin, Cout, H, m1, m2, s),
                  "spectral_unpack_grad")
        return None, dx, dw1, dw2, None


def spectral_conv2d(module, x):
    H = x.shape[1]
    return SpectralConv2dFn.apply((module.modes1, module.modes2, module.out_channels), x, module.weights1,
                                  module.weights2, module.packed(H))


class SpectralConv3dFn(torch.autograd.Function):
    """SpectralConv3d.forward (proc_fno.py:334-376) and its torch.fft / complex-einsum backward, axis by
    axis with the 2-D kernels (include/nps.h, SpectralConv3d)."""

    @staticmethod
    def forward(ctx, meta, x, w1, w2, w3, w4, wpack):
        m1, m2, m3, Cout, D = meta
        x = _c(x)  # (B, D*H, W, Cin)
        B, DH, W, Cin = x.shape
        H = DH // D
        y = ops.empty_nhwc(B, DH, W, Cout, x)
        X3 = ops.spectral_conv3d_stages([Src(x)], D, H, W, Cin, wpack, m1, m2, m3, Cout, y)
        ctx.meta, ctx.shape = meta, (B, D, H, W, Cin)
        ctx.save_for_backward(X3, wpack)
        return y

    @staticmethod
    def backward(ctx, gy):
        m1, m2, m3, Cout, D = ctx.meta
        B, D, H, W, Cin = ctx.shape
        X3, wpack = ctx.saved_tensors
        R1, R2 = min(D, 2 * m1), min(H, 2 * m2)
        gy = _c(gy)
        dev = gy.device
        c64 = torch.complex64
        s = stream_ptr()
        gZ2 = torch.empty((B, D * H, m3, Cout), dtype=c64, device=dev)
        gZ1 = torch.empty((B * D, R2, m3, Cout), dtype=c64, device=dev)
        gY = torch.empty((B, R1, R2 * m3, Cout), dtype=c64, device=dev)
        gX3 = torch.empty((B, R1, R2 * m3, Cin), dtype=c64, device=dev)
        gwp = torch.empty((R1, R2, m3, Cin, Cout), dtype=c64, device=dev)
        check(lib.nps_spectral_idft_w_bwd(ptr(gy), ptr(gZ2), B, D * H, W, m3, Cout, s), "spectral3d idft_w_bwd")
        check(lib.nps_spectral_dft_h(ptr(gZ2), ptr(gZ1), B * D, H, m2, m3, Cout, s), "spectral3d dft_h (H, bwd)")
        check(lib.nps_spectral_dft_h(ptr(gZ1), ptr(gY), B, D, m1, R2 * m3, Cout, s), "spectral3d dft_h (D, bwd)")
        check(lib.nps_spectral_mix_bwd(ptr(X3), ptr(wpack), ptr(gY), ptr(gX3), ptr(gwp), B, R1, R2 * m3, Cin, Cout,
                                       s), "spectral3d mix_bwd")
        dx = None
        gws = [None] * 4
        if ctx.needs_input_grad[1]:
            gX2 = torch.empty((B, D, R2 * m3, Cin), dtype=c64, device=dev)
            gX1 = torch.empty((B * D, H, m3, Cin), dtype=c64, device=dev)
            check(lib.nps_spectral_idft_h(ptr(gX3), ptr(gX2), B, D, m1, R2 * m3, Cin, s), "spectral3d idft_h (D, bwd)")
            check(lib.nps_spectral_idft_h(ptr(gX2), ptr(gX1), B * D, H, m2, m3, Cin, s), "spectral3d idft_h (H, bwd)")
            dx = torch.empty((B, D * H, W, Cin), dtype=torch.float32, device=dev)
            check(lib.nps_spectral_dft_w_bwd(ptr(gX1), ptr(dx), B, D * H, W, m3, Cin, s), "spectral3d dft_w_bwd")
        if any(ctx.needs_input_grad[2:6]):
            gws = [torch.empty((Cin, Cout, m1, m2, m3), dtype=c64, device=dev) for _ in range(4)]
            check(lib.nps_spectral3d_unpack_grad(ptr(gwp), *[ptr(g) for g in gws], Cin, Cout, D, H, m1, m2, m3, s),
                  "spectral3d_unpack_grad")
        return (None, dx, *gws, None)


def spectral_conv3d(module, x, D):
    """x: (B, D*H, W, Cin) NDHWC view -> (B, D*H, W, Cout)."""
    H = x.shape[1] // D
    return SpectralConv3dFn.apply((module.modes1, module.modes2, module.modes3, module.out_channels, D), x,
                                  module.weights1, module.weights2, module.weights3, module.weights4,
                                  module.packed(D, H))


# ------------------------------------------------------------------------- decoder / wrapper / loss
class TimeConvDecodeFn(torch.autograd.Function):
    """TimeConvDense conv1d chain + add_delta('per_step') + tanh + spatial-cond mask
    (dec_grid.py:126-146, :8-31; activation_wrapper.py:34-35)."""

    @staticmethod
    def forward(ctx, meta, pre, u, w1, b1, w2, b2, dtcum, mask):
        mask_ch, act_tanh, num_c, tw = meta
        pre, u = _c(pre), _c(u)
        out = ops.timeconv_decode(pre, u, w1.detach().contiguous(), b1.detach(), w2.detach().contiguous(),
                                  b2.detach(), dtcum, mask, mask_ch, act_tanh, num_c, tw)
        ctx.meta = meta
        ctx.save_for_backward(pre, u, w1, b1, w2, b2, dtcum, mask if mask is not None else torch.empty(0))
        ctx.has_mask = mask is not None
        return out

    @staticmethod
    def backward(ctx, gout):
        mask_ch, act_tanh, num_c, tw = ctx.meta
        pre, u, w1, b1, w2, b2, dtcum, mask = ctx.saved_tensors
        mask = mask if ctx.has_mask else None
        gout = _c(gout)
        B, _, _, H, W = u.shape
        ka, kb = w1.shape[2], w2.shape[2]
        C2 = 2 * num_c
        nparams = C2 * num_c * ka + C2 + num_c * C2 * kb + num_c
        nblk = B * ((H * W + 63) // 64)
        ws = torch.empty((nblk, nparams), dtype=torch.float32, device=gout.device)
        gpre = torch.empty_like(pre)
        S = 0 if mask is None else mask.shape[1]
        check(lib.nps_timeconv_decode_bwd(ptr(pre), ptr(u), ptr(w1.detach().contiguous()), ptr(b1.detach()),
                                          ptr(w2.detach().contiguous()), ptr(b2.detach()), ptr(dtcum), ptr(mask), S,
                                          mask_ch, ptr(gout), ptr(gpre), ptr(ws), B, num_c, tw, H, W,
                                          1 if act_tanh else 0, stream_ptr()), "timeconv_decode_bwd")
        red = channel_sums(ws)
        o = 0
        gw1 = red[o:o + C2 * num_c * ka].view_as(w1)
        o += C2 * num_c * ka
        gb1 = red[o:o + C2]
        o += C2
        gw2 = red[o:o + num_c * C2 * kb].view_as(w2)
        o += num_c * C2 * kb
        gb2 = red[o:o + num_c]
        return None, gpre, None, gw1, gb1, gw2, gb2, None, None


class VolumeRescaleFn(torch.autograd.Function):
    """activation_wrapper 'individual_static' volume preservation + re-applied mask
    (activation_wrapper.py:80-105); x (the model input) is data and gets no gradient."""

    @staticmethod
    def forward(ctx, meta, u, x, mpdcum, mask):
        mask_ch = meta
        u = _c(u)
        B, c, tw, H, W = u.shape
        xc = _c(x)
        new_tot = ops.plane_sums(u, 0, H * W, H * W, B * c * tw)
        prev_tot = ops.plane_sums(xc, (xc.shape[2] - 1) * H * W, xc.shape[2] * H * W, H * W, B * c)
        out = u.clone()
        ops.volume_rescale(out, new_tot, prev_tot, mpdcum, mask, mask_ch)
        ctx.meta = meta
        ctx.has_mask = mask is not None
        ctx.save_for_backward(u, new_tot, prev_tot, mpdcum, mask if mask is not None else torch.empty(0))
        return out

    @staticmethod
    def backward(ctx, g):
        mask_ch = ctx.meta
        u, new_tot, prev_tot, mpdcum, mask = ctx.saved_tensors
        mask = mask if ctx.has_mask else None
        g = _c(g)
        B, c, tw, H, W = u.shape
        S = 0 if mask is None else mask.shape[1]
        D = torch.empty(B * c * tw, dtype=torch.float64, device=g.device)
        check(lib.nps_plane_dot(ptr(g), ptr(u), ptr(mask), S, mask_ch, B, c * tw, H, W, ptr(D), stream_ptr()),
              "plane_dot")
        gu = torch.empty_like(u)
        check(lib.nps_volume_rescale_bwd(ptr(g), ptr(new_tot), ptr(prev_tot), ptr(mpdcum), ptr(mask), S, mask_ch,
                                         ptr(D), ptr(gu), B, c, tw, H, W, stream_ptr()), "volume_rescale_bwd")
        return None, gu, None, None, None


class SqrtMseSumFn(torch.autograd.Function):
    """torch.sqrt(nn.MSELoss(reduction='sum')(pred, labels)) — autoregressivepushforwardtrainer.py:158-162."""

    @staticmethod
    def forward(ctx, pred, labels):
        pred, labels = _c(pred), _c(labels)
        L = ops.sq_err_sum(pred, labels)        # fp64 on device
        r = torch.sqrt(L)
        ctx.save_for_backward(pred, labels, r)
        return r.float()

    @staticmethod
    def backward(ctx, g):
        pred, labels, r = ctx.saved_tensors
        scale = (g.double() / r).reshape(1)      # d sqrt(L) / d pred = (pred - labels) / sqrt(L)
        out = torch.empty_like(pred)
        check(lib.nps_scaled_diff(ptr(pred), ptr(labels), ptr(scale), ptr(out), pred.numel(), stream_ptr()),
              "scaled_diff")
        return out, None


def sqrt_mse_sum(pred, labels):
    return SqrtMseSumFn.apply(pred, labels)


class MseSumFn(torch.autograd.Function):
    """nn.MSELoss(reduction='sum')(pred, labels) as an fp64 device scalar with a HIP backward — a rank's
    part S_r of the global sum under data parallelism (trainers.distributed.global_sqrt_loss)."""

    @staticmethod
    def forward(ctx, pred, labels):
        pred, labels = _c(pred), _c(labels)
        ctx.save_for_backward(pred, labels)
        return ops.sq_err_sum(pred, labels)     # fp64

    @staticmethod
    def backward(ctx, g):
        pred, labels = ctx.saved_tensors
        scale = (2.0 * g.double()).reshape(1)     # d S / d pred = 2 (pred - labels)
        out = torch.empty_like(pred)
        check(lib.nps_scaled_diff(ptr(pred), ptr(labels), ptr(scale), ptr(out), pred.numel(), stream_ptr()),
              "scaled_diff")
        return out, None


def mse_sum(pred, labels):
    return MseSumFn.apply(pred, labels)
