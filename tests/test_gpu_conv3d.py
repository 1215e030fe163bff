"""nps_conv3d (csrc/conv3d.hip): the 3-D U-Net convolutions of the 3-D U-FNO (BASELINE config C5) against
torch fp64 references of the same ops — nn.Conv3d valid / stride 2 (proc_unet_modern.py:222-227, :445-449),
the GroupNorm + GELU prologue on a torch.cat / crop_Nd frame (:245-247, :188-191), the 1x1 shortcut / final
conv, the residual accumulate at the crop offset (:250), and this build's 3-D Upsample (circular pad 1 +
ConvTranspose3d(k=4, s=2), DESIGN.md "3-D U-FNO").  fp32 storage runs on exact-fp32 MFMA (tolerance: rel-L2
< 1e-5); bf16 storage is compared with the fp64 op on the same bf16-rounded operands (rel-L2 < 1e-2)."""
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = {torch.float32: 1e-5, torch.bfloat16: 1e-2}
DTYPES = [torch.float32, torch.bfloat16]


def _ndhwc(x, dt):
    return x.permute(0, 2, 3, 4, 1).contiguous().to(DEV, dt)


def _ncdhw(y):
    return y.float().cpu().permute(0, 4, 1, 2, 3).double()


def _frame(srcs, B, dhw):
    """torch.cat of crop_Nd-placed sources (NCDHW fp64)."""
    C = sum(s.shape[1] for s, _ in srcs)
    fr = torch.zeros(B, C, *dhw, dtype=torch.float64)
    c = 0
    for s, off in srcs:
        D, H, W = s.shape[2:]
        lo = [max(0, o) for o in off]
        hi = [min(n, o + m) for n, o, m in zip(dhw, off, (D, H, W))]
        if all(h > l for l, h in zip(lo, hi)):
            fr[:, c:c + s.shape[1], lo[0]:hi[0], lo[1]:hi[1], lo[2]:hi[2]] = \
                s[:, :, lo[0] - off[0]:hi[0] - off[0], lo[1] - off[1]:hi[1] - off[1], lo[2] - off[2]:hi[2] - off[2]]
        c += s.shape[1]
    return fr


def _rt(x, dt):
    """the operand as the kernel sees it (bf16-rounded for bf16 storage)."""
    return x.to(dt).double() if dt == torch.bfloat16 else x.double()


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("K,stride,shape", [(3, 1, (2, 9, 20, 40)), (3, 2, (2, 9, 19, 37)), (1, 1, (1, 5, 7, 33))])
def test_conv3d_valid(dt, K, stride, shape):
    from nps_hip import ops
    torch.manual_seed(0)
    B, D, H, W = shape
    x1, x2 = torch.randn(B, 64, D, H, W), torch.randn(B, 4, D, H, W)
    w = torch.randn(48, 68, K, K, K) * 0.05
    b = torch.randn(48) * 0.1
    ref = F.conv3d(torch.cat([_rt(x1, dt), _rt(x2, dt)], 1), _rt(w, dt), b.double(), stride=stride)
    wp = ops.pack_conv3d_weight(w.to(DEV), bf16=dt == torch.bfloat16)
    y = ops.conv3d([ops.Src3(_ndhwc(x1, dt)), ops.Src3(_ndhwc(x2, dt))], (D, H, W), wp, b.to(DEV), 48, K,
                   stride=stride)
    assert rel_l2(_ncdhw(y), ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
def test_conv3d_gn_prologue_on_crop_frame(dt):
    """UpBlock shape: cat(h, crop_Nd(skip), crop_Nd(vb)) -> GroupNorm(1) -> GELU -> 3x3x3 valid conv; the
    skip is cropped on one axis and zero-padded on another, so the frame has uncovered (zero) voxels that
    the GroupNorm counts and normalises."""
    from nps_hip import ops
    torch.manual_seed(1)
    B, dhw = 2, (8, 12, 36)
    h = torch.randn(B, 32, *dhw)
    s = torch.randn(B, 32, 10, 10, 36) * 2 + 0.5
    v = torch.rand(B, 4, 6, 12, 36)
    offs = [(0, 0, 0), (-1, 1, 0), (1, 0, 0)]
    gamma, beta = 1 + 0.2 * torch.randn(68), 0.1 * torch.randn(68)
    fr = _frame([(_rt(h, dt), offs[0]), (_rt(s, dt), offs[1]), (_rt(v, dt), offs[2])], B, dhw)
    n = F.gelu(F.group_norm(fr, 1, gamma.double(), beta.double(), eps=1e-5))
    w = torch.randn(40, 68, 3, 3, 3) * 0.05
    ref = F.conv3d(_rt(n, dt), _rt(w, dt))
    srcs = [ops.Src3(_ndhwc(t, dt), *o) for t, o in zip((h, s, v), offs)]
    st = ops.gn_stats3d(srcs, dhw, 1)
    # (per-voxel channel runs are summed in fp32, the runs in fp64)
    torch.testing.assert_close(st[:, 0, 0].cpu(), fr.sum((1, 2, 3, 4)), rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(st[:, 0, 1].cpu(), (fr ** 2).sum((1, 2, 3, 4)), rtol=1e-6, atol=1e-3)
    gn = ops.GN(st, gamma.to(DEV), beta.to(DEV), 1, 1e-5)
    wp = ops.pack_conv3d_weight(w.to(DEV), bf16=dt == torch.bfloat16)
    y = ops.conv3d(srcs, dhw, wp, None, 40, 3, gn=gn, pre_act=1)
    # bf16: the kernel rounds the normalised frame to bf16 once more (as the LDS image) — the reference does too
    assert rel_l2(_ncdhw(y), ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("inside", [True, False])
def test_gn_stats3d_groups_across_unaligned_sources(dt, inside):
    """GroupNorm(2) moments of a [4 | 8 | 4]-channel frame (8 channels per group): the 8-channel source starts at
    channel 4, so each of its 8-channel pieces spans both groups — the per-element path, not the one-group-per-
    piece fast paths (for a source inside the frame and for a cropped one)."""
    from nps_hip import ops
    torch.manual_seed(5)
    B, dhw = 2, (4, 6, 10)
    xs = [torch.randn(B, c, *dhw) + k for k, c in enumerate((4, 8, 4))]
    offs = [(0, 0, 0), (0, 0, 0) if inside else (0, -1, 1), (0, 0, 0)]
    fr = _frame([(_rt(x, dt), o) for x, o in zip(xs, offs)], B, dhw)
    st = ops.gn_stats3d([ops.Src3(_ndhwc(x, dt), *o) for x, o in zip(xs, offs)], dhw, 2).cpu()
    g = fr.view(B, 2, 8, *dhw)
    torch.testing.assert_close(st[:, :, 0], g.sum((2, 3, 4, 5)), rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(st[:, :, 1], (g ** 2).sum((2, 3, 4, 5)), rtol=1e-6, atol=1e-3)


@pytest.mark.parametrize("dt", DTYPES)
def test_conv3d_residual_accumulate_and_final_crop(dt):
    """ResidualBlock tail: conv2 accumulated at crop offset (2, 2, 2) into the 1x1 shortcut output; and the
    U-Net final GroupNorm(8) + GELU + 1x1 conv written at a negative crop offset with addend + GELU
    (GELU(h_fno + h_unet), proc_ufno.py:118)."""
    from nps_hip import ops
    torch.manual_seed(2)
    B, dhw = 1, (9, 14, 40)
    x = torch.randn(B, 24, *dhw)
    ws, bs = torch.randn(32, 24, 1, 1, 1) * 0.2, torch.randn(32) * 0.1
    w2, b2 = torch.randn(32, 24, 3, 3, 3) * 0.05, torch.randn(32) * 0.1
    sc = F.conv3d(_rt(x, dt), _rt(ws, dt), bs.double())
    h = F.conv3d(_rt(x, dt), _rt(w2, dt), b2.double())
    ref = sc.clone()
    ref[:, :, 1:-1, 1:-1, 1:-1] += h  # crop_Nd(h, shortcut) + shortcut (valid 3^3 conv: offset 1 here)
    xd = _ndhwc(x, dt)
    out = ops.conv3d([ops.Src3(xd)], dhw, ops.pack_conv3d_weight(ws.to(DEV), bf16=dt == torch.bfloat16), bs.to(DEV),
                     32, 1)
    ops.conv3d([ops.Src3(xd)], dhw, ops.pack_conv3d_weight(w2.to(DEV), bf16=dt == torch.bfloat16), b2.to(DEV), 32, 3,
               out=out, out_off=(1, 1, 1), accumulate=True)
    assert rel_l2(_ncdhw(out), ref) < TOL[dt]
    # final: GN(8) -> GELU -> 1x1 -> crop to (7, 12, 36) at offset -1, -1, -2, + addend, GELU
    gamma, beta = 1 + 0.1 * torch.randn(32), 0.1 * torch.randn(32)
    wf, bf = torch.randn(32, 32, 1, 1, 1) * 0.2, torch.randn(32) * 0.1
    r = _rt(ref, dt) if dt == torch.bfloat16 else ref
    fin = F.conv3d(_rt(F.gelu(F.group_norm(r, 8, gamma.double(), beta.double(), eps=1e-5)), dt), _rt(wf, dt),
                   bf.double())[:, :, 1:8, 1:13, 2:38]
    addend = torch.randn(B, 32, 7, 12, 36)
    want = F.gelu(fin + _rt(addend, dt))
    st = ops.gn_stats3d([ops.Src3(out)], dhw, 8)
    o2 = torch.empty(B, 7, 12, 36, 32, dtype=dt, device=DEV)
    ops.conv3d([ops.Src3(out)], dhw, ops.pack_conv3d_weight(wf.to(DEV), bf16=dt == torch.bfloat16), bf.to(DEV), 32,
               1, gn=ops.GN(st, gamma.to(DEV), beta.to(DEV), 8, 1e-5), pre_act=1, out=o2, out_off=(-1, -1, -2),
               addend=_ndhwc(addend, dt), act=1)
    assert rel_l2(_ncdhw(o2), want) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("shape", [(2, 5, 7, 20), (1, 4, 16, 33)])
def test_conv3d_upsample_transposed(dt, shape):
    """3-D Upsample: circular pad 1 on every axis, then ConvTranspose3d(k=4, s=2, p=0) — 8 phase convs."""
    from nps_hip import ops
    torch.manual_seed(3)
    B, D, H, W = shape
    x = torch.randn(B, 48, D, H, W)
    w, b = torch.randn(48, 40, 4, 4, 4) * 0.05, torch.randn(40) * 0.1
    xp = F.pad(_rt(x, dt), (1, 1, 1, 1, 1, 1), mode="circular")
    ref = F.conv_transpose3d(xp, _rt(w, dt), b.double(), stride=2)
    assert ref.shape[2:] == (2 * D + 6, 2 * H + 6, 2 * W + 6)
    wp = ops.pack_conv3d_weight(w.to(DEV), transposed=True, bf16=dt == torch.bfloat16)
    y = ops.conv3d([ops.Src3(_ndhwc(x, dt))], (D, H, W), wp, b.to(DEV), 40, 2, transposed=True, circ=1, zpad=1)
    assert y.shape[1:4] == ref.shape[2:]
    assert rel_l2(_ncdhw(y), ref) < TOL[dt]


@pytest.mark.parametrize("dt", DTYPES)
@pytest.mark.parametrize("groups", [1, 2, 4])
def test_gn_stats3d_and_frame_pack3d_channels_mod4(dt, groups):
    """C5's 64 + 4 = 68-channel frames (C % 8 == 4): the moments sweep the source as a flat element array
    (16-B loads, a group per 4-element half) when the channels per group are a multiple of 4 (GroupNorm 1, 2)
    and fall back to per-element pieces otherwise (4 groups of 17); the frame pack reads 4-channel halves.
    Against the fp64 GroupNorm + GELU of the same frame."""
    from nps_hip import ops
    torch.manual_seed(7)
    B, dhw = 2, (5, 6, 11)
    x = torch.randn(B, 68, *dhw) * 1.5 + 0.3
    fr = _rt(x, dt)
    st = ops.gn_stats3d([ops.Src3(_ndhwc(x, dt))], dhw, groups).cpu()
    g = fr.view(B, groups, 68 // groups, *dhw)
    torch.testing.assert_close(st[:, :, 0], g.sum((2, 3, 4, 5)), rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(st[:, :, 1], (g ** 2).sum((2, 3, 4, 5)), rtol=1e-6, atol=1e-3)
    gamma, beta = 1 + 0.2 * torch.randn(68), 0.1 * torch.randn(68)
    gn = ops.GN(st.to(DEV), gamma.to(DEV), beta.to(DEV), groups, 1e-5)
    packed = ops.frame_pack3d([ops.Src3(_ndhwc(x, dt))], dhw, gn, pre_act=1)
    assert packed.shape[-1] == 80 and float(packed[..., 68:].abs().max()) == 0.0
    want = F.gelu(F.group_norm(fr, groups, gamma.double(), beta.double(), eps=1e-5))
    got = packed[..., :68].float().cpu().permute(0, 4, 1, 2, 3).double()
    assert rel_l2(got, _rt(want, dt) if dt == torch.bfloat16 else want) < (1e-2 if dt == torch.bfloat16 else 1e-6)


@pytest.mark.parametrize("dt", DTYPES)
def test_conv3d_out_stats_carry_moments(dt):
    """nps_conv3d_t.out_stats: a plain-epilogue conv adds the GroupNorm(1) moments of the values it stores (as
    stored: bf16-rounded for bf16) — the ResidualBlock's norm2 statistics of h1 without a gn_stats3d pass;
    equal to gn_stats3d over the output, and to the fp64 sums of it."""
    from nps_hip import ops
    torch.manual_seed(9)
    B, dhw = 2, (6, 10, 21)
    x = torch.randn(B, 36, *dhw)
    w, b = torch.randn(24, 36, 3, 3, 3) * 0.05, torch.randn(24) * 0.1
    gamma, beta = 1 + 0.2 * torch.randn(36), 0.1 * torch.randn(36)
    src = [ops.Src3(_ndhwc(x, dt))]
    gn = ops.GN(ops.gn_stats3d(src, dhw, 1), gamma.to(DEV), beta.to(DEV), 1, 1e-5)
    st = ops.new_stats(B, src[0].t)
    y = ops.conv3d(src, dhw, ops.pack_conv3d_weight(w.to(DEV), bf16=dt == torch.bfloat16), b.to(DEV), 24, 3, gn=gn,
                   pre_act=1, out_stats=st)
    got = ops._stats_sum([st], B, ops.new_stats(B, y, 1)).cpu()[:, 0]
    ref = ops.gn_stats3d([ops.Src3(y)], y.shape[1:4], 1).cpu()[:, 0]
    yd = y.float().cpu().double().reshape(B, -1)
    torch.testing.assert_close(got, ref, rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(got[:, 0], yd.sum(1), rtol=1e-6, atol=1e-3)
    torch.testing.assert_close(got[:, 1], (yd ** 2).sum(1), rtol=1e-6, atol=1e-3)


@pytest.mark.parametrize("dt", DTYPES)
def test_conv3d_out_stats_with_accumulate_addend_act_and_phases(dt):
    """out_stats for the 3-D producers whose outputs feed the next GroupNorm(1) (ops.group_norm_stats3d carries them
    instead of a gn_stats3d pass): conv2 accumulating into the shortcut output (the CHANGE's moments, added to a
    buffer seeded with the old output's), the U-Net's final conv with the U-FNO addend + GELU, and the 8 phases of
    the 3-D Upsample — each equal to a gn_stats3d pass over the stored tensor."""
    from nps_hip import ops
    torch.manual_seed(11)
    B, dhw = 2, (6, 10, 21)
    bf = dt == torch.bfloat16
    x = _ndhwc(torch.randn(B, 32, *dhw), dt)
    w, b = torch.randn(32, 32, 3, 3, 3) * 0.05, torch.randn(32) * 0.1

    def passes(t):
        return ops.gn_stats3d([ops.Src3(t)], t.shape[1:4], 1).cpu()[:, 0]

    def carried(st):
        return ops._stats_sum([st], B, ops.new_stats(B, st, 1)).cpu()[:, 0]

    # accumulate into a (cropped) output seeded with its own moments
    out = _ndhwc(torch.randn(B, 32, 6, 12, 23), dt)
    st = ops.copy_stats(ops.gn_stats3d([ops.Src3(out)], out.shape[1:4], 1))
    ops.conv3d([ops.Src3(x)], dhw, ops.pack_conv3d_weight(w.to(DEV), bf16=bf), b.to(DEV), 32, 3, zpad=1, out=out,
               out_off=(0, 1, 1), accumulate=True, out_stats=st)
    torch.testing.assert_close(carried(st), passes(out), rtol=1e-5, atol=1e-2)
    # addend + GELU
    add = _ndhwc(torch.randn(B, 32, *dhw), dt)
    st = ops.new_stats(B, x)
    y = ops.conv3d([ops.Src3(x)], dhw, ops.pack_conv3d_weight(w.to(DEV), bf16=bf), b.to(DEV), 32, 3, zpad=1,
                   addend=add, act=1, out_stats=st)
    torch.testing.assert_close(carried(st), passes(y), rtol=1e-5, atol=1e-2)
    # the 3-D Upsample's 8 phases (circular pad 1, ConvTranspose3d k4 s2)
    wt = torch.randn(32, 32, 4, 4, 4) * 0.05
    st = ops.new_stats(B, x)
    u = ops.conv3d([ops.Src3(x)], dhw, ops.pack_conv3d_weight(wt.to(DEV), transposed=True, bf16=bf), None, 32, 2,
                   transposed=True, circ=1, zpad=1, out_stats=st)
    torch.testing.assert_close(carried(st), passes(u), rtol=1e-5, atol=1e-2)


@pytest.mark.parametrize("cout", [64, 96, 128])
@pytest.mark.parametrize("chans,offs", [((64, 4), ((0, 0, 0), (0, 0, 0))),
                                        ((64, 64, 4), ((0, 0, 0), (-1, 1, 0), (1, 0, 0))),
                                        ((192, 8), ((0, 0, 0), (0, -2, 1)))])
def test_conv3d_1x1x1_bf16_streaming(cout, chans, offs):
    """The bf16 1x1x1 kernel (conv3d_1x1_kernel: weights resident in LDS, every K-step's load of a 32-voxel tile in
    flight at once): the ResidualBlock shortcut over cat(h, crop_Nd(skip), crop_Nd(vb)) at Cin 68 / 132 / 200 (5, 9
    and 16 K-step register sets), Cout 64 / 96 / 128 (2 and 4 channel blocks), a volume that is not a multiple of
    32 voxels; bias, out_stats; against fp64 on the bf16-rounded operands, and the moments against a gn_stats3d pass."""
    from nps_hip import ops
    torch.manual_seed(13)
    B, dhw = 2, (5, 9, 37)
    xs = []
    for k, (c, o) in enumerate(zip(chans, offs)):
        shp = tuple(n - 2 * oo for n, oo in zip(dhw, o))  # crop (< 0): larger; zero-pad (> 0): smaller
        xs.append(torch.randn(B, c, *shp) * (1 + 0.5 * k))
    dt = torch.bfloat16
    cin = sum(chans)
    w, b = torch.randn(cout, cin, 1, 1, 1) / cin ** 0.5, torch.randn(cout) * 0.1
    fr = _frame([(_rt(x, dt), o) for x, o in zip(xs, offs)], B, dhw)
    ref = F.conv3d(fr, _rt(w, dt), b.double())
    srcs = [ops.Src3(_ndhwc(x, dt), *o) for x, o in zip(xs, offs)]
    st = ops.new_stats(B, srcs[0].t)
    y = ops.conv3d(srcs, dhw, ops.pack_conv3d_weight(w.to(DEV), bf16=True), b.to(DEV), cout, 1, out_stats=st)
    assert rel_l2(_ncdhw(y), ref) < 1e-2
    got = ops._stats_sum([st], B, ops.new_stats(B, y, 1)).cpu()[:, 0]
    torch.testing.assert_close(got, ops.gn_stats3d([ops.Src3(y)], dhw, 1).cpu()[:, 0], rtol=1e-5, atol=1e-2)


def test_conv3d_1x1x1_bf16_streaming_prologue_epilogue():
    """The same kernel with the GroupNorm(2) + GELU prologue on a cropped two-source frame, written at a crop offset
    with addend + GELU, and accumulating (the change's moments into a buffer seeded with the old output's)."""
    from nps_hip import ops
    torch.manual_seed(14)
    dt = torch.bfloat16
    B, dhw = 2, (6, 10, 35)
    h, v = torch.randn(B, 64, *dhw) + 0.3, torch.rand(B, 4, 6, 8, 35)
    offs = [(0, 0, 0), (0, 1, 0)]
    gamma, beta = 1 + 0.2 * torch.randn(68), 0.1 * torch.randn(68)
    fr = _frame([(_rt(h, dt), offs[0]), (_rt(v, dt), offs[1])], B, dhw)
    n = _rt(F.gelu(F.group_norm(fr, 2, gamma.double(), beta.double(), eps=1e-5)), dt)
    w, b = torch.randn(64, 68, 1, 1, 1) / 68 ** 0.5, torch.randn(64) * 0.1
    srcs = [ops.Src3(_ndhwc(t, dt), *o) for t, o in zip((h, v), offs)]
    gn = ops.GN(ops.gn_stats3d(srcs, dhw, 2), gamma.to(DEV), beta.to(DEV), 2, 1e-5)
    wp = ops.pack_conv3d_weight(w.to(DEV), bf16=True)
    # crop to (4, 8, 33) at offset -1 with addend + GELU
    addend = torch.randn(B, 64, 4, 8, 33)
    want = F.gelu(F.conv3d(n, _rt(w, dt), b.double())[:, :, 1:5, 1:9, 1:34] + _rt(addend, dt))
    o2 = torch.empty(B, 4, 8, 33, 64, dtype=dt, device=DEV)
    ops.conv3d(srcs, dhw, wp, b.to(DEV), 64, 1, gn=gn, pre_act=1, out=o2, out_off=(-1, -1, -1),
               addend=_ndhwc(addend, dt), act=1)
    assert rel_l2(_ncdhw(o2), want) < 1e-2
    # accumulate into a seeded output
    base = torch.randn(B, 64, *dhw)
    out = _ndhwc(base, dt)
    st = ops.copy_stats(ops.gn_stats3d([ops.Src3(out)], dhw, 1))
    ops.conv3d(srcs, dhw, wp, b.to(DEV), 64, 1, gn=gn, pre_act=1, out=out, accumulate=True, out_stats=st)
    assert rel_l2(_ncdhw(out), F.conv3d(n, _rt(w, dt), b.double()) + _rt(base, dt)) < 1e-2
    got = ops._stats_sum([st], B, ops.new_stats(B, out, 1)).cpu()[:, 0]
    torch.testing.assert_close(got, ops.gn_stats3d([ops.Src3(out)], dhw, 1).cpu()[:, 0], rtol=1e-5, atol=1e-2)


# the bf16 fast paths (one 16-channel-aligned source, no prologue): stage copies by LDS-DMA into one stage buffer
# with the half-swap swizzle on the source address and a zero line for the padding (conv3d.hip GLT / SB): 3x3x3
# stride 1 on 1 / 3 / 5 channel chunks, one or two 64-channel co tiles, zero / circular / both paddings, odd extents
# (row and column tails); 3x3x3 stride 2; the 8 phases of the 3-D Upsample (2x2x2, circular + zero pad)
FAST_CASES = [(16, 40, 0, 1, (2, 5, 9, 37), 3, 1, False), (48, 64, 1, 0, (1, 6, 17, 33), 3, 1, False),
              (80, 96, 1, 1, (2, 4, 8, 70), 3, 1, False), (64, 64, 0, 0, (1, 3, 12, 64), 3, 1, False),
              (64, 64, 0, 1, (1, 9, 19, 37), 3, 2, False), (48, 40, 1, 1, (2, 5, 7, 20), 2, 1, True)]


def _fast_case(cin, cout, circ, zpad, shape, k, stride, transposed):
    from nps_hip import ops
    torch.manual_seed(0)
    B, D, H, W = shape
    x = torch.randn(B, cin, D, H, W)
    w = torch.randn(*((cin, cout) if transposed else (cout, cin)), *(4 if transposed else k,) * 3) * 0.05
    b = torch.randn(cout) * 0.1
    wp = ops.pack_conv3d_weight(w.to(DEV), transposed=transposed, bf16=True)
    y = ops.conv3d([ops.Src3(_ndhwc(x, torch.bfloat16))], (D, H, W), wp, b.to(DEV), cout, k, stride=stride,
                   transposed=transposed, circ=circ, zpad=zpad)
    return x, w, b, y


@pytest.mark.parametrize("cin,cout,circ,zpad,shape,k,stride,transposed", FAST_CASES)
def test_conv3d_bf16_fast_path_lds_dma(cin, cout, circ, zpad, shape, k, stride, transposed):
    x, w, b, y = _fast_case(cin, cout, circ, zpad, shape, k, stride, transposed)
    xr = _rt(x, torch.bfloat16)
    if circ:
        xr = F.pad(xr, (circ,) * 6, mode="circular")
    if transposed:  # the 3-D Upsample: circular pad, then ConvTranspose3d(k=4, s=2) (zpad 1 = its full extent)
        ref = F.conv_transpose3d(xr, _rt(w, torch.bfloat16), b.double(), stride=2)
    else:
        if zpad:
            xr = F.pad(xr, (zpad,) * 6)
        ref = F.conv3d(xr, _rt(w, torch.bfloat16), b.double(), stride=stride)
    assert y.shape[1:4] == ref.shape[2:]
    assert rel_l2(_ncdhw(y), ref) < TOL[torch.bfloat16]


# multi-source frames: the bf16 1x1x1 over three sources (generic kernel at four waves per SIMD) and the GroupNorm +
# GELU frame pack — flat (every source covers the frame at offset 0: no coordinate decode) and cropped / zero-padded
# sources (crop offsets of either sign on every axis: the general decode)
MULTI_CASES = [((64, 64, 4), ((0, 0, 0), (0, 0, 0), (0, 0, 0)), 64, (2, 5, 9, 37)),
               ((64, 64, 4), ((0, 0, 0), (-1, 1, 0), (1, 0, 0)), 96, (1, 6, 17, 33)),
               ((64, 4), ((0, 0, 0), (0, 0, 0)), 64, (2, 4, 8, 70)), ((4, 48, 12), ((0, 0, 0),) * 3, 40, (1, 3, 12, 64)),
               ((64, 4), ((0, 0, 0), (1, -1, 2)), 64, (2, 5, 9, 37)), ((48, 16), ((-1, 0, -2), (0, 2, 1)), 40, (1, 6, 11, 20))]


def _multi_case(chans, offs, cout, shape):
    from nps_hip import ops
    torch.manual_seed(1)
    B, D, H, W = shape
    dt = torch.bfloat16
    xs = [torch.randn(B, c, *(n - 2 * oo for n, oo in zip((D, H, W), o))) * (1 + 0.5 * k)
          for k, (c, o) in enumerate(zip(chans, offs))]
    srcs = [ops.Src3(_ndhwc(x, dt), *o) for x, o in zip(xs, offs)]
    cin = sum(chans)
    w, b = torch.randn(cout, cin, 1, 1, 1) / cin ** 0.5, torch.randn(cout) * 0.1
    y = ops.conv3d(srcs, (D, H, W), ops.pack_conv3d_weight(w.to(DEV), bf16=True), b.to(DEV), cout, 1)
    gamma, beta = 1 + 0.2 * torch.randn(cin), 0.1 * torch.randn(cin)
    gn = ops.GN(ops.gn_stats3d(srcs, (D, H, W), 2), gamma.to(DEV), beta.to(DEV), 2, 1e-5)
    packed = ops.frame_pack3d(srcs, (D, H, W), gn, 1)
    return xs, gamma, beta, y, packed


@pytest.mark.parametrize("chans,offs,cout,shape", MULTI_CASES)
def test_frame_pack3d_multi_source_vs_fp64(chans, offs, cout, shape):
    xs, gamma, beta, _, packed = _multi_case(chans, offs, cout, shape)
    B, D, H, W = shape
    dt = torch.bfloat16
    fr = _frame([(_rt(x, dt), o) for x, o in zip(xs, offs)], B, (D, H, W))
    want = F.gelu(F.group_norm(fr, 2, gamma.double(), beta.double(), eps=1e-5))
    cin = sum(chans)
    assert packed.shape[-1] % 16 == 0 and bool((packed[..., cin:] == 0).all())
    assert rel_l2(_ncdhw(packed[..., :cin]), want) < 1e-2


def test_conv3d_bf16_fast_path_lds_dma_matches_register_staging(tmp_path):
    """The LDS-DMA staging changes only how a stage reaches LDS (and how many work-groups share a CU): the same
    image, the same MFMA order — the output is bit-identical to the register-staged double-buffered kernels
    (NPS_C3D_GLDS=0, read once per process: a child process).  Likewise the four-waves-per-SIMD 1x1x1 and the flat
    multi-source frame pack against their previous forms."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    f = tmp_path / "staged.pt"
    code = (f"import sys, torch; sys.path[:0] = [{here!r}, {os.path.dirname(here)!r}, "
            f"{os.path.join(os.path.dirname(here), 'neural-pde-surrogates_amd')!r}]\n"
            "import test_gpu_conv3d as t\n"
            f"torch.save([[t._fast_case(*c)[3].cpu() for c in t.FAST_CASES], "
            f"[[r.cpu() for r in t._multi_case(*c)[3:]] for c in t.MULTI_CASES]], {str(f)!r})\n")
    # (and the multi-source defaults: the 1x1x1 at three waves per SIMD, the frame pack through the general decode —
    # NPS_PACK3D_MFLAT=0 also turns off the flat pack kernel)
    env = dict(os.environ, NPS_C3D_GLDS="0", NPS_C3D_K1O4="0", NPS_PACK3D_MFLAT="0")
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=240)
    staged, multi = torch.load(f, weights_only=True)
    for c, ys in zip(FAST_CASES, staged):
        assert torch.equal(_fast_case(*c)[3].cpu(), ys), c
    for c, (ys, ps) in zip(MULTI_CASES, multi):
        _, _, _, y, p = _multi_case(*c)
        assert torch.equal(y.cpu(), ys), c
        assert torch.equal(p.cpu(), ps), c
