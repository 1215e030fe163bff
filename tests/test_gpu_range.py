"""Range safety of the split-fp16 convs (3-pass hi/lo fp16 MFMA, the default arithmetic of every 1x1 / 2x2 /
3x3 / 5x5 conv): activations far from O(1) — tiny (1e-4), large (1e3) and beyond fp16's range (7e4, 1.5e5)
— must keep the fp32 bar of BASELINE.json (rel-L2 < 1e-5 against an fp64 reference of the same op).

The kernels scale their input by a power of 2 from the RANGE TAG the tensor carries (include/nps.h,
nps_conv2d_t.in_scale / in_tag*; ops.py): produced by the epilogue of the kernel that wrote the tensor, or
by nps_absmax for a tensor that arrives untagged.  Reference semantics: the convs of
proc_unet_modern.py / proc_dilatedresnet.py:71-76 / enc_grid.py / dec_grid.py, in fp64.
"""
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_l2

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda"
SCALES = [1e-4, 1e3, 7e4, 1.5e5]

# (Cin, Cout, k, stride, dil, padding, padding_mode, H, W): one shape per split-fp16 kernel class
KERNELS = {
    "3x3": (196, 192, 3, 1, 1, 0, "zeros", 33, 35),               # conv2d_x3_kernel<9,*>
    "3x3_circ": (64, 64, 3, 1, 1, 1, "circular", 20, 24),         # circular frame extension
    "1x1_lds_weights": (196, 192, 1, 1, 1, 0, "zeros", 37, 29),   # conv1x1_wl_kernel
    "1x1_coblock": (48, 388, 1, 1, 1, 0, "zeros", 15, 17),        # conv1x1_x3_kernel
    "5x5_dilated": (132, 128, 5, 1, 4, "same", "circular", 40, 36),  # conv2d_x3_kernel<25,2> on the lattice
    "3x3_s2": (32, 32, 3, 2, 1, 0, "zeros", 31, 29),              # space-to-depth 2x2 (<4,*>)
}


def _ref_conv(x, w, b, s, d, p, pm):
    x, w, b = x.double(), w.double(), b.double()
    if pm == "circular":
        k = w.shape[-1]
        tot = d * (k - 1)
        pad = tot // 2 if p == "same" else p
        x = F.pad(x, (pad, tot - pad if p == "same" else pad) * 2, mode="circular")
        return F.conv2d(x, w, b, stride=s, dilation=d)
    return F.conv2d(x, w, b, stride=s, dilation=d, padding=p)


@pytest.mark.parametrize("scale", SCALES)
@pytest.mark.parametrize("kind", list(KERNELS))
def test_split_fp16_conv_range(kind, scale):
    from models.common import Conv2d
    from nps_hip import ops
    Cin, Cout, k, s, d, p, pm, H, W = KERNELS[kind]
    torch.manual_seed(0)
    m = Conv2d(Cin, Cout, k, stride=s, dilation=d, padding=p, padding_mode=pm)
    x = torch.randn(2, Cin, H, W) * scale
    ref = _ref_conv(x, m.weight.detach(), m.bias.detach(), s, d, p, pm)
    md = m.to(DEV)
    xd = ops.nchw_to_nhwc(x.to(DEV))
    y = md.run([ops.Src(xd)], (H, W))
    if s == 1:  # (the stride-2 form reads a space-to-depth copy, which carries the tag instead)
        assert ops.tag_value(xd) == pytest.approx(float(x.abs().max()), rel=1e-6)  # nps_absmax on first use
    out = ops.nhwc_to_nchw(y).cpu()
    assert rel_l2(out, ref) < TOL, (kind, scale)
    # the epilogue tagged the output with its exact max |value|
    assert ops.tag_value(y) == pytest.approx(float(out.abs().max()), rel=1e-6)


@pytest.mark.parametrize("scale", [1e-4, 7e4])
def test_conv_transpose_range(scale):
    """ConvTranspose2d(k=4, s=2) as four 2x2 phase convs writing one output (one shared output tag)."""
    from models.common import ConvTranspose2d_padded
    from oracle import functional as Fo
    torch.manual_seed(0)
    m = ConvTranspose2d_padded(1, 24, 20, kernel_size=4, stride=2)
    x = torch.randn(2, 24, 13, 11) * scale
    sd = {"weight": m.weight.detach().double(), "bias": m.bias.detach().double()}
    ref = Fo.conv_transpose_ref(x.double(), sd, "", stride=2, padding=0, circ_pre_pad=1)
    y = m.to(DEV)(x.to(DEV)).cpu()
    assert rel_l2(y, ref) < TOL


def test_concat_sources_of_different_ranges():
    """One virtual frame of three sources at 1e-3, 1 and 2e4 (cat + crop, proc_unet_modern.py:188-191):
    the conv scales by the max of the sources' tags; the small source keeps an absolute error far below
    the fp32 rounding of the output."""
    from nps_hip import ops
    torch.manual_seed(3)
    B, H, W = 2, 22, 20
    h = torch.randn(B, 32, H, W) * 1e-3
    sk = torch.randn(B, 16, 19, 17)
    v = torch.randn(B, 16, 25, 23) * 2e4
    w = torch.randn(24, 64, 3, 3) * 0.05
    b = torch.randn(24) * 0.1
    oy1, ox1 = ops.crop_offset(19, H), ops.crop_offset(17, W)
    oy2, ox2 = ops.crop_offset(25, H), ops.crop_offset(23, W)
    frame = torch.zeros(B, 64, H, W, dtype=torch.float64)
    frame[:, :32] = h.double()
    frame[:, 32:48, oy1:oy1 + 19, ox1:ox1 + 17] = sk.double()
    frame[:, 48:] = v.double()[:, :, -oy2:-oy2 + H, -ox2:-ox2 + W]
    ref = F.conv2d(frame, w.double(), b.double())
    srcs = [ops.Src(ops.nchw_to_nhwc(h.to(DEV))), ops.Src(ops.nchw_to_nhwc(sk.to(DEV)), oy1, ox1),
            ops.Src(ops.nchw_to_nhwc(v.to(DEV)), oy2, ox2)]
    wp = ops.pack_conv_weight(w.to(DEV))
    y = ops.nhwc_to_nchw(ops.conv2d(srcs, (H, W), wp, b.to(DEV), 24, 3, 3)).cpu()
    assert rel_l2(y, ref) < TOL


@pytest.mark.parametrize("scale", [1e-4, 5e3])
def test_dilated_resnet_block_chain(scale):
    """A DRN block (7 dilated 5x5 convs, GELU after each, proc_dilatedresnet.py:53-84) on an input far from
    O(1): every intermediate is produced and range-tagged by the previous conv's epilogue."""
    from models.enc_proc_dec_components.proc_dilatedresnet import DilatedResnetBlock
    from nps_hip import ops
    from torch import nn
    torch.manual_seed(5)
    blk = DilatedResnetBlock(2, 24, 5, (1, 2, 4, 8, 4, 2, 1), nn.GELU(), "circular", hidden_features_out=24)
    x = torch.randn(2, 24, 32, 28) * scale
    h = x.double()
    for conv in [m for m in blk.layers if isinstance(m, torch.nn.Conv2d)]:
        h = F.gelu(_ref_conv(h, conv.weight.detach(), conv.bias.detach(), 1, conv.dilation[0], "same", "circular"))
    blk = blk.to(DEV)
    y = ops.nhwc_to_nchw(blk.run([ops.Src(ops.nchw_to_nhwc(x.to(DEV)))])).cpu()
    assert rel_l2(y, h) < TOL


def test_accumulating_conv_tag_covers_prior_contents():
    """A conv accumulating into an untagged tensor seeds the tag with the tensor's current max (the
    residual `crop_Nd(h) + shortcut` into a cloned input, proc_unet_modern.py:250)."""
    from nps_hip import ops
    torch.manual_seed(7)
    base = (torch.randn(2, 18, 18, 16) * 3e4).to(DEV)
    x = torch.randn(2, 18, 18, 8).to(DEV)
    wp = ops.pack_conv_weight((torch.randn(16, 8, 3, 3) * 0.1).to(DEV))
    out = base.clone()
    ops.conv2d([ops.Src(x)], (18, 18), wp, None, 16, 3, 3, out=out, out_off=(1, 1), accumulate=True)
    assert ops.tag_value(out) >= float(out.abs().max().cpu()) * (1 - 1e-6)


@pytest.mark.parametrize("cout", [192, 64])  # 192: the wide 192-channel tile, 64: the 512-pixel tile
@pytest.mark.parametrize("xscale,gscale", [(1e-4, 1.0), (7e4, 1e-3), (1.0, 3e2), (1.0, 1e-4)])
def test_fused_groupnorm_prologue_range(cout, xscale, gscale):
    """The 3x3 conv applying GroupNorm(8) + GELU while staging its patch (proc_unet_modern.py:62-99): the
    normalised values do not carry the input's range tag; the kernel scales them from gamma, beta and the
    group size (gn_prologue_scale), so a GroupNorm affine far from O(1) keeps the fp32 bar."""
    from nps_hip import ops
    if not ops.FUSE_PROLOGUE:
        pytest.skip("fused prologue off (NPS_FUSE_PROLOGUE=0)")
    torch.manual_seed(7)
    B, Cin, H, W, G = 2, 192, 34, 30, 8
    x = torch.randn(B, Cin, H, W) * xscale + 0.3 * xscale
    gamma = (torch.rand(Cin) + 0.5) * gscale
    beta = (torch.rand(Cin) - 0.5) * gscale
    w = torch.randn(cout, Cin, 3, 3) * 0.03
    b = torch.randn(cout) * 0.1
    ref = F.conv2d(F.gelu(F.group_norm(x.double(), G, gamma.double(), beta.double(), 1e-5)), w.double(), b.double(),
                   padding=1)
    packs = []
    real_pack = ops.frame_pack
    try:
        ops.frame_pack = lambda *a, **k: packs.append(1) or real_pack(*a, **k)
        xd = ops.nchw_to_nhwc(x.to(DEV))
        st = ops.group_norm_stats([ops.Src(xd)], (H, W), G)
        gn = ops.GN(st, gamma.to(DEV), beta.to(DEV), G, 1e-5)
        y = ops.conv2d([ops.Src(xd)], (H, W), ops.pack_conv_weight(w.to(DEV)), b.to(DEV), cout, 3, 3, pad=(1, 1),
                       gn=gn, pre_act=1)
    finally:
        ops.frame_pack = real_pack
    assert not packs, "GroupNorm prologue went through frame_pack"
    assert rel_l2(ops.nhwc_to_nchw(y).cpu(), ref) < TOL, (cout, xscale, gscale)


def test_tag_arena_wrap_inside_a_conv_keeps_range():
    """a conv reads its inputs' tag pointers and then allocates its output tag.  With one arena
    slot left, the output allocation used to wrap the arena (zeroing every tag) after the input's tag
    pointer was taken, so the split-fp16 conv ran unscaled and overflowed fp16 at 1e5.  conv2d now
    reserves every tag it needs before reading any."""
    from models.common import Conv2d
    from nps_hip import ops
    torch.manual_seed(0)
    m = Conv2d(64, 64, 3)
    x = torch.randn(2, 64, 20, 24) * 1.5e5
    ref = _ref_conv(x, m.weight.detach(), m.bias.detach(), 1, 1, 0, "zeros")
    md = m.to(DEV)
    xd = ops.nchw_to_nhwc(x.to(DEV))
    ar = ops._arena(xd.device)
    xd._nps_tag = None                   # untagged input: the conv's input_tag allocates the last slot
    ar.next = ops._ARENA_TAGS - 1
    gen = ar.gen
    y = md.run([ops.Src(xd)], (20, 24))
    assert ar.gen == gen + 1             # the wrap happened, before the launch
    out = ops.nhwc_to_nchw(y).cpu()
    assert torch.isfinite(out).all()
    assert rel_l2(out, ref) < TOL


def test_tag_invalidated_by_torch_inplace_write():
    """a range tag is recorded with the tensor's version; a torch in-place write drops it, so
    the next split-fp16 conv re-measures the input (nps_absmax) instead of trusting a stale bound."""
    from models.common import Conv2d
    from nps_hip import ops
    torch.manual_seed(0)
    m = Conv2d(64, 64, 3).to(DEV)
    xd = ops.nchw_to_nhwc(torch.randn(2, 64, 20, 24).to(DEV))
    m.run([ops.Src(xd)], (20, 24))       # tags xd with max|x| ~ 4
    assert ops.tag_of(xd) is not None
    xd.mul_(1e5)                         # torch in-place: the bound is stale
    assert ops.tag_of(xd) is None
    y = m.run([ops.Src(xd)], (20, 24))
    ref = _ref_conv(ops.nhwc_to_nchw(xd).cpu(), m.weight.detach().cpu(), m.bias.detach().cpu(), 1, 1, 0, "zeros")
    assert rel_l2(ops.nhwc_to_nchw(y).cpu(), ref) < TOL


@pytest.mark.parametrize("stride,cin,cout,pad", [(1, 64, 64, 1), (2, 12, 40, 1)])
def test_tag_arena_wrap_inside_conv_backward_keeps_gradient_range(stride, cin, cout, pad):
    """the conv backward passes gy's range-tag pointer to the input-gradient conv(s) and to
    the weight gradient; a reserve between them used to wrap the arena (zeroing gy's tag), so the split-fp16
    dgrad / wgrad of a tiny gradient ran unscaled and flushed to zero.  The backward now reserves every tag it
    needs before taking the pointer.  The wrap point is swept over every position inside one backward."""
    from models.common import Conv2d
    from nps_hip import ops
    torch.manual_seed(3)
    m = Conv2d(cin, cout, 3, stride=stride, padding=pad)
    x = torch.randn(2, cin, 20, 22)
    xr = x.clone().double().requires_grad_(True)
    w = m.weight.detach().double().requires_grad_(True)
    ref = F.conv2d(xr, w, m.bias.detach().double(), stride=stride, padding=pad)
    g = torch.randn_like(ref) * 1e-8             # far below fp16's subnormals unless range-scaled
    ref.backward(g)
    md = m.to(DEV)
    for left in range(1, 14):
        xd = x.to(DEV).requires_grad_(True)
        md.weight.grad = None
        y = md(xd)
        ar = ops._arena(y.device)
        ar.next = ops._ARENA_TAGS - left
        y.backward(g.float().to(DEV))
        assert rel_l2(xd.grad, xr.grad) < TOL, left
        assert rel_l2(md.weight.grad, w.grad) < TOL, left
