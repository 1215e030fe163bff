"""GPU parity: the HIP path (through the C ABI) vs the pinned CPU oracle / reference goldens.

Tolerance: fp32 rel-L2 < 1e-5 (BASELINE.json north star; fp32 noise floor ~1e-7).
"""
import pytest
import torch
import torch.nn.functional as F
from torch import nn

import oracle
from oracle import functional as Fo
from conftest import load_golden, rel_l2

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda"


def _gelu():
    return nn.GELU()


# ------------------------------------------------------------------ conv unit tests
CONV_CASES = [
    # (Cin, Cout, k, stride, dil, padding, padding_mode, H, W)
    (16, 64, 3, 1, 1, 0, "zeros", 20, 20),          # valid 3x3
    (196, 192, 3, 1, 1, 0, "zeros", 33, 35),        # U-FNO shape, chunk tail (196 = 12*16 + 4)
    (7, 5, 3, 1, 1, 1, "zeros", 17, 13),            # zero pad, odd channels (scalar gather path)
    (12, 12, 3, 2, 1, 0, "zeros", 31, 29),          # downsample s2 valid
    (12, 40, 3, 2, 1, 1, "zeros", 16, 16),          # downsample s2 pad 1
    (32, 40, 3, 2, 1, 0, "zeros", 31, 29),          # downsample s2 valid, space-to-depth view (C % 16 == 0)
    (48, 192, 3, 2, 1, 1, "zeros", 27, 30),         # downsample s2 pad 1, view, wide tile
    (192, 192, 3, 2, 1, 0, "zeros", 65, 64),        # U-FNO Downsample shape, view
    (8, 8, 5, 1, 2, "same", "circular", 24, 24),    # DRN dilated circular
    (8, 8, 5, 1, 8, "same", "circular", 20, 20),    # dilation 8 > tile lattice
    (132, 128, 5, 1, 4, "same", "circular", 40, 36),
    (81, 192, 1, 1, 1, 0, "zeros", 19, 23),         # encoder 1x1, Cin % 4 != 0
    (192, 75, 1, 1, 1, 0, "zeros", 16, 16),         # pre-decoder 1x1, Cout % 32 != 0
    # 1x1 kernels: LDS-weight (Cout <= 192) and co-block waves (Cout > 192, 512-channel grid split)
    (196, 192, 1, 1, 1, 0, "zeros", 37, 29),        # LDS weights, 32-channel stage tail (196 = 6*32 + 4)
    (20, 192, 1, 1, 1, 1, "zeros", 13, 11),         # LDS weights, single partial stage, zero pad 1 (frame offset)
    (48, 388, 1, 1, 1, 0, "zeros", 15, 17),         # co-block waves, 7 waves
    (36, 600, 1, 1, 1, 0, "circular", 9, 10),       # co-block waves, two 512-channel groups
    (12, 16, 5, 1, 1, 2, "zeros", 19, 21),          # undilated 5x5, zero pad (split-fp16 25-tap kernel)
    (16, 24, 5, 1, 2, 4, "zeros", 23, 18),          # dilated 5x5 on the lattice, zero pad
    # packing boundaries (a latent over-read must be caught by a shape, not by allocation luck):
    # packed_ncb pads Cout to a multiple of 192 (6 x 32-channel blocks), the 1x1 co-block grid splits at 512
    (16, 193, 3, 1, 1, 1, "zeros", 18, 21),         # 3x3, 64-channel tiles, one channel past a 192 pack
    (36, 385, 3, 1, 1, 1, "circular", 12, 17),      # 3x3, 7 co tiles, packs of 2 x 192 + 1
    (40, 160, 3, 1, 1, 1, "zeros", 19, 22),         # 3x3 wide tile, Cout = 160: the last blocks are pack padding
    (20, 577, 1, 1, 1, 0, "zeros", 11, 13),         # 1x1 co-block waves, 512-channel group 2 of 65 channels
    (20, 193, 1, 1, 1, 0, "zeros", 14, 9),          # 1x1 co-block waves, one channel past the LDS-weight kernel
    (33, 192, 1, 1, 1, 0, "zeros", 16, 15),         # 1x1 LDS weights, Cin tail of 1 (frame-packed to 36)
    (388, 192, 3, 1, 1, 1, "zeros", 17, 19),        # 3x3 wide, 25 stages, Cin tail 4 (the odd tap-pair count)
    (388, 196, 3, 1, 1, 1, "zeros", 13, 12),        # 3x3, Cout 196: 64-channel tiles, last tile 4 channels
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_vs_torch(case):
    from models.common import Conv2d
    Cin, Cout, k, s, d, p, pm, H, W = case
    torch.manual_seed(0)
    m = Conv2d(Cin, Cout, k, stride=s, dilation=d, padding=p, padding_mode=pm)
    x = torch.randn(2, Cin, H, W)
    ref = Fo.conv2d_ref(x, {"weight": m.weight.detach(), "bias": m.bias.detach()}, "", stride=s, padding=p,
                        dilation=d, padding_mode=pm)
    y = m.to(DEV)(x.to(DEV)).cpu()
    assert y.shape == ref.shape
    assert rel_l2(y, ref) < TOL


@pytest.mark.parametrize("C,Cout,p,H,W", [(32, 40, 0, 31, 29), (192, 192, 0, 65, 64), (64, 192, 1, 20, 23)])
def test_downsample_s2d_view_equals_copy(C, Cout, p, H, W):
    """The Downsample's 2x2 conv reading the space-to-depth view of its input (nps_conv2d_t.s2d) gives the same
    values as the same conv over the materialised space_to_depth copy (same kernel, same operands)."""
    from models.common import Conv2d
    from nps_hip import ops
    torch.manual_seed(3)
    m = Conv2d(C, Cout, 3, stride=2, padding=p).to(DEV)
    x = ops.nchw_to_nhwc(torch.randn(2, C, H, W, device=DEV))
    old = ops.S2D_VIEW
    try:
        ops.S2D_VIEW = True
        y_view = m.run([ops.Src(x)], x.shape[1:3]).cpu()
        ops.S2D_VIEW = False
        y_copy = m.run([ops.Src(x)], x.shape[1:3]).cpu()
    finally:
        ops.S2D_VIEW = old
    assert rel_l2(y_view, y_copy) < 1e-7


@pytest.mark.parametrize("circ", [True, False])
def test_conv_transpose_vs_torch(circ):
    from models.common import ConvTranspose2d, ConvTranspose2d_padded
    torch.manual_seed(0)
    if circ:
        m = ConvTranspose2d_padded(1, 24, 20, kernel_size=4, stride=2)
    else:
        m = ConvTranspose2d(24, 20, kernel_size=4, stride=2, padding=1)
    x = torch.randn(2, 24, 13, 11)
    sd = {"weight": m.weight.detach(), "bias": m.bias.detach()}
    ref = Fo.conv_transpose_ref(x, sd, "", stride=2, padding=0 if circ else 1, circ_pre_pad=1 if circ else 0)
    y = m.to(DEV)(x.to(DEV)).cpu()
    assert y.shape == ref.shape
    assert rel_l2(y, ref) < TOL


def test_residual_block_concat_crop_groupnorm():
    """UpBlock-style input cat(h, crop(s), crop(vb)) with GN(1)+GELU prologues and crop-pad residual."""
    from models.enc_proc_dec_components.proc_unet_modern import ResidualBlock
    from nps_hip import ops
    torch.manual_seed(0)
    rb = ResidualBlock(20 + 16 + 4, 16, activation=_gelu(), norm=True, num_spatial_dims=2,
                       padding_kwargs=dict(padding_mode="circular"))
    with torch.no_grad():
        for n in (rb.norm1, rb.norm2):
            n.weight.uniform_(0.5, 1.5)
            n.bias.uniform_(-0.3, 0.3)
    h = torch.randn(2, 20, 30, 30)
    s = torch.randn(2, 16, 27, 27)   # crop_Nd pads 27 -> 30 (1 top, 2 bottom)
    v = torch.rand(2, 4, 33, 33)     # crop_Nd crops 33 -> 30
    x = torch.cat([h, Fo.crop_nd(s, h.shape), Fo.crop_nd(v, h.shape)], dim=1)
    ref = Fo.residual_block({k: t.detach() for k, t in rb.state_dict().items()}, "", x, True,
                            dict(padding_mode="circular"))
    rb = rb.to(DEV)
    hd, sd_, vd = (ops.nchw_to_nhwc(t.to(DEV)) for t in (h, s, v))
    srcs = [ops.Src(hd), ops.Src(sd_, ops.crop_offset(27, 30), ops.crop_offset(27, 30)),
            ops.Src(vd, ops.crop_offset(33, 30), ops.crop_offset(33, 30))]
    y = ops.nhwc_to_nchw(rb.run(srcs, (30, 30))).cpu()
    assert rel_l2(y, ref) < TOL


@pytest.mark.parametrize("pm", ["circular", "zeros"])
def test_residual_block_fused_prologue(monkeypatch, pm):
    """The split-fp16 3x3 conv applying GroupNorm + GELU itself (NPS_FUSE_PROLOGUE=1): 16-channel aligned
    concat with a padded crop (frame pixels no source covers get act(GN(0)), as frame_pack gives them)."""
    from models.enc_proc_dec_components.proc_unet_modern import ResidualBlock
    from nps_hip import ops
    if ops.CONV_PRECISION != ops.PREC_X3F16:
        pytest.skip("fused prologue is a split-fp16 kernel feature")
    monkeypatch.setattr(ops, "FUSE_PROLOGUE", True)
    packs = []
    real_pack = ops.frame_pack
    monkeypatch.setattr(ops, "frame_pack", lambda *a, **k: packs.append(k.get("gn")) or real_pack(*a, **k))
    torch.manual_seed(1)
    rb = ResidualBlock(32 + 16 + 4, 32, activation=_gelu(), norm=True, num_spatial_dims=2,
                       padding_kwargs=dict(padding_mode=pm))
    with torch.no_grad():
        for n in (rb.norm1, rb.norm2):
            n.weight.uniform_(0.5, 1.5)
            n.bias.uniform_(-0.3, 0.3)
    h = torch.randn(2, 32, 40, 36)
    s = torch.randn(2, 16, 37, 33)   # crop_Nd pads 37x33 -> 40x36: uncovered frame rows / columns
    v = torch.rand(2, 4, 40, 36)
    x = torch.cat([h, Fo.crop_nd(s, h.shape), v], dim=1)
    ref = Fo.residual_block({k: t.detach() for k, t in rb.state_dict().items()}, "", x, True, dict(padding_mode=pm))
    rb = rb.to(DEV)
    hd, sd_, vd = (ops.nchw_to_nhwc(t.to(DEV)) for t in (h, s, v))
    srcs = [ops.Src(hd), ops.Src(sd_, ops.crop_offset(37, 40), ops.crop_offset(33, 36)), ops.Src(vd)]
    y = ops.nhwc_to_nchw(rb.run(srcs, (40, 36))).cpu()
    assert not any(g is not None for g in packs), "GroupNorm prologue went through frame_pack"
    assert rel_l2(y, ref) < TOL


@pytest.mark.parametrize("cout", [192, 64])     # 192: wide tiles, 64: 512-pixel tiles (PB=4 kernels)
@pytest.mark.parametrize("nchw", [False, True])  # LDS-staged vs register-store epilogue
def test_split_fp16_persistent_tiles(cout, nchw):
    """Every work-group walks many tiles (persistent grid of 8 work-groups, nps_x3_set_grid) for both
    epilogue layouts — the register-store one walks tiles too since the producer fetches became
    compiler-visible loads (round 1 kept it on one tile per work-group): bias + GELU epilogue vs fp64."""
    from nps_hip import lib, ops
    import torch.nn.functional as F
    torch.manual_seed(2)
    B, Cin, H, W = 2, 48, 66, 70
    x = torch.randn(B, Cin, H, W)
    w = torch.randn(cout, Cin, 3, 3) * 0.05
    b = torch.randn(cout) * 0.1
    ref = F.gelu(F.conv2d(x.double(), w.double(), b.double()))
    lib.nps_x3_set_grid(8)
    try:
        y = ops.conv2d([ops.Src(ops.nchw_to_nhwc(x.to(DEV)))], (H, W), ops.pack_conv_weight(w.to(DEV)), b.to(DEV),
                       cout, 3, 3, act=ops.GELU, out_nchw=nchw)
        torch.cuda.synchronize()
    finally:
        lib.nps_x3_set_grid(0)
    y = y.cpu() if nchw else ops.nhwc_to_nchw(y).cpu()
    assert rel_l2(y, ref) < TOL


def _moments(t):
    """fp64 (sum, sum of squares) per sample.  The carried moments match to ~1e-8 relative: the epilogues
    sum in fp64, nps_group_norm_stats (the seed of an identity shortcut's) sums fp32 quads first."""
    x = t.detach().cpu().double().reshape(t.shape[0], -1)
    return torch.stack([x.sum(1), (x * x).sum(1)], 1)


@pytest.mark.parametrize("C", [192, 32])  # 192: wide 192-channel tiles, 32: 64-channel tiles
def test_groupnorm_moments_carried_by_conv_epilogues(C):
    """GroupNorm(1) moments (proc_unet_modern.py:235-236) produced by the epilogues of the convs that write
    a tensor (ResidualBlock conv2 accumulating onto its shortcut, the 4 transposed-conv phases, the
    space-to-depth Downsample conv) equal the fp64 sums of the stored tensor, and the next block's
    GroupNorm reads them without a statistics pass over its frame."""
    from models.common import ConvTranspose2d_padded
    from models.enc_proc_dec_components.proc_unet_modern import Downsample, ResidualBlock
    from nps_hip import ops
    if ops.CONV_PRECISION != ops.PREC_X3F16:
        pytest.skip("moments come from the split-fp16 epilogues")
    torch.manual_seed(4)
    pk = dict(padding_mode="circular")
    rb1 = ResidualBlock(C, C, activation=_gelu(), norm=True, num_spatial_dims=2, padding_kwargs=pk).to(DEV)
    rb2 = ResidualBlock(C + 4, C, activation=_gelu(), norm=True, num_spatial_dims=2, padding_kwargs=pk).to(DEV)
    up = ConvTranspose2d_padded(1, C, C, kernel_size=4, stride=2).to(DEV)
    down = Downsample(C, 2, 0, pk).to(DEV)
    x = ops.nchw_to_nhwc(torch.randn(2, C, 18, 20, device=DEV))
    h = rb1.run([ops.Src(x)], (18, 20))
    assert torch.allclose(ops.stats_of(h).sum(1).cpu(), _moments(h), rtol=1e-7, atol=1e-4)
    u = up.run(h)                                         # (2 * (18 + 2) + 2) x (2 * (20 + 2) + 2)
    assert tuple(u.shape[1:3]) == (42, 46)
    assert torch.allclose(ops.stats_of(u).sum(1).cpu(), _moments(u), rtol=1e-7, atol=1e-4)
    v = ops.nchw_to_nhwc(torch.rand(2, 4, 42, 46, device=DEV))
    passes = []
    real = ops.lib.nps_group_norm_stats
    try:
        ops.lib.nps_group_norm_stats = lambda *a: passes.append(a[1]) or real(*a)
        y = rb2.run([ops.Src(u), ops.Src(v)], (42, 46))   # norm1 over cat(u, v): u's moments + one pass over v
    finally:
        ops.lib.nps_group_norm_stats = real
    assert passes == [1], passes                          # only v (untagged) was read for statistics
    d = down.run(y, None)[0]
    assert torch.allclose(ops.stats_of(d).sum(1).cpu(), _moments(d), rtol=1e-7, atol=1e-4)
    # the block output against the oracle on the same inputs
    ref = Fo.residual_block({k: t.detach().cpu() for k, t in rb2.state_dict().items()}, "",
                            torch.cat([ops.nhwc_to_nchw(u).cpu(), ops.nhwc_to_nchw(v).cpu()], 1), True, pk)
    assert rel_l2(ops.nhwc_to_nchw(y).cpu(), ref) < TOL


# ------------------------------------------------------------------ spectral
@pytest.mark.parametrize("name", ["spectral2d_a", "spectral2d_overlap", "spectral2d_nyq"])
def test_spectral2d_golden(name):
    from models.enc_proc_dec_components.proc_fno import SpectralConv2d
    g = load_golden(name)
    kw = g["kwargs"]
    m = SpectralConv2d(kw["in_channels"], kw["out_channels"], tuple(kw["modes"]))
    m.load_state_dict(g["state_dict"])
    y = m.to(DEV)(g["x"].to(DEV)).cpu()
    assert rel_l2(y, g["y"]) < TOL


@pytest.mark.parametrize("H,W,m", [(128, 128, 12), (256, 256, 10), (96, 64, 10)])
def test_spectral2d_full_size(H, W, m):
    """U-FNO spectral conv at the BASELINE sizes (196 -> 192 channels) vs the torch.fft oracle."""
    from models.enc_proc_dec_components.proc_fno import SpectralConv2d
    torch.manual_seed(1)
    sc = SpectralConv2d(196, 192, (m, m))
    x = torch.randn(2, 196, H, W)
    ref = Fo.spectral_conv2d(x, sc.weights1.detach(), sc.weights2.detach())
    y = sc.to(DEV)(x.to(DEV)).cpu()
    assert rel_l2(y, ref) < TOL


def test_fno_layer_golden():
    from models.enc_proc_dec_components.proc_fno import FNO_Layer
    g = load_golden("fno_layer")
    m = FNO_Layer(**g["kwargs"])
    m.load_state_dict(g["state_dict"])
    y = m.to(DEV)(g["x"].to(DEV)).cpu()
    assert rel_l2(y, g["y"]) < TOL


@pytest.mark.parametrize("H,W,m,cin,cout", [(256, 256, 10, 196, 192), (128, 128, 12, 196, 192), (64, 128, 5, 36, 44)])
def test_fno_layer_fused_synthesis(H, W, m, cin, cout, monkeypatch):
    """FNO_Layer (proc_fno.py:142-146: act(conv(x) + w(x))) with the spectral conv's W-pass synthesis done by the
    1x1 `w`'s epilogue (nps_conv2d_t.spec_z, no idft_w launch) against the unfused HIP path (1x1, then idft_w
    accumulating) and against torch (the oracle's spectral conv + a 1x1 conv + GELU)."""
    from models.enc_proc_dec_components.proc_fno import FNO_Layer
    from nps_hip import ops
    if not ops.spectral_fusable(W, m, cout):
        pytest.skip("fused synthesis off (split-fp16 1x1 on the LDS-weight kernel only)")
    torch.manual_seed(3)
    layer = FNO_Layer(cin, num_spatial_dims=2, modes=m, hidden_dim_out=cout).to(DEV)
    x = torch.randn(2, cin, H, W)
    calls = []
    real = ops.lib.nps_spectral_idft_w
    monkeypatch.setattr(ops.lib, "nps_spectral_idft_w", lambda *a: calls.append(1) or real(*a))
    with torch.no_grad():  # (the inference path: the differentiable one runs the unfused kernels)
        y = layer(x.to(DEV)).cpu()
        assert calls == []  # synthesised in the 1x1 epilogue
        monkeypatch.setattr(ops, "FUSE_IDFT", False)
        y_ref = layer(x.to(DEV)).cpu()
    assert calls == [1]
    assert rel_l2(y, y_ref) < 1e-6
    sc = layer.conv
    ref = F.gelu(Fo.spectral_conv2d(x, sc.weights1.detach().cpu(), sc.weights2.detach().cpu()) +
                 F.conv2d(x, layer.w.weight.detach().cpu(), layer.w.bias.detach().cpu()))
    assert rel_l2(y, ref) < TOL


# ------------------------------------------------------------------ processors
def _proc(name):
    from models.enc_proc_dec_components import UNetModern, DilatedResnet, UFNO, FNO
    cls = {"unet_ufno_style": UNetModern, "unet_cfg": UNetModern, "unet_ones": UNetModern, "drn": DilatedResnet,
           "ufno": UFNO, "fno": FNO}[name]
    g = load_golden(name)
    kw = dict(g["kwargs"])
    if cls is not FNO:
        kw["activation"] = _gelu()
    m = cls(pde=None, **kw)
    m.load_state_dict(g["state_dict"])
    return m.to(DEV), g


@pytest.mark.parametrize("name", ["unet_ufno_style", "unet_cfg", "unet_ones", "drn", "ufno", "fno"])
def test_processor_golden(name):
    m, g = _proc(name)
    with torch.no_grad():
        y = m(h=g["h"].to(DEV), variables_broadcast=g["vb"].to(DEV)).cpu()
    assert y.shape == g["y"].shape
    assert rel_l2(y, g["y"]) < TOL


@pytest.mark.parametrize("min_idle", [0.0, 0.25])
def test_side_stream_forks_match_serial(monkeypatch, min_idle):
    """ops.Fork (the U-FNO block's FNO layer and the ResidualBlock shortcuts on side streams): the U-FNO
    processor golden, forks on (every shortcut forked at min_idle 0) vs all launches on one stream — the same
    kernels on the same inputs, so equal up to the order of the moments' float atomics (rel-L2 < 1e-6)."""
    from nps_hip import ops
    m, g = _proc("ufno")
    h, vb = g["h"].to(DEV), g["vb"].to(DEV)
    monkeypatch.setattr(ops, "SIDE_STREAM", False)
    with torch.no_grad():
        y0 = m(h=h, variables_broadcast=vb)
    monkeypatch.setattr(ops, "SIDE_STREAM", True)
    monkeypatch.setattr(ops, "SIDE_MIN_IDLE", min_idle)
    with torch.no_grad():
        y1 = m(h=h, variables_broadcast=vb)
        y2 = m(h=h, variables_broadcast=vb)
    torch.cuda.synchronize()
    assert rel_l2(y1, y0) < 1e-6 and rel_l2(y2, y0) < 1e-6
    assert rel_l2(y1.cpu(), g["y"]) < TOL


# ------------------------------------------------------------------ full models + rollout
def _build_model(g):
    import models
    from pdes import PDE2D
    cfg = dict(g["cfg"])
    cfg.pop("object")
    cfg["activation"] = _gelu()
    cfg["activation_final"] = nn.Tanh()
    p = g["pde"]
    pde = PDE2D(tmin=p["tmin"], tmax=p["tmax"], nt=p["nt"], L1=1.0, L2=1.0, nx1=p["nx1"], nx2=p["nx2"], x=None,
                name="twophase", n_cond_static=p["n_cond_static"], n_cond_spatial=p["n_cond_spatial"])
    m = models.activation_wrapper(**cfg, pde=pde)
    m.load_state_dict(g["state_dict"])
    return m.to(DEV).eval(), pde


@pytest.mark.parametrize("name", ["model_ufno", "model_unet", "model_drn", "model_ufno_fno"])
def test_model_and_simulate_golden(name):
    import argparse
    import types
    from common.interfaces import D
    from trainers.autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer
    g = load_golden(name)
    m, pde = _build_model(g)
    tw = g["cfg"]["time_window"]
    u, cond, pos, sc = (g[k].to(DEV) for k in ("u", "cond", "pos", "spatial_cond"))
    with torch.no_grad():
        y = m(u[:, :, :tw], cond=cond, bc=None, pos=pos, t_cond=None, spatial_cond=sc).cpu()
    assert rel_l2(y, g["y"]) < TOL
    T = u.shape[2]
    cfg = argparse.Namespace(time_window=tw, base_resolution=(T, u.shape[3], u.shape[4]), device=DEV, nr_gt_steps=1)
    tr = AutoregressivePushforwardTrainer(model=m, data=types.SimpleNamespace(pde=pde, data_interface=D.sim2d),
                                          criterion=nn.MSELoss(reduction="sum"), config=cfg)
    with torch.no_grad():
        losses, (gt, preds) = tr.simulate(u, cond, pos, compute_loss=True, include_data=True, nr_gt_steps=1, t_res=T,
                                          spatial_conditioning=sc)
    pred = torch.cat(preds[1:], dim=2).cpu()
    assert rel_l2(pred, g["sim_pred"]) < TOL
    assert rel_l2(torch.stack([l.cpu() for l in losses]), g["sim_losses"]) < TOL


def test_ufno_c3_full_size_one_call():
    """North-star config C3: U-FNO twophase cfg (hidden 192, 3 blocks, modes 10) at 256x256, 3 fields,
    obstacle, B=1 — one rollout model call vs the CPU oracle."""
    import __graft_entry__  # noqa: F401
    from bench import build_model, ORACLE_PDE
    from trainers.synthetic import twophase_batch
    m, ocfg, opde = build_model("ufno", res=256, num_c=3, device=DEV)
    u, cond, pos, sc = twophase_batch(1, 3, 25, 256, 256, seed=7, obstacle="disc")
    with torch.no_grad():
        y = m(u.to(DEV), cond=cond.to(DEV), bc=None, pos=pos.to(DEV), t_cond=None, spatial_cond=sc.to(DEV)).cpu()
    ref = oracle.build_oracle_model(ocfg, opde, {k: v.cpu() for k, v in m.state_dict().items()})(
        u, cond=cond, pos=pos, spatial_cond=sc)
    assert rel_l2(y, ref) < TOL


def test_c1_unet_cfg_simulate_golden():
    """BASELINE C1: the exact cfg_twophase_unet model (hidden 32, ch_mults [2,2,1,2]), 64x64, no obstacle,
    B=2, t_res=150 — the 5-call rollout through the mirror's simulate on the GPU against the reference's
    own simulate (tests/golden/make_golden_c1.py), every window and every loss."""
    import argparse
    import types
    from common.interfaces import D
    from trainers.autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer
    from c1_fixture import c1_golden, c1_inputs, c1_model
    g = c1_golden()
    u, cond, pos, sc = (t.to(DEV) for t in c1_inputs(g))
    m, pde = c1_model(g)
    m = m.to(DEV)
    tw, T = g["cfg"]["time_window"], u.shape[2]
    cfg = argparse.Namespace(time_window=tw, base_resolution=(T, u.shape[3], u.shape[4]), device=DEV, nr_gt_steps=1)
    tr = AutoregressivePushforwardTrainer(model=m, data=types.SimpleNamespace(pde=pde, data_interface=D.sim2d),
                                          criterion=nn.MSELoss(reduction="sum"), config=cfg)
    with torch.no_grad():
        losses, (gt, preds) = tr.simulate(u, cond, pos, compute_loss=True, include_data=True, nr_gt_steps=1, t_res=T,
                                          spatial_conditioning=sc)
    assert len(preds) == 6
    for k in range(5):  # every window of the rollout (errors would compound through the feedback)
        assert rel_l2(preds[k + 1].cpu(), g["sim_pred"][:, :, k * tw:(k + 1) * tw]) < TOL, k
    assert rel_l2(torch.stack([l.cpu() for l in losses]), g["sim_losses"]) < TOL


@pytest.mark.parametrize("name", ["ufno", "unet", "drn"])
def test_native_geometry_simulate_golden(name):
    """The geometry an unchanged train.py feeds the drop-in: every twophase cfg sets base_resolution
    (501, 96, 64) (reference cfg_twophase_ufno.py:6-7).  The full-width cfg model (U-FNO hidden 192 / U-Net
    hidden 32 ch_mults [2,2,1,2] / DRN hidden 128), num_c = 1, B = 2, through the mirror's simulate on the GPU at
    t_res = 110 — 3 calls, the partial last window skipped as at autoregressivepushforwardtrainer.py:354-358 —
    against the reference's own simulate (tests/golden/make_golden_native.py), every window and every loss."""
    import argparse
    import types
    from common.interfaces import D
    from trainers.autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer
    from native_fixture import native_golden, native_inputs, native_model
    g = native_golden(name)
    u, cond, pos, sc = (t.to(DEV) for t in native_inputs(g))
    m, pde = native_model(g)
    m = m.to(DEV)
    tw, T = g["cfg"]["time_window"], u.shape[2]
    cfg = argparse.Namespace(time_window=tw, base_resolution=(T, u.shape[3], u.shape[4]), device=DEV, nr_gt_steps=1)
    tr = AutoregressivePushforwardTrainer(model=m, data=types.SimpleNamespace(pde=pde, data_interface=D.sim2d),
                                          criterion=nn.MSELoss(reduction="sum"), config=cfg)
    with torch.no_grad():
        losses, (gt, preds) = tr.simulate(u, cond, pos, compute_loss=True, include_data=True, nr_gt_steps=1, t_res=T,
                                          spatial_conditioning=sc)
    assert len(preds) == 4
    for k in range(3):
        assert rel_l2(preds[k + 1].cpu(), g["sim_pred"][:, :, k * tw:(k + 1) * tw]) < TOL, k
    assert rel_l2(torch.stack([l.cpu() for l in losses]), g["sim_losses"]) < TOL


def test_drn_c4_full_size_one_call():
    """BASELINE C4: the cfg_twophase_drn model (DilatedResnet hidden 128, k 5, 2 blocks, dilations
    1,2,4,8,4,2,1, circular; decoder kernel 5) at 256x256, 1 field, B=1 — one rollout model call vs the CPU
    oracle (cf. test_ufno_c3_full_size_one_call)."""
    import __graft_entry__  # noqa: F401
    from bench import build_model
    from trainers.synthetic import twophase_batch
    m, ocfg, opde = build_model("drn", res=256, num_c=1, device=DEV)
    u, cond, pos, sc = twophase_batch(1, 1, 25, 256, 256, seed=13, obstacle="disc")
    with torch.no_grad():
        y = m(u.to(DEV), cond=cond.to(DEV), bc=None, pos=pos.to(DEV), t_cond=None, spatial_cond=sc.to(DEV)).cpu()
    ref = oracle.build_oracle_model(ocfg, opde, {k: v.cpu() for k, v in m.state_dict().items()})(
        u, cond=cond, pos=pos, spatial_cond=sc)
    assert rel_l2(y, ref) < TOL


def test_ufno_c2_full_size_one_call():
    """BASELINE C2: U-FNO twophase cfg with 12 Fourier modes (hidden 192, 3 blocks) at 128x128, 1 field,
    B=2 — one rollout model call vs the CPU oracle (cf. test_ufno_c3_full_size_one_call)."""
    import __graft_entry__  # noqa: F401
    from bench import build_model
    from trainers.synthetic import twophase_batch
    m, ocfg, opde = build_model("ufno", res=128, num_c=1, device=DEV, fno_modes=12)
    u, cond, pos, sc = twophase_batch(2, 1, 25, 128, 128, seed=11, obstacle="random")
    with torch.no_grad():
        y = m(u.to(DEV), cond=cond.to(DEV), bc=None, pos=pos.to(DEV), t_cond=None, spatial_cond=sc.to(DEV)).cpu()
    ref = oracle.build_oracle_model(ocfg, opde, {k: v.cpu() for k, v in m.state_dict().items()})(
        u, cond=cond, pos=pos, spatial_cond=sc)
    assert rel_l2(y, ref) < TOL


@pytest.mark.parametrize("cin,cout,hw", [(192, 225, (37, 29)), (36, 200, (16, 21)), (84, 256, (9, 40))])
def test_conv1x1_planar_output_vs_torch(cin, cout, hw):
    """The decoder's pre-output 1x1 (dec_grid.py:126-130) writes NCHW planes with 192 < Cout <= 256: the
    resident-weight kernel (conv1x1_res.hip, two channel groups of 128) with planar stores."""
    from models.common import Conv2d
    from nps_hip import ops
    torch.manual_seed(5)
    m = Conv2d(cin, cout, 1)
    x = torch.randn(2, cin, *hw)
    ref = Fo.conv2d_ref(x, {"weight": m.weight.detach(), "bias": m.bias.detach()}, "", stride=1, padding=0,
                        dilation=1, padding_mode="zeros")
    md = m.to(DEV)
    y = md.run([ops.Src(ops.nchw_to_nhwc(x.to(DEV)))], hw, out_nchw=True)
    assert tuple(y.shape) == (2, cout) + hw
    assert rel_l2(y.cpu(), ref) < TOL


@pytest.mark.parametrize("cin,cout,groups,pad,xscale", [(192, 192, 8, 0, 1.0), (196, 75, 1, 1, 3e3), (36, 192, 3, 0, 1e-3)])
def test_conv1x1_fused_groupnorm_gelu_prologue(cin, cout, groups, pad, xscale):
    """The U-Net's final GN(8) + GELU + 1x1 (proc_unet_modern.py:191-196) as ONE launch: the LDS-weight 1x1
    kernel applies the GroupNorm affine and GELU to each loaded element (no frame_pack materialisation); frame
    pixels get act(GN(x)), the conv's zero padding stays 0."""
    from nps_hip import ops
    torch.manual_seed(11)
    B, H, W = 2, 21, 18
    x = torch.randn(B, cin, H, W) * xscale + 0.2 * xscale
    gamma = torch.rand(cin) + 0.5
    beta = torch.rand(cin) - 0.5
    w = torch.randn(cout, cin, 1, 1) * 0.05
    b = torch.randn(cout) * 0.1
    ref = F.conv2d(F.gelu(F.group_norm(x.double(), groups, gamma.double(), beta.double(), 1e-5)), w.double(),
                   b.double(), padding=pad)
    packs = []
    real_pack = ops.frame_pack
    try:
        ops.frame_pack = lambda *a, **k: packs.append(1) or real_pack(*a, **k)
        xd = ops.nchw_to_nhwc(x.to(DEV))
        st = ops.group_norm_stats([ops.Src(xd)], (H, W), groups)
        gn = ops.GN(st, gamma.to(DEV), beta.to(DEV), groups, 1e-5)
        ost = ops.new_stats(B, xd)  # the U-Net's final conv also carries its output's GroupNorm(1) moments
        y = ops.conv2d([ops.Src(xd)], (H, W), ops.pack_conv_weight(w.to(DEV)), b.to(DEV), cout, 1, 1, pad=(pad, pad),
                       gn=gn, pre_act=1, out_stats=ost)
    finally:
        ops.frame_pack = real_pack
    assert not packs, "GroupNorm prologue of the 1x1 went through frame_pack"
    assert rel_l2(ops.nhwc_to_nchw(y).cpu(), ref) < TOL
    if cout % 4:  # (moments need an NHWC output with 4-aligned channels: the buffer is marked incomplete)
        assert getattr(ost, "_nps_incomplete", False)
        return
    assert not getattr(ost, "_nps_incomplete", False)
    got = ost.sum(1).cpu()
    want = torch.stack([ref.sum((1, 2, 3)), (ref * ref).sum((1, 2, 3))], 1)
    assert rel_l2(got, want) < TOL
