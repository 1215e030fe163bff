"""GPU parity of the backward (training) path: HIP gradients vs autograd through the CPU oracle and the
reference's own golden gradients.

Every gradient here is produced by libnps_hip.so kernels (nps_hip.autograd): conv input gradients as
forward convs of dy, weight gradients on the MFMA wgrad kernel, GroupNorm/GELU frame backward,
spectral-conv backward, TimeConvDense / volume-rescale backward.  Tolerance: fp32 rel-L2 < 1e-5 per
gradient tensor (BASELINE.json north star), measured 1e-7 ... 1e-6.
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


def _grads_ok(named_ref, named_got, tol=TOL, tensor_tol=1e-4):
    """All parameter gradients as one vector: rel-L2 < tol (1e-5).  Per tensor: rel-L2 < tensor_tol, or an
    error below tol x the norm of the whole gradient — bias / GroupNorm-affine gradients are sums over every
    pixel that largely cancel (fp32 noise of such a sum is ~eps x the cancellation factor, on the CPU
    reference as much as here), and a bias feeding a per-channel GroupNorm (e.g. the last UpBlock's
    shortcut bias before GroupNorm(8, 8)) has an analytically zero gradient that both sides only resolve
    to rounding noise."""
    keys = list(named_ref)
    for k in keys:
        assert named_got[k] is not None, f"no gradient for {k}"
    ref = torch.cat([torch.view_as_real(named_ref[k]).reshape(-1) if named_ref[k].is_complex()
                     else named_ref[k].reshape(-1) for k in keys]).double()
    got = torch.cat([(torch.view_as_real(named_got[k]) if named_got[k].is_complex() else named_got[k])
                     .reshape(-1).cpu() for k in keys]).double()
    e_all = (torch.linalg.vector_norm(got - ref) / torch.linalg.vector_norm(ref)).item()
    total = torch.linalg.vector_norm(ref).item()
    bad = []
    for k in keys:
        r = named_ref[k].detach().cpu()
        g = named_got[k].detach().cpu()
        if r.is_complex():
            r, g = torch.view_as_real(r), torch.view_as_real(g)
        r, g = r.double(), g.double()
        d = torch.linalg.vector_norm(g - r).item()
        e = d / max(torch.linalg.vector_norm(r).item(), 1e-30)
        if not (e < tensor_tol or d < tol * total):
            bad.append((k, e, d / total))
    assert e_all < tol and not bad, (e_all, bad)


# ------------------------------------------------------------------ conv
CONV_CASES = [
    # (Cin, Cout, k, stride, dil, padding, padding_mode, H, W)
    (16, 64, 3, 1, 1, 0, "zeros", 20, 20),          # valid 3x3 (U-Net)
    (196, 192, 3, 1, 1, 0, "zeros", 33, 35),        # U-FNO shape, chunk tails
    (7, 5, 3, 1, 1, 1, "zeros", 17, 13),            # 'ones' zero pad, odd channels
    (12, 12, 3, 2, 1, 0, "zeros", 31, 29),          # Downsample s2 valid, odd size
    (12, 40, 3, 2, 1, 1, "zeros", 16, 16),          # Downsample s2 pad 1
    (2, 2, 3, 2, 1, 0, "zeros", 21, 22),            # vb Downsample, C % 4 != 0
    (8, 8, 5, 1, 2, "same", "circular", 24, 24),    # DRN dilated circular
    (8, 8, 5, 1, 8, "same", "circular", 20, 20),
    (132, 128, 5, 1, 4, "same", "circular", 40, 36),
    (81, 192, 1, 1, 1, 0, "zeros", 19, 23),         # encoder 1x1, Cin % 4 != 0
    (192, 75, 1, 1, 1, 0, "zeros", 16, 16),         # pre-decoder 1x1
    # packing boundaries: dgrad Cin / wgrad M one past a 192 pack, 4-channel tails
    (36, 193, 3, 1, 1, 1, "zeros", 14, 15),         # wgrad M = 193 (pad-4 path), dgrad 193 -> 36
    (196, 388, 1, 1, 1, 0, "zeros", 12, 13),        # 1x1: wgrad 388 x 196, dgrad 388 -> 196
    (388, 192, 3, 1, 1, 1, "zeros", 11, 12),        # the U-Net up-block 3x3: dgrad 192 -> 388 (Cout tail 4)
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_backward_vs_torch(case):
    from models.common import Conv2d
    Cin, Cout, k, s, d, p, pm, H, W = case
    torch.manual_seed(0)
    m = Conv2d(Cin, Cout, k, stride=s, dilation=d, padding=p, padding_mode=pm)
    x = torch.randn(2, Cin, H, W)
    w = m.weight.detach().clone().requires_grad_(True)
    b = m.bias.detach().clone().requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    ref = Fo.conv2d_ref(xr, {"weight": w, "bias": b}, "", stride=s, padding=p, dilation=d, padding_mode=pm)
    g = torch.randn_like(ref)
    ref.backward(g)
    m = m.to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    y = m(xd)
    assert y.shape == ref.shape
    y.backward(g.to(DEV))
    assert rel_l2(y, ref) < TOL
    assert rel_l2(xd.grad, xr.grad) < TOL
    assert rel_l2(m.weight.grad, w.grad) < TOL
    assert rel_l2(m.bias.grad, b.grad) < TOL


WGRAD_X3_CASES = [
    # (B, M, N, k, pad, circ, Ha, Wa, a_scale, x_scale)
    (2, 192, 196, 3, 1, 0, 33, 35, 1.0, 1.0),       # U-FNO shape: channel tails, ragged pixel tiles
    (2, 64, 64, 3, 0, 1, 40, 36, 1.0, 1.0),         # circular 'same' (frame extended by 1)
    (1, 20, 96, 2, 0, 0, 17, 19, 1.0, 1.0),         # space-to-depth / phase form
    (2, 76, 84, 1, 0, 0, 19, 23, 1.0, 1.0),         # 1x1, channel tails (not multiples of 64)
    (2, 64, 48, 3, 1, 0, 64, 64, 1e-4, 1e3),        # range: tiny gradients x large activations
    (2, 32, 40, 3, 1, 0, 24, 24, 1.5e5, 1e-3),      # range: gradients past fp16's max
    (3, 128, 128, 3, 0, 1, 96, 96, 1.0, 1.0),       # many pixel tiles per split
    (2, 192, 81, 1, 0, 0, 32, 32, 1.0, 1.0),        # the encoder's 81-channel 1x1: zero-padded to 84
    (2, 30, 22, 3, 1, 0, 20, 20, 1.0, 1.0),         # both channel counts off the 4-channel quads
    # 1x1 on the 192 x 192 work-group kernel (wgrad1_wide_kernel): M, N past one 192-row tile, ragged last
    # 32-pixel tile, many tiles per split, range cases
    (2, 388, 196, 1, 0, 0, 37, 29, 1.0, 1.0),
    (4, 192, 192, 1, 0, 0, 64, 64, 1.0, 1.0),
    (1, 196, 388, 1, 0, 0, 13, 11, 1e-4, 1e3),
    (2, 84, 192, 1, 0, 0, 40, 40, 1.5e5, 1e-3),
    # 2x2 on the 128 x 128 work-group kernel (wgrad2_wide_kernel): the space-to-depth Downsample / transposed-conv
    # phase shape (M = 192, N = 4 x 192), padding, circular extension, tails past one 128-row tile, range
    (2, 192, 768, 2, 0, 0, 33, 31, 1.0, 1.0),
    (1, 100, 136, 2, 1, 0, 19, 21, 1e-4, 1e3),
    (2, 132, 80, 2, 0, 1, 20, 24, 1.0, 1.0),
    # N tails of <= 8 channels past the 64-channel tiles on wgrad_tail_kernel (the 388 / 196-channel U-Net frames):
    # padding, circular extension, 2x2 with an 8-channel tail, range
    (2, 192, 388, 3, 1, 0, 29, 31, 1.0, 1.0),
    (2, 64, 68, 3, 0, 1, 22, 26, 1e-4, 1e3),
    (1, 48, 136, 2, 1, 0, 18, 21, 1.0, 1.0),
    (2, 40, 72, 3, 1, 0, 16, 19, 1.5e5, 1e-3),
]


@pytest.mark.parametrize("case", WGRAD_X3_CASES)
def test_wgrad_x3_vs_fp64(case):
    """nps_conv2d_wgrad_x3 (split-fp16 MFMA) against the fp64 weight gradient of the same geometry:
    G[m][n][ky][kx] = sum_{b,p} a[b][p][m] Xext[b][p + (ky, kx) - pad][n], Xext circularly extended by circ
    and zero outside; range-scaled operands must keep the fp32 bar at any magnitude."""
    from nps_hip import autograd as ad
    from nps_hip import ops
    B, M, N, k, pad, circ, Ha, Wa, sa, sx = case
    Hx, Wx = Ha + k - 1 - 2 * pad - 2 * circ, Wa + k - 1 - 2 * pad - 2 * circ
    torch.manual_seed(1)
    a = torch.randn(B, M, Ha, Wa, dtype=torch.float64) * sa
    x = torch.randn(B, N, Hx, Wx, dtype=torch.float64) * sx
    xe = F.pad(x, (circ,) * 4, mode="circular") if circ else x
    xe = F.pad(xe, (pad,) * 4)
    ref = torch.nn.grad.conv2d_weight(xe, (M, N, k, k), a)
    assert ops.CONV_PRECISION == ops.PREC_X3F16
    ad_a = a.float().permute(0, 2, 3, 1).contiguous().to(DEV)
    ad_x = x.float().permute(0, 2, 3, 1).contiguous().to(DEV)
    got = ad.wgrad(ad_a, ad_x, k, k, pad=(pad, pad), circ=circ)
    got32 = torch.nn.grad.conv2d_weight(xe.float(), (M, N, k, k), a.float())  # fp32 CPU: the reference class
    assert rel_l2(got, ref) < TOL, (rel_l2(got, ref), rel_l2(got32, ref))


@pytest.mark.parametrize("circ", [True, False])
def test_conv_transpose_backward_vs_torch(circ):
    from models.common import ConvTranspose2d, ConvTranspose2d_padded
    torch.manual_seed(0)
    m = ConvTranspose2d_padded(1, 24, 20, kernel_size=4, stride=2) if circ else \
        ConvTranspose2d(24, 20, kernel_size=4, stride=2, padding=1)
    x = torch.randn(2, 24, 13, 11)
    sd = {"weight": m.weight.detach().clone().requires_grad_(True),
          "bias": m.bias.detach().clone().requires_grad_(True)}
    xr = x.clone().requires_grad_(True)
    ref = Fo.conv_transpose_ref(xr, sd, "", stride=2, padding=0 if circ else 1, circ_pre_pad=1 if circ else 0)
    g = torch.randn_like(ref)
    ref.backward(g)
    m = m.to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    y = m(xd)
    y.backward(g.to(DEV))
    assert rel_l2(y, ref) < TOL
    assert rel_l2(xd.grad, xr.grad) < TOL
    assert rel_l2(m.weight.grad, sd["weight"].grad) < TOL
    assert rel_l2(m.bias.grad, sd["bias"].grad) < TOL


@pytest.mark.parametrize("quad", [True, False])
def test_frame_backward_source_gradient_range_tags(quad):
    """nps_frame_pack_bwd_tagged: each source gradient's range tag equals max |dsrc| (the quad kernel publishes it
    per wave, the element-wise path runs one absmax per source), so the conv backward that reads it as dy scales
    by it instead of an absmax pass; gradients as the untagged entry point's."""
    import ctypes
    from nps_hip import ops, lib, ptr, stream_ptr, check, Conv2dArgs
    torch.manual_seed(11)
    c1 = 12 if quad else 6  # 6 channels (and 5 per group): off the quad kernels
    B, H, W = 2, 13, 17
    s1, s2 = torch.randn(B, H, W, c1, device=DEV), torch.randn(B, H + 2, W + 2, 4, device=DEV) * 3
    srcs = [ops.Src(s1), ops.Src(s2, -1, -1)]
    st = ops.group_norm_stats(srcs, (H, W), 2)
    C = c1 + 4
    gamma, beta = 1 + 0.1 * torch.randn(C, device=DEV), 0.1 * torch.randn(C, device=DEV)
    gy = torch.randn(B, H, W, C, device=DEV)
    outs = []
    for tagged in (False, True):
        a = Conv2dArgs()
        a.nsrc, a.src = 2, ops._c_src(srcs)
        a.B, a.Hin, a.Win, a.Cin = B, H, W, C
        a.gn_stats, a.gn_gamma, a.gn_beta, a.gn_groups, a.gn_eps = ptr(st), ptr(gamma), ptr(beta), 2, 1e-5
        a.pre_act = 1
        d = [torch.empty_like(s1), torch.empty_like(s2)]
        dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        work = torch.empty((B, 2, C), dtype=torch.float64, device=DEV)
        arr = (ctypes.c_void_p * 3)(d[0].data_ptr(), d[1].data_ptr(), None)
        if tagged:
            ops.reserve_tags(gy.device, 2)
            tags = (ctypes.c_void_p * 3)(ops.new_tag(d[0]), ops.new_tag(d[1]), None)
            check(lib.nps_frame_pack_bwd_tagged(ctypes.byref(a), ptr(gy), arr, tags, ptr(dg), ptr(db), ptr(work),
                                                stream_ptr()), "frame_pack_bwd_tagged")
            for t in d:
                assert ops.tag_value(t) == float(t.abs().max())
        else:
            check(lib.nps_frame_pack_bwd(ctypes.byref(a), ptr(gy), arr, ptr(dg), ptr(db), ptr(work), stream_ptr()),
                  "frame_pack_bwd")
        outs.append(d)
    for u, t in zip(*outs):  # (the GroupNorm reduction's float atomics make two runs differ in the last bits)
        torch.testing.assert_close(u, t, rtol=1e-5, atol=1e-6)


def test_residual_block_backward_concat_crop_groupnorm():
    """cat(h, crop(s), crop(vb)) -> GN(1)+GELU -> conv1 -> GN+GELU -> conv2, + crop-padded 1x1 shortcut."""
    from models.enc_proc_dec_components.proc_unet_modern import ResidualBlock
    from nps_hip import ops
    from nps_hip import autograd as ad
    torch.manual_seed(0)
    rb = ResidualBlock(20 + 16 + 4, 16, activation=nn.GELU(), norm=True, num_spatial_dims=2,
                       padding_kwargs=dict(padding_mode="circular"))
    with torch.no_grad():
        for n in (rb.norm1, rb.norm2):
            n.weight.uniform_(0.5, 1.5)
            n.bias.uniform_(-0.3, 0.3)
    h, s, v = torch.randn(2, 20, 30, 30), torch.randn(2, 16, 27, 27), torch.rand(2, 4, 33, 33)
    sd = {k: t.detach().clone().requires_grad_(True) for k, t in rb.state_dict().items()}
    hr, sr, vr = (t.clone().requires_grad_(True) for t in (h, s, v))
    x = torch.cat([hr, Fo.crop_nd(sr, h.shape), Fo.crop_nd(vr, h.shape)], dim=1)
    ref = Fo.residual_block(sd, "", x, True, dict(padding_mode="circular"))
    g = torch.randn_like(ref)
    ref.backward(g)
    rb = rb.to(DEV)
    hd, sdd, vd = (ops.nchw_to_nhwc(t.to(DEV)).requires_grad_(True) for t in (h, s, v))
    srcs = [ops.Src(hd), ops.Src(sdd, ops.crop_offset(27, 30), ops.crop_offset(27, 30)),
            ops.Src(vd, ops.crop_offset(33, 30), ops.crop_offset(33, 30))]
    y = rb.run_ad(srcs, (30, 30))
    y.backward(ops.nchw_to_nhwc(g.to(DEV)))
    assert rel_l2(ops.nhwc_to_nchw(y.detach()), ref) < TOL
    for got, want in ((hd, hr), (sdd, sr), (vd, vr)):
        assert rel_l2(ops.nhwc_to_nchw(got.grad), want.grad) < TOL
    _grads_ok({k: t.grad for k, t in sd.items()}, dict((k, p.grad) for k, p in rb.named_parameters()))


# ------------------------------------------------------------------ spectral
@pytest.mark.parametrize("name", ["spectral2d_a", "spectral2d_overlap", "spectral2d_nyq"])
def test_spectral2d_backward_golden(name):
    """dx, dweights1, dweights2 vs the reference's own autograd (torch.fft + complex einsum)."""
    from models.enc_proc_dec_components.proc_fno import SpectralConv2d
    g = load_golden(name)
    kw = g["kwargs"]
    m = SpectralConv2d(kw["in_channels"], kw["out_channels"], tuple(kw["modes"]))
    m.load_state_dict(g["state_dict"])
    m = m.to(DEV)
    x = g["x"].to(DEV).requires_grad_(True)
    y = m(x)
    y.backward(g["g"].to(DEV))
    assert rel_l2(y, g["y"]) < TOL
    assert rel_l2(x.grad, g["dx"]) < TOL
    assert rel_l2(m.weights1.grad, g["dw1"]) < TOL
    assert rel_l2(m.weights2.grad, g["dw2"]) < TOL


@pytest.mark.parametrize("H,W,m", [(64, 64, 12), (96, 64, 10)])
def test_spectral2d_backward_full_channels(H, W, m):
    from models.enc_proc_dec_components.proc_fno import SpectralConv2d
    torch.manual_seed(1)
    sc = SpectralConv2d(196, 192, (m, m))
    x = torch.randn(2, 196, H, W)
    w1 = sc.weights1.detach().clone().requires_grad_(True)
    w2 = sc.weights2.detach().clone().requires_grad_(True)
    xr = x.clone().requires_grad_(True)
    ref = Fo.spectral_conv2d(xr, w1, w2)
    g = torch.randn_like(ref)
    ref.backward(g)
    sc = sc.to(DEV)
    xd = x.to(DEV).requires_grad_(True)
    sc(xd).backward(g.to(DEV))
    assert rel_l2(xd.grad, xr.grad) < TOL
    assert rel_l2(sc.weights1.grad, w1.grad) < TOL
    assert rel_l2(sc.weights2.grad, w2.grad) < TOL


# ------------------------------------------------------------------ processors
def _proc(name):
    from models.enc_proc_dec_components import UNetModern, DilatedResnet, UFNO, FNO
    cls = {"unet_ufno_style": UNetModern, "unet_cfg": UNetModern, "unet_ones": UNetModern, "drn": DilatedResnet,
           "ufno": UFNO, "fno": FNO}[name]
    g = load_golden(name)
    kw = dict(g["kwargs"])
    if cls is not FNO:
        kw["activation"] = nn.GELU()
    m = cls(pde=None, **kw)
    m.load_state_dict(g["state_dict"])
    return m, g, cls


_ORACLE_PROC = {"unet_ufno_style": Fo.unet_modern, "unet_cfg": Fo.unet_modern, "unet_ones": Fo.unet_modern,
                "drn": Fo.dilated_resnet, "ufno": Fo.ufno, "fno": Fo.fno}


@pytest.mark.parametrize("B,Cin,Cout", [(1, 20, 12), (2, 196, 192), (5, 67, 64), (16, 64, 32), (17, 40, 44),
                                         (32, 24, 16), (33, 20, 12)])
def test_spectral_mix_backward_vs_fp64(B, Cin, Cout):
    """nps_spectral_mix_bwd (MFMA for B <= 32, the scalar kernel above) vs the fp64 adjoint of the per-mode
    contraction y[b][o] = sum_i x[b][i] W[i][o] (proc_fno.py:253-255): gX = gY W^H, gW = sum_b conj(x) gY."""
    from nps_hip import lib, ptr, stream_ptr, check
    g = torch.Generator().manual_seed(B * 1000 + Cin)
    nm = 6  # modes

    def crand(*sh):
        return torch.complex(torch.randn(*sh, generator=g), torch.randn(*sh, generator=g))

    X = crand(B, nm, Cin)
    W = crand(nm, Cin, Cout)
    gY = crand(B, nm, Cout)
    gX = torch.einsum("bmo,mio->bmi", gY.to(torch.complex128), W.to(torch.complex128).conj())
    gW = torch.einsum("bmi,bmo->mio", X.to(torch.complex128).conj(), gY.to(torch.complex128))
    Xd, Wd, gYd = X.to(DEV), W.to(DEV), gY.to(DEV)
    gXd = torch.empty_like(Xd)
    gWd = torch.empty_like(Wd)
    check(lib.nps_spectral_mix_bwd(ptr(Xd), ptr(Wd), ptr(gYd), ptr(gXd), ptr(gWd), B, 2, nm // 2, Cin, Cout,
                                   stream_ptr()), "spectral_mix_bwd")
    assert rel_l2(gXd.cpu(), gX) < 1e-6
    assert rel_l2(gWd.cpu(), gW) < 1e-6


@pytest.mark.parametrize("name", ["unet_ufno_style", "unet_cfg", "unet_ones", "drn", "ufno", "fno"])
def test_processor_backward_vs_oracle(name):
    m, g, _ = _proc(name)
    sd = {k: t.detach().clone().requires_grad_(True) for k, t in m.state_dict().items()}
    hr = g["h"].clone().requires_grad_(True)
    vr = g["vb"].clone().requires_grad_(True)
    cfg = dict(g["kwargs"])
    ref = _ORACLE_PROC[name](sd, "", cfg, hr, vr)
    torch.manual_seed(3)
    gy = torch.randn_like(ref)
    ref.backward(gy)
    m = m.to(DEV)
    hd = g["h"].to(DEV).requires_grad_(True)
    vd = g["vb"].to(DEV).requires_grad_(True)
    y = m(h=hd, variables_broadcast=vd)
    y.backward(gy.to(DEV))
    assert rel_l2(y, g["y"]) < TOL
    assert rel_l2(hd.grad, hr.grad) < TOL
    assert rel_l2(vd.grad, vr.grad) < TOL
    _grads_ok({k: t.grad for k, t in sd.items() if t.grad is not None},
              {k: p.grad for k, p in m.named_parameters()})


# ------------------------------------------------------------------ full model training loss
def _build_model(g):
    import models
    from pdes import PDE2D
    cfg = dict(g["cfg"])
    cfg.pop("object")
    cfg["activation"] = nn.GELU()
    cfg["activation_final"] = nn.Tanh()
    p = g["pde"]
    pde = PDE2D(tmin=p["tmin"], tmax=p["tmax"], nt=p["nt"], L1=1.0, L2=1.0, nx1=p["nx1"], nx2=p["nx2"], x=None,
                name="twophase", n_cond_static=p["n_cond_static"], n_cond_spatial=p["n_cond_spatial"])
    m = models.activation_wrapper(**cfg, pde=pde)
    m.load_state_dict(g["state_dict"])
    return m, pde


@pytest.mark.parametrize("name", ["model_ufno", "model_unet", "model_drn", "model_ufno_fno"])
def test_model_train_loss_grads_vs_oracle(name):
    """loss = sqrt(MSE_sum(model(x), labels)) (autoregressivepushforwardtrainer.py:158-162) and every
    parameter gradient, vs autograd through the oracle on the same state_dict."""
    from nps_hip import autograd as ad
    g = load_golden(name)
    m, pde = _build_model(g)
    tw = g["cfg"]["time_window"]
    u, cond, pos, sc = g["u"], g["cond"], g["pos"], g["spatial_cond"]
    x, labels = u[:, :, :tw], u[:, :, tw:2 * tw]
    om = oracle.build_oracle_model({k: v for k, v in g["cfg"].items() if k != "object"}, g["pde"], g["state_dict"])
    om.sd = {k: v.detach().clone().requires_grad_(True) for k, v in om.sd.items()}
    ref_pred = om(x, cond=cond, pos=pos, spatial_cond=sc)
    ref_loss = torch.sqrt(torch.sum((ref_pred - labels) ** 2))
    ref_loss.backward()
    m = m.to(DEV).train()
    pred = m(x.to(DEV), cond=cond.to(DEV), bc=None, pos=pos.to(DEV), t_cond=None, spatial_cond=sc.to(DEV))
    loss = ad.sqrt_mse_sum(pred, labels.to(DEV))
    loss.backward()
    assert rel_l2(pred, ref_pred) < TOL
    assert abs(loss.item() - ref_loss.item()) / ref_loss.item() < TOL
    _grads_ok({k: t.grad for k, t in om.sd.items() if t.grad is not None},
              {k: p.grad for k, p in m.named_parameters()})


def test_ufno_c3_full_size_train_grads():
    """North-star config C3 (U-FNO twophase cfg: hidden 192, 3 blocks, modes 10, 256x256, 3 fields,
    obstacle), B=1: sqrt(MSE_sum) training loss and every parameter gradient vs the CPU oracle."""
    import __graft_entry__  # noqa: F401
    from bench import build_model
    from nps_hip import autograd as ad
    from trainers.synthetic import twophase_batch
    m, ocfg, opde = build_model("ufno", res=256, num_c=3, device=DEV)
    m.train()
    u, cond, pos, sc = twophase_batch(1, 3, 50, 256, 256, seed=7, obstacle="disc")
    x, labels = u[:, :, :25], u[:, :, 25:50]
    om = oracle.build_oracle_model(ocfg, opde, {k: v.cpu() for k, v in m.state_dict().items()})
    om.sd = {k: v.detach().clone().requires_grad_(True) for k, v in om.sd.items()}
    ref_loss = torch.sqrt(torch.sum((om(x, cond=cond, pos=pos, spatial_cond=sc) - labels) ** 2))
    ref_loss.backward()
    loss = ad.sqrt_mse_sum(m(x.to(DEV), cond=cond.to(DEV), bc=None, pos=pos.to(DEV), t_cond=None,
                             spatial_cond=sc.to(DEV)), labels.to(DEV))
    loss.backward()
    assert abs(loss.item() - ref_loss.item()) / ref_loss.item() < TOL
    _grads_ok({k: t.grad for k, t in om.sd.items() if t.grad is not None},
              {k: p.grad for k, p in m.named_parameters()})


def test_pushforward_train_one_epoch():
    """trainers/base.py:472-507 loop with the pushforward train_step (:43-163) and Adam on the MI355X:
    finite losses, every parameter updated, loss goes down over a few steps on a fixed batch."""
    import argparse
    import types
    import random
    from bench import build_model
    from common.interfaces import D
    from trainers.autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer
    from trainers.synthetic import twophase_batch
    random.seed(0)
    m, _, _ = build_model("ufno", res=32, num_c=1, device=DEV)
    m.train()
    # T = 50: the only valid window starts at step 25, so successive losses are comparable
    u, cond, pos, sc = twophase_batch(2, 1, 50, 32, 32, seed=3, obstacle="random", device=DEV)
    batch = (u[:, :, :1], u, pos, cond, torch.empty(u.shape[0], 0, device=DEV), sc)
    cfg = argparse.Namespace(time_window=25, base_resolution=(50, 32, 32), device=DEV, batch_size=2,
                             lr_step_interval=1, unrolling=2)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    tr = AutoregressivePushforwardTrainer(model=m, data=types.SimpleNamespace(pde=m.pde, data_interface=D.sim2d),
                                          criterion=nn.MSELoss(reduction="sum"), optimizer=opt, config=cfg)
    before = {k: p.detach().clone() for k, p in m.named_parameters()}
    losses = [float(tr.train_one_epoch([batch], epoch=0)) for _ in range(6)]
    assert all(l == l and l < 1e6 for l in losses), losses
    assert losses[-1] < losses[0], losses
    for k, p in m.named_parameters():
        assert not torch.equal(p.detach(), before[k]), f"{k} not updated"
    # epoch >= lr_step_interval: random unroll depth (no-grad pushforward calls) before the grad call
    u2, _, _, _ = twophase_batch(2, 1, 125, 32, 32, seed=4, obstacle="random", device=DEV)
    cfg.base_resolution = (125, 32, 32)
    tr2 = AutoregressivePushforwardTrainer(model=m, data=types.SimpleNamespace(pde=m.pde, data_interface=D.sim2d),
                                           criterion=nn.MSELoss(reduction="sum"), optimizer=opt, config=cfg)
    for _ in range(3):
        l2 = float(tr2.train_one_epoch([(u2[:, :, :1], u2, pos, cond, torch.empty(u2.shape[0], 0, device=DEV), sc)], epoch=3))
        assert l2 == l2


@pytest.mark.parametrize("cout,cin,k,dil", [(192, 388, 3, 1), (192, 196, 1, 1), (4, 16, 2, 1), (40, 84, 1, 1),
                                            (64, 64, 5, 3), (8, 12, 3, 1)])
def test_dgrad_packing_equals_flipped_transpose(cout, cin, k, dil):
    """pack_weights mode -3 (the input-gradient conv's weight, transposed + flipped inside the pack kernel)
    is bit-identical to packing the torch flip/transpose of w (both arithmetics: 5x5 dilated packs fp32)."""
    from nps_hip import ops
    torch.manual_seed(cout + cin + k)
    w = (torch.randn(cout, cin, k, k) * 0.1).to(DEV)
    got = ops.pack_conv_weight_dgrad(w, dil)
    ref = ops.pack_conv_weight(w.flip(2, 3).transpose(0, 1).contiguous(), 1, dil)
    assert got.nps_precision == ref.nps_precision
    body = got.numel() - 64 + 1  # fragment body + trailer[0] (max|w|); the rest of the trailer is unwritten
    assert torch.equal(got[:body], ref[:body])


@pytest.mark.parametrize("off,src_hw,C", [((1, -1), (10, 16), 8), ((0, 0), (12, 14), 4), ((-2, 3), (15, 9), 6)])
def test_add_at_forward_and_backward(off, src_hw, C):
    """ad.add_at (the residual crop_Nd(h) + shortcut, proc_unet_modern.py:250) — the one-pass nps_add_at_copy for
    C % 4 == 0, clone + nps_add_at otherwise — and its gradients, against torch on the same placement."""
    from nps_hip import autograd as ad
    torch.manual_seed(2)
    base = torch.randn(2, 12, 14, C, device=DEV, requires_grad=True)
    src = torch.randn(2, *src_hw, C, device=DEV, requires_grad=True)
    y = ad.add_at(base, src, off)
    g = torch.randn_like(y)
    y.backward(g)
    bd, sd = base.detach().cpu().double(), src.detach().cpu().double()
    ref = bd.clone()
    oy, ox = off
    Hs, Ws = src_hw
    y0, y1 = max(0, oy), min(12, oy + Hs)
    x0, x1 = max(0, ox), min(14, ox + Ws)
    ref[:, y0:y1, x0:x1] += sd[:, y0 - oy:y1 - oy, x0 - ox:x1 - ox]
    assert torch.allclose(y.detach().cpu().double(), ref, atol=1e-6)
    from nps_hip import ops
    st = ops.stats_of(y)  # the one-pass form carries y's GroupNorm(1) moments for the next frame
    if C % 4 == 0 and ad.ADD_AT_COPY and ad.CARRY_ADD and ops.CONV_PRECISION == ops.PREC_X3F16:
        assert st is not None
        m = st.detach().cpu().sum(1)
        assert torch.allclose(m[:, 0], ref.sum((1, 2, 3)), rtol=1e-6, atol=1e-6)
        assert torch.allclose(m[:, 1], (ref * ref).sum((1, 2, 3)), rtol=1e-6)
    else:
        assert st is None
    gd = g.cpu().double()
    assert torch.allclose(base.grad.cpu().double(), gd, atol=1e-6)
    gs = torch.zeros_like(sd)
    gs[:, y0 - oy:y1 - oy, x0 - ox:x1 - ox] = gd[:, y0:y1, x0:x1]
    assert torch.allclose(src.grad.cpu().double(), gs, atol=1e-6)


CARRY_CASES = [
    # (kind, Cin, Cout, k, stride, padding, padding_mode, H, W) — the autograd outputs that carry their GroupNorm(1)
    # moments from the conv epilogues (autograd._carry_buffer)
    ("conv", 16, 64, 3, 1, 0, "zeros", 21, 19),       # valid 3x3, ragged tiles
    ("conv", 192, 192, 3, 1, 0, "zeros", 20, 22),     # wide 192-channel tiles
    ("conv", 12, 40, 3, 2, 0, "zeros", 31, 29),       # Downsample s2: out_hw one row / column short of the grid
    ("conv", 12, 40, 3, 2, 1, "zeros", 16, 16),       # Downsample s2, pad 1
    ("conv", 8, 8, 5, 1, "same", "circular", 24, 24),  # DRN 5x5 dilated circular
    ("conv", 196, 192, 1, 1, 0, "zeros", 19, 23),     # 1x1, Cout <= 192 (LDS-weight kernel)
    ("conv", 192, 75, 1, 1, 0, "zeros", 16, 16),      # 1x1, Cout % 4 != 0: no carried moments
    ("convT", 64, 64, 4, 2, 0, 1, 13, 11),            # Upsample: circular pre-pad 1, 4 phase launches
    ("convT", 40, 40, 4, 2, 1, 0, 9, 12),             # transposed conv with padding 1 (crop of every phase)
]


@pytest.mark.parametrize("case", CARRY_CASES)
def test_autograd_outputs_carry_exact_moments(case):
    """the GroupNorm(1) moments the training forward's convs carry (Conv2dFn stride 1 / 2, 1x1,
    ConvTranspose2dFn's 4 phases with a crop offset) equal the fp64 (sum, sum of squares) of the stored output."""
    from models.common import Conv2d, ConvTranspose2d, ConvTranspose2d_padded
    from nps_hip import autograd as ad
    from nps_hip import ops
    kind, Cin, Cout, k, s, p, pm, H, W = case
    torch.manual_seed(1)
    if kind == "conv":
        m = Conv2d(Cin, Cout, k, stride=s, padding=p, padding_mode=pm, dilation=2 if k == 5 else 1).to(DEV)
    elif pm:
        m = ConvTranspose2d_padded(pm, Cin, Cout, k, stride=s, padding=p).to(DEV)
    else:
        m = ConvTranspose2d(Cin, Cout, k, stride=s, padding=p).to(DEV)
    x = (torch.randn(2, H, W, Cin, device=DEV) + 0.3).requires_grad_(True)
    y = ad.conv2d(m, x) if kind == "conv" else ad.conv_transpose2d(m, x)
    st = ops.stats_of(y)
    if not (ad.CARRY_TRAIN and ops.CONV_PRECISION == ops.PREC_X3F16):
        pytest.skip("moments not carried in training (NPS_CARRY_TRAIN=0 / exact fp32 convs)")
    if Cout % 4 != 0:
        assert st is None  # the planar / off-quad epilogue cannot take them: a statistics pass instead
        return
    assert st is not None
    yd = y.detach().double().cpu()
    m1 = st.detach().cpu().sum(1)
    ref = torch.stack([yd.sum((1, 2, 3)), (yd * yd).sum((1, 2, 3))], 1)
    assert torch.allclose(m1, ref, rtol=1e-6, atol=1e-6 * ref.abs().max().item()), (m1, ref)
    y.sum().backward()  # the carried buffer does not disturb the backward
    assert x.grad is not None and torch.isfinite(x.grad).all()


def test_batched_repack_equals_individual_packs():
    """ops._repack_stale (one nps_conv2d_pack_weights_x3_batch call after an optimizer step) writes, into the cached
    buffers, exactly the bytes of fresh nps_conv2d_pack_weights_x3 calls: forward, input-gradient (mode -3),
    space-to-depth (-2) and transposed-conv phase packings, over more weights than one batch launch takes (48)."""
    from nps_hip import ops
    if ops.CONV_PRECISION != ops.PREC_X3F16 or not ops.PACK_BATCH:
        pytest.skip("split-fp16 batched packing off")
    torch.manual_seed(9)
    shapes = [(192, 196, 3, 3), (192, 388, 3, 3), (64, 36, 1, 1), (225, 192, 1, 1), (128, 132, 5, 5), (40, 12, 3, 3)]
    ws = [torch.nn.Parameter(torch.randn(*shapes[i % len(shapes)], device=DEV) * 10 ** (i % 5 - 2)) for i in range(30)]
    convT = torch.nn.Parameter(torch.randn(64, 48, 4, 4, device=DEV))
    kinds = []
    for i, w in enumerate(ws):
        kinds.append((w, "conv", lambda p: ops.pack_conv_weight(p)))
        if w.shape[2] != 5:
            kinds.append((w, "dgrad", lambda p: ops.pack_conv_weight_dgrad(p)))
        if w.shape[2] == 3:
            kinds.append((w, "s2d", ops.pack_conv_weight_s2d))
    kinds.append((convT, "convT", ops.pack_convT_phases))
    for w, kind, fn in kinds:
        ops.cached_pack(w, kind, fn)
    assert sum(len(ops._replay_jobs(w, w._nps_packs[k][1]) or []) for w, k, _ in kinds) > 48
    with torch.no_grad():  # the optimizer's in-place step: every version bumps
        for w in ws + [convT]:
            w.mul_(-1.5).add_(0.25)
    got = [ops.cached_pack(w, kind, fn) for w, kind, fn in kinds]  # the first lookup repacks everything in a batch
    for (w, kind, fn), g in zip(kinds, got):
        ref = fn(w)
        gs, rs = (g, ref) if isinstance(g, list) else ([g], [ref])
        for a, b in zip(gs, rs):
            n = a.numel() - 64 + 1  # the fragment body and trailer[0] = max|w| (the rest: absmax partials / unused)
            assert torch.equal(a[:n].view(torch.int32), b[:n].view(torch.int32)), kind


@pytest.mark.parametrize("case", [c for c in WGRAD_X3_CASES if c[1] % 4 == 0 and c[2] % 4 == 0])
def test_wgrad_x3_bias_gradient_from_staging(case):
    """nps_wgrad_t.db: the split-fp16 weight-gradient launch also stores sum_pix a[pix][m] (the conv's bias gradient,
    a = dy) from its own staging of a — on wgrad_x3_kernel (1x1 / 2x2 / 3x3 64 x 64 tiles), wgrad1_wide_kernel and
    wgrad2_wide_kernel, with m-tails past one tile and several n-tiles (only n-tile 0 adds) — against the fp64 sums;
    the weight gradient itself is unchanged by it."""
    from nps_hip import autograd as ad
    B, M, N, k, pad, circ, Ha, Wa, sa, sx = case
    Hx, Wx = Ha + k - 1 - 2 * pad - 2 * circ, Wa + k - 1 - 2 * pad - 2 * circ
    torch.manual_seed(2)
    a = torch.randn(B, M, Ha, Wa, dtype=torch.float64) * sa + 0.1 * sa
    x = torch.randn(B, N, Hx, Wx, dtype=torch.float64) * sx
    ad_a = a.float().permute(0, 2, 3, 1).contiguous().to(DEV)
    ad_x = x.float().permute(0, 2, 3, 1).contiguous().to(DEV)
    db = torch.full((M,), float("nan"), device=DEV)
    g1 = ad.wgrad(ad_a, ad_x, k, k, pad=(pad, pad), circ=circ, db=db)
    g0 = ad.wgrad(ad_a, ad_x, k, k, pad=(pad, pad), circ=circ)
    assert rel_l2(g1, g0) < 1e-6  # (split-K fp32 atomics: equal up to the order of the partial sums)
    ref = a.sum((0, 2, 3))
    assert rel_l2(db.cpu().double(), ref) < 1e-6, rel_l2(db.cpu().double(), ref)


@pytest.mark.parametrize("cout", [388, 196, 256])
def test_conv1x1_channel_groups_vs_fp64(cout):
    """1x1 convs with Cout > 192 (the input-gradient convs 192 -> 388 / 196 of the shortcut and FNO 1x1s) on the
    LDS-weight kernel's channel groups of 192: the groups of one pixel tile, the tail group's empty blocks skipped,
    bias and an addend at an output channel stride, against fp64."""
    from nps_hip import ops
    torch.manual_seed(6)
    B, H, W, cin = 2, 23, 37, 192
    x = torch.randn(B, H, W, cin, dtype=torch.float64)
    w = torch.randn(cout, cin, dtype=torch.float64) / cin ** 0.5
    b = torch.randn(cout, dtype=torch.float64) * 0.1
    add = torch.randn(B, H, W, cout, dtype=torch.float64)
    ref = x @ w.T + b + add
    wp = ops.pack_conv_weight(w.float().view(cout, cin, 1, 1).to(DEV))
    y = ops.conv2d([ops.Src(x.float().to(DEV))], (H, W), wp, b.float().to(DEV), cout, 1, 1,
                   addends=(add.float().to(DEV),))
    assert rel_l2(y.cpu().double(), ref) < TOL


def test_wgrad_x3_bias_row_accumulates_like_g():
    """nps_conv2d_wgrad_x3 (+= mode) through ctypes: db follows g's semantics — a second launch adds into it."""
    import ctypes
    from nps_hip import WgradArgs, lib, ops
    from nps_hip import autograd as ad
    torch.manual_seed(23)
    B, H, W, M, N = 2, 17, 21, 64, 36
    a = torch.randn(B, H, W, M, device=DEV)
    x = torch.randn(B, H, W, N, device=DEV)
    g = torch.zeros(M, N, 3, 3, device=DEV)
    db = torch.zeros(M, device=DEV)
    p = WgradArgs()
    p.a, p.B, p.Ha, p.Wa, p.M = a.data_ptr(), B, H, W, M
    p.x, p.Hx, p.Wx, p.N = x.data_ptr(), H, W, N
    p.KH = p.KW = 3
    p.dil, p.pad_y, p.pad_x, p.circ, p.g, p.db = 1, 1, 1, 0, g.data_ptr(), db.data_ptr()
    ops.reserve_tags(a.device, 2)
    ar, xr = ad._range_ptr(a), ad._range_ptr(x)
    ws = torch.empty(lib.nps_wgrad_x3_ws_floats(M, N, 3, 3), device=DEV)
    for _ in range(2):
        assert lib.nps_conv2d_wgrad_x3(ctypes.byref(p), ar, xr, ws.data_ptr(), ops.stream_ptr()) == 0
    ref = 2 * a.double().sum((0, 1, 2))
    assert rel_l2(db.cpu().double(), ref.cpu()) < 1e-6
    gref = 2 * ad.wgrad(a, x, 3, 3, pad=(1, 1))
    assert rel_l2(g.cpu(), gref.cpu()) < 1e-6
