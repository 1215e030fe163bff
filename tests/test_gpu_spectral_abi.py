"""GPU parity of the one-call spectral C ABI (include/nps.h "one call per module"; VERDICT r5 Missing #1):
nps_spectral_conv2d_fwd / _bwd, nps_fno_layer2d_fwd and nps_spectral_conv3d_fwd / _bwd called through ctypes on
raw device pointers with a caller-provided workspace — no nps_hip.ops sequencing — against the reference's own
golden vectors (tests/golden/make_golden*.py) and the CPU oracle at the BASELINE sizes.

Tolerance: fp32 rel-L2 < 1e-5 (north star), gradients compared on (re, im).
"""
import ctypes

import pytest
import torch
import torch.nn.functional as F

from oracle import functional as Fo
from conftest import load_golden, rel_l2

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda"


def _lib():
    from nps_hip import lib
    return lib


def _p(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _s():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _ok(rc, what):
    if rc != 0:
        raise AssertionError(f"{what}: rc {rc}: {_lib().nps_last_error().decode()}")


def _nhwc(x):  # (B, C, *spatial) -> channels-last contiguous on the GPU
    return x.movedim(1, -1).contiguous().to(DEV)


def _nchw(y):
    return y.movedim(-1, 1).cpu()


def _ws(nbytes):
    assert nbytes > 0
    return torch.empty(nbytes, dtype=torch.uint8, device=DEV)


def spectral2d_abi(x, w1, w2, y=None, accumulate=0, act=0):
    """x (B, Cin, H, W) CPU -> y (B, Cout, H, W) through nps_spectral_conv2d_fwd."""
    lib = _lib()
    B, Cin, H, W = x.shape
    Cout, m1, m2 = w1.shape[1], w1.shape[2], w1.shape[3]
    xd = _nhwc(x)
    yd = _nhwc(y) if y is not None else torch.empty(B, H, W, Cout, device=DEV)
    w1d, w2d = w1.contiguous().to(DEV), w2.contiguous().to(DEV)  # (held until the launches have run)
    ws = _ws(lib.nps_spectral_conv2d_workspace(B, Cin, Cout, H, W, m1, m2))
    _ok(lib.nps_spectral_conv2d_fwd(_p(xd), _p(w1d), _p(w2d), _p(yd), _p(ws),
                                    B, Cin, Cout, H, W, m1, m2, accumulate, act, _s()), "spectral_conv2d_fwd")
    torch.cuda.synchronize()
    return _nchw(yd)


def spectral2d_abi_bwd(x, w1, w2, g):
    lib = _lib()
    B, Cin, H, W = x.shape
    Cout, m1, m2 = w1.shape[1], w1.shape[2], w1.shape[3]
    xd, gd = _nhwc(x), _nhwc(g)
    dx = torch.empty(B, H, W, Cin, device=DEV)
    dw1 = torch.empty_like(w1, device=DEV)
    dw2 = torch.empty_like(w2, device=DEV)
    w1d, w2d = w1.contiguous().to(DEV), w2.contiguous().to(DEV)
    ws = _ws(lib.nps_spectral_conv2d_workspace(B, Cin, Cout, H, W, m1, m2))
    _ok(lib.nps_spectral_conv2d_bwd(_p(xd), _p(w1d), _p(w2d), _p(gd), _p(dx),
                                    _p(dw1), _p(dw2), _p(ws), B, Cin, Cout, H, W, m1, m2, _s()), "spectral_conv2d_bwd")
    torch.cuda.synchronize()
    return _nchw(dx), dw1.cpu(), dw2.cpu()


@pytest.mark.parametrize("name", ["spectral2d_a", "spectral2d_overlap", "spectral2d_nyq"])
def test_spectral2d_abi_golden_forward_backward(name):
    g = load_golden(name)
    w1, w2 = g["state_dict"]["weights1"], g["state_dict"]["weights2"]
    assert rel_l2(spectral2d_abi(g["x"], w1, w2), g["y"]) < TOL
    dx, dw1, dw2 = spectral2d_abi_bwd(g["x"], w1, w2, g["g"])
    assert rel_l2(dx, g["dx"]) < TOL
    assert rel_l2(dw1, g["dw1"]) < TOL
    assert rel_l2(dw2, g["dw2"]) < TOL


@pytest.mark.parametrize("B,H,W,m", [(2, 256, 256, 10), (2, 96, 64, 10), (1, 128, 128, 12)])
def test_spectral2d_abi_full_size(B, H, W, m):
    """The U-FNO spectral conv (196 -> 192 channels) at the BASELINE sizes vs the torch.fft oracle; the accumulate
    + GELU form is FNO_Layer's act(conv(x) + w(x)) tail (proc_fno.py:142-146)."""
    torch.manual_seed(2)
    Cin, Cout = 196, 192
    w1 = (torch.rand(Cin, Cout, m, m, dtype=torch.cfloat)) / (Cin * Cout)
    w2 = (torch.rand(Cin, Cout, m, m, dtype=torch.cfloat)) / (Cin * Cout)
    x = torch.randn(B, Cin, H, W)
    ref = Fo.spectral_conv2d(x, w1, w2)
    assert rel_l2(spectral2d_abi(x, w1, w2), ref) < TOL
    y0 = torch.randn(B, Cout, H, W)
    assert rel_l2(spectral2d_abi(x, w1, w2, y=y0, accumulate=1, act=1), F.gelu(y0 + ref)) < TOL


def test_spectral2d_abi_backward_vs_autograd():
    """Backward at a U-FNO-like shape (channel tails, 2 m1 > H / 2) vs torch autograd through the oracle."""
    torch.manual_seed(4)
    B, Cin, Cout, H, W, m1, m2 = 2, 36, 44, 24, 40, 7, 9
    w1 = (torch.rand(Cin, Cout, m1, m2, dtype=torch.cfloat) / (Cin * Cout)).requires_grad_(True)
    w2 = (torch.rand(Cin, Cout, m1, m2, dtype=torch.cfloat) / (Cin * Cout)).requires_grad_(True)
    x = torch.randn(B, Cin, H, W, requires_grad=True)
    y = Fo.spectral_conv2d(x, w1, w2)
    g = torch.randn_like(y)
    y.backward(g)
    dx, dw1, dw2 = spectral2d_abi_bwd(x.detach(), w1.detach(), w2.detach(), g)
    assert rel_l2(dx, x.grad) < TOL
    assert rel_l2(dw1, w1.grad) < TOL
    assert rel_l2(dw2, w2.grad) < TOL


def test_spectral_abi_refuses_bad_modes():
    """proc_fno.py:134-139: modes above the spatial dims (W // 2 + 1 for the last) are refused, workspace 0."""
    lib = _lib()
    assert lib.nps_spectral_conv2d_workspace(1, 4, 4, 16, 16, 17, 3) == 0
    assert lib.nps_spectral_conv2d_workspace(1, 4, 4, 16, 16, 4, 10) == 0
    t = torch.zeros(64, device=DEV)
    rc = lib.nps_spectral_conv2d_fwd(_p(t), _p(t), _p(t), _p(t), _p(t), 1, 4, 4, 16, 16, 4, 10, 0, 0, _s())
    assert rc < 0 and "modes" in lib.nps_last_error().decode()


def _fno_args(srcs, w1x1, bias, out, act):
    """A planned nps_conv2d_t of the layer's 1x1 `w` over the virtual frame `srcs` (NHWC device tensors)."""
    from nps_hip import Conv2dArgs
    lib = _lib()
    a = Conv2dArgs()
    a.nsrc = len(srcs)
    for i, s in enumerate(srcs):
        a.src[i].ptr, a.src[i].C, a.src[i].H, a.src[i].W = s.data_ptr(), s.shape[3], s.shape[1], s.shape[2]
    B, H, W = srcs[0].shape[:3]
    Cin = sum(s.shape[3] for s in srcs)
    Cout = w1x1.shape[0]
    a.B, a.Hin, a.Win, a.Cin = B, H, W, Cin
    a.KH = a.KW = a.stride = a.dil = 1
    a.Hout, a.Wout = H, W
    wpk = torch.empty(lib.nps_conv2d_packed_size(Cout, Cin, 1), device=DEV)
    wd = w1x1.contiguous().to(DEV)
    _ok(lib.nps_conv2d_pack_weights_x3(_p(wd), _p(wpk), Cout, Cin, 1, 1, -1, _s()), "pack")
    torch.cuda.synchronize()
    a.wpack, a.bias, a.Cout = wpk.data_ptr(), bias.data_ptr(), Cout
    a.out, a.out_C, a.out_H, a.out_W, a.out_os = out.data_ptr(), Cout, H, W, 1
    a.act = act
    a.precision = 1  # NPS_PREC_X3F16
    assert lib.nps_conv2d_plan(ctypes.byref(a)) >= 0
    return a, wpk


@pytest.mark.parametrize("H,W,m,fused", [(64, 256, 10, True), (96, 64, 10, False), (40, 128, 6, True)])
def test_fno_layer2d_abi(H, W, m, fused):
    """FNO_Layer (proc_fno.py:142-146) in one call: act(SpectralConv2d(x) + w(x)) over the U-FNO block's frame
    cat(h, vb) (two sources); W % 128 == 0 takes the synthesis fused into the 1x1's epilogue, the native 96 x 64
    grid the 1x1 + accumulating idft_w pass — both against torch."""
    lib = _lib()
    torch.manual_seed(5)
    B, Ch, Cv, Cout = 2, 192, 4, 192
    Cin = Ch + Cv
    h, vb = torch.randn(B, Ch, H, W), torch.rand(B, Cv, H, W)
    w1 = torch.rand(Cin, Cout, m, m, dtype=torch.cfloat) / (Cin * Cout)
    w2 = torch.rand(Cin, Cout, m, m, dtype=torch.cfloat) / (Cin * Cout)
    wc = torch.randn(Cout, Cin, 1, 1) / Cin ** 0.5
    bc = torch.randn(Cout) * 0.1
    hd, vd = _nhwc(h), _nhwc(vb)
    out = torch.empty(B, H, W, Cout, device=DEV)
    bd, w1d, w2d = bc.to(DEV), w1.to(DEV), w2.to(DEV)  # (a holds raw pointers: keep the tensors alive)
    a, _wpk = _fno_args([hd, vd], wc, bd, out, act=1)
    ws = _ws(lib.nps_fno_layer2d_workspace(B, Cin, Cout, H, W, m, m))
    _ok(lib.nps_fno_layer2d_fwd(ctypes.byref(a), _p(w1d), _p(w2d), m, m, _p(ws), _s()), "fno_layer2d")
    torch.cuda.synchronize()
    x = torch.cat([h, vb], 1)
    ref = F.gelu(Fo.spectral_conv2d(x, w1, w2) + F.conv2d(x, wc, bc))
    assert rel_l2(_nchw(out), ref) < TOL


def spectral3d_abi(x, ws4, y=None, accumulate=0, act=0):
    lib = _lib()
    B, Cin, D, H, W = x.shape
    Cout, m1, m2, m3 = ws4[0].shape[1:]
    xd = _nhwc(x)
    yd = _nhwc(y) if y is not None else torch.empty(B, D, H, W, Cout, device=DEV)
    wd = [w.contiguous().to(DEV) for w in ws4]
    ws = _ws(lib.nps_spectral_conv3d_workspace(B, Cin, Cout, D, H, W, m1, m2, m3))
    _ok(lib.nps_spectral_conv3d_fwd(_p(xd), *[_p(w) for w in wd], _p(yd), _p(ws), B, Cin, Cout, D, H, W, m1, m2, m3,
                                    accumulate, act, _s()), "spectral_conv3d_fwd")
    torch.cuda.synchronize()
    return _nchw(yd)


def spectral3d_abi_bwd(x, ws4, g):
    lib = _lib()
    B, Cin, D, H, W = x.shape
    Cout, m1, m2, m3 = ws4[0].shape[1:]
    xd, gd = _nhwc(x), _nhwc(g)
    wd = [w.contiguous().to(DEV) for w in ws4]
    dx = torch.empty(B, D, H, W, Cin, device=DEV)
    dws = [torch.empty_like(w) for w in wd]
    ws = _ws(lib.nps_spectral_conv3d_workspace(B, Cin, Cout, D, H, W, m1, m2, m3))
    _ok(lib.nps_spectral_conv3d_bwd(_p(xd), *[_p(w) for w in wd], _p(gd), _p(dx), *[_p(d) for d in dws], _p(ws),
                                    B, Cin, Cout, D, H, W, m1, m2, m3, _s()), "spectral_conv3d_bwd")
    torch.cuda.synchronize()
    return _nchw(dx), [d.cpu() for d in dws]


@pytest.mark.parametrize("name", ["spectral3d", "spectral3d_overlap", "spectral3d_nyq"])
def test_spectral3d_abi_golden(name):
    g = load_golden(name)
    ws4 = [g["state_dict"][f"weights{i}"] for i in range(1, 5)]
    assert rel_l2(spectral3d_abi(g["x"], ws4), g["y"]) < TOL
    if "g" in g:
        dx, dws = spectral3d_abi_bwd(g["x"], ws4, g["g"])
        assert rel_l2(dx, g["dx"]) < TOL
        for i in range(4):
            assert rel_l2(dws[i], g["dw"][i]) < TOL, f"weights{i + 1}"


def test_spectral3d_abi_c5_volume():
    """SpectralConv3d at the C5 volume (16 x 128 x 128, 68 -> 64 channels, modes (8, 12, 12)) vs the oracle, and the
    accumulate + GELU tail of the 3-D FNO layer."""
    torch.manual_seed(6)
    B, Cin, Cout, D, H, W = 1, 68, 64, 16, 128, 128
    m = (8, 12, 12)
    ws4 = [torch.rand(Cin, Cout, *m, dtype=torch.cfloat) / (Cin * Cout) for _ in range(4)]
    x = torch.randn(B, Cin, D, H, W)
    ref = Fo.spectral_conv3d(x, *ws4)
    assert rel_l2(spectral3d_abi(x, ws4), ref) < TOL
    y0 = torch.randn(B, Cout, D, H, W)
    assert rel_l2(spectral3d_abi(x, ws4, y=y0, accumulate=1, act=1), F.gelu(y0 + ref)) < TOL
