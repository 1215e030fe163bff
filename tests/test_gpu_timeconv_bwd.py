"""TimeConvDense + add_delta('per_step') + tanh + spatial-cond mask backward (csrc/pointwise.hip
nps_timeconv_decode_bwd) against torch fp64 autograd of the same chain (dec_grid.py:126-146, :8-31;
activation_wrapper.py:34-35): the gradient of the planar pre-decoder output and of both conv1d layers.

tw = 25 (the twophase cfgs, num_c 1 and 3) runs timeconv_bwd_fast_kernel: blocks walk 16-pixel groups, so the
shapes cover a ragged last group (H*W % 16 != 0), several groups per block (the grid is one resident pass)
and the mask / tanh switches.  tw = 8 runs the generic one-wave kernel.  Tolerance: rel-L2 < 1e-5 per tensor
(fp32 kernels vs fp64)."""
import pytest
import torch
import torch.nn.functional as F

from conftest import rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _sizes(tw):
    ka = (tw + 1) // 2
    kb = (tw + 3) // 4 + 1 + (1 if tw % 4 == 0 else 0)
    return ka, kb


def _dtcum(tw):
    return torch.cumsum(torch.full((tw,), 0.04) * (1 + 0.1 * torch.arange(tw)), 0)


def _reference(pre, u, w1, b1, w2, b2, dt, mask, mask_ch, act_tanh, nc, tw):
    """fp64 chain per pixel: conv1d(s2) -> GELU -> conv1d -> u_last + dt * d -> tanh -> v - m v."""
    B, _, H, W = pre.shape
    x = pre.view(B, nc, 3 * tw, H * W).permute(0, 3, 1, 2).reshape(B * H * W, nc, 3 * tw)
    d = F.conv1d(F.gelu(F.conv1d(x, w1, b1, stride=2)), w2, b2)          # (BHW, nc, tw)
    d = d.view(B, H * W, nc, tw).permute(0, 2, 3, 1).reshape(B, nc, tw, H, W)
    v = u[:, :, -1:] + dt.view(1, 1, tw, 1, 1) * d
    if act_tanh:
        v = torch.tanh(v)
    if mask is not None:
        m = mask[:, mask_ch:mask_ch + 1].unsqueeze(2)
        v = v - m * v
    return v


@pytest.mark.parametrize("nc,tw,B,H,W,use_mask,act_tanh", [
    (3, 25, 2, 37, 29, True, True),      # ragged last group, C3's num_c
    (3, 25, 1, 96, 64, False, True),     # native 96x64 grid: many groups per block
    (1, 25, 2, 33, 17, True, False),     # C2/C4's num_c, no tanh
    (3, 25, 1, 256, 256, True, True),    # C3 full size
    (2, 8, 2, 19, 23, True, True),       # generic kernel
])
def test_timeconv_decode_bwd_vs_fp64(nc, tw, B, H, W, use_mask, act_tanh):
    from nps_hip import autograd as ad
    torch.manual_seed(nc * 100 + tw + H)
    ka, kb = _sizes(tw)
    L = 3 * tw
    pre = torch.randn(B, nc * L, H, W)
    u = torch.rand(B, nc, tw, H, W)
    w1, b1 = torch.randn(2 * nc, nc, ka) * 0.2, torch.randn(2 * nc) * 0.1
    w2, b2 = torch.randn(nc, 2 * nc, kb) * 0.2, torch.randn(nc) * 0.1
    dt = _dtcum(tw)
    mask = (torch.rand(B, 2, H, W) > 0.7).float() if use_mask else None
    gout = torch.randn(B, nc, tw, H, W)

    ref_in = [t.double().requires_grad_(True) for t in (pre, w1, b1, w2, b2)]
    ref = _reference(ref_in[0], u.double(), *ref_in[1:], dt.double(), None if mask is None else mask.double(), 1,
                     act_tanh, nc, tw)
    ref.backward(gout.double())

    got_in = [t.to(DEV).requires_grad_(True) for t in (pre, w1, b1, w2, b2)]
    y = ad.TimeConvDecodeFn.apply((1, act_tanh, nc, tw), got_in[0], u.to(DEV), got_in[1], got_in[2], got_in[3],
                                  got_in[4], dt.to(DEV), None if mask is None else mask.to(DEV))
    y.backward(gout.to(DEV))
    assert rel_l2(y, ref) < 1e-5
    for name, g, r in zip(("pre", "w1", "b1", "w2", "b2"), got_in, ref_in):
        assert rel_l2(g.grad, r.grad) < 1e-5, name
