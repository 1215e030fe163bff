"""BASELINE config C5 — the 3-D U-FNO (time-bundled D x H x W volume, bf16) on the GPU.

* Pinned to the REFERENCE where it can build the model: its 3-D UNetModern / U-FNO with a single U-Net
  resolution and its 3-D Downsample (tests/golden/make_golden_3d.py), fp32 storage, rel-L2 < 1e-5.
* Multi-resolution 3-D U-Nets need a 3-D Upsample the reference lacks; this build defines it (circular pad 1
  + ConvTranspose3d(k=4, s=2), DESIGN.md "3-D U-FNO").  Those models are checked against the CPU oracle's
  restatement of the same definition (oracle/functional.py ufno3d / unet_modern3d: PARITY UNPINNED beyond
  the Upsample semantics), fp32 at rel-L2 < 1e-5, including the full C5 volume 16 x 128 x 128.
* bf16 storage (the C5 arithmetic) has no reference (the reference's CPU FFT rejects bf16): it is checked
  against this build's fp32 path on the same input at rel-L2 < 2e-2.
"""
import pytest
import torch

import oracle
from oracle import functional as Fo
from conftest import load_golden, rel_l2

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 1e-5
BF16_TOL = 2e-2


def _model(cls, kw, sd=None, seed=42):
    import models.enc_proc_dec_components as comps
    kw = dict(kw)
    if "fno_modes" in kw and isinstance(kw["fno_modes"], list):
        kw["fno_modes"] = tuple(kw["fno_modes"])
    torch.manual_seed(seed)
    m = getattr(comps, cls)(pde=None, **kw)
    if sd is not None:
        m.load_state_dict(sd)
    return m.to(DEV).eval()


def test_unet3d_single_resolution_golden():
    g = load_golden("unet3d_single")
    m = _model("UNetModern", g["kwargs"], g["state_dict"])
    with torch.no_grad():
        y = m(g["h"].to(DEV), variables_broadcast=g["vb"].to(DEV)).cpu()
    assert rel_l2(y, g["y"]) < TOL


def test_downsample3d_golden():
    from models.enc_proc_dec_components.proc_unet_modern import Downsample
    g = load_golden("downsample3d")
    m = Downsample(8, num_spatial_dims=3, n_cond=2, padding_kwargs=dict(padding_mode="circular"))
    m.load_state_dict(g["state_dict"])
    m = m.to(DEV).eval()
    with torch.no_grad():
        yh, yv = m(g["h"].to(DEV), variables_broadcast=g["vb"].to(DEV))
    assert rel_l2(yh.cpu(), g["yh"]) < TOL and rel_l2(yv.cpu(), g["yv"]) < TOL


def test_ufno3d_single_resolution_golden():
    g = load_golden("ufno3d_single")
    m = _model("UFNO", g["kwargs"], g["state_dict"])
    with torch.no_grad():
        y = m(g["h"].to(DEV), variables_broadcast=g["vb"].to(DEV)).cpu()
    assert rel_l2(y, g["y"]) < TOL


@pytest.mark.parametrize("shape,ch_mults", [((2, 11, 20, 24), [1, 2]), ((1, 23, 26, 35), [1, 1, 2])])
def test_unet3d_multires_vs_oracle(shape, ch_mults):
    """Down / Downsample / Middle / Upsample / Up with odd sizes (crop_Nd crops and pads), 2 and 3 levels
    (the valid 3x3x3 convs of the middle block need >= 5 voxels per axis at the lowest level)."""
    B, D, H, W = shape
    kw = dict(num_spatial_dims=3, n_cond=4, hidden_features=16, cond_mode="concat", norm=True, ch_mults=ch_mults,
              is_attn=[False] * len(ch_mults), mid_attn=False, n_blocks=1, use1x1=True, padding_mode="circular")
    m = _model("UNetModern", kw)
    g = torch.Generator().manual_seed(5)
    h = torch.randn(B, 16, D, H, W, generator=g)
    vb = torch.rand(B, 4, D, H, W, generator=g)
    with torch.no_grad():
        y = m(h.to(DEV), variables_broadcast=vb.to(DEV)).cpu()
    sd = {k: v.cpu() for k, v in m.state_dict().items()}
    ref = Fo.unet_modern3d(sd, "", kw, h, vb)
    assert y.shape == ref.shape
    assert rel_l2(y, ref) < TOL


def _c5(blocks):
    from bench import C5_UFNO_CFG
    return dict(C5_UFNO_CFG, hidden_blocks=blocks)


def test_ufno3d_c5_volume_fp32_vs_oracle_and_bf16_vs_fp32():
    """C5 shape: U-FNO 3D, 64 hidden + 4 conditioning channels, modes (8, 12, 12), U-Nets with ch_mults
    [1, 1] (one Downsample / Upsample), on the full 16 x 128 x 128 volume (2 blocks to bound the CPU
    oracle's time): fp32 GPU vs oracle, then bf16 storage vs the fp32 GPU result."""
    from models.common import to_ndhwc, to_ncdhw
    from nps_hip import ops
    kw = _c5(2)
    m = _model("UFNO", kw)
    g = torch.Generator().manual_seed(11)
    D, H, W = 16, 128, 128
    h = torch.rand(1, kw["hidden_features"], D, H, W, generator=g) * 2 - 1
    vb = torch.rand(1, kw["n_cond"], D, H, W, generator=g)
    hd, vd = h.to(DEV), vb.to(DEV)
    with torch.no_grad():
        y32 = m(hd, variables_broadcast=vd)
    sd = {k: v.cpu() for k, v in m.state_dict().items()}
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    ref = Fo.ufno3d(sd, "", dict(kw, fno_modes=tuple(kw["fno_modes"])), h, vb)
    assert rel_l2(y32.cpu(), ref) < TOL
    # bf16 storage, NDHWC in HBM like the bench
    hb, vbb = ops.to_bf16(to_ndhwc(hd)), ops.to_bf16(to_ndhwc(vd))
    with torch.no_grad():
        yb = to_ncdhw(ops.to_f32(m.run3d(hb, vbb)))
    err = rel_l2(yb.cpu(), y32.cpu())
    print(f"C5 U-FNO 3D bf16 vs fp32 rel-L2 {err:.3e}")
    assert err < BF16_TOL
