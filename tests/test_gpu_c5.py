"""BASELINE config C5 — the 3-D spectral path at its full shape (time-bundled 16 x 128 x 128 volume) in fp32
and in bf16 storage.

* fp32 FNO-3D (proc_fno.py:22-155, SpectralConv3d :291-376) at the C5 volume vs the CPU oracle: the fp32
  bar of BASELINE.json, rel-L2 < 1e-5.
* bf16 storage (activations and packed weights in bf16, every sum in fp32): the reference has no bf16 path
  (CPU FFT rejects bf16), so it is checked against the fp32 HIP path — itself pinned to the
  oracle above — at a stated bf16 tolerance: rel-L2 < 1e-2 for the 4-block FNO-3D and 5e-3 for one
  SpectralConv3d (bf16 keeps 8 significant bits: rounding one tensor costs ~1e-3 rel-L2; measured values in
  the test log).  The bf16 pointwise conv is checked against fp64 on the same bf16-rounded operands.
"""
import pytest
import torch

from conftest import rel_l2
from oracle import functional as Fo

pytestmark = pytest.mark.gpu
DEV = "cuda"
# C5: FNO-3D processor over a (D, H, W) = (16, 128, 128) volume, hidden 64 + 4 conditioning channels,
# modes (8, 12, 12), 4 blocks (bench.py --model fno3d)
C5 = dict(num_spatial_dims=3, n_cond=4, hidden_features=64, fno_modes=(8, 12, 12), hidden_blocks=4,
          cond_mode="concat", fno_kernel_size=1)
VOL = (16, 128, 128)


def _fno3d(seed=11):
    from models.enc_proc_dec_components.proc_fno import FNO
    torch.manual_seed(seed)
    return FNO(pde=None, **C5)


def _inputs(B=1, seed=12):
    g = torch.Generator().manual_seed(seed)
    h = torch.rand(B, C5["hidden_features"], *VOL, generator=g) * 2 - 1
    vb = torch.rand(B, C5["n_cond"], *VOL, generator=g)
    return h, vb


def test_fno3d_c5_fp32_vs_oracle():
    m = _fno3d()
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    h, vb = _inputs()
    ref = Fo.fno3d(sd, "", dict(hidden_blocks=C5["hidden_blocks"]), h, vb)
    with torch.no_grad():
        y = m.to(DEV)(h.to(DEV), variables_broadcast=vb.to(DEV)).cpu()
    err = rel_l2(y, ref)
    print(f"C5 fp32 FNO-3D vs oracle: rel-L2 {err:.3e}")
    assert err < 1e-5


def test_fno3d_c5_bf16_vs_fp32():
    m = _fno3d().to(DEV)
    h, vb = _inputs(B=2)
    h, vb = h.to(DEV), vb.to(DEV)
    with torch.no_grad():
        y32 = m(h, variables_broadcast=vb)
        y16 = m(h.to(torch.bfloat16), variables_broadcast=vb.to(torch.bfloat16))
    assert y16.dtype == torch.bfloat16 and y16.shape == y32.shape
    err = rel_l2(y16.float(), y32)
    print(f"C5 bf16 FNO-3D vs fp32 HIP path: rel-L2 {err:.3e}")
    assert err < 1e-2


def test_spectral_conv3d_bf16_vs_fp32():
    from models.enc_proc_dec_components.proc_fno import SpectralConv3d
    torch.manual_seed(3)
    m = SpectralConv3d(68, 64, (8, 12, 12)).to(DEV)
    x = (torch.rand(1, 68, *VOL, device=DEV) * 2 - 1)
    with torch.no_grad():
        y32 = m(x)
        y16 = m(x.to(torch.bfloat16))
    err = rel_l2(y16.float(), y32)
    print(f"C5 bf16 SpectralConv3d vs fp32: rel-L2 {err:.3e}")
    assert err < 5e-3


@pytest.mark.parametrize("cin,cout", [(68, 64), (20, 32), (132, 192)])
def test_conv1x1_bf16_vs_fp64(cin, cout):
    """nps_conv1x1_bf16 (two bf16 sources, the last one's channel tail partial) vs fp64 on the same
    bf16-rounded operands: only the bf16 rounding of the output separates them."""
    from nps_hip import ops
    torch.manual_seed(5)
    c0 = (cin // 8 - 1) * 8  # first source: a multiple of 8 channels; second: the rest
    x0 = (torch.randn(2, 24, 40, c0) * 0.5).to(torch.bfloat16)
    x1 = (torch.randn(2, 24, 40, cin - c0) * 0.5).to(torch.bfloat16)
    w = torch.randn(cout, cin) * 0.1
    b = torch.randn(cout) * 0.1
    y = ops.conv1x1_bf16([ops.Src(x0.to(DEV)), ops.Src(x1.to(DEV))], ops.pack_1x1_bf16(w.to(DEV)), b.to(DEV), cout,
                         act=ops.GELU).cpu()
    x = torch.cat([x0, x1], dim=-1).double()
    ref = torch.nn.functional.gelu(x @ w.to(torch.bfloat16).double().T + b.double())
    err = rel_l2(y.float(), ref)
    assert err < 4e-3, err
