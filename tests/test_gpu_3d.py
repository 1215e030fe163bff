"""GPU parity of the 3-D spectral path (SpectralConv3d, FNO-3D processor):
the HIP pipeline through the C ABI vs the reference's own golden vectors (tests/golden/make_golden*.py)
and vs the pinned CPU oracle at a larger size.

Tolerance: fp32 rel-L2 < 1e-5 (north star); gradients compared as whole vectors at the same bar.
"""
import pytest
import torch

from oracle import functional as Fo
from conftest import load_golden, rel_l2

pytestmark = pytest.mark.gpu
TOL = 1e-5
DEV = "cuda"


def _r(t):
    return torch.view_as_real(t) if t.is_complex() else t


def _spectral3d(g):
    from models.enc_proc_dec_components.proc_fno import SpectralConv3d
    kw = dict(g["kwargs"])
    kw["modes"] = tuple(kw["modes"])
    m = SpectralConv3d(**kw)
    m.load_state_dict(g["state_dict"])
    return m.to(DEV)


@pytest.mark.parametrize("name", ["spectral3d", "spectral3d_overlap", "spectral3d_nyq"])
def test_spectral3d_forward_golden(name):
    g = load_golden(name)
    m = _spectral3d(g)
    with torch.no_grad():
        y = m(g["x"].to(DEV)).cpu()
    assert y.shape == g["y"].shape
    assert rel_l2(y, g["y"]) < TOL


@pytest.mark.parametrize("name", ["spectral3d_overlap", "spectral3d_nyq"])
def test_spectral3d_backward_golden(name):
    g = load_golden(name)
    m = _spectral3d(g)
    x = g["x"].to(DEV).requires_grad_(True)
    y = m(x)
    assert rel_l2(y.detach().cpu(), g["y"]) < TOL
    y.backward(g["g"].to(DEV))
    assert rel_l2(x.grad.cpu(), g["dx"]) < TOL
    for i in range(4):
        gw = getattr(m, f"weights{i + 1}").grad.cpu()
        assert rel_l2(_r(gw), _r(g["dw"][i])) < TOL, f"weights{i + 1}"


def _fno3d(g):
    from models.enc_proc_dec_components.proc_fno import FNO
    kw = dict(g["kwargs"])
    kw["fno_modes"] = tuple(kw["fno_modes"])
    m = FNO(pde=None, **kw)
    m.load_state_dict(g["state_dict"])
    return m.to(DEV)


def test_fno3d_golden_forward_backward():
    g = load_golden("fno3d")
    m = _fno3d(g)
    with torch.no_grad():
        y0 = m(g["h"].to(DEV), variables_broadcast=g["vb"].to(DEV)).cpu()
    assert rel_l2(y0, g["y"]) < TOL
    h = g["h"].to(DEV).requires_grad_(True)
    y = m(h, variables_broadcast=g["vb"].to(DEV))
    assert rel_l2(y.detach().cpu(), g["y"]) < TOL
    y.backward(g["g"].to(DEV))
    assert rel_l2(h.grad.cpu(), g["dh"]) < TOL


def test_fno3d_larger_vs_oracle():
    """C5-shaped (reduced channels/batch so the CPU oracle finishes in seconds): 16 x 64 x 64 volume,
    modes (6, 12, 12), 24 hidden + 4 cond channels, 2 blocks."""
    from models.enc_proc_dec_components.proc_fno import FNO
    torch.manual_seed(7)
    m = FNO(pde=None, num_spatial_dims=3, n_cond=4, hidden_features=24, fno_modes=(6, 12, 12), hidden_blocks=2,
            cond_mode="concat", fno_kernel_size=1)
    sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
    h = torch.rand(2, 24, 16, 64, 64) * 2 - 1
    vb = torch.rand(2, 4, 16, 64, 64)
    ref = Fo.fno3d(sd, "", dict(hidden_blocks=2), h, vb)
    with torch.no_grad():
        y = m.to(DEV)(h.to(DEV), variables_broadcast=vb.to(DEV)).cpu()
    assert rel_l2(y, ref) < TOL
