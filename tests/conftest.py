import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "neural-pde-surrogates_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs on the GPU box)")


def load_golden(name):
    import torch
    return torch.load(os.path.join(GOLDEN, f"{name}.pt"), weights_only=True)


def _as_f64(t):
    """fp64 CPU copy; complex tensors are compared through their (re, im) pairs, so both parts count."""
    import torch
    t = t.detach().cpu()
    if t.is_complex():
        t = torch.view_as_real(t.resolve_conj())
    return t.to(torch.float64)


def rel_l2(a, b):
    import torch
    a, b = _as_f64(a), _as_f64(b)
    if a.shape != b.shape:
        raise AssertionError(f"rel_l2: shape mismatch {tuple(a.shape)} vs {tuple(b.shape)}")
    return (torch.linalg.vector_norm(a - b) / torch.linalg.vector_norm(b)).item()


@pytest.fixture
def golden():
    return load_golden
