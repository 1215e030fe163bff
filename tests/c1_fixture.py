"""BASELINE config C1 (tests/golden/c1_unet_cfg_sim.pt, written by tests/golden/make_golden_c1.py from the
reference): the exact cfg_twophase_unet model at 64x64, B=2, t_res=150 (5 model calls).  The fixture holds
no weights and no trajectory; both are regenerated here and checked against its checksums — to 1e-7
relative, not bit for bit: torch's vectorised CPU tanh / sin round differently on different host ISAs (the
GPU box's CPU is not this container's), a last-ulp change that moves the outputs far below the 1e-5 bar."""
import torch
from torch import nn

from conftest import load_golden


def _checksums(sd):
    out = {}
    for k, v in sd.items():
        v = v.detach()
        v = (torch.view_as_real(v) if v.is_complex() else v).double()  # both parts of complex weights count
        out[k] = torch.stack([v.sum(), (v ** 2).sum()])
    return out


def assert_checksums(got, want, what):
    assert set(got) == set(want), what
    for k in want:
        torch.testing.assert_close(got[k], want[k], rtol=1e-7, atol=1e-9, msg=f"{what}: {k}")


def c1_golden():
    return load_golden("c1_unet_cfg_sim")


def c1_inputs(g):
    from trainers.synthetic import twophase_batch
    d = g["data"]
    u, cond, pos, sc = twophase_batch(d["B"], d["num_c"], d["T"], d["res"], d["res"], seed=d["seed"],
                                      obstacle=d["obstacle"])
    assert_checksums(_checksums(dict(u=u, cond=cond, pos=pos, sc=sc)), g["input_checksums"], "C1 inputs")
    return u, cond, pos, sc


def c1_model(g):
    """The mirror's cfg_twophase_unet model, torch.manual_seed(42) construction (CPU), pinned to the
    reference's seeded weights by checksum."""
    import models
    from pdes import PDE2D
    cfg = dict(g["cfg"], activation=nn.GELU(), activation_final=nn.Tanh())
    p = g["pde"]
    pde = PDE2D(tmin=p["tmin"], tmax=p["tmax"], nt=p["nt"], L1=1.0, L2=1.0, nx1=p["nx1"], nx2=p["nx2"], x=None,
                name="twophase", n_cond_static=p["n_cond_static"], n_cond_spatial=p["n_cond_spatial"])
    torch.manual_seed(42)
    m = models.activation_wrapper(**cfg, pde=pde).eval()
    assert_checksums(_checksums(m.state_dict()), g["state_checksums"], "C1 weights")
    return m, pde
