"""The twophase cfgs' native geometry (tests/golden/native_{ufno,unet,drn}_96x64.pt, written by
tests/golden/make_golden_native.py from the reference): the full-width cfg_twophase_{ufno,unet,drn} models at
base_resolution (501, 96, 64) (reference src/configs/train/cfg_twophase_ufno.py:6-7), num_c = 1, disc obstacle,
B = 2, t_res = 110 — a 3-call `simulate` whose partial last window [100, 110) is skipped
(autoregressivepushforwardtrainer.py:354-358).  Weights and inputs are regenerated from seeds and checked against
the fixture's checksums (c1_fixture.assert_checksums)."""
import torch
from torch import nn

from c1_fixture import _checksums, assert_checksums
from conftest import load_golden

NATIVE_MODELS = ("ufno", "unet", "drn")


def native_golden(name):
    return load_golden(f"native_{name}_96x64")


def native_inputs(g):
    from trainers.synthetic import twophase_batch
    d = g["data"]
    u, cond, pos, sc = twophase_batch(d["B"], d["num_c"], d["T"], d["H"], d["W"], seed=d["seed"],
                                      obstacle=d["obstacle"])
    assert_checksums(_checksums(dict(u=u, cond=cond, pos=pos, sc=sc)), g["input_checksums"], "native inputs")
    return u, cond, pos, sc


def native_model(g):
    """The mirror's cfg model, torch.manual_seed(42) construction on the CPU, pinned to the reference's seeded
    weights by checksum."""
    import models
    from pdes import PDE2D
    cfg = dict(g["cfg"], activation=nn.GELU(), activation_final=nn.Tanh())
    p = g["pde"]
    pde = PDE2D(tmin=p["tmin"], tmax=p["tmax"], nt=p["nt"], L1=1.0, L2=1.0, nx1=p["nx1"], nx2=p["nx2"], x=None,
                name="twophase", n_cond_static=p["n_cond_static"], n_cond_spatial=p["n_cond_spatial"])
    torch.manual_seed(42)
    m = models.activation_wrapper(**cfg, pde=pde).eval()
    assert_checksums(_checksums(m.state_dict()), g["state_checksums"], "native weights")
    return m, pde


def native_oracle(g, m):
    import oracle
    return oracle.build_oracle_model(dict(g["cfg"]), dict(g["pde"]), {k: v.detach().cpu()
                                                                     for k, v in m.state_dict().items()})
