"""train.py as a drop-in: the call sequence of reference src/train.py:102-165 —
get_dataloaders, the pre-train trainer.test(valid_loader), get_parameters / set_optimizer /
set_lr_scheduler, trainer.train() (3 epochs: pushforward train_one_epoch, validation, checkpoint,
test pass on improvement) and the final trainer.test(test_loader) — run on the MI355X mirror, against
the numbers the REFERENCE's own packages produce for the same sequence on the CPU
(tests/golden/make_golden_trainer.py -> trainer_ufno.pt).

The sample order and random unroll choices match the reference exactly (DeviceLoader draws the RNG as
torch's DataLoader does), so the comparison is value-for-value.  Tolerances: rel 1e-5 on every loss
and metric (fp32 rel-L2 bar of BASELINE.json; measured ~1e-7); the trained weights rel-L2 < 1e-4 over
the whole state and the update (trained - initial) rel-L2 < 1e-2 — Adam's first steps move every weight
by ≈ lr·sign(g), so weights whose gradient is analytically zero (a bias feeding a GroupNorm) move by
rounding noise in either implementation.
"""
import os

import pytest
import torch

from conftest import load_golden, rel_l2
import trainer_scenario

DEV = "cuda"


def _close(a, b, tol=1e-5, what=""):
    assert abs(a - b) <= tol * max(abs(b), 1e-12), f"{what}: {a} vs {b}"


@pytest.mark.gpu
def test_train_py_sequence_matches_reference(tmp_path):
    import data
    import models
    import trainers
    g = load_golden("trainer_ufno")
    root = trainer_scenario.write_dataset(str(tmp_path / "ds"))
    save_dir = str(tmp_path / "ckpt")
    os.makedirs(save_dir)
    cwd = os.getcwd()
    os.chdir(tmp_path)  # train() creates experiments/ and models/output relative to cwd, as the reference
    os.makedirs("models", exist_ok=True)
    try:
        got = trainer_scenario.run(models, trainers, data, DEV, root, save_dir)
    finally:
        os.chdir(cwd)
    assert got["shape"] == g["shape"] and got["n_params"] == g["n_params"]
    assert got["checkpoints"] == g["checkpoints"]
    assert got["lr"] == pytest.approx(g["lr"], rel=1e-12)
    _close(got["valid_loss"], g["valid_loss"], what="pre-train valid loss")
    _close(got["test_loss"], g["test_loss"], what="final test loss")
    for which in ("valid_summary", "test_summary"):
        assert set(got[which]) == set(g[which])
        for k, v in g[which].items():
            _close(got[which][k], v, what=f"{which}[{k}]")
    assert len(got["train_losses"]) == len(g["train_losses"])
    for a, b in zip(got["train_losses"], g["train_losses"]):
        _close(a, b, what="train loss")
    for name, vs in g["val_losses"].items():
        for a, b in zip(got["val_losses"][name], vs):
            _close(a, b, what="val loss")
        for sa, sb in zip(got["val_stats"][name], g["val_stats"][name]):
            assert set(sa) == set(sb)
            for k in sb:
                _close(sa[k], sb[k], what=f"val stat {k}")
    # trained weights
    fin_ref = g["final_state"]
    fin = got["final_state"]
    assert set(fin) == set(fin_ref)
    vec = lambda sd: torch.cat([torch.view_as_real(t).flatten() if t.is_complex() else t.flatten().float()  # noqa
                                for t in (sd[k] for k in sorted(sd))])
    assert rel_l2(vec(fin), vec(fin_ref)) < 1e-4
    torch.manual_seed(trainer_scenario.SEED)
    from pdes import PDE2D
    init = models.activation_wrapper(**{k: v for k, v in trainer_scenario.MODEL.items() if k != "object"},
                                     pde=PDE2D(tmin=0.0, tmax=1.0, nt=101, L1=1.0, L2=1.0, nx1=32, nx2=32, x=None,
                                               name="twophase", n_cond_static=3, n_cond_spatial=1)).state_dict()
    assert rel_l2(vec(fin) - vec(init), vec(fin_ref) - vec(init)) < 1e-2
