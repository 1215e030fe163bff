"""Golden vectors of the on-disk dataset path (PDE2DDataset / MemMapDataset / DataCreator.create_data).

CONTAINER-ONLY TOOL, same contract as make_golden.py: writes the deterministic dataset of
tests/data_fixture.py to a temp dir, loads it with the REFERENCE's data classes (twophase cfg arguments),
and saves what they return (only plain tensors / numbers travel):
    python tests/golden/make_golden_data.py
"""
import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]
from make_golden import REF_SRC, OUT_DIR, _install_stubs  # noqa: E402
from data_fixture import write_twophase_dataset, DATASET_KW  # noqa: E402


def main():
    _install_stubs()
    root = tempfile.mkdtemp()
    write_twophase_dataset(root)
    write_twophase_dataset(os.path.join(root, "nosplit"), with_split=False)
    os.chdir(tempfile.mkdtemp())
    sys.path.insert(0, REF_SRC)
    import torch
    from data.PDE2D import PDE2DDataset
    from common.data_creator import DataCreator

    out = {}
    ds = PDE2DDataset(base_path=root, **DATASET_KW)
    p = ds.pde
    out["pde"] = {k: float(getattr(p, k)) for k in ("tmin", "tmax", "nt", "L1", "L2", "nx1", "nx2", "dt", "dx1",
                                                    "dx2", "n_cond_static", "n_cond_dynamic", "n_cond_spatial")}
    out["x"] = p.x
    for split in ("train", "valid", "test"):
        sub = getattr(ds, split)
        out[f"{split}_indices"] = torch.tensor([int(i) for i in sub.indices])
        items = [sub[i] for i in range(len(sub))]
        for j, name in enumerate(("u_base", "u", "x", "cond", "t_cond", "sc")):
            out[f"{split}_{name}"] = torch.stack([it[j] for it in items])
    ds2 = PDE2DDataset(base_path=os.path.join(root, "nosplit"), **dict(DATASET_KW, split_file=None,
                                                                       split_val=0.2, split_test=0.15))
    for split in ("train", "valid", "test"):
        out[f"nosplit_{split}_indices"] = torch.tensor([int(i) for i in getattr(ds2, split).indices])
    dc = DataCreator(pde=p, neighbors=3, time_window=3, t_resolution=11, x_resolution=(8, 6))
    u = out["train_u"]
    steps = [3, 5, 8, 4]
    d, l = dc.create_data(u, steps)
    out.update(cd_steps=torch.tensor(steps), cd_data=d, cd_labels=l)
    torch.save(out, os.path.join(OUT_DIR, "data_twophase.pt"))
    print("wrote data_twophase.pt")


if __name__ == "__main__":
    main()
