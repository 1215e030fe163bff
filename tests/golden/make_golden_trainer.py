"""Golden numbers of the train.py call sequence (pre-train validation, 3 epochs of pushforward training with
validation / test passes and checkpoints, final test) run by the REFERENCE's own packages on the CPU.

CONTAINER-ONLY TOOL, same contract as make_golden.py: writes the synthetic dataset of
tests/trainer_scenario.py to a temp dir, imports the reference (two unused import-time dependencies
stubbed), runs tests/trainer_scenario.run against the reference's `models` / `trainers` / `data` and
saves the returned numbers and final state_dict (plain tensors only) as trainer_ufno.pt:
    python tests/golden/make_golden_trainer.py
"""
import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [HERE, os.path.dirname(HERE)]
from make_golden import REF_SRC, OUT_DIR, _install_stubs  # noqa: E402
import trainer_scenario  # noqa: E402


def main():
    _install_stubs()
    root = trainer_scenario.write_dataset(tempfile.mkdtemp())
    work = tempfile.mkdtemp()
    os.chdir(work)  # the reference's train() mkdirs experiments/ and models/output relative to cwd
    os.makedirs("models", exist_ok=True)
    save_dir = os.path.join(work, "ckpt")
    os.makedirs(save_dir)
    sys.path.insert(0, REF_SRC)
    import torch
    torch.set_num_threads(8)
    import data
    import models
    import trainers
    out = trainer_scenario.run(models, trainers, data, "cpu", root, save_dir)
    torch.save(out, os.path.join(OUT_DIR, "trainer_ufno.pt"))
    print({k: v for k, v in out.items() if k != "final_state"})
    print("wrote trainer_ufno.pt")


if __name__ == "__main__":
    main()
