"""train.py's order of operations under `torchrun --nproc-per-node 2`, with NO wrapper and no
init_process_group call of its own (VERDICT r4 Missing #2; reference src/train.py:17-19 imports, :32 model
.to(device), :70 trainer by name, :135-144 optimizer, then steps).  Importing the mirror's packages opens the
group (common/launch.py); the trainer then wires data parallelism.  Each rank trains on its half of the
global batches of tests/test_ddp_training.py's torch-only grid model and writes its results to argv[1].

Run by tests/test_ddp_training.py::test_torchrun_train_py_without_wrapper (gloo, CPU)."""
import os
import random
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "neural-pde-surrogates_amd"))
sys.path.insert(0, HERE)

import torch.distributed as dist  # noqa: E402

assert not dist.is_initialized()
import data  # noqa: E402,F401   train.py:17
import models  # noqa: E402,F401  train.py:18
import trainers  # noqa: E402     train.py:19

from test_ddp_training import GLOBAL_B, _GridToy, _global_batch, _run, _shard  # noqa: E402


def main(out):
    assert dist.is_initialized(), "importing the mirror's packages under torchrun must open the group"
    world, rank = dist.get_world_size(), dist.get_rank()
    assert dist.get_backend() == "gloo"
    torch.set_num_threads(1)
    torch.manual_seed(100 + rank)      # rank 1 builds different parameters: the trainer broadcasts rank 0's
    random.seed(1000 + rank)           # ... and a different Python RNG state
    model = _GridToy().to("cpu")       # train.py:32
    import argparse
    from common.interfaces import D
    cfg = argparse.Namespace(device="cpu", batch_size=GLOBAL_B // world, time_window=2, base_resolution=(10, 6, 6),
                             neighbors=3, lr_step_interval=1, unrolling=2, nr_gt_steps=1, num_epochs=1)
    tr = getattr(trainers, "AutoregressivePushforwardTrainer")(  # train.py:70
        model=model, data=argparse.Namespace(data_interface=D.sim2d, pde=None, train=None, valid=None, test=None),
        config=cfg, criterion=torch.nn.MSELoss(reduction="sum"), save_path="unused")
    assert tr.grad_sync is not None and tr.world == world
    b = _global_batch()
    lo, hi = rank * GLOBAL_B // world, (rank + 1) * GLOBAL_B // world
    train_loader = [_shard(b, lo, hi), _shard(_global_batch(seed=2), lo, hi)]
    v = _global_batch(5, seed=3)
    val = [_shard(v, 0, 2), _shard(v, 2, 3)] if rank == 0 else [_shard(v, 3, 5)]
    res = _run(tr, train_loader, val)
    torch.save(dict(rank=rank, world=world, res=res), os.path.join(out, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1])
