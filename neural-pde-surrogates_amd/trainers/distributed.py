"""Data-parallel training over RCCL/xGMI: bucketed gradient all-reduce overlapped with backward.

The reference has no distributed code (single process, single
device).  The MI355X build shards the batch over one process per GPU
(torch.distributed, backend "nccl" = RCCL on ROCm) and all-reduces gradients
once per optimizer step: trainers/base.py:492-493 becomes
`loss.backward(); grad_sync.finish(); optimizer.step()`.

The sharded step is the 1-process step on the concatenated global batch, not an
approximation of it.  The reference's training loss is sqrt(MSE_sum) over the
whole batch (autoregressivepushforwardtrainer.py:158-162), whose gradient is
∇S / (2·√S) with S = Σ_r S_r the ranks' squared-error sums.  Each rank therefore
all-reduces its fp64 S_r *before* backward (`global_sqrt_loss`) and backpropagates
S_r / (2·√S) — its exact share of the global gradient — and the gradients are
SUMMED over the ranks (`GradAllReducer`, op SUM, no 1/N).  `sync_python_random`
gives every rank rank 0's Python RNG state, so the per-step unroll depth and the
random start steps (drawn for the global batch, each rank taking its slice) are
those of the 1-process run.

Buckets are filled in reverse parameter order (the order backward produces
gradients) and each is launched as one asynchronous all-reduce the moment its
last gradient is accumulated, so RCCL's ring over xGMI overlaps the rest of
backward; `finish()` waits and writes the reduced (summed) gradients back.  Buckets are
launched strictly in index order so every rank issues the same collective
sequence.  Complex parameters (SpectralConv2d weights1/weights2) are reduced as
their float32 (re, im) pairs, the sum of which is the sum of the complex values.
"""
import random
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist

# ~64 MB buckets: U-FNO's 278 MB of gradients in 5 collectives, each large enough that the
# per-link (~150 GB/s) ring bandwidth of xGMI, not latency, bounds it
DEFAULT_BUCKET_BYTES = 64 * 1024 * 1024


def _flat(g: torch.Tensor) -> torch.Tensor:
    return torch.view_as_real(g).reshape(-1) if g.is_complex() else g.reshape(-1)


def world_and_rank(group=None):
    """(world_size, rank) of the default (or given) process group; (1, 0) without one."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def global_sqrt_loss(s_local: torch.Tensor, count_local: Optional[int] = None, group=None,
                     grad_scale: float = 1.0) -> torch.Tensor:
    """sqrt of a sum over the GLOBAL batch from this rank's part of it, with this rank's share of the
    global gradient.  Value: sqrt(S) (or sqrt(S / N) with element counts, nn.MSELoss(reduction='mean')),
    S = Σ_r s_r all-reduced in fp64 before backward.  Gradient: ∇s_local / (2·sqrt(S)) (/ N) — the
    ranks' gradients, summed by GradAllReducer, are ∇sqrt(S) of the 1-process step on the concatenated
    batch (autoregressivepushforwardtrainer.py:158-162: loss = torch.sqrt(criterion(pred, labels))).
    grad_scale multiplies the gradient only (not the value): the world size when the gradients are
    AVERAGED instead of summed (GradAllReducer(average=True), torch DDP)."""
    world, _ = world_and_rank(group)
    tot = s_local.detach().to(torch.float64).reshape(1).clone()
    if count_local is not None:
        tot = torch.cat([tot, torch.tensor([float(count_local)], dtype=torch.float64, device=tot.device)])
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM, group=group)
    S = tot[0] / tot[1] if count_local is not None else tot[0]
    scale = 1.0 / tot[1] if count_local is not None else 1.0
    root = torch.sqrt(S)
    out_dtype = torch.float32 if s_local.dtype == torch.float64 else s_local.dtype
    # value root; d/ds_local = scale / (2 root)
    share = (s_local - s_local.detach()).to(torch.float64) * (scale * grad_scale / (2.0 * root))
    return (root + share).to(out_dtype).reshape(s_local.shape)


def check_rank_device(params: Iterable, current_device: Optional[int] = None) -> None:
    """Raise when a rank's model sits on a GPU other than the one this rank is bound to.

    Under torchrun every rank binds its own card (`common/launch.py`: set_device(LOCAL_RANK)), but train.py takes the
    device string from the cfg (reference src/train.py:24,32) — `--trainer.device=cuda:0` would put every rank's model
    on card 0 and all ranks would silently share it.  Every CUDA parameter must be on `current_device` (default
    torch.cuda.current_device()); CPU parameters (gloo runs) are not checked."""
    cur = None
    for p in params:
        dev = p.device
        if dev.type != "cuda":
            continue
        if cur is None:
            cur = current_device if current_device is not None else torch.cuda.current_device()
        idx = dev.index if dev.index is not None else cur
        if idx != cur:
            raise RuntimeError(f"data-parallel rank bound to cuda:{cur} holds a model parameter on {dev}: give the "
                               f"trainer device as 'cuda' (this rank's card) instead of a fixed index, or bind the "
                               f"rank with torch.cuda.set_device before building the model")


def sync_python_random(group=None, src: int = 0):
    """Give every rank rank `src`'s Python `random` state (one object broadcast), so the unroll depth and
    start steps the trainer draws per step are the same on every rank and equal the 1-process draws."""
    world, rank = world_and_rank(group)
    if world == 1:
        return
    obj = [random.getstate() if rank == src else None]
    dist.broadcast_object_list(obj, src=src, group=group)
    random.setstate(obj[0])


class GradAllReducer:
    """Bucketed gradient all-reduce.  average=False (default): the SUM over the ranks, for losses whose
    per-rank backward is already its share of the global loss (global_sqrt_loss); average=True: the
    mean, for a loss that is the mean of per-rank losses."""

    def __init__(self, params: Iterable[torch.nn.Parameter], bucket_bytes: int = DEFAULT_BUCKET_BYTES,
                 group=None, overlap: bool = True, average: bool = False):
        self.group = group
        self.world = dist.get_world_size(group)
        self.average = bool(average)
        self.params: List[torch.nn.Parameter] = [p for p in params if p.requires_grad]
        self.buckets: List[List[int]] = []
        cur, cur_bytes = [], 0
        for i in reversed(range(len(self.params))):
            p = self.params[i]
            nbytes = p.numel() * p.element_size()
            if cur and cur_bytes + nbytes > bucket_bytes:
                self.buckets.append(cur)
                cur, cur_bytes = [], 0
            cur.append(i)
            cur_bytes += nbytes
        if cur:
            self.buckets.append(cur)
        self.bucket_of = {}
        for b, idxs in enumerate(self.buckets):
            for i in idxs:
                self.bucket_of[i] = b
        self.overlap = overlap
        self._hooks = []
        if overlap:
            for i, p in enumerate(self.params):
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
        self._reset()

    def _reset(self):
        self.ready = [0] * len(self.buckets)
        self.next = 0
        self.inflight = []

    def _make_hook(self, i):
        def hook(p):
            b = self.bucket_of[i]
            self.ready[b] += 1
            while self.next < len(self.buckets) and self.ready[self.next] == len(self.buckets[self.next]):
                self._launch(self.next)
                self.next += 1
        return hook

    def _launch(self, b):
        grads = []
        for i in self.buckets[b]:
            p = self.params[i]
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            grads.append(_flat(p.grad))
        buf = torch.cat(grads)
        if self.average:
            buf.div_(self.world)
        work = dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True)
        self.inflight.append((b, buf, work))

    def finish(self):
        """Launch what backward did not (unused parameters count as zero), wait, write the reduced grads back."""
        while self.next < len(self.buckets):
            self._launch(self.next)
            self.next += 1
        for b, buf, work in self.inflight:
            work.wait()
            off = 0
            for i in self.buckets[b]:
                g = _flat(self.params[i].grad)
                n = g.numel()
                g.copy_(buf[off:off + n])
                off += n
        self._reset()

    def broadcast_parameters(self, src: int = 0):
        """Make every rank start from rank `src`'s parameters (one collective per parameter)."""
        with torch.no_grad():
            for p in self.params:
                dist.broadcast(torch.view_as_real(p.data) if p.is_complex() else p.data, src, group=self.group)

    def remove(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
