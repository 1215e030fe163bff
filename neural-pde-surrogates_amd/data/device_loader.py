"""Device-resident batch loader: replaces the reference's DataLoader(pin_memory=True) + per-batch and
per-step `.to(device)` (trainers/base.py:157-179, 484; autoregressivepushforwardtrainer.py:105-106, 363-364).

A background thread reads each batch from the memmaps with one sorted fancy-indexed read per array
(MemMapDataset.load_batch), pins it, and issues the host->device copies on a dedicated HIP stream;
the consumer's stream waits on the copy's event, so the PCIe transfer of batch i+1 overlaps the
rollout / training step of batch i.  Everything the step touches afterwards (windows, labels,
conditioning) is already in HBM; windows are cut on the device by nps_gather_windows.
"""
import queue
import threading
from typing import Optional

import numpy as np
import torch
from torch.utils.data import Subset


def _base_and_indices(ds):
    """(MemMapDataset, absolute indices) of a MemMapDataset or a (nested) Subset of one."""
    idx = np.arange(len(ds))
    while isinstance(ds, Subset):
        idx = np.asarray(ds.indices)[idx]
        ds = ds.dataset
    if not hasattr(ds, "load_batch"):
        raise TypeError(f"DeviceLoader needs a MemMapDataset (or Subset of one), got {type(ds).__name__}")
    return ds, idx


def _draw_int64(generator):
    return int(torch.empty((), dtype=torch.int64).random_(generator=generator).item())


class DeviceLoader:
    """Iterable of batches (u_base, u, x, conditioning, t_conditioning, spatial_conditioning) on `device`,
    the default-collated layout of the reference's DataLoader over the same dataset.

    Sample order is the one torch's DataLoader would produce from the same RNG state, so a run driven by
    this loader sees the reference's batches (trainers/base.py:169-179: DataLoader(shuffle=True)):
      * single process: each epoch draws the iterator's base seed and then RandomSampler's seed from
        `generator` (torch's global RNG when None), exactly as DataLoader + RandomSampler do, and permutes
        with randperm on a generator seeded by the latter;
        With an explicit `generator`, a fully iterated epoch also draws the trailing randperm RandomSampler
        makes for its empty remainder slice (torch 2.10 sampler.py), so later epochs stay in step;
      * num_replicas > 1 (one process per GPU): the samples of `rank` under DistributedSampler semantics
         — a permutation seeded by `seed + epoch` (set_epoch), padded by wrapping (or cut
        with drop_last) to a multiple of num_replicas, rank r taking positions r, r + R, ...; the shards
        of one epoch are disjoint and cover the split once when its size divides by num_replicas.
        pad=False (evaluation): no wrap-around duplicates — rank r takes positions r, r + R, ... < n, so
        the shards differ in length by at most one sample and together are the split exactly once.
    prefetch: batches read / in flight ahead of the consumer."""

    def __init__(self, dataset, batch_size: int, shuffle: bool = False, drop_last: bool = False,
                 device="cuda", prefetch: int = 2, generator: Optional[torch.Generator] = None,
                 num_replicas: int = 1, rank: int = 0, seed: int = 0, pad: bool = True):
        self.base, self.indices = _base_and_indices(dataset)
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.device = torch.device(device)
        self.prefetch = max(1, int(prefetch))
        self.generator = generator
        if not (num_replicas >= 1 and 0 <= rank < num_replicas):
            raise ValueError(f"invalid rank {rank} of {num_replicas} replicas")
        self.num_replicas, self.rank, self.seed = int(num_replicas), int(rank), int(seed)
        self.pad = bool(pad)
        self.epoch = 0

    def set_epoch(self, epoch: int):
        """DistributedSampler.set_epoch: a different permutation per epoch, the same on every rank."""
        self.epoch = int(epoch)

    def _num_samples(self):
        n, R = len(self.indices), self.num_replicas
        if R == 1:
            return n
        if not self.pad:
            return len(range(self.rank, n, R))
        # DistributedSampler: with drop_last the tail that does not fill every replica is cut
        return (n - R) // R + 1 if (self.drop_last and n % R != 0) else -(-n // R)

    def __len__(self):
        n = self._num_samples()
        # drop_last of a sharded loader applies to the shard split (above), the batch split keeps the tail
        if self.drop_last and self.num_replicas == 1:
            return n // self.batch_size
        return (n + self.batch_size - 1) // self.batch_size

    def shard_positions(self):
        """Positions (into this split) of the samples this rank visits this epoch, in visiting order.
        Consumes RNG exactly as iterating a torch DataLoader over the same split does."""
        n = len(self.indices)
        _draw_int64(self.generator)  # DataLoader iterator base seed (drawn even with num_workers=0)
        if self.num_replicas == 1:
            if not self.shuffle:
                return torch.arange(n)
            if self.generator is None:  # RandomSampler without a generator: a private one, freshly seeded
                g = torch.Generator()
                g.manual_seed(_draw_int64(None))
            else:
                g = self.generator
            return torch.randperm(n, generator=g)
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            order = torch.randperm(n, generator=g)
        else:
            order = torch.arange(n)
        if not self.pad:
            return order[self.rank:n:self.num_replicas]
        total = self._num_samples() * self.num_replicas
        if total > n:
            order = order.repeat(-(-total // n))  # wrap-around padding
        order = order[:total]
        return order[self.rank:total:self.num_replicas]

    def _batches(self):
        order = self.indices[self.shard_positions().numpy()]
        for i in range(len(self)):
            yield order[i * self.batch_size:(i + 1) * self.batch_size]
        if self.num_replicas == 1 and self.shuffle and self.generator is not None:
            # RandomSampler.__iter__'s trailing randperm (num_samples % n == 0 remainder slice), drawn
            # when the epoch's iteration runs to its end
            torch.randperm(len(self.indices), generator=self.generator)

    def __iter__(self):
        if self.device.type != "cuda":
            for idx in self._batches():
                yield self.base.load_batch(idx)
            return
        yield from self._iter_device()

    def _iter_device(self):
        dev = self.device
        copy_stream = torch.cuda.Stream(device=dev)
        q = queue.Queue(maxsize=self.prefetch)
        stop = threading.Event()

        def producer():
            try:
                for idx in self._batches():
                    if stop.is_set():
                        return
                    host = [t.pin_memory() for t in self.base.load_batch(idx)]
                    with torch.cuda.stream(copy_stream):
                        dev_t = [t.to(dev, non_blocking=True) for t in host]
                        ev = torch.cuda.Event()
                        ev.record(copy_stream)
                    q.put((dev_t, host, ev))  # host buffers stay referenced until the copy is consumed
                q.put(None)
            except BaseException as e:  # surface loader errors in the consumer
                q.put(e)

        th = threading.Thread(target=producer, daemon=True)
        th.start()
        try:
            while True:
                item = q.get()
                if item is None:
                    return
                if isinstance(item, BaseException):
                    raise item
                dev_t, _host, ev = item
                cur = torch.cuda.current_stream(dev)
                cur.wait_event(ev)
                for t in dev_t:
                    t.record_stream(cur)  # allocated on copy_stream, consumed on the compute stream
                yield tuple(dev_t)
        finally:
            stop.set()
            while th.is_alive():
                try:
                    q.get_nowait()
                except queue.Empty:
                    pass
                th.join(timeout=0.05)
