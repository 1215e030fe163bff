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


class DeviceLoader:
    """Iterable of batches (u_base, u, x, conditioning, t_conditioning, spatial_conditioning) on `device`,
    the default-collated layout of the reference's DataLoader over the same dataset.

    shuffle: a fresh permutation per epoch from `generator` (torch.Generator) or torch's global RNG, as
    RandomSampler.  prefetch: batches read / in flight ahead of the consumer."""

    def __init__(self, dataset, batch_size: int, shuffle: bool = False, drop_last: bool = False,
                 device="cuda", prefetch: int = 2, generator: Optional[torch.Generator] = None):
        self.base, self.indices = _base_and_indices(dataset)
        self.batch_size = int(batch_size)
        self.shuffle = shuffle
        self.drop_last = drop_last
        self.device = torch.device(device)
        self.prefetch = max(1, int(prefetch))
        self.generator = generator

    def __len__(self):
        n = len(self.indices)
        return n // self.batch_size if self.drop_last else (n + self.batch_size - 1) // self.batch_size

    def _batches(self):
        order = self.indices
        if self.shuffle:
            perm = torch.randperm(len(order), generator=self.generator).numpy()
            order = order[perm]
        for i in range(len(self)):
            yield order[i * self.batch_size:(i + 1) * self.batch_size]

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
