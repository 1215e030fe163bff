"""CPU (gloo, world_size 2) tests of the data-parallel gradient all-reduce (trainers/distributed.py) and the
batch sharding the rollout bench uses.  The same code runs over RCCL on the MI355X node."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Toy(torch.nn.Module):
    """Real + complex parameters (like SpectralConv2d's weights1/weights2), one unused parameter."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(0)
        self.lin = torch.nn.Linear(6, 5)
        with torch.no_grad():
            self.lin.weight.copy_(torch.randn(5, 6, generator=g))
            self.lin.bias.copy_(torch.randn(5, generator=g))
        self.wc = torch.nn.Parameter(torch.randn(5, 3, dtype=torch.cfloat, generator=g))
        self.unused = torch.nn.Parameter(torch.ones(4))

    def forward(self, x):
        h = self.lin(x)
        z = torch.einsum("bi,io->bo", h.to(torch.cfloat), self.wc)
        return (z.real ** 2 + z.imag).sum()


def _worker(rank, world, port, bucket_bytes, overlap, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "neural-pde-surrogates_amd")]
    from trainers.distributed import GradAllReducer
    torch.manual_seed(0)
    m = _Toy()
    sync = GradAllReducer(m.parameters(), bucket_bytes=bucket_bytes, overlap=overlap)
    x = torch.randn(8, 6, generator=torch.Generator().manual_seed(1))
    for _ in range(2):  # two steps: the hook state resets between steps
        m.zero_grad()
        m(x[rank * 4:(rank + 1) * 4]).backward()
        sync.finish()
    q.put((rank, {k: p.grad.clone() for k, p in m.named_parameters()}, len(sync.buckets)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_bytes,overlap", [(64, True), (1 << 20, True), (64, False)])
def test_grad_allreduce_matches_full_batch(bucket_bytes, overlap):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, bucket_bytes, overlap, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # reference: gradient of the mean of the two shard losses = average of per-shard gradients
    m = _Toy()
    x = torch.randn(8, 6, generator=torch.Generator().manual_seed(1))
    grads = []
    for r in range(world):
        m.zero_grad()
        m(x[r * 4:(r + 1) * 4]).backward()
        grads.append({k: (p.grad.clone() if p.grad is not None else torch.zeros_like(p))
                      for k, p in m.named_parameters()})
    want = {k: (grads[0][k] + grads[1][k]) / 2 for k in grads[0]}
    for rank, got, nb in res:
        if bucket_bytes == 64:
            assert nb > 1
        for k in want:
            torch.testing.assert_close(got[k], want[k], rtol=1e-6, atol=1e-6)
