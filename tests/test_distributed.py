"""CPU (gloo, world_size 2) tests of the data-parallel gradient all-reduce (trainers/distributed.py) and the
batch sharding the rollout bench uses.  The same code runs over RCCL on the MI355X node."""
import os
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _init_file():
    """A fresh file:// rendezvous (no TCP port to race for with other processes or earlier cases)."""
    d = tempfile.mkdtemp(prefix="nps_pg_")
    return os.path.join(d, "init")


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


def _worker(rank, world, init_file, bucket_bytes, overlap, q):
    dist.init_process_group("gloo", init_method="file://" + init_file, rank=rank, world_size=world)
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
    # numpy copies travel by value: torch tensors would go through a file-descriptor server that dies with
    # this process, racing the parent's unpickling (the round-2 flake)
    q.put((rank, {k: p.grad.clone().numpy() for k, p in m.named_parameters()}, len(sync.buckets)))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("bucket_bytes,overlap", [(64, True), (1 << 20, True), (64, False)])
def test_grad_allreduce_matches_full_batch(bucket_bytes, overlap):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init_file = _init_file()
    procs = [ctx.Process(target=_worker, args=(r, world, init_file, bucket_bytes, overlap, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # reference: gradient of the sum of the two shard losses = sum of per-shard gradients (GradAllReducer
    # sums: each rank's loss is its share of the global loss, trainers/distributed.py)
    m = _Toy()
    x = torch.randn(8, 6, generator=torch.Generator().manual_seed(1))
    grads = []
    for r in range(world):
        m.zero_grad()
        m(x[r * 4:(r + 1) * 4]).backward()
        grads.append({k: (p.grad.clone() if p.grad is not None else torch.zeros_like(p))
                      for k, p in m.named_parameters()})
    want = {k: grads[0][k] + grads[1][k] for k in grads[0]}
    for rank, got, nb in res:
        if bucket_bytes == 64:
            assert nb > 1
        for k in want:
            torch.testing.assert_close(torch.from_numpy(got[k]), want[k], rtol=1e-6, atol=1e-6)


# ----------------------------------------------------------------- model-shaped all-reduce, shards, bench
class _ModelShaped(torch.nn.Module):
    """The U-FNO block's parameter shapes: SpectralConv2d weights1/weights2 complex (196, 192, 10, 10), a
    3x3 conv (192, 196, 3, 3) + bias, a GroupNorm affine pair and a 1x1 conv (278 MB of
    gradients for the full model, reduced as real pairs in several buckets)."""

    def __init__(self):
        super().__init__()
        g = torch.Generator().manual_seed(0)
        s = 1.0 / (196 * 192)
        self.w1 = torch.nn.Parameter(s * torch.rand(196, 192, 10, 10, dtype=torch.cfloat, generator=g))
        self.w2 = torch.nn.Parameter(s * torch.rand(196, 192, 10, 10, dtype=torch.cfloat, generator=g))
        self.conv = torch.nn.Parameter(0.02 * torch.randn(192, 196, 3, 3, generator=g))
        self.bias = torch.nn.Parameter(0.1 * torch.randn(192, generator=g))
        self.gamma = torch.nn.Parameter(1 + 0.1 * torch.randn(196, generator=g))
        self.beta = torch.nn.Parameter(0.1 * torch.randn(196, generator=g))
        self.pw = torch.nn.Parameter(0.05 * torch.randn(192, 196, generator=g))

    def forward(self, x):  # x (B, 196, 20, 20): a spectral-style contraction + a conv + a pointwise map
        xf = torch.fft.rfft2(x)[:, :, :10, :10]
        y = torch.einsum("bixy,ioxy->boxy", xf, self.w1) + torch.einsum("bixy,ioxy->boxy", xf.conj(), self.w2)
        h = torch.nn.functional.group_norm(x, 1, self.gamma, self.beta)
        c = torch.nn.functional.conv2d(h, self.conv, self.bias)
        p = torch.einsum("oi,bixy->boxy", self.pw, x)
        return (y.abs() ** 2).sum() + (c ** 2).mean() + p.square().mean()


def _model_worker(rank, world, init_file, q, done):
    dist.init_process_group("gloo", init_method="file://" + init_file, rank=rank, world_size=world)
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, "neural-pde-surrogates_amd"), os.path.join(root, "tests")]
    from trainers.distributed import GradAllReducer
    import bench
    torch.set_num_threads(2)
    m = _ModelShaped()
    sync = GradAllReducer(m.parameters(), bucket_bytes=16 * 1024 * 1024, average=True)
    sync.broadcast_parameters(0)
    x = torch.randn(4, 196, 20, 20, generator=torch.Generator().manual_seed(1))
    lo, hi = bench.shard_bounds(4, world, rank)
    m.zero_grad()
    m(x[lo:hi]).backward()
    sync.finish()
    grads = {k: p.grad.clone() for k, p in m.named_parameters()}
    # data shards of a DeviceLoader over an on-disk split (DistributedSampler semantics)
    from data_fixture import write_twophase_dataset, DATASET_KW
    from data import PDE2DDataset, DeviceLoader
    import tempfile
    d = tempfile.mkdtemp() if rank == 0 else None
    obj = [d]
    dist.broadcast_object_list(obj, src=0)
    if rank == 0:
        write_twophase_dataset(obj[0], shape=(10, 8, 11, 8, 6), with_split=False)
    dist.barrier()
    ds = PDE2DDataset(base_path=obj[0], **dict(DATASET_KW, split_file=None, split_val=0.0, split_test=0.0))
    dl = DeviceLoader(ds.test, batch_size=2, shuffle=True, device="cpu", num_replicas=world, rank=rank)
    shards = {}
    for epoch in (0, 1):
        dl.set_epoch(epoch)
        seen = [int(i) for b in dl for i in b[1].flatten(1).sum(1).mul(1e4).round().tolist()]
        allseen = [None] * world
        dist.all_gather_object(allseen, seen)
        shards[epoch] = allseen
    elapsed = bench.max_over_ranks(1.0 + rank, torch.device("cpu"))
    times = bench.per_rank_times(1.0 + rank, torch.device("cpu"))
    info = bench.dist_info(world)
    q.put((rank, grads, len(sync.buckets), (lo, hi), shards, (elapsed, times, info)))
    done.wait(timeout=120)  # keep the tensors' shared memory alive until the parent has received them
    dist.destroy_process_group()


def test_model_shaped_allreduce_shards_and_bench_reduction():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    done = ctx.Event()
    init_file = _init_file()
    procs = [ctx.Process(target=_model_worker, args=(r, world, init_file, q, done)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=150) for _ in range(world)], key=lambda r: r[0])
    done.set()
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    m = _ModelShaped()
    x = torch.randn(4, 196, 20, 20, generator=torch.Generator().manual_seed(1))
    m.zero_grad()
    (m(x[:2]) + m(x[2:])).div(2).backward()  # 1-process gradient of the mean of the two shard losses
    want = {k: p.grad for k, p in m.named_parameters()}
    for rank, grads, nb, (lo, hi), shards, (elapsed, times, info) in res:
        assert nb >= 3  # 60 MB of complex weights + the rest in 16 MB buckets
        assert (lo, hi) == (2 * rank, 2 * rank + 2)
        assert elapsed == 2.0  # the slowest rank's time on every rank
        assert times == [1.0, 2.0]  # every rank's own time, in rank order
        assert info["backend"] == "gloo" and info["world_size"] == 2
        for k in want:
            torch.testing.assert_close(grads[k], want[k], rtol=1e-5, atol=1e-7)
    # every epoch: the ranks' shards are disjoint and cover the 10-sample split exactly once
    shards = res[0][4]
    ds_ids = None
    for epoch, per_rank in shards.items():
        allids = sorted(per_rank[0] + per_rank[1])
        assert len(per_rank[0]) == len(per_rank[1]) == 5
        assert len(set(allids)) == 10
        ds_ids = allids if ds_ids is None else ds_ids
        assert allids == ds_ids
    assert shards[0][0] != shards[1][0]  # set_epoch reshuffles


def test_bench_traffic_keyed_on_per_gpu_workload():
    """bench.py attaches the committed PMC bytes per launch only to the per-GPU workload those passes
    profiled; at N > 1 (per-GPU batch 16/N) or any other workload traffic is null, with the reason."""
    import bench
    roof = dict(kclass="x3f16_9tap", traffic=None)
    got = bench.attach_traffic(dict(roof), dict(bench.PMC_WORKLOAD))
    assert got["traffic"] is not None and got["traffic"] > 1e8
    for n in (2, 4, 8):
        w = dict(bench.PMC_WORKLOAD, per_gpu_batch=16 // n)
        got = bench.attach_traffic(dict(roof), w)
        assert got["traffic"] is None and "no PMC pass" in got["traffic_note"]


def test_rank_device_guard():
    """a rank whose model sits on another card (train.py's cfg device `cuda:0` under torchrun)
    is refused before any collective runs; the rank's own card, an index-less 'cuda' and CPU parameters pass.
    (torch.device objects only: no CUDA call is made.)"""
    from trainers.distributed import check_rank_device

    class P:
        def __init__(self, dev):
            self.device = torch.device(dev)

    check_rank_device([P("cuda:3"), P("cuda:3")], current_device=3)
    check_rank_device([P("cuda"), P("cpu")], current_device=5)
    check_rank_device([P("cpu")])  # no CUDA parameter: nothing to check, no CUDA call
    with pytest.raises(RuntimeError, match="cuda:0"):
        check_rank_device([P("cuda:3"), P("cuda:0")], current_device=3)
