"""Data-parallel training reproduces the 1-process global-batch step.

World-size-2 gloo processes run the MIRROR's AutoregressivePushforwardTrainer (train_one_epoch, train_step,
test) on a torch-only grid model, each on its half of a global batch, and are compared against ONE process
on the concatenated batch:
  * the trainer wires data parallelism itself (as under an unchanged train.py + torchrun): rank 1 starts
    from different parameters and a different Python RNG state and still takes rank 0's;
  * every rank's gradient of the reference loss sqrt(MSE_sum) (autoregressivepushforwardtrainer.py:158-162)
    equals the 1-process gradient to 1e-6, and so do the logged epoch loss and the updated parameters
    (random unroll depth and start steps included: epoch 3 allows up to 2 no-grad unrolls);
  * test(): unpadded validation shards of different lengths give the 1-process sample-weighted loss.
The same code runs over RCCL on the MI355X node (the model there is the HIP one; the loss's local part is
the fp64 HIP reduction ad.mse_sum)."""
import argparse
import os
import random
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C, TW, T, H, W = 1, 2, 10, 6, 6
GLOBAL_B = 4


def _paths():
    for p in (os.path.join(ROOT, "neural-pde-surrogates_amd"),):
        if p not in sys.path:
            sys.path.insert(0, p)


class _GridToy(torch.nn.Module):
    """A time-bundled grid model with the reference's forward signature (enc_proc_dec.py:117)."""

    def __init__(self):
        super().__init__()
        from common.interfaces import D, M
        self.model_interface = M.AR_TB
        self.data_interface = [D.sim2d]
        self.conv = torch.nn.Conv2d(C * TW + 2 + 3, C * TW, 3, padding=1, padding_mode="circular")

    def forward(self, x, cond=None, bc=None, pos=None, t_cond=None, spatial_cond=None):
        B = x.shape[0]
        vb = cond[:, :, None, None].expand(B, cond.shape[1], H, W)
        h = torch.cat([x.flatten(1, 2), pos.permute(0, 3, 1, 2), vb], 1)
        return x + 0.1 * torch.tanh(self.conv(h)).view(B, C, TW, H, W)


def _global_batch(n=GLOBAL_B, seed=1):
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(n, C, T, H, W, generator=g)
    pos = torch.stack(torch.meshgrid(torch.linspace(0, 1, H), torch.linspace(0, 1, W), indexing="ij"), -1)
    pos = pos.expand(n, H, W, 2).contiguous()
    cond = torch.rand(n, 3, generator=g)
    # (u_base, u_super, x, conditioning, t_conditioning, spatial_conditioning): no baseline / t / spatial cond
    return (torch.empty(n, 0), u, pos, cond, torch.empty(n, 0), torch.empty(n, 0))


def _shard(batch, lo, hi):
    return tuple(t[lo:hi] for t in batch)


def _trainer(model, batch_size, grad_sync=None):
    from common.interfaces import D
    from trainers import AutoregressivePushforwardTrainer
    data = argparse.Namespace(data_interface=D.sim2d, pde=None, train=None, valid=None, test=None)
    config = argparse.Namespace(device="cpu", batch_size=batch_size, time_window=TW, base_resolution=(T, H, W),
                                neighbors=3, lr_step_interval=1, unrolling=2, nr_gt_steps=1, num_epochs=1)
    return AutoregressivePushforwardTrainer(model=model, data=data, criterion=torch.nn.MSELoss(reduction="sum"),
                                            config=config, save_path="unused", grad_sync=grad_sync)


def _run(tr, train_loader, val_loader):
    opt = torch.optim.SGD(tr.get_parameters(), lr=0.05)
    tr.set_optimizer(opt)
    ep_loss = tr.train_one_epoch(train_loader, epoch=3)
    grads = {k: p.grad.clone() for k, p in tr.model.named_parameters()}
    params = {k: p.detach().clone() for k, p in tr.model.named_parameters()}
    val_loss, metrics = tr.test(val_loader)
    return float(ep_loss), grads, params, float(val_loss), {k: float(v) for k, v in metrics.items()}


def _worker(rank, world, init_file, q, done, mode="auto"):
    _paths()
    dist.init_process_group("gloo", init_method="file://" + init_file, rank=rank, world_size=world)
    torch.set_num_threads(1)
    torch.manual_seed(100 + rank)       # rank 1 builds different parameters: the trainer broadcasts rank 0's
    random.seed(1000 + rank)            # ... and a different Python RNG state: the trainer broadcasts rank 0's
    model = _GridToy()
    if mode == "average":
        # an explicit, AVERAGING reducer ("an explicit grad_sync replaces it"): the caller
        # broadcasts the parameters; the trainer still syncs the Python RNG and scales the loss share's gradient
        from trainers.distributed import GradAllReducer
        gs = GradAllReducer(model.parameters(), average=True)
        gs.broadcast_parameters(0)
        tr = _trainer(model, GLOBAL_B // world, grad_sync=gs)
        assert tr.grad_sync is gs and tr.grad_world_scale == world
    else:
        tr = _trainer(model, GLOBAL_B // world)
        assert tr.grad_sync is not None and not tr.grad_sync.average and tr.grad_world_scale == 1
    b = _global_batch()
    lo, hi = rank * GLOBAL_B // world, (rank + 1) * GLOBAL_B // world
    train_loader = [_shard(b, lo, hi), _shard(_global_batch(seed=2), lo, hi)]
    # validation: 5 samples in batches of 2 -> rank 0 holds samples {0,1},{2} (two batches), rank 1 {3,4}
    v = _global_batch(5, seed=3)
    val = [_shard(v, 0, 2), _shard(v, 2, 3)] if rank == 0 else [_shard(v, 3, 5)]
    q.put((rank, _run(tr, train_loader, val)))
    done.wait(timeout=120)
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["auto", "average"])
def test_ddp_train_step_equals_one_process_global_batch(tmp_path, mode):
    world = 2
    ctx = mp.get_context("spawn")
    q, done = ctx.Queue(), ctx.Event()
    init_file = str(tmp_path / "pg_init")
    procs = [ctx.Process(target=_worker, args=(r, world, init_file, q, done, mode)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = []
        while len(res) < world:  # fail fast if a worker dies instead of waiting out the queue timeout
            try:
                res.append(q.get(timeout=2))
            except Exception:
                assert all(p.is_alive() or p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        res.sort(key=lambda r: r[0])
    finally:
        done.set()
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    _check_against_one_process(res)


def _one_process():
    """1 process, concatenated global batch, rank 0's initial parameters and Python RNG state."""
    _paths()
    torch.manual_seed(100)
    random.seed(1000)
    model = _GridToy()
    tr = _trainer(model, GLOBAL_B)
    assert tr.grad_sync is None
    v = _global_batch(5, seed=3)
    return _run(tr, [_global_batch(), _global_batch(seed=2)], [_shard(v, 0, 2), _shard(v, 2, 4), _shard(v, 4, 5)])


def _check_against_one_process(res):
    w_loss, w_grads, w_params, w_val, w_metrics = _one_process()
    for rank, (loss, grads, params, val, metrics) in res:
        assert loss == pytest.approx(w_loss, rel=1e-6)
        for k in w_grads:
            torch.testing.assert_close(grads[k], w_grads[k], rtol=1e-6, atol=1e-7)
            torch.testing.assert_close(params[k], w_params[k], rtol=1e-6, atol=1e-7)
        assert val == pytest.approx(w_val, rel=1e-6)
        assert metrics.keys() == w_metrics.keys()
        for k in w_metrics:
            assert metrics[k] == pytest.approx(w_metrics[k], rel=1e-6), k


def test_global_sqrt_loss_single_process_is_sqrt():
    _paths()
    from trainers.distributed import global_sqrt_loss
    x = torch.randn(7, dtype=torch.float64, requires_grad=True)
    s = (x ** 2).sum()
    out = global_sqrt_loss(s)
    out.backward()
    assert out.dtype == torch.float32  # fp64 sums (the HIP S_r) come back as the reference's fp32 loss
    torch.testing.assert_close(out.detach(), torch.sqrt(s.detach()).float())
    torch.testing.assert_close(x.grad, x.detach() / torch.sqrt(s.detach()))
    x.grad = None
    out = global_sqrt_loss((x ** 2).sum(), count_local=7)  # MSELoss(reduction='mean')
    out.backward()
    m = (x.detach() ** 2).mean()
    torch.testing.assert_close(out.detach(), torch.sqrt(m).float())
    torch.testing.assert_close(x.grad, x.detach() / (7 * torch.sqrt(m)))


def test_torchrun_train_py_without_wrapper(tmp_path):
    """An unchanged train.py under `torch.distributed.run --nproc-per-node 2`: no init_process_group, no
    sitecustomize — importing the mirror's data / models / trainers opens the group from torchrun's
    environment (common/launch.py), and the 2-rank run equals the 1-process global-batch run."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "NPS_AUTO_DIST"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port),
                        os.path.join(ROOT, "tests", "ddp_torchrun_scenario.py"), str(tmp_path)],
                       env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    res = []
    for rank in range(2):
        d = torch.load(tmp_path / f"rank{rank}.pt", weights_only=False)
        assert d["rank"] == rank and d["world"] == 2
        res.append((rank, d["res"]))
    _check_against_one_process(res)


def test_launch_env_parsing(monkeypatch):
    _paths()
    from common import launch
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR"):
        monkeypatch.delenv(k, raising=False)
    assert launch.torchrun_env() is None
    monkeypatch.setenv("WORLD_SIZE", "1")
    assert launch.torchrun_env() is None
    monkeypatch.setenv("WORLD_SIZE", "4")
    monkeypatch.setenv("RANK", "3")
    assert launch.torchrun_env() is None            # no rendezvous address: not a launcher's env
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    monkeypatch.setenv("LOCAL_RANK", "1")
    assert launch.torchrun_env() == (4, 3, 1)
