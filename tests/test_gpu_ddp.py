"""The PRODUCT model's data-parallel training step on the GPU (VERDICT r3 missing #3).

Two ranks share the box's one MI355X over gloo (the NPS_BENCH_REHEARSAL arrangement; the 8-GPU node uses RCCL,
the same code).  Each rank runs the mirror's HIP U-FNO — SpectralConv2d layers with complex weights, the U-Net
with its fused GroupNorm+GELU convs, the TimeConvDense decoder, the activation wrapper — through
`TrainInterface.train_one_epoch` (trainers/base.py:472-507) on its half of a global batch: the HIP fp64
`ad.mse_sum` feeds `global_sqrt_loss`, `GradAllReducer`'s post-accumulate hooks fire on the HIP autograd outputs
and the complex spectral gradients go through the bucketed SUM as (re, im) pairs.  Every rank's gradients
(complex included) and SGD-updated parameters must equal ONE process on the concatenated batch at rel-L2 < 1e-5
(reference: autoregressivepushforwardtrainer.py:43-163 with loss = sqrt(MSE_sum) at :158-162).  Rank 1 starts
from different parameters and Python RNG state; epoch 3 allows up to 2 no-grad unrolls, so the shared unroll
depth and the global-batch start-step draw are exercised."""
import os
import random
import sys
import types

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import rel_l2

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GLOBAL_B, T, RES, TW = 4, 100, 32, 25
TOL = 1e-5


def _paths():
    for p in (ROOT, os.path.join(ROOT, "neural-pde-surrogates_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)


def _batch(lo, hi, dev, seed):
    from trainers.synthetic import twophase_batch
    u, cond, pos, sc = twophase_batch(GLOBAL_B, 1, T, RES, RES, seed=seed, obstacle="disc")
    s = slice(lo, hi)
    n = hi - lo
    # collated (u_base, u_super, x, conditioning, t_conditioning, spatial_conditioning)
    return tuple(t.to(dev) for t in (u[s, :, :1], u[s], pos[s], cond[s], torch.empty(n, 0), sc[s]))


def _train(model_seed, rng_seed, lo, hi, dev):
    from torch import nn
    from common.interfaces import D
    from trainers.autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer
    import __graft_entry__
    m, _, _ = __graft_entry__._tiny_ufno(dev, seed=model_seed, num_c=1)
    m.train()
    random.seed(rng_seed)
    cfg = types.SimpleNamespace(time_window=TW, base_resolution=(T, RES, RES), device=dev, batch_size=hi - lo,
                                lr_step_interval=1, unrolling=2)
    tr = AutoregressivePushforwardTrainer(model=m, data=types.SimpleNamespace(pde=m.pde, data_interface=D.sim2d),
                                          criterion=nn.MSELoss(reduction="sum"), config=cfg)
    tr.set_optimizer(torch.optim.SGD(m.parameters(), lr=0.05))
    loader = [_batch(lo, hi, dev, 1), _batch(lo, hi, dev, 2)]
    loss = tr.train_one_epoch(loader, epoch=3)
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters()}
    params = {k: p.detach().cpu().clone() for k, p in m.named_parameters()}
    return float(loss), grads, params, tr.grad_sync is not None


def _worker(rank, world, init_file, q, done):
    _paths()
    torch.cuda.set_device(0)  # both ranks on the one GPU (rehearsal arrangement)
    dist.init_process_group("gloo", init_method="file://" + init_file, rank=rank, world_size=world)
    try:
        per = GLOBAL_B // world
        q.put((rank, _train(100 + rank, 1000 + rank, rank * per, (rank + 1) * per, torch.device("cuda", 0))))
    except BaseException as e:  # report instead of hanging the parent on the queue
        q.put((rank, repr(e)))
    done.wait(timeout=120)
    dist.destroy_process_group()


def test_hip_ufno_ddp_train_step_equals_one_process_global_batch(tmp_path):
    world = 2
    ctx = mp.get_context("spawn")
    q, done = ctx.Queue(), ctx.Event()
    procs = [ctx.Process(target=_worker, args=(r, world, str(tmp_path / "pg"), q, done)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = []
        while len(res) < world:
            try:
                res.append(q.get(timeout=2))
            except Exception:
                assert all(p.is_alive() or p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        res.sort(key=lambda r: r[0])
    finally:
        done.set()
        for p in procs:
            p.join(timeout=60)
    for rank, r in res:
        assert not isinstance(r, str), f"rank {rank}: {r}"
    _paths()
    w_loss, w_grads, w_params, synced = _train(100, 1000, 0, GLOBAL_B, torch.device("cuda", 0))
    assert not synced
    assert any(g.is_complex() for g in w_grads.values())  # the spectral weights are in the comparison
    for rank, (loss, grads, params, synced) in res:
        assert synced
        assert loss == pytest.approx(w_loss, rel=TOL)
        bad = [(k, rel_l2(grads[k], w_grads[k])) for k in w_grads if rel_l2(grads[k], w_grads[k]) >= TOL]
        assert not bad, f"rank {rank} gradients: {bad}"
        bad = [(k, rel_l2(params[k], w_params[k])) for k in w_params if rel_l2(params[k], w_params[k]) >= TOL]
        assert not bad, f"rank {rank} parameters: {bad}"
