"""Dev tool (GPU box): every conv launch of one C3 model call with its geometry and HIP-event time.

python tools/call_shapes.py [--model ufno --res 256 --b 16] [--train]   -> one line per launch, then per-shape
totals (--train: one pushforward training step, forward + backward incl. weight gradients, as bench.py --mode train)
"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "neural-pde-surrogates_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from nps_hip import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="ufno")
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--b", type=int, default=16)
    ap.add_argument("--num-c", type=int, default=3)
    ap.add_argument("--train", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda")
    ops.SIDE_STREAM = False  # one stream: a forked launch would be timed from its dispatch (bench.probe_roofline)
    if a.train:
        return train_shapes(a, dev)
    model, _, _ = bench.build_model(a.model, a.res, a.num_c, dev)
    from trainers.synthetic import twophase_batch
    u, cond, pos, sc = twophase_batch(B=a.b, num_c=a.num_c, T=50, H=a.res, W=a.res, seed=1)
    x = u[:, :, :25].to(dev)
    cond, pos, sc = cond.to(dev), pos.to(dev), sc.to(dev)
    with torch.no_grad():
        for _ in range(2):
            model(x, cond=cond, bc=None, pos=pos, t_cond=None, spatial_cond=sc)
        torch.cuda.synchronize()
        ops.conv_probe, ops.conv_shape_log = [], []
        model(x, cond=cond, bc=None, pos=pos, t_cond=None, spatial_cond=sc)
        torch.cuda.synchronize()
    report()


def train_shapes(a, dev):
    import types
    import torch.nn as nn
    from common.interfaces import D
    from trainers.autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer
    from trainers.synthetic import twophase_batch
    tw = 25
    model, _, _ = bench.build_model(a.model, a.res, a.num_c, dev)
    model.train()
    u, cond, pos, sc = twophase_batch(a.b, a.num_c, 2 * tw, a.res, a.res, seed=1234, obstacle="disc", device=dev)
    batch = (u[:, :, :1], u, pos, cond, torch.empty(a.b, 0, device=dev), sc)
    cfg = types.SimpleNamespace(time_window=tw, base_resolution=(2 * tw, a.res, a.res), device=dev,
                                batch_size=a.b, lr_step_interval=25, unrolling=0)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    tr = AutoregressivePushforwardTrainer(model=model, data=types.SimpleNamespace(pde=model.pde, data_interface=D.sim2d),
                                          criterion=nn.MSELoss(reduction="sum"), optimizer=opt, config=cfg)
    for _ in range(2):
        tr.train_one_epoch([batch], epoch=0)
    torch.cuda.synchronize()
    ops.conv_probe, ops.conv_shape_log = [], []
    tr.train_one_epoch([batch], epoch=0)
    torch.cuda.synchronize()
    report()


def report():
    tot = collections.defaultdict(lambda: [0, 0.0, 0.0])
    for (e0, e1, fl, cls, nb), d in zip(ops.conv_probe, ops.conv_shape_log):
        ms = e0.elapsed_time(e1)
        print(f"{ms * 1e3:8.1f} us  {fl / ms / 1e9:7.1f} TF/s  {nb / ms / 1e9:6.2f} TB/s  {cls}  {d}")
        key = (d["k"], d["cin"], d["cout"], d["out"], d["nsrc"], d["acc"], d["addends"], d["act"], d["gn"], d["stats"],
               cls[0])
        t = tot[key]
        t[0] += 1
        t[1] += ms
        t[2] += nb
    print("--- per shape: launches, ms, TB/s (algorithmic bytes)")
    for k, (n, ms, nb) in sorted(tot.items(), key=lambda kv: -kv[1][1]):
        print(f"{n:3d} {ms:8.3f} ms {nb / ms / 1e9:6.2f} TB/s  k={k[0]} cin={k[1]} cout={k[2]} out={k[3]} nsrc={k[4]} "
              f"acc={k[5]} add={k[6]} act={k[7]} gn={k[8]} stats={k[9]} {k[10]}")


if __name__ == "__main__":
    main()
