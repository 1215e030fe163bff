"""Seeded synthetic two-phase trajectories (the real twophase dataset is not available offline).

u = 0.5 + 0.5 tanh((y - 0.3 - 0.4 t - 0.1 sin(2 pi x + phi)) / 0.05) + 0.02 U[0,1)
cond ~ U[0,1]^(B x 3); spatial_cond channel 0 = obstacle mask; pos = unit meshgrid (B, H, W, 2).
"""
import math

import torch


def twophase_batch(B, num_c, T, H, W, seed=1234, obstacle="random", device="cpu"):
    g = torch.Generator(device="cpu").manual_seed(seed)
    xs = torch.linspace(0, 1, H)
    ys = torch.linspace(0, 1, W)
    X, Y = torch.meshgrid(xs, ys, indexing="ij")
    phase = torch.rand(B, num_c, 1, 1, 1, generator=g) * 2 * math.pi
    noise_seed = int(torch.randint(0, 2 ** 31 - 1, (1,), generator=g))
    cond = torch.rand(B, 3, generator=g)
    if obstacle == "random":
        sc = (torch.rand(B, 1, H, W, generator=g) > 0.9).float()
    elif obstacle == "disc":
        sc = (((X - 0.5) ** 2 + (Y - 0.35) ** 2) < 0.1 ** 2).float()[None, None].repeat(B, 1, 1, 1)
    else:
        sc = torch.zeros(B, 1, H, W)
    pos = torch.stack([X, Y], dim=-1)[None].repeat(B, 1, 1, 1)
    dev = torch.device(device)
    ts = torch.linspace(0, 1, T, device=dev)
    Xd, Yd = X.to(dev), Y.to(dev)
    u = 0.5 + 0.5 * torch.tanh((Yd[None, None, None] - 0.3 - 0.4 * ts[None, None, :, None, None]
                                - 0.1 * torch.sin(2 * math.pi * Xd[None, None, None] + phase.to(dev))) / 0.05)
    gd = torch.Generator(device=dev).manual_seed(noise_seed)
    u = u + 0.02 * torch.rand(u.shape, generator=gd, device=dev)
    return u.float().contiguous(), cond.to(dev), pos.to(dev), sc.to(dev)
