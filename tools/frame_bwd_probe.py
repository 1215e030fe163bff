"""Dev tool (GPU box): HBM rate of the training frame kernels (frame_pack forward, frame backward reduce + apply)
at the U-Net's frame shapes, B = 16.

python tools/frame_bwd_probe.py   -> per shape: ms and TB/s of algorithmic bytes (reduce: gy + src read; apply:
gy + src read, dsrc written; pack: src read, frame written)
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "neural-pde-surrogates_amd")]
import torch  # noqa: E402

from nps_hip import autograd as ad  # noqa: E402
from nps_hip.ops import Src  # noqa: E402


def run(B, H, W, chans, reps=10):
    dev = torch.device("cuda")
    srcs = [torch.randn(B, H, W, c, device=dev, requires_grad=True) for c in chans]
    C = sum(chans)
    norm = torch.nn.GroupNorm(1, C).to(dev)
    ss = [Src(t, 0, 0) for t in srcs]
    g = torch.randn(B, H, W, C, device=dev)
    for _ in range(2):
        y = ad.frame(ss, (H, W), norm, 1)
        y.backward(g)
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    tf = tb = 0.0
    for _ in range(reps):
        e[0].record()
        y = ad.frame(ss, (H, W), norm, 1)
        e[1].record()
        y.backward(g)
        e[2].record()
        torch.cuda.synchronize()
        tf += e[0].elapsed_time(e[1])
        tb += e[1].elapsed_time(e[2])
    n = 4.0 * B * H * W * C
    tf, tb = tf / reps, tb / reps
    print(f"B={B} {H}x{W} C={chans}: forward {tf:.3f} ms ({2 * n / tf / 1e9:.2f} TB/s incl. statistics), "
          f"backward {tb:.3f} ms ({5 * n / tb / 1e9:.2f} TB/s of reduce 2N + apply 3N)", flush=True)


if __name__ == "__main__":
    for hw, chans in [(258, (192, 196)), (256, (192,)), (125, (192, 196)), (123, (192,)), (260, (388,))]:
        run(16, hw, hw, chans)
