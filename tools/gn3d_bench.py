"""Dev micro-benchmark (GPU): nps_gn_stats3d / nps_frame_pack3d on C5-shaped bf16 frames vs a torch read of the
same bytes.  usage: python tools/gn3d_bench.py"""
import os
import sys
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "neural-pde-surrogates_amd"))
from nps_hip import ops  # noqa: E402


def timeit(f, n=20):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


B, D, H, W = 8, 16, 128, 128
dev = "cuda"
h = torch.randn(B, D, H, W, 64, device=dev).to(torch.bfloat16)
h68 = torch.randn(B, D, H, W, 68, device=dev).to(torch.bfloat16)
vb = torch.randn(B, D + 2, H + 2, W + 2, 4, device=dev).to(torch.bfloat16)
mb = lambda t: t.numel() * t.element_size() / 1e6
print(f"torch sum h (64ch, {mb(h):.0f} MB): {timeit(lambda: h.sum()):.1f} us")
for name, srcs, dhw in [("h 64ch exact", [ops.Src3(h)], (D, H, W)),
                        ("h68 exact", [ops.Src3(h68)], (D, H, W)),
                        ("h + vb(cropped, 4ch)", [ops.Src3(h), ops.Src3(vb, -1, -1, -1)], (D, H, W))]:
    t1 = timeit(lambda: ops.gn_stats3d(srcs, dhw, 1))
    st = ops.gn_stats3d(srcs, dhw, 1)
    C = sum(s.t.shape[-1] for s in srcs)
    gn = ops.GN(st, torch.ones(C, device=dev), torch.zeros(C, device=dev), 1, 1e-5)
    t2 = timeit(lambda: ops.frame_pack3d(srcs, dhw, gn, pre_act=1))
    t3 = timeit(lambda: ops.frame_pack3d(srcs, dhw, None, pre_act=0))
    by = B * D * H * W * C * 2 / 1e6
    print(f"{name}: gn_stats3d {t1:.1f} us ({by / t1:.2f} TB/s read), frame_pack3d GN+GELU {t2:.1f} us, "
          f"frame_pack3d copy {t3:.1f} us")
