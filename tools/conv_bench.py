"""Micro-benchmark of one fused conv launch shape (dev tool, not part of the product).

python tools/conv_bench.py [--cin 388 --cout 192 --k 3 --hw 260 --b 16 --gn 1 --iters 20]
Prints algorithmic TFLOP/s of nps_conv2d_fwd measured with HIP events; with --check compares a
B=1 slice against torch.nn.functional.conv2d on the CPU.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "neural-pde-surrogates_amd")]
import torch  # noqa: E402

from nps_hip import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=388)
    ap.add_argument("--cout", type=int, default=192)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--dil", type=int, default=1)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--circ", type=int, default=0)
    ap.add_argument("--hw", type=int, default=260)
    ap.add_argument("--b", type=int, default=16)
    ap.add_argument("--gn", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--prec", default="x3f16", choices=["x3f16", "f32"])
    ap.add_argument("--data", default="randn", choices=["randn", "zero", "const", "wzero"],
                    help="input / weight content (data-dependence of the kernel's clock: zero / constant operands)")
    a = ap.parse_args()
    ops.CONV_PRECISION = ops.PREC_F32 if a.prec == "f32" else ops.PREC_X3F16
    dev = "cuda"
    torch.manual_seed(0)
    x = torch.randn(a.b, a.hw, a.hw, a.cin, device=dev)
    w = torch.randn(a.cout, a.cin, a.k, a.k, device=dev) * (1.0 / (a.cin * a.k * a.k) ** 0.5)
    if a.data == "zero":
        x.zero_()
    elif a.data == "const":
        x.fill_(0.75)
    elif a.data == "wzero":
        w.zero_()
    bias = torch.randn(a.cout, device=dev)
    wp = ops.pack_conv_weight(w, a.stride, a.dil)
    gn = None
    if a.gn:
        st = ops.group_norm_stats([ops.Src(x)], (a.hw, a.hw), 1)
        gn = ops.GN(st, torch.rand(a.cin, device=dev) + 0.5, torch.rand(a.cin, device=dev) - 0.5, 1, 1e-5)
    kw = dict(stride=a.stride, dil=a.dil, circ=a.circ, gn=gn, pre_act=1 if a.gn else 0)
    out = ops.conv2d([ops.Src(x)], (a.hw, a.hw), wp, bias, a.cout, a.k, a.k, **kw)
    torch.cuda.synchronize()
    Ho, Wo = out.shape[1:3]
    flops = 2.0 * a.b * Ho * Wo * a.cout * a.cin * a.k * a.k
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        ops.conv2d([ops.Src(x)], (a.hw, a.hw), wp, bias, a.cout, a.k, a.k, out=out, **kw)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    print(f"conv[{a.prec}] cin={a.cin} cout={a.cout} k={a.k} d={a.dil} s={a.stride} hw={a.hw} B={a.b} gn={a.gn}: "
          f"{ms:.3f} ms  {flops / ms / 1e9:.1f} TFLOP/s  ({flops / ms / 1e9 / 157.3 * 100:.1f}% of fp32 MFMA peak)")
    if a.check:
        import torch.nn.functional as F
        for bi in sorted({0, a.b // 2, a.b - 1}):
            check_sample(a, x, gn, w, bias, out, bi)


def check_sample(a, x, gn, w, bias, out, bi):
    if True:
        import torch.nn.functional as F
        xc = x[bi:bi + 1].permute(0, 3, 1, 2).cpu()
        if a.gn:
            xc = F.gelu(F.group_norm(xc, 1, gn.gamma.cpu(), gn.beta.cpu(), 1e-5))
        if a.circ:
            xc = F.pad(xc, (a.circ,) * 4, mode="circular")
        ref = F.conv2d(xc, w.cpu(), bias.cpu(), stride=a.stride, dilation=a.dil)
        y = out[bi:bi + 1].permute(0, 3, 1, 2).cpu()
        err = (torch.linalg.vector_norm(y.double() - ref.double()) / torch.linalg.vector_norm(ref.double())).item()
        print(f"  sample {bi}: rel-L2 vs torch CPU: {err:.2e}")
        if err > 1e-5 and os.environ.get("NPS_DIAG"):
            d = (y.double() - ref.double()).abs()[0]  # (C, H, W)
            bad = d > 1e-3 * ref.double().abs().max()
            ch = bad.flatten(1).any(1).nonzero().flatten().tolist()
            ys, xs = bad.any(0).nonzero(as_tuple=True)
            print(f"    bad channels {ch[:8]}..{ch[-8:]} ({len(ch)}); bad px {bad.any(0).sum().item()} "
                  f"rows {sorted(set(ys.tolist()))[:40]} cols {sorted(set(xs.tolist()))[:40]}")


if __name__ == "__main__":
    main()
