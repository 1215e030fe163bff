"""Micro-benchmark of one nps_conv3d launch shape (dev tool, not part of the product).

python tools/conv3d_bench.py [--srcs 64,4 --cout 64 --k 1 --stride 1 --dhw 16,128,128 --b 8 --gn 0 --iters 20] [--save F]
Prints HIP-event time, algorithmic TB/s (sources + weights + output, bf16) and TFLOP/s.  --save writes the output
tensor (torch.save) so two processes with different dev knobs (e.g. NPS_C3D_1X1=0) can be compared bit for bit
with --compare F.
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
    ap.add_argument("--srcs", default="64,4")
    ap.add_argument("--cout", type=int, default=64)
    ap.add_argument("--k", type=int, default=1)
    ap.add_argument("--dhw", default="16,128,128")
    ap.add_argument("--b", type=int, default=8)
    ap.add_argument("--gn", type=int, default=0)
    ap.add_argument("--stride", type=int, default=1)
    ap.add_argument("--pack-only", type=int, default=0, help="time nps_frame_pack3d of the frame alone")
    ap.add_argument("--stats", type=int, default=1)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--save", default=None)
    ap.add_argument("--compare", default=None)
    a = ap.parse_args()
    dev = "cuda"
    torch.manual_seed(0)
    chans = [int(c) for c in a.srcs.split(",")]
    dhw = tuple(int(n) for n in a.dhw.split(","))
    srcs = [ops.Src3(torch.randn(a.b, *dhw, c, device=dev).to(torch.bfloat16)) for c in chans]
    cin = sum(chans)
    w = torch.randn(a.cout, cin, a.k, a.k, a.k, device=dev) / (cin * a.k ** 3) ** 0.5
    bias = torch.randn(a.cout, device=dev) * 0.1
    wp = ops.pack_conv3d_weight(w, bf16=True)
    gn = None
    if a.gn:
        gn = ops.GN(ops.gn_stats3d(srcs, dhw, 1), torch.ones(cin, device=dev), torch.zeros(cin, device=dev), 1, 1e-5)
    st = ops.new_stats(a.b, srcs[0].t) if a.stats else None

    def run():
        if a.pack_only:
            return ops.frame_pack3d(srcs, dhw, gn, 1 if a.gn else 0)
        return ops.conv3d(srcs, dhw, wp, bias, a.cout, a.k, stride=a.stride, gn=gn, pre_act=1 if a.gn else 0,
                          out_stats=st)

    y = run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.iters
    nv = a.b * ((dhw[0] - a.k) // a.stride + 1) * ((dhw[1] - a.k) // a.stride + 1) * ((dhw[2] - a.k) // a.stride + 1)
    nbytes = 2 * (sum(s.t.numel() for s in srcs) + w.numel() + nv * a.cout)
    if a.pack_only:  # frame in, padded frame out
        nbytes = 2 * (sum(s.t.numel() for s in srcs) + y.numel())
    fl = 2.0 * nv * a.cout * cin * a.k ** 3
    knob = os.environ.get("NPS_C3D_1X1", "1")
    if a.pack_only:
        print(f"frame_pack3d[bf16] srcs={a.srcs} dhw={a.dhw} B={a.b} gn={a.gn}: {ms * 1e3:.1f} us "
              f"{nbytes / ms / 1e9:.2f} TB/s", flush=True)
        fl = 0.0
    print(f"conv3d[bf16] srcs={a.srcs} cout={a.cout} k={a.k} dhw={a.dhw} B={a.b} gn={a.gn} knob={knob}: {ms * 1e3:.1f} us "
          f"{nbytes / ms / 1e9:.2f} TB/s {fl / ms / 1e9:.1f} TFLOP/s", flush=True)
    if a.save:
        torch.save(y.cpu(), a.save)
    if a.compare:
        ref = torch.load(a.compare, weights_only=True)
        same = torch.equal(ref, y.cpu())
        print(f"bit-identical to {a.compare}: {same}", flush=True)
        if not same:
            d = (ref.float() - y.cpu().float()).abs()
            print(f"  max |diff| {float(d.max()):.3e}, differing {int((d > 0).sum())} of {d.numel()}", flush=True)
            sys.exit(1)


if __name__ == "__main__":
    main()
