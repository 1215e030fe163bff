"""Per-stage timing of the SpectralConv2d HIP pipeline at a given shape (default: the C3 FNO layer, B=16,
256x256, Cin 196 -> Cout 192, 10 modes): HIP-event time per launch, algorithmic bytes and the fraction of
the 8 TB/s HBM peak (MI355X_MICROARCH.md).  Algorithmic bytes per stage = its inputs read once + its
outputs written once (+ the packed weights for the mixer).  `--mix-valu` times the scalar-FMA mixer."""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "neural-pde-surrogates_amd")]
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=16)
    ap.add_argument("--hw", type=int, default=256)
    ap.add_argument("--cin", type=int, default=196)
    ap.add_argument("--cout", type=int, default=192)
    ap.add_argument("--m", type=int, default=10)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from nps_hip import lib, check, ptr, stream_ptr, ops
    B, H, W, Ci, Co, m = args.b, args.hw, args.hw, args.cin, args.cout, args.m
    R = min(H, 2 * m)
    dev = "cuda"
    c64 = torch.complex64
    x = torch.randn(B, H, W, Ci, device=dev)
    w1 = torch.rand(Ci, Co, m, m, dtype=c64, device=dev) / (Ci * Co)
    w2 = torch.rand(Ci, Co, m, m, dtype=c64, device=dev) / (Ci * Co)
    wp = ops.pack_spectral_weight(w1, w2, H)
    X1 = torch.empty(B, H, m, Ci, dtype=c64, device=dev)
    X2 = torch.empty(B, R, m, Ci, dtype=c64, device=dev)
    Y = torch.empty(B, R, m, Co, dtype=c64, device=dev)
    Z = torch.empty(B, H, m, Co, dtype=c64, device=dev)
    out = torch.empty(B, H, W, Co, device=dev)
    s = stream_ptr()
    src = ops._c_src([ops.Src(x)])
    stages = [
        ("dft_w", lambda: lib.nps_spectral_dft_w(src, 1, B, H, W, Ci, m, ptr(X1), s), x.numel() * 4 + X1.numel() * 8),
        ("dft_h", lambda: lib.nps_spectral_dft_h(ptr(X1), ptr(X2), B, H, m, m, Ci, s), X1.numel() * 8 + X2.numel() * 8),
        ("mix", lambda: lib.nps_spectral_mix(ptr(X2), ptr(wp), ptr(Y), B, R, m, Ci, Co, s),
         X2.numel() * 8 + wp.numel() * 8 + Y.numel() * 8),
        ("idft_h", lambda: lib.nps_spectral_idft_h(ptr(Y), ptr(Z), B, H, m, m, Co, s), Y.numel() * 8 + Z.numel() * 8),
        ("idft_w", lambda: lib.nps_spectral_idft_w(ptr(Z), ptr(out), B, H, W, m, Co, 0, None, 0, None, s),
         Z.numel() * 8 + out.numel() * 4),
    ]
    for name, fn, nbytes in stages:
        for _ in range(3):
            check(fn(), name)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.reps
        print(f"{name:7s} {ms * 1e3:8.1f} us  {nbytes / 1e6:8.1f} MB  {nbytes / (ms * 1e-3) / 1e12:6.2f} TB/s  "
              f"{nbytes / (ms * 1e-3) / 8e12:5.3f} of 8 TB/s", flush=True)


if __name__ == "__main__":
    main()
