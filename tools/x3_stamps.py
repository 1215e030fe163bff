"""Dev diagnostic: per-work-group timing of the split-fp16 conv from the NPS_X3_STAMP build.

NPS_HIP_LIB=.../libnps_x3stamp.so python tools/x3_stamps.py [--cin 192 --cout 192 --k 3 --hw 258 --b 16]
Prints the in-kernel clock (s_memtime / s_memrealtime x 100 MHz) and the median prologue / main-loop /
epilogue cycles per work-group against the MFMA-only cycles of the main loop.
"""
import argparse
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "neural-pde-surrogates_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from nps_hip import lib, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=192)
    ap.add_argument("--cout", type=int, default=192)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--hw", type=int, default=258)
    ap.add_argument("--b", type=int, default=16)
    ap.add_argument("--gn", type=int, default=0, help="1: fused GroupNorm(1) + GELU prologue")
    a = ap.parse_args()
    x = torch.randn(a.b, a.hw, a.hw, a.cin, device="cuda")
    w = torch.randn(a.cout, a.cin, a.k, a.k, device="cuda") * 0.05
    wp = ops.pack_conv_weight(w)
    kw = {}
    if a.gn:
        st = ops.group_norm_stats([ops.Src(x)], (a.hw, a.hw), 1)
        kw = dict(gn=ops.GN(st, torch.rand(a.cin, device="cuda") + 0.5, torch.rand(a.cin, device="cuda") - 0.5, 1,
                            1e-5), pre_act=1)
    for _ in range(5):
        out = ops.conv2d([ops.Src(x)], (a.hw, a.hw), wp, None, a.cout, a.k, a.k, **kw)
    torch.cuda.synchronize()
    ho = out.shape[1]
    n = 1 << 20
    buf = (ctypes.c_ulonglong * n)()
    fn = lib.nps_x3_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert fn(ctypes.addressof(buf), n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 16).astype(np.int64)
    wide = os.environ.get("NPS_X3_WIDE", "1") != "0" and a.k in (2, 3) and 128 < a.cout <= 192
    tile = 128 if wide else (512 if a.hw >= 64 else 256)
    nwg = int(np.count_nonzero(st[:, 3]))
    st = st[:nwg]
    clk = (st[:, 3] - st[:, 0]) / np.maximum(st[:, 5] - st[:, 4], 1) * 100.0  # MHz
    pro, loop, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
    groups = ((a.cin + 15) // 16) * a.k * a.k
    ideal = groups * (3 * 2 if wide else 2 * (tile // 128)) * 3 * 32  # MFMAs per K-group per consumer wave
    span = (st[:, 5].max() - st[:, 4].min()) / 100.0  # us
    print(f"work-groups {nwg}, out {ho}x{ho}, span {span:.1f} us, clock median {np.median(clk):.0f} MHz")
    print(f"cycles per WG (median): prologue {np.median(pro):.0f}  loop {np.median(loop):.0f} "
          f"(MFMA-only {ideal})  epilogue {np.median(epi):.0f}; loop p10/p90 {np.percentile(loop, 10):.0f}/"
          f"{np.percentile(loop, 90):.0f}")
    print(f"epilogue split (median cycles): acc->LDS + barrier {np.median(st[:, 8] - st[:, 2]):.0f}, store phase "
          f"{np.median(st[:, 9] - st[:, 8]):.0f}, final barrier {np.median(st[:, 3] - st[:, 9]):.0f}; first 2 K-groups "
          f"{np.median(st[:, 7] - st[:, 1]):.0f} (MFMA-only {2 * ideal // groups})")
    print(f"loop efficiency {ideal / np.median(loop) * 100:.1f}%; consumer wave 0 waits at stage barriers "
          f"{np.median(st[:, 6]):.0f} cycles per WG (median)")


if __name__ == "__main__":
    main()
