"""Dev diagnostic: per-work-group timeline of the LDS-weight 1x1 conv (conv1x1_wl_kernel) from the
NPS_X3_STAMP build (tools/build_stamp.sh).

NPS_HIP_LIB=.../libnps_x3stamp.so python tools/x1_stamps.py [--cin 196 --cout 192 --hw 256 --b 16]
Prints, for the last launch: work-groups, launch span, in-kernel clock, the median cycles of the weight
prologue / stage loop / epilogue (incl. the store drain) per work-group, the MFMA-only cycles of the loop,
and how many work-groups were resident at once (from the realtime start / end stamps).
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
    ap.add_argument("--cin", type=int, default=196)
    ap.add_argument("--cout", type=int, default=192)
    ap.add_argument("--hw", type=int, default=256)
    ap.add_argument("--b", type=int, default=16)
    a = ap.parse_args()
    x = torch.randn(a.b, a.hw, a.hw, a.cin, device="cuda")
    w = torch.randn(a.cout, a.cin, 1, 1, device="cuda") * 0.05
    wp = ops.pack_conv_weight(w)
    tag = ops.absmax(x)
    for _ in range(5):
        ops.conv2d([ops.Src(x)], (a.hw, a.hw), wp, None, a.cout, 1, 1, in_scale=tag)
    torch.cuda.synchronize()
    n = 1 << 20
    buf = (ctypes.c_ulonglong * n)()
    fn = lib.nps_x3_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert fn(ctypes.addressof(buf), n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 16).astype(np.int64)
    nwg = int(np.count_nonzero(st[:, 3]))
    st = st[:nwg]
    clk = (st[:, 3] - st[:, 0]) / np.maximum(st[:, 5] - st[:, 4], 1) * 100.0  # MHz
    pro, loop, epi = st[:, 1] - st[:, 0], st[:, 2] - st[:, 1], st[:, 3] - st[:, 2]
    t0, t1 = st[:, 4] - st[:, 4].min(), st[:, 5] - st[:, 4].min()  # realtime ticks (100 MHz)
    span = t1.max() / 100.0
    nst = (a.cin + 31) // 32
    ideal = nst * 2 * 6 * 3 * 32  # 2 K-groups x 6 co blocks x 3 passes x 32 cycles per stage, one wave
    grid = np.linspace(0, t1.max(), 200)
    resident = [int(np.count_nonzero((t0 <= g) & (t1 > g))) for g in grid]
    life = (t1 - t0) / 100.0
    print(f"work-groups {nwg}, span {span:.1f} us, clock median {np.median(clk):.0f} MHz")
    print(f"cycles per WG (median): weight prologue {np.median(pro):.0f}  stage loop {np.median(loop):.0f} "
          f"(MFMA-only one wave {ideal})  epilogue+drain {np.median(epi):.0f}")
    print(f"WG lifetime median {np.median(life):.2f} us (p10 {np.percentile(life, 10):.2f}, p90 "
          f"{np.percentile(life, 90):.2f}); resident WGs median {np.median(resident):.0f}, max {max(resident)}")
    starts = np.sort(t0) / 100.0
    print(f"start times: first 768 WGs by {starts[min(767, nwg - 1)]:.2f} us; WG starts per us (median gap "
          f"{np.median(np.diff(starts)) * 1e3:.1f} ns)")


if __name__ == "__main__":
    main()
