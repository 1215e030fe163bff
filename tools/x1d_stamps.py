"""Dev diagnostic: per-work-group cycle split of the DMA-stream 1x1 conv (NPS_X3_STAMP build).

NPS_HIP_LIB=.../libnps_x3stamp.so python tools/x1d_stamps.py [--cin 388 --cout 192 --hw 260 --b 16]
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
    ap.add_argument("--cin", type=int, default=388)
    ap.add_argument("--cout", type=int, default=192)
    ap.add_argument("--hw", type=int, default=260)
    ap.add_argument("--b", type=int, default=16)
    a = ap.parse_args()
    x = torch.randn(a.b, a.hw, a.hw, a.cin, device="cuda")
    w = torch.randn(a.cout, a.cin, 1, 1, device="cuda") * 0.05
    wp = ops.pack_conv_weight(w)
    for _ in range(5):
        ops.conv2d([ops.Src(x)], (a.hw, a.hw), wp, None, a.cout, 1, 1)
    torch.cuda.synchronize()
    n = 1 << 20
    buf = (ctypes.c_ulonglong * n)()
    fn = lib.nps_x3_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    assert fn(ctypes.addressof(buf), n) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(-1, 16).astype(np.int64)
    nwg = int(np.count_nonzero(st[:, 4]))
    st = st[:nwg]
    clk = (st[:, 4] - st[:, 0]) / np.maximum(st[:, 9] - st[:, 8], 1) * 100.0
    tot = st[:, 4] - st[:, 0]
    U = np.median(st[:, 7])
    print(f"work-groups {nwg}, stages per WG {U:.0f}, clock median {np.median(clk):.0f} MHz, "
          f"span {(st[:, 9].max() - st[:, 8].min()) / 100.0:.1f} us")
    med = lambda v: float(np.median(v))  # noqa: E731
    print(f"MFMA wave 0 (median cycles per WG): total {med(tot):.0f}, start {med(st[:, 1] - st[:, 0]):.0f}, "
          f"barriers {med(st[:, 2]):.0f}, epilogues {med(st[:, 3]):.0f}; per stage {med(tot) / U:.0f}")
    print(f"loader wave 4: vmcnt waits {med(st[:, 5]):.0f}, barriers {med(st[:, 6]):.0f}")


if __name__ == "__main__":
    main()
