"""CPU checks of the C-ABI boundary: libnps_hip.so loads and exports every symbol include/nps.h declares
(no compute calls without a GPU), and the ctypes struct layouts match the header."""
import ctypes
import os
import re

from conftest import ROOT


def _header_functions():
    src = open(os.path.join(ROOT, "include", "nps.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nps_\w+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    import nps_hip
    names = _header_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(nps_hip.lib, n)]
    assert not missing, missing
    assert set(names) == set(nps_hip.EXPORTED), set(names) ^ set(nps_hip.EXPORTED)
    assert nps_hip.lib.nps_version().startswith(b"nps_hip")


import pytest


@pytest.mark.parametrize("cstruct,pyname,srcname,pysrc", [("nps_conv2d_t", "Conv2dArgs", "nps_src_t", "Src"),
                                                         ("nps_conv3d_t", "Conv3dArgs", "nps_src3_t", "Src3"),
                                                         ("nps_pack_job_t", "PackJob", "nps_src_t", "Src"),
                                                         ("nps_wgrad_t", "WgradArgs", "nps_src_t", "Src")])
def test_struct_layout_matches_header(cstruct, pyname, srcname, pysrc):
    """ctypes mirror vs a C compile of the header (offsetof / sizeof)."""
    import subprocess
    import tempfile
    import nps_hip
    Args, SrcT = getattr(nps_hip, pyname), getattr(nps_hip, pysrc)
    fields = [f for f, _ in Args._fields_]
    prog = "#include <stdio.h>\n#include <stddef.h>\n#include \"nps.h\"\nint main(){\n"
    prog += f'printf("%zu %zu\\n", sizeof({cstruct}), sizeof({srcname}));\n'
    for f in fields:
        prog += f'printf("%zu\\n", offsetof({cstruct}, {f}));\n'
    prog += "return 0;}\n"
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        open(c, "w").write(prog)
        exe = os.path.join(d, "t")
        subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), c, "-o", exe], check=True)
        out = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split()
    assert int(out[0]) == ctypes.sizeof(Args)
    assert int(out[1]) == ctypes.sizeof(SrcT)
    for f, off in zip(fields, out[2:]):
        assert getattr(Args, f).offset == int(off), f


def test_ops_refuse_cpu_tensors():
    """The product path has no CPU fallback: a CPU tensor is an error, not a silent torch path."""
    import pytest
    import torch
    from nps_hip import ops
    with pytest.raises(RuntimeError, match="MI355X"):
        ops.nchw_to_nhwc(torch.zeros(1, 2, 3, 4))


def _plan_args(Cin, Cout, k, H=40, W=36, pad=0, out_nchw=0, gn=False, nphase=1):
    import nps_hip
    from nps_hip import ops
    a = nps_hip.Conv2dArgs()
    a.nsrc = 1
    a.src[0].ptr, a.src[0].C, a.src[0].H, a.src[0].W = 0x1000, Cin, H, W
    a.B, a.Hin, a.Win, a.Cin = 2, H, W, Cin
    a.KH = a.KW = k
    a.stride, a.dil, a.pad_y, a.pad_x = 1, 1, pad, pad
    a.Hout, a.Wout = H + 2 * pad - k + 1, W + 2 * pad - k + 1
    a.Cout, a.out_C, a.out_H, a.out_W, a.out_os = Cout, Cout, a.Hout, a.Wout, 1
    a.out_nchw = out_nchw
    a.precision = ops.PREC_X3F16
    if gn:
        a.gn_stats, a.gn_gamma, a.gn_beta, a.gn_groups, a.gn_eps, a.pre_act = 0x2000, 0x3000, 0x4000, 1, 1e-5, 1
    if nphase > 1:
        a.nphase, a.phase_wstride = nphase, nps_hip.lib.nps_conv2d_packed_size(Cout, Cin, k * k)
    return a


@pytest.mark.parametrize("k", [1, 2, 3])
def test_x3_weight_reads_stay_inside_the_packing(k):
    """every split-fp16 conv launch reads its packed weight only inside the buffer, for the kernel the
    launcher picks (host arithmetic of nps_conv2d_x3_weight_span: block / chunk / K-group indices of each kernel,
    checked against nps_conv2d_packed_size) — at the packing boundaries (Cout 193, 385, 577: one past a 192-channel
    pack; 225, 256: the resident 1x1's two channel groups) and with channel tails (Cin 20, 36, 196, 388)."""
    import nps_hip
    lib = nps_hip.lib
    checked = 0
    for Cout in (4, 32, 64, 75, 128, 160, 192, 193, 196, 225, 256, 385, 388, 577, 600):
        for Cin in (4, 16, 20, 36, 84, 192, 196, 388):
            variants = [dict()]
            if k == 1:
                variants += [dict(out_nchw=1), dict(gn=True)]
            if k == 3:
                variants += [dict(gn=True), dict(pad=1)]
            if k == 2:
                variants += [dict(nphase=4)]
            for v in variants:
                if v.get("gn") and (k == 1 and Cout > 192):
                    continue  # (a 1x1 prologue needs the LDS-weight kernel: the host materialises the frame otherwise)
                a = _plan_args(Cin, Cout, k, **v)
                assert lib.nps_conv2d_plan(ctypes.byref(a)) >= 0, (Cin, Cout, k, v)
                span = lib.nps_conv2d_x3_weight_span(ctypes.byref(a))
                size = 4 * lib.nps_conv2d_packed_size(Cout, Cin, k * k) * v.get("nphase", 1)
                assert 0 < span <= size, (Cin, Cout, k, v, span, size)
                checked += 1
    assert checked > 100


def test_fork_gate_reads_the_planners_tiles():
    """the shortcut-fork gate (ops.last_round_idle) counts the tiles nps_conv2d_plan actually picks
    (ops.x3_plan_tiles), not an assumed 16 x 8 plan.  C3 shapes: the 258^2 conv1 at B = 2 leaves >= 25 % of a
    256-work-group grid idle in its last round (the shortcut forks), the 256^2 / 128-tile shapes fill exact rounds."""
    from nps_hip import ops
    for (Ho, Wo, B, Cout, Cin) in ((258, 258, 2, 192, 388), (256, 256, 2, 192, 192), (125, 125, 2, 192, 388),
                                   (258, 258, 16, 192, 388), (40, 36, 2, 64, 36)):
        a = _plan_args(Cin, Cout, 3, H=Ho + 2, W=Wo + 2)
        a.B = B
        assert ops.lib.nps_conv2d_plan(ctypes.byref(a)) >= 0
        nco = 192 if a.TH * a.TW == 128 else 64
        want = -(-Ho // a.TH) * -(-Wo // a.TW) * B * -(-Cout // nco)
        assert ops.x3_plan_tiles(Ho, Wo, B, Cout, Cin) == want
    assert ops.idle_fraction(ops.x3_plan_tiles(258, 258, 2, 192, 388), 256) >= ops.SIDE_MIN_IDLE
    assert ops.idle_fraction(ops.x3_plan_tiles(256, 256, 2, 192, 192), 256) == 0.0


def test_fused_synthesis_arguments_are_checked_on_the_host():
    """nps_conv2d_t.spec_z (the FNO layer's W-pass synthesis in the 1x1 epilogue) is refused by nps_conv2d_fwd's
    host checks — before any launch — outside its conditions (an accumulating conv, a 3x3, a row not a multiple of
    128 pixels, m2 > 16); ops.spectral_fusable mirrors them on the Python side."""
    import nps_hip
    from nps_hip import ops
    lib = nps_hip.lib
    bad = []
    for tweak in ("accumulate", "k3", "w", "m2"):
        k = 3 if tweak == "k3" else 1
        W = 200 if tweak == "w" else 256
        a = _plan_args(192, 192, k, H=8 + k - 1, W=W + k - 1)
        a.out = 0x5000
        a.wpack = 0x6000
        a.spec_z, a.spec_m2, a.spec_scale = 0x7000, (20 if tweak == "m2" else 10), 1.0 / (8 * W)
        if tweak == "accumulate":
            a.accumulate = 1
        assert lib.nps_conv2d_plan(ctypes.byref(a)) >= 0
        rc = lib.nps_conv2d_fwd(ctypes.byref(a), None)
        bad.append((tweak, rc, lib.nps_last_error().decode()))
    assert all(rc < 0 and "spec_z" in msg for _, rc, msg in bad), bad
    assert ops.spectral_fusable(256, 10, 192) == (ops.FUSE_IDFT and ops.CONV_PRECISION == ops.PREC_X3F16)
    assert not ops.spectral_fusable(200, 10, 192) and not ops.spectral_fusable(256, 17, 192)
    assert not ops.spectral_fusable(256, 10, 225)


def test_wgrad_workspace_holds_the_bias_row():
    """nps_wgrad_x3_ws_floats: the split-K partials [KH*KW][M][N] plus the bias-gradient row [M] (nps_wgrad_t.db)."""
    import nps_hip
    lib = nps_hip.lib
    for M, N, k in [(192, 388, 3), (196, 192, 1), (40, 768, 2)]:
        assert lib.nps_wgrad_x3_ws_floats(M, N, k, k) == M * N * k * k + M


def test_fp32_wgrad_refuses_the_bias_row():
    """The exact-fp32 weight gradient computes no bias gradient: a non-NULL db is an error, not a silent skip."""
    import ctypes
    import nps_hip
    p = nps_hip.WgradArgs()
    p.a, p.B, p.Ha, p.Wa, p.M = 0x1000, 1, 4, 4, 8
    p.x, p.Hx, p.Wx, p.N = 0x2000, 4, 4, 8
    p.KH = p.KW = 3
    p.dil, p.pad_y, p.pad_x, p.circ, p.g = 2, 1, 1, 0, 0x3000
    p.db = 0x4000
    assert nps_hip.lib.nps_conv2d_wgrad(ctypes.byref(p), None) < 0
    assert b"bias gradient" in nps_hip.lib.nps_last_error()
