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
                                                         ("nps_conv3d_t", "Conv3dArgs", "nps_src3_t", "Src3")])
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
