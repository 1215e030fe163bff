"""Dev diagnostic: the failing fused-prologue test case run first in a fresh process."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "neural-pde-surrogates_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from conftest import rel_l2  # noqa: E402
from nps_hip import ops  # noqa: E402

for rep in range(3):
    for cin, cout, g, pad, xs in [(196, 75, 1, 1, 3e3), (196, 75, 1, 1, 1.0), (196, 75, 1, 0, 3e3), (192, 75, 1, 1, 3e3)]:
        torch.manual_seed(11)
        B, H, W = 2, 21, 18
        x = torch.randn(B, cin, H, W) * xs + 0.2 * xs
        gamma = torch.rand(cin) + 0.5
        beta = torch.rand(cin) - 0.5
        w = torch.randn(cout, cin, 1, 1) * 0.05
        b = torch.randn(cout) * 0.1
        ref = F.conv2d(F.gelu(F.group_norm(x.double(), g, gamma.double(), beta.double(), 1e-5)), w.double(),
                       b.double(), padding=pad)
        xd = ops.nchw_to_nhwc(x.to("cuda"))
        st = ops.group_norm_stats([ops.Src(xd)], (H, W), g)
        gn = ops.GN(st, gamma.to("cuda"), beta.to("cuda"), g, 1e-5)
        y = ops.conv2d([ops.Src(xd)], (H, W), ops.pack_conv_weight(w.to("cuda")), b.to("cuda"), cout, 1, 1,
                       pad=(pad, pad), gn=gn, pre_act=1)
        yc = ops.nhwc_to_nchw(y).cpu()
        print(rep, cin, cout, g, pad, xs, rel_l2(yc, ref), "stats", st.cpu().tolist(), flush=True)
