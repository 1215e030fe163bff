"""Dev diagnostic: UNet golden (unet_ufno_style) forward, no-grad and grad, under the NPS_RANGE_TAGS setting."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "neural-pde-surrogates_amd"), os.path.join(ROOT, "tests")]
import torch
from torch import nn
from conftest import load_golden, rel_l2
from models.enc_proc_dec_components import UNetModern
for name in sys.argv[1:]:
    g = load_golden(name)
    kw = dict(g["kwargs"]); kw["activation"] = nn.GELU()
    m = UNetModern(pde=None, **kw); m.load_state_dict(g["state_dict"]); m = m.cuda()
    with torch.no_grad():
        y = m(h=g["h"].cuda(), variables_broadcast=g["vb"].cuda())
    e1 = rel_l2(y, g["y"])
    y2 = m(h=g["h"].cuda().requires_grad_(True), variables_broadcast=g["vb"].cuda())
    e2 = rel_l2(y2, g["y"])
    print(os.environ.get("NPS_RANGE_TAGS", "1"), name, "nograd", e1, "grad", e2, tuple(y.shape), flush=True)
    bad = (y.cpu() - g["y"]).abs().amax(dim=(2, 3))
    print("  per (b,c) max err > 1e-3:", (bad > 1e-3).nonzero().tolist()[:20])
