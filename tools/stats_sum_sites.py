"""Dev tool (GPU box): histogram of the nps_stats_sum call sites (caller chain, parts, sub-slots) of one C3 model
call at B = 2.  python tools/stats_sum_sites.py"""
import collections, os, sys, traceback
ROOT = os.environ.get("GRAFT_REPO_ROOT", "/root/repo")
sys.path[:0] = [ROOT, os.path.join(ROOT, "neural-pde-surrogates_amd")]
import torch
import bench
from nps_hip import ops
dev = torch.device("cuda")
model, _, _ = bench.build_model("ufno", 256, 3, dev)
from trainers.synthetic import twophase_batch
u, cond, pos, sc = twophase_batch(B=2, num_c=3, T=50, H=256, W=256, seed=1)
x = u[:, :, :25].to(dev); cond, pos, sc = cond.to(dev), pos.to(dev), sc.to(dev)
cnt = collections.Counter()
orig = ops._stats_sum
def wrapped(parts, B, out):
    st = traceback.extract_stack(limit=4)[:-1]
    key = " <- ".join(f"{f.name}:{f.lineno}" for f in reversed(st)) + f" parts={len(parts)} sub={[p.shape[1] for p in parts]}"
    cnt[key] += 1
    return orig(parts, B, out)
with torch.no_grad():
    model(x, cond=cond, bc=None, pos=pos, t_cond=None, spatial_cond=sc)
    ops._stats_sum = wrapped
    model(x, cond=cond, bc=None, pos=pos, t_cond=None, spatial_cond=sc)
for k, v in cnt.most_common(): print(v, k)
print(sum(cnt.values()))
