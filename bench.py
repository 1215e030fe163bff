"""Rollout throughput bench: U-FNO twophase cfg, 256x256, 3 fields, obstacle (BASELINE.json config C3).

python bench.py [--gpus N --steps K --warmup W]
  * one step = one autoregressive model call (advances tw=25 timesteps for every sample) plus the
    per-window MSE_sum loss, i.e. one iteration of AutoregressivePushforwardTrainer.simulate
    (reference trainers/autoregressivepushforwardtrainer.py:354-432), trajectory resident in HBM;
  * strong scaling: a fixed global batch (16) is sharded over the ranks (one process per GPU,
    torchrun); no collective inside the rollout, one barrier + max-reduction of the timings;
  * value = global samples x tw x K / max-over-ranks wall time  [sample-timesteps/s];
  * roofline: the dominant conv class (the split-fp16 implicit-GEMM kernel conv2d_x3_kernel<9,*> at C3),
    timed live with HIP events on its stream during one extra model call after the timed region:
    achieved = sum(algorithmic fp32 conv flops) / sum(kernel durations) vs the kernel's fp32-equivalent
    ceiling, 2.5 PF/s dense f16 MFMA / 3 products (MI355X_MICROARCH.md); traffic = PMC HBM bytes per
    launch from the committed profiles/pmc_traffic.json (tools/pmc_traffic.sh; FETCH_SIZE scaled per access
    shape as calibrated by tools/calib/pmc_calib.hip: x1 for the conv producers' 64-B reads);
  * cpu_baseline: the CPU oracle (oracle/, the reference restated in fp32 PyTorch-CPU) on a bounded
    sample (2 model calls at B=2, after one untimed warm-up call) on rank 0 only, with the GPU-vs-CPU
    rel-L2 of that sample.
  * --gpus N > 1 without torchrun: this process starts the N ranks itself (torch.distributed.run children,
    launch_ranks) before any GPU call; under a launcher, WORLD_SIZE must equal --gpus.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "neural-pde-surrogates_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

# bench.py opens its own process group (init_ranks); the mirror packages' torchrun bring-up
# (common/launch.py) must not open one first when run_fno3d imports models before init_ranks
os.environ.setdefault("NPS_AUTO_DIST", "0")

import torch  # noqa: E402
from torch import nn  # noqa: E402

FP32_MFMA_PEAK_TFLOPS = 157.3
ORACLE_PDE = dict(tmin=0.0, tmax=1.0, nt=501, n_cond_static=3, n_cond_spatial=1)

# cfg_twophase_*.py model dicts (reference src/configs/train/), wrapper args included
_WRAP = dict(activation_final=nn.Tanh(), enforce_spatial_cond=True, spatial_cond_channel=0,
             approx_volume_preserve=True, approx_volume_preserve_mode="individual_static", max_pct_dif=1 / 25,
             model_class="EncProcDec", num_spatial_dims=2, time_window=25, data_structure="grid",
             processor_residual=False, encoder="enc_grid.ElementWise", decoder="dec_grid.TimeConvDense",
             dec_delta_mode="per_step")
CFGS = {
    "ufno": dict(processor="UFNO", fno_modes=10, hidden_blocks=3, hidden_features=192, fno_kernel_size=1,
                 fno_conv_mode="single", padding_mode="circular", ch_mults=[1, 1], is_attn=[False, False],
                 mid_attn=False, norm=True, use1x1=True),
    "unet": dict(processor="UNetModern", ch_mults=[2, 2, 1, 2], is_attn=[False] * 4, mid_attn=False,
                 hidden_features=32, norm=True, use1x1=True, cond_mode="concat", padding_mode="circular",
                 dec_kernel_size=5, dec_padding_mode="circular"),
    "drn": dict(processor="DilatedResnet", kernel_size=5, hidden_blocks=2, hidden_features=128,
                padding_mode="circular", dec_kernel_size=5, dec_padding_mode="circular"),
}


def build_model(kind, res, num_c, device, fno_modes=None, seed=42):
    """Random-init (seed 42, configs/train/defaults/base.py:4) twophase model of the given cfg."""
    import models
    from pdes import PDE2D
    cfg = dict(_WRAP, activation=nn.GELU(), num_c=num_c, **CFGS[kind])
    if fno_modes is not None:
        cfg["fno_modes"] = fno_modes
    pde = PDE2D(tmin=ORACLE_PDE["tmin"], tmax=ORACLE_PDE["tmax"], nt=ORACLE_PDE["nt"], L1=1.0, L2=1.0, nx1=res,
                nx2=res, x=None, name="twophase", n_cond_static=3, n_cond_spatial=1)
    torch.manual_seed(seed)
    m = models.activation_wrapper(**cfg, pde=pde).to(device).eval()
    ocfg = {k: v for k, v in cfg.items() if k not in ("activation", "activation_final")}
    return m, ocfg, dict(ORACLE_PDE, nx1=res, nx2=res)


# dense MFMA peaks, MI355X_MICROARCH.md: f32 (v_mfma_f32_32x32x2_f32) 157.3 TF; f16 2.5 PF.  A split-fp16
# conv spends 3 f16 MFMA products per algorithmic fp32 product, so its fp32-equivalent ceiling is 2.5 PF / 3.
PEAK_TFLOPS = {"f32": FP32_MFMA_PEAK_TFLOPS, "x3f16": 2500.0 / 3.0, "f32w": FP32_MFMA_PEAK_TFLOPS,
               "x3w": 2500.0 / 3.0, "bf16_3d": 2500.0, "f32_3d": FP32_MFMA_PEAK_TFLOPS}
KERNEL_NAMES = {("x3f16", 9): "conv2d_x3_kernel<9,*> (3x3, split-fp16 MFMA)",
                ("x3f16", 4): "conv2d_x3_kernel<4,*> (2x2 phase / space-to-depth, split-fp16 MFMA)",
                ("x3f16", 1): "conv2d_x3_kernel<1,*> (1x1, split-fp16 MFMA)",
                ("x3f16", 25): "conv2d_x3_kernel<25,2> (5x5 dilated on the lattice, split-fp16 MFMA)",
                ("f32", 1): "conv2d_pc_kernel<1,32,2,3,2> (1x1, f32 MFMA)",
                ("f32w", 9): "wgrad_kernel (3x3 weight gradient, f32 MFMA)",
                ("f32w", 4): "wgrad_kernel (2x2 weight gradient, f32 MFMA)",
                ("f32w", 1): "wgrad_kernel (1x1 weight gradient, f32 MFMA)",
                ("x3w", 9): "wgrad_x3_kernel<3,3> (3x3 weight gradient, split-fp16 MFMA)",
                ("x3w", 4): "wgrad_x3_kernel<2,2> (2x2 weight gradient, split-fp16 MFMA)",
                ("x3w", 1): "wgrad_x3_kernel<1,1> (1x1 weight gradient, split-fp16 MFMA)",
                ("bf16_3d", 27): "conv3d_kernel<bf16,3,*> (3x3x3, bf16 MFMA)",
                ("bf16_3d", 8): "conv3d_kernel<bf16,2,1,8> (ConvTranspose3d phases, bf16 MFMA)",
                ("bf16_3d", 1): "conv3d_kernel<bf16,1,1,8> (1x1x1, bf16 MFMA)",
                ("f32_3d", 27): "conv3d_kernel<f32,3,*> (3x3x3, f32 MFMA)"}


def conv_roofline(model, x, cond, pos, sc):
    """One model call with every conv launch bracketed by HIP events on its stream; the roofline is
    reported for the conv class with the largest total time (the dominant kernel)."""
    def call():
        with torch.no_grad():
            model(x, cond=cond, bc=None, pos=pos, t_cond=None, spatial_cond=sc)
    return probe_roofline(call)


def probe_roofline(fn):
    """Run fn() with every conv / weight-gradient launch bracketed by HIP events on its stream
    (ops.conv_probe); roofline of the class with the largest total time.  The probe call runs on one stream
    (ops.SIDE_STREAM off): a launch on a side stream would be timed from its dispatch, including the wait for
    CUs a concurrent launch holds, not its own duration (the timed steps keep the side streams)."""
    from nps_hip import ops
    ops.conv_probe = []
    side, ops.SIDE_STREAM = ops.SIDE_STREAM, False
    try:
        fn()
        torch.cuda.synchronize()
    finally:
        probe, ops.conv_probe = ops.conv_probe, None
        ops.SIDE_STREAM = side
    groups = {}
    for e0, e1, f, (prec, ntaps, waves), nb in probe:
        g = groups.setdefault((prec, ntaps), [0.0, 0.0, 0, 0.0])
        g[0] += e0.elapsed_time(e1)
        g[1] += f
        g[2] += 1
        g[3] += nb
    key = max(groups, key=lambda k: groups[k][0])
    ms, flops, n, nbytes = groups[key]
    achieved = flops / (ms * 1e-3) / 1e12
    peak = PEAK_TFLOPS[key[0]]
    all_ms = sum(g[0] for g in groups.values())
    classes = {f"{p}_{t}tap": dict(launches=c, ms=round(m, 3), tflops=round(fl / (m * 1e-3) / 1e12, 2))
               for (p, t), (m, fl, c, _) in groups.items()}
    return dict(bound="mfma", achieved=round(achieved, 3), peak=round(peak, 1), unit="TFLOP/s",
                frac=round(achieved / peak, 4), traffic=None,
                kernel=KERNEL_NAMES.get(key, f"conv {key}"), arithmetic=key[0], kclass=f"{key[0]}_{key[1]}tap",
                launches=n,
                avg_launch_ms=round(ms / max(1, n), 4), flops_per_launch=flops / max(1, n),
                algorithmic_bytes_per_launch=nbytes / max(1, n),
                conv_ms_per_call=round(all_ms, 3), conv_classes=classes)


def _dtype():
    from nps_hip import ops
    return "f32" if ops.CONV_PRECISION == ops.PREC_F32 else "f32 (1x1/2x2/3x3/5x5 convs: 3-pass split-fp16 MFMA)"


PMC_FILE = os.path.join(ROOT, "profiles", "pmc_traffic.json")


# the workload the committed PMC passes profiled (one process, the default command): the launches of a
# rank carry these per-launch bytes only when the rank runs this exact per-GPU workload
PMC_WORKLOAD = dict(model="ufno", res=256, num_c=3, per_gpu_batch=16, fno_modes=None)


def attach_traffic(roof, workload):
    """roofline.traffic: HBM bytes per launch of the dominant kernel from the committed rocprofv3 --pmc
    passes (tools/pmc_traffic.sh: separate FETCH_SIZE and WRITE_SIZE passes; FETCH_SIZE x1 for the conv
    producers' 64-B-per-line reads as calibrated by tools/calib/pmc_calib.hip, x2 for 16 B/lane sweeps;
    see profiles/pmc_traffic.json's note).  Those passes profiled PMC_WORKLOAD; a rank running any other
    per-GPU workload (another model / size, or a per-GPU batch of 16/N at N > 1) reports traffic null."""
    if workload != PMC_WORKLOAD:
        roof["traffic_note"] = "null: no PMC pass for this per-GPU workload " + json.dumps(workload)
        return roof
    try:
        with open(PMC_FILE) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return roof
    rec = pmc.get("classes", {}).get(roof["kclass"])
    if rec:
        roof["traffic"] = rec["hbm_bytes_per_launch"]
        roof["traffic_source"] = f"{os.path.relpath(PMC_FILE, ROOT)} ({pmc.get('command', '')})"
    return roof


def shard_bounds(global_batch, world, rank):
    """[lo, hi) of this rank's samples of the global batch: equal contiguous shards (strong scaling; the
    rollout samples are independent, so no collective touches the data path)."""
    if global_batch % world != 0:
        raise SystemExit(f"global batch {global_batch} not divisible by {world} ranks")
    per = global_batch // world
    return rank * per, (rank + 1) * per


def launch_ranks(argv, n):
    """`bench.py --gpus N` (N > 1) without a launcher: start N ranks, one process per GPU, as
    `torch.distributed.run --nproc-per-node N` children on a free 127.0.0.1 port, and return their exit
    status.  This parent never touches the GPU (no HIP call before or after the children run); each child
    binds its LOCAL_RANK's card and opens the RCCL group in init_ranks."""
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    return subprocess.call(cmd)


def check_world(gpus):
    """The launcher's world size must be the --gpus the line will report."""
    env = os.environ.get("WORLD_SIZE")
    if env is not None and int(env) != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={env} ranks")


def init_ranks(check=False):
    """(world, rank, device) of this process: one process per GPU (torchrun env), RCCL process group.

    NPS_BENCH_REHEARSAL=1 (dev only, never a reported number): every rank on cuda:0 over gloo, so the
    N > 1 code path (sharding, barriers, max-over-ranks) can run on a one-GPU box.  check=True
    (--launch-check): gloo on the host, no GPU call at all."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if check:
        if world > 1:
            import torch.distributed as dist
            dist.init_process_group("gloo")
        return world, rank, torch.device("cpu")
    if world > 1:
        import torch.distributed as dist
        if os.environ.get("NPS_BENCH_REHEARSAL") == "1":
            local_rank = 0
            torch.cuda.set_device(0)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    return world, rank, torch.device("cuda", local_rank)


def launch_check(args):
    """--launch-check: bring the ranks up exactly as a measured run would (launcher, world size, rank ->
    shard), print what the process group is and every rank's shard of the mode's global batch, touch no
    GPU.  Used by tests/test_bench_launch.py on the CPU."""
    world, rank, _ = init_ranks(check=True)
    gb = args.global_batch if not (args.model in ("fno3d", "ufno3d") and args.global_batch == 16) else 8
    lo, hi = shard_bounds(gb, world, rank)
    shards = [[lo, hi]]
    if world > 1:
        import torch.distributed as dist
        shards = [None] * world
        dist.all_gather_object(shards, [lo, hi])
    if rank == 0:
        print(json.dumps({"launch_check": True, "mode": args.mode, "model": args.model, "n_gpus": world,
                          "gpus_arg": args.gpus, "global_batch": gb, "shards": shards,
                          "dist": dist_info(world)}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def max_over_ranks(elapsed, device):
    """The job's wall time: the slowest rank's (one all-reduce MAX; identity in a single process)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return elapsed
    on_cpu = dist.get_backend() == "gloo"
    t = torch.tensor([elapsed], device="cpu" if on_cpu else device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return t.item()


def per_rank_times(elapsed, device):
    """Every rank's elapsed seconds (all-gather; [elapsed] in a single process)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [elapsed]
    on_cpu = dist.get_backend() == "gloo"
    t = torch.tensor([elapsed], device="cpu" if on_cpu else device, dtype=torch.float64)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [float(x.item()) for x in out]


def dist_info(world):
    """What the process group actually is (read back from torch.distributed, not from the arguments)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dict(backend=str(dist.get_backend()), world_size=dist.get_world_size(), launcher_world=world,
                    rehearsal=os.environ.get("NPS_BENCH_REHEARSAL") == "1")
    return dict(backend=None, world_size=1, launcher_world=world, rehearsal=False)


def timing_fields(elapsed, times, steps):
    return dict(ms_per_step=round(elapsed / steps * 1e3, 3),
                ms_per_step_per_rank=[round(t / steps * 1e3, 3) for t in times])


def cpu_baseline(model, ocfg, opde, res, num_c, calls=2, B=2):
    import oracle
    from trainers.synthetic import twophase_batch
    threads = int(os.environ.get("OMP_NUM_THREADS", len(os.sched_getaffinity(0))))
    torch.set_num_threads(threads)
    om = oracle.build_oracle_model(ocfg, opde, {k: v.detach().cpu() for k, v in model.state_dict().items()})
    u, cond, pos, sc = twophase_batch(B, num_c, 25 * (calls + 1), res, res, seed=99, obstacle="disc")
    tw = 25
    with torch.no_grad():  # one untimed call: allocator / thread-pool warm-up, as the GPU legs get
        om(u[:, :, :tw], cond=cond, pos=pos, spatial_cond=sc)
    t0 = time.perf_counter()
    with torch.no_grad():
        losses, preds = oracle.simulate(om, u, cond, pos, sc, tw, 25 * (calls + 1))
    dt = time.perf_counter() - t0
    # parity of the same sample on the GPU path
    dev = next(model.parameters()).device
    pred = u[:, :, :tw].to(dev)
    err = 0.0
    with torch.no_grad():
        for k in range(calls):
            pred = model(pred, cond=cond.to(dev), bc=None, pos=pos.to(dev), t_cond=None, spatial_cond=sc.to(dev))
            ref = preds[k + 1].double()
            e = (torch.linalg.vector_norm(pred.cpu().double() - ref) / torch.linalg.vector_norm(ref)).item()
            err = max(err, e)
    return dict(value=round(B * tw * calls / dt, 3), unit="sample-timesteps/s", cores=threads, kind="port",
                sample=f"oracle (fp32 PyTorch-CPU restatement of the reference) simulate: {calls} model calls, "
                       f"B={B}, {res}x{res}, {num_c} fields, {dt:.1f} s",
                rel_l2_gpu_vs_cpu=err)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--model", default="ufno", choices=list(CFGS) + ["fno3d", "ufno3d"],
                    help="ufno3d = BASELINE config C5 (3-D U-FNO over a 16x128x128 time-bundled volume); fno3d = "
                         "its FNO-3D processor alone")
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--num-c", type=int, default=3)
    ap.add_argument("--global-batch", type=int, default=16)
    ap.add_argument("--fno-modes", type=int, default=None)
    ap.add_argument("--cpu-calls", type=int, default=2, help="CPU-baseline sample size (model calls, 0 = skip)")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"],
                    help="fno3d only: activation / weight storage of the C5 3-D spectral path")
    ap.add_argument("--mode", default="rollout", choices=["rollout", "train"],
                    help="rollout = the headline metric; train = pushforward train_step + backward + RCCL "
                         "all-reduce + Adam (samples/s)")
    ap.add_argument("--launch-check", action="store_true",
                    help="bring the N ranks up (launcher, process group, shards), print them and exit; no GPU")
    args = ap.parse_args()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU: this parent starts the N ranks and only waits for them
        raise SystemExit(launch_ranks(sys.argv[1:], args.gpus))
    check_world(args.gpus)
    if args.launch_check:
        return launch_check(args)
    if args.mode == "train":
        return run_train(args)
    if args.model in ("fno3d", "ufno3d"):
        return run_fno3d(args)

    world, rank, dev = init_ranks()
    lo, hi = shard_bounds(args.global_batch, world, rank)
    B = hi - lo
    tw = 25

    import argparse as _ap
    import types
    from common.interfaces import D
    from trainers.autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer
    from trainers.synthetic import twophase_batch

    model, ocfg, opde = build_model(args.model, args.res, args.num_c, dev, fno_modes=args.fno_modes)
    # this rank's shard of the global synthetic batch: samples [rank*B, (rank+1)*B)
    T = tw * (max(args.steps, args.warmup) + 1)
    u, cond, pos, sc = twophase_batch(args.global_batch, args.num_c, 1, args.res, args.res, seed=1234,
                                      obstacle="disc")
    u_all, _, _, _ = twophase_batch(B, args.num_c, T, args.res, args.res, seed=1234 + rank, obstacle="disc",
                                    device=dev)
    cond = cond[lo:hi].to(dev)
    pos = pos[lo:hi].to(dev)
    sc = sc[lo:hi].to(dev)
    cfg = _ap.Namespace(time_window=tw, base_resolution=(T, args.res, args.res), device=dev, nr_gt_steps=1)
    tr = AutoregressivePushforwardTrainer(model=model, data=types.SimpleNamespace(pde=model.pde, data_interface=D.sim2d),
                                          criterion=nn.MSELoss(reduction="sum"), config=cfg)

    def rollout(nsteps):
        with torch.no_grad():
            return tr.simulate(u_all, cond, pos, compute_loss=True, include_data=False, nr_gt_steps=1,
                               t_res=tw * (nsteps + 1), spatial_conditioning=sc)

    if args.warmup > 0:
        rollout(args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses = rollout(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    mine = time.perf_counter() - t0
    elapsed = max_over_ranks(mine, dev)
    times = per_rank_times(mine, dev)
    value = args.global_batch * tw * args.steps / elapsed

    if rank == 0:
        workload = dict(model=args.model, res=args.res, num_c=args.num_c, per_gpu_batch=B, fno_modes=args.fno_modes)
        roof = attach_traffic(conv_roofline(model, u_all[:, :, :tw], cond, pos, sc), workload)
        cpu = cpu_baseline(model, ocfg, opde, args.res, args.num_c, calls=args.cpu_calls) if (
            args.cpu_calls > 0 and world == 1) else None
        if cpu is not None and B >= 2:
            # the north star's 10x is defined at the CPU sample's batch (B = 2): the same rollout on this
            # GPU at B = 2, timed like the headline
            def rollout2(nsteps):
                with torch.no_grad():
                    return tr.simulate(u_all[:2], cond[:2], pos[:2], compute_loss=True, include_data=False,
                                       nr_gt_steps=1, t_res=tw * (nsteps + 1), spatial_conditioning=sc[:2])
            rollout2(1)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            rollout2(args.steps)
            torch.cuda.synchronize()
            v2 = 2 * tw * args.steps / (time.perf_counter() - t2)
            cpu["gpu_at_same_batch"] = dict(value=round(v2, 3), batch=2, gpu_over_cpu=round(v2 / cpu["value"], 1))
        line = {
            "metric": f"rollout timesteps/sec on {args.res}x{args.res} two-phase grid (sample-timesteps/s); "
                      "rel-L2 vs CPU reference",
            "value": round(value, 3), "unit": "sample-timesteps/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, **timing_fields(elapsed, times, args.steps), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": _dtype(), "data": "synthetic",
            "dist": dist_info(world),
            "config": {"workload": f"{args.model.upper()} twophase cfg rollout (simulate), {args.res}x{args.res}, "
                                   f"{args.num_c} fields, obstacle mask, tw=25", "model": args.model,
                       "global_batch": args.global_batch, "per_gpu_batch": B, "res": args.res,
                       "num_c": args.num_c, "parallelism": f"dp{world} (batch-sharded rollout, no collective)"},
            "roofline": roof, "cpu_baseline": cpu,
            "rel_l2_vs_cpu": None if cpu is None else cpu["rel_l2_gpu_vs_cpu"],
            "loss_last_window": float(losses[-1].item()),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


# BASELINE config C5: FNO-3D processor (proc_fno.py:22-83 with SpectralConv3d :291-376) over a time-bundled
# (D, H, W) = (16, 128, 128) volume, 64 hidden + 4 conditioning channels, modes (8, 12, 12), 4 blocks
C5_CFG = dict(num_spatial_dims=3, n_cond=4, hidden_features=64, fno_modes=(8, 12, 12), hidden_blocks=4,
              cond_mode="concat", fno_kernel_size=1)
C5_VOL = (16, 128, 128)
# the 3-D U-FNO of C5: the same FNO-3D layers plus, per block, a 3-D U-Net as the twophase U-FNO cfg builds it
# (ch_mults [1, 1], n_blocks 1, GroupNorm, 1x1 final, circular; cfg_twophase_ufno.py) — its Upsample is this
# build's 3-D definition (DESIGN.md "3-D U-FNO")
C5_UFNO_CFG = dict(C5_CFG, ch_mults=[1, 1], is_attn=[False, False], mid_attn=False, norm=True, n_blocks=1,
                   use1x1=True, padding_mode="circular")


def run_fno3d(args):
    """C5 throughput: one step = one 3-D processor forward over the batch (16 bundled timesteps per
    sample) — the U-FNO 3D (--model ufno3d: FNO-3D layers + 3-D U-Nets) or the FNO-3D alone (fno3d) —
    fp32 or bf16 storage; batch-sharded over the ranks like the rollout."""
    from models.enc_proc_dec_components.proc_fno import FNO
    from models.enc_proc_dec_components.proc_ufno import UFNO
    from nps_hip import ops
    world, rank, dev = init_ranks()
    gb = args.global_batch if args.global_batch != 16 else 8  # C5: global batch 8 (one volume per GPU at 8)
    lo, hi = shard_bounds(gb, world, rank)
    B = hi - lo
    torch.manual_seed(42)
    ufno = args.model == "ufno3d"
    m = (UFNO(pde=None, **C5_UFNO_CFG) if ufno else FNO(pde=None, **C5_CFG)).to(dev).eval()
    D, H, W = C5_VOL
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    h = torch.rand(B, C5_CFG["hidden_features"], D * H, W, device=dev, generator=g) * 2 - 1
    vb = torch.rand(B, C5_CFG["n_cond"], D * H, W, device=dev, generator=g)
    bf16 = args.dtype == "bf16"
    # NDHWC (viewed as (B, D*H, W, C)) resident in HBM in the storage dtype before timing
    hn, vn = ops.nchw_to_nhwc(h), ops.nchw_to_nhwc(vb)
    if bf16:
        hn, vn = ops.to_bf16(hn), ops.to_bf16(vn)
    if ufno:  # NDHWC volumes
        hn = hn.view(B, D, H, W, hn.shape[3])
        vn = vn.view(B, D, H, W, vn.shape[3])

    def step():
        with torch.no_grad():
            if ufno:
                return m.run3d(hn, vn)
            return m.run_bf16(hn, vn, D) if bf16 else m.run(hn, vn, D)

    for _ in range(max(1, args.warmup)):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        y = step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    mine = time.perf_counter() - t0
    elapsed = max_over_ranks(mine, dev)
    times = per_rank_times(mine, dev)
    if rank == 0 and ufno:
        return print_ufno3d_line(args, m, step, hn, vn, gb, B, world, elapsed, times, bf16)
    if rank == 0:
        # bytes one layer must move at least: input frame read by the pointwise conv and by the W-DFT, the
        # output written and re-read by the spectral accumulate, the per-mode weights once
        es = 2 if bf16 else 4
        Cin, Co = C5_CFG["hidden_features"] + C5_CFG["n_cond"], C5_CFG["hidden_features"]
        m1, m2, m3 = C5_CFG["fno_modes"]
        npx = B * D * H * W
        wbytes = min(D, 2 * m1) * min(H, 2 * m2) * m3 * Cin * Co * (4 if bf16 else 8)
        layer_bytes = npx * es * (2 * Cin + 3 * Co) + wbytes
        ms = elapsed / args.steps * 1e3
        print(json.dumps({
            "metric": "C5 FNO-3D processor throughput (sample-timesteps/s, 16 time-bundled steps per volume)",
            "value": round(gb * D * args.steps / elapsed, 3), "unit": "sample-timesteps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, **timing_fields(elapsed, times, args.steps),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
            "dtype": "bf16 storage, fp32 arithmetic" if bf16 else "f32", "data": "synthetic", "dist": dist_info(world),
            "config": {"workload": "FNO-3D (C5) over a 16x128x128 volume, 64 hidden + 4 cond, modes (8,12,12), "
                                   "4 blocks", "model": "fno3d", "global_batch": gb, "per_gpu_batch": B,
                       "parallelism": f"dp{world} (batch-sharded, no collective)"},
            "hbm_bytes_per_step_min": layer_bytes * C5_CFG["hidden_blocks"],
            "achieved_hbm_TBps": round(layer_bytes * C5_CFG["hidden_blocks"] / (ms * 1e-3) / 1e12, 3),
            "out_abs_mean": float(y.float().abs().mean())}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def print_ufno3d_line(args, m, step, hn, vn, gb, B, world, elapsed, times, bf16):
    """The C5 U-FNO 3D line: throughput, the conv3d roofline (HIP events on every conv launch of one step)
    and the CPU oracle on a bounded sample (one of the 4 blocks, B=1, fp32 PyTorch-CPU restatement, scaled
    to the 4-block call) with the GPU-vs-oracle rel-L2 of that block."""
    import oracle  # noqa: F401  (CPU baseline only, outside the timed region)
    from oracle import functional as Fo
    from models.common import to_ncdhw
    from nps_hip import ops
    D = C5_VOL[0]
    roof = probe_roofline(step)
    cpu = None
    if args.cpu_calls > 0 and world == 1:
        threads = int(os.environ.get("OMP_NUM_THREADS", len(os.sched_getaffinity(0))))
        torch.set_num_threads(threads)
        sd = {k: v.detach().cpu() for k, v in m.state_dict().items() if k.split(".")[1] == "0"}
        h1 = to_ncdhw(ops.to_f32(hn[:1]) if bf16 else hn[:1]).cpu()
        v1 = to_ncdhw(ops.to_f32(vn[:1]) if bf16 else vn[:1]).cpu()
        cfg1 = dict(C5_UFNO_CFG, hidden_blocks=1)
        t0 = time.perf_counter()
        with torch.no_grad():
            ref = Fo.ufno3d(sd, "", cfg1, h1, v1)
        dt = time.perf_counter() - t0
        nblk = C5_UFNO_CFG["hidden_blocks"]
        with torch.no_grad():  # the GPU's first block on the same volume
            fl, ul = m.fno_layers, m.unet_layers
            m.fno_layers, m.unet_layers = fl[:1], ul[:1]
            try:
                y1 = m.run3d(hn[:1], vn[:1])
            finally:
                m.fno_layers, m.unet_layers = fl, ul
        y1 = to_ncdhw(ops.to_f32(y1) if bf16 else y1).cpu().double()
        err = (torch.linalg.vector_norm(y1 - ref.double()) / torch.linalg.vector_norm(ref.double())).item()
        cpu = dict(value=round(D / (nblk * dt), 4), unit="sample-timesteps/s", cores=threads, kind="port",
                   sample=f"oracle (fp32 PyTorch-CPU restatement) U-FNO 3D block 1 of {nblk}, B=1, "
                          f"{'x'.join(map(str, C5_VOL))}: {dt:.1f} s, scaled x{nblk} to the whole processor call",
                   rel_l2_gpu_vs_cpu_block1=err)
    ms = elapsed / args.steps * 1e3
    print(json.dumps({
        "metric": "C5 U-FNO 3D processor throughput (sample-timesteps/s, 16 time-bundled steps per volume)",
        "value": round(gb * D * args.steps / elapsed, 3), "unit": "sample-timesteps/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, **timing_fields(elapsed, times, args.steps),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "bf16 storage, bf16 MFMA / fp32 accumulate" if bf16 else "f32", "data": "synthetic",
        "dist": dist_info(world),
        "config": {"workload": "U-FNO 3D (C5) over a 16x128x128 volume, 64 hidden + 4 cond, modes (8,12,12), "
                               "4 blocks, 3-D U-Nets ch_mults [1,1]", "model": "ufno3d", "global_batch": gb,
                   "per_gpu_batch": B, "parallelism": f"dp{world} (batch-sharded, no collective)"},
        "roofline": roof, "cpu_baseline": cpu}), flush=True)


def cpu_baseline_train(model, args, B=1):
    """The training step on the host: the oracle (fp32 PyTorch-CPU restatement) forward, sqrt(MSE_sum)
    loss and autograd backward for one sample (trainers/autoregressivepushforwardtrainer.py:43-163,
    unroll 0), plus Adam — samples/s on the host cores."""
    import oracle
    from trainers.synthetic import twophase_batch
    _, ocfg, opde = build_model(args.model, args.res, args.num_c, "cpu", fno_modes=args.fno_modes)
    threads = int(os.environ.get("OMP_NUM_THREADS", len(os.sched_getaffinity(0))))
    torch.set_num_threads(threads)
    om = oracle.build_oracle_model(ocfg, opde, {k: v.detach().cpu() for k, v in model.state_dict().items()})
    om.sd = {k: v.detach().clone().requires_grad_(True) for k, v in om.sd.items()}
    opt = torch.optim.Adam([t for t in om.sd.values() if t.is_floating_point() or t.is_complex()], lr=1e-4)
    u, cond, pos, sc = twophase_batch(B, args.num_c, 50, args.res, args.res, seed=99, obstacle="disc")
    t0 = time.perf_counter()
    loss = torch.sqrt(torch.sum((om(u[:, :, :25], cond=cond, pos=pos, spatial_cond=sc) - u[:, :, 25:50]) ** 2))
    loss.backward()
    opt.step()
    dt = time.perf_counter() - t0
    return dict(value=round(B / dt, 4), unit="samples/s", cores=threads, kind="port",
                sample=f"oracle train step (forward + sqrt(MSE_sum) + autograd backward + Adam), B={B}, "
                       f"{args.res}x{args.res}, {args.num_c} fields, {dt:.1f} s")


def run_train(args):
    """Training throughput: trainers/base.py:472-507 steps of the pushforward train_step (unroll 0, the
    epoch-0 case) on a fixed global batch sharded over the ranks; under a process group the trainer wires
    data parallelism itself (parameter broadcast, global sqrt(MSE_sum) loss, summed RCCL gradient
    all-reduce overlapped with backward: trainers/distributed.py), Adam(lr=1e-4) as in the cfgs."""
    import types
    from common.interfaces import D
    from trainers.autoregressivepushforwardtrainer import AutoregressivePushforwardTrainer
    from trainers.synthetic import twophase_batch
    world, rank, dev = init_ranks()
    lo, hi = shard_bounds(args.global_batch, world, rank)
    B = hi - lo
    tw = 25
    model, _, _ = build_model(args.model, args.res, args.num_c, dev, fno_modes=args.fno_modes)
    model.train()
    u, cond, pos, sc = twophase_batch(B, args.num_c, 2 * tw, args.res, args.res, seed=1234 + rank,
                                      obstacle="disc", device=dev)
    batch = (u[:, :, :1], u, pos, cond, torch.empty(B, 0, device=dev), sc)  # collated layout (B, 0)
    cfg = types.SimpleNamespace(time_window=tw, base_resolution=(2 * tw, args.res, args.res), device=dev,
                                batch_size=B, lr_step_interval=25, unrolling=0)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    tr = AutoregressivePushforwardTrainer(model=model, data=types.SimpleNamespace(pde=model.pde,
                                                                                  data_interface=D.sim2d),
                                          criterion=nn.MSELoss(reduction="sum"), optimizer=opt, config=cfg)
    assert (tr.grad_sync is not None) == (world > 1)
    for _ in range(max(1, args.warmup)):
        tr.train_one_epoch([batch], epoch=0)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    t0 = time.perf_counter()
    loss = None
    for _ in range(args.steps):
        loss = tr.train_one_epoch([batch], epoch=0)
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    mine = time.perf_counter() - t0
    elapsed = max_over_ranks(mine, dev)
    times = per_rank_times(mine, dev)
    # the probe step runs on every rank: under a process group a training step holds collectives (the global
    # loss and the gradient all-reduce), which a rank-0-only step would leave unmatched
    roof = probe_roofline(lambda: tr.train_one_epoch([batch], epoch=0))
    if rank == 0:
        cpu = cpu_baseline_train(model, args) if (args.cpu_calls > 0 and world == 1) else None
        print(json.dumps({
            "metric": "pushforward training samples/sec (train_step + backward + all-reduce + Adam)",
            "value": round(args.global_batch * args.steps / elapsed, 3), "unit": "samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, **timing_fields(elapsed, times, args.steps),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": _dtype(),
            "data": "synthetic", "dist": dist_info(world),
            "config": {"workload": f"{args.model.upper()} twophase cfg train_step, {args.res}x{args.res}, "
                                   f"{args.num_c} fields, tw=25", "global_batch": args.global_batch,
                       "per_gpu_batch": B, "parallelism": f"dp{world} (RCCL gradient all-reduce)"},
            "roofline": roof, "cpu_baseline": cpu, "loss_last": float(loss)}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
