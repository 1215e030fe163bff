"""Torch-tensor front end of the HIP kernels (include/nps.h).

Activations are NHWC fp32 tensors of shape (B, H, W, C).  A conv input is a
*virtual frame*: a list of `Src(tensor, off_y, off_x)` slices concatenated
along channels, each placed at an offset of the frame (crop_Nd, cat), so no
cat / pad / crop is ever materialised.
"""
import math
import os
import weakref
from typing import List, NamedTuple, Optional, Sequence, Union

import torch

from . import Conv2dArgs, Conv3dArgs, PackJob, Src as _CSrc, Src3 as _CSrc3, check, lib, ptr, stream_ptr

GELU = 1

# Conv arithmetic (include/nps.h NPS_PREC_*): exact fp32 MFMA, or the 3-pass split-fp16 MFMA products
# (~2^-21 relative per product, 5.3x the fp32 MFMA rate) for the stride-1 undilated 1x1 / 2x2 / 3x3 convs.
PREC_F32, PREC_X3F16 = 0, 1
# split-fp16 3x3 convs apply their GroupNorm / GELU prologue while staging (nps_conv2d_x3_prologue_ok)
# instead of a frame_pack pass in front of the conv (dev knob NPS_FUSE_PROLOGUE=0: off).  Pays off on the
# wide 192-channel tiles, whose producers stage each patch once for all output channels.
FUSE_PROLOGUE = os.environ.get("NPS_FUSE_PROLOGUE", "1") == "1"
# dev knob NPS_FUSE_PROLOGUE_1X1=0: the 1x1 convs' GroupNorm + GELU prologue materialised by frame_pack (A/B of the
# LDS-weight kernel's fused prologue, conv1x1_wl_kernel<6, 2, true>)
FUSE_PROLOGUE_1X1 = os.environ.get("NPS_FUSE_PROLOGUE_1X1", "1") != "0"
CONV_PRECISION = PREC_F32 if os.environ.get("NPS_CONV_PRECISION", "x3f16") == "f32" else PREC_X3F16
# the Downsample's 2x2 conv reads the space-to-depth view of its input directly (nps_conv2d_t.s2d) instead of
# a space_to_depth copy (dev knob NPS_S2D_VIEW=0: the copy)
S2D_VIEW = os.environ.get("NPS_S2D_VIEW", "1") == "1"
# split-fp16 transposed convs run their 4 phases in one launch (dev knob NPS_CONVT_MERGE=0: 4 launches)
MERGE_CONVT_PHASES = os.environ.get("NPS_CONVT_MERGE", "1") == "1"


def conv_precision(KH, KW, stride=1, dil=1):
    """Arithmetic a conv of this geometry runs in under the current CONV_PRECISION setting."""
    if CONV_PRECISION == PREC_X3F16 and lib.nps_conv2d_x3_eligible(KH, KW, stride, dil):
        return PREC_X3F16
    return PREC_F32

# Optional live probe of the conv kernel (bench.py): when a list, every conv2d launch appends
# (start_event, end_event, algorithmic_flops) recorded on the launching stream.
conv_probe = None
conv_shape_log = None  # dev (tools/call_shapes.py): with conv_probe, one launch-geometry dict per conv launch


class Src(NamedTuple):
    t: torch.Tensor          # (B, H, W, C) NHWC contiguous
    off_y: int = 0
    off_x: int = 0


# ----------------------------------------------------------------- range tags ----
# A split-fp16 conv scales its input by a power of 2 picked from an upper bound of |x| (include/nps.h,
# nps_conv2d_t.in_scale / in_tag*), so fp32-class accuracy holds for activations of any magnitude.  The
# bound travels with the tensor as a RANGE TAG: NPS_TAG_FLOATS floats of a per-device arena, raised by
# the kernel that writes the tensor (conv / frame_pack / spectral epilogues: out_tag).  A tensor without
# a live tag (model inputs, views, torch-made tensors) gets one from nps_absmax the first time a
# split-fp16 conv reads it.  Tags are only ever raised, so a tag shared by several tensors (a clone,
# a space-to-depth copy) or written by several kernels (accumulating convs) stays an upper bound.
TAG_FLOATS = 64 * 64        # NPS_TAG_FLOATS
# dev knob NPS_RANGE_TAGS: "1" (default) input + output tags, "in" / "out" one side only, "0" none
_TAGS = os.environ.get("NPS_RANGE_TAGS", "1")
USE_IN_TAGS, USE_OUT_TAGS = _TAGS in ("1", "in"), _TAGS in ("1", "out")
_ARENA_TAGS = 2048          # 32 MiB per device; re-zeroed (new generation) when exhausted


class _TagArena:
    def __init__(self, device):
        self.buf = torch.zeros(_ARENA_TAGS * TAG_FLOATS, dtype=torch.float32, device=device)
        self.gen = 0
        self.next = 0

    def reserve(self, k: int):
        """Start a new generation now unless k more tags fit in this one: a launch that needs several
        tags reserves them all before it reads any tag pointer, so no wrap (which zeroes the buffer)
        can happen between reading an input tag and launching the kernel that reads it."""
        if self.next + k > _ARENA_TAGS:
            # stream-ordered after every kernel that used the old generation; once side streams (Fork) have
            # carried launches, the device drains before and after the zero so no stream's kernel can read
            # or raise a tag across it (a wrap comes every few model calls)
            fenced = _forked and self.buf.is_cuda
            if fenced:
                torch.cuda.synchronize(self.buf.device)
            self.buf.zero_()
            if fenced:
                torch.cuda.synchronize(self.buf.device)
            self.gen += 1
            self.next = 0

    def alloc(self):
        self.reserve(1)
        i = self.next
        self.next += 1
        return _Tag(self, self.gen, self.buf.data_ptr() + 4 * i * TAG_FLOATS)


class _Tag(NamedTuple):
    arena: "_TagArena"
    gen: int
    ptr: int

    @property
    def live(self):
        return self.arena.gen == self.gen


_arenas = {}
_forked = False  # set by the first Fork that runs launches on a side stream


# ----------------------------------------------------------------- side streams ----
# Launches that do not depend on the one just issued (the ResidualBlock's 1x1 shortcut beside conv1, the U-FNO
# block's FNO layer beside its U-Net) go to a second HIP stream, so their work-groups take the CUs a
# persistent 3x3 launch leaves idle in its last round (B = 2: the 258^2 convs are 1122 tiles on 256 CUs,
# 4.4 rounds).  Each lane is one stream per device (one hardware queue).  dev knob NPS_SIDE_STREAM=0: off.
SIDE_STREAM = os.environ.get("NPS_SIDE_STREAM", "1") == "1"
SIDE_FNO = os.environ.get("NPS_SIDE_FNO", "1") == "1"      # dev knob: the U-FNO block's FNO layer fork
# ... for 2-D activations of at most this many elements (B=2 C3: 25 M; at B=16, 201 M, the U-Net's launches
# keep the CUs busy: within noise, profiles/r4/experiments/side_stream_*; the 3-D U-FNO forks at every size)
SIDE_FNO_MAX_ELEMS = int(float(os.environ.get("NPS_SIDE_FNO_MAX_ELEMS", "6.4e7")))


# dev knob NPS_SIDE_WGRAD=1: the training backward's weight gradients on a side stream (see
# nps_hip.autograd.Conv2dFn.backward)
SIDE_WGRAD = os.environ.get("NPS_SIDE_WGRAD", "0") == "1"


def fno_fork(h: torch.Tensor, settle: Sequence[torch.Tensor] = ()) -> "Fork":
    """The U-FNO block's fork for its FNO layer (lane 1): on for small activations (see SIDE_FNO_MAX_ELEMS)."""
    return Fork(h, lane=1, on=SIDE_FNO and h.numel() <= SIDE_FNO_MAX_ELEMS, settle=settle)
# dev knob: the shortcut fork needs conv1's last round to leave at least this fraction of the CUs idle
SIDE_MIN_IDLE = float(os.environ.get("NPS_SIDE_MIN_IDLE", "0.25"))
_side_streams = {}
_side_depth = 0   # > 0 while launches go to a side stream


_ncu = {}


def x3_plan_tiles(Ho: int, Wo: int, B: int, Cout: int, Cin: int, K: int = 3) -> int:
    """Work-group tiles of a stride-1 split-fp16 KxK launch with that output, as nps_conv2d_plan tiles it
    (wide 192-channel or 64-channel tiles, the planner's TH x TW): host-only, cached per shape."""
    key = (Ho, Wo, B, Cout, Cin, K)
    n = _plan_tiles.get(key)
    if n is None:
        a = Conv2dArgs()
        a.nsrc = 1
        a.src[0].ptr, a.src[0].C, a.src[0].H, a.src[0].W = 0x1000, Cin, Ho + K - 1, Wo + K - 1
        a.B, a.Hin, a.Win, a.Cin = B, Ho + K - 1, Wo + K - 1, Cin
        a.KH = a.KW = K
        a.stride, a.dil = 1, 1
        a.Hout, a.Wout, a.Cout = Ho, Wo, Cout
        a.out_C, a.out_H, a.out_W, a.out_os = Cout, Ho, Wo, 1
        a.precision = PREC_X3F16
        if lib.nps_conv2d_plan(ctypes_byref(a)) < 0:
            raise RuntimeError("conv2d_plan failed: " + lib.nps_last_error().decode())
        nco = 192 if a.TH * a.TW == 128 else 64
        n = _plan_tiles[key] = -(-Ho // a.TH) * -(-Wo // a.TW) * B * -(-Cout // nco)
    return n


_plan_tiles = {}


def last_round_idle(Ho: int, Wo: int, B: int, Cout: int, device, Cin: int = 192) -> float:
    """Fraction of the CUs left idle in the last round of a split-fp16 3x3 launch: the persistent grid of
    nps_launch_conv2d_x3 (one work-group per CU, multi_processor_count & ~7 of them) over the tiles
    nps_conv2d_plan picks (x3_plan_tiles).  A fork beside such a launch pays only when this is large: every
    cross-stream wait costs ~15 us (profiles/r4/experiments/side_stream_forks_ab.txt)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    n = _ncu.get(idx)
    if n is None:
        n = _ncu[idx] = torch.cuda.get_device_properties(idx).multi_processor_count & ~7
    return idle_fraction(x3_plan_tiles(Ho, Wo, B, Cout, Cin), n)


def idle_fraction(tiles: int, workgroups: int) -> float:
    """Idle share of a persistent grid of `workgroups` in the last round of `tiles` tiles."""
    last = tiles % workgroups
    return 0.0 if last == 0 else 1.0 - last / workgroups


class Fork:
    """`f = Fork(t)` marks the fork point on the current stream (t: any tensor of the device);
    `with f:` issues the enclosed launches on side stream `lane`, which starts at the fork point;
    `f.join(*outs)` makes the current stream wait for them and hands it the tensors they allocated.
    Moments buffers made inside (new_stats) are private zeros of the side stream; the tag arena fences a
    wrap across all streams.  `settle`: fp32 tensors both streams may read as split-fp16 conv inputs — their
    range tags are made live here, before the fork point, because a tag one stream computes lazily (absmax)
    could be read by the other before that absmax ran.  A no-op on the CPU or with NPS_SIDE_STREAM=0."""

    def __init__(self, like: torch.Tensor, lane: int = 0, on: bool = True, settle: Sequence[torch.Tensor] = ()):
        d = like.device
        self.on = on and SIDE_STREAM and d.type == "cuda"
        self.done = None
        if not self.on:
            return
        if USE_IN_TAGS and CONV_PRECISION == PREC_X3F16:
            ts = [t for t in settle if t is not None and t.dtype == torch.float32]
            reserve_tags(d, len(ts))
            for t in ts:
                input_tag(t)
        idx = d.index if d.index is not None else torch.cuda.current_device()
        key = (idx, lane)
        self.side = _side_streams.get(key)
        if self.side is None:
            self.side = _side_streams[key] = torch.cuda.Stream(device=idx)
        self.main = torch.cuda.current_stream(idx)
        self.start = torch.cuda.Event()
        self.start.record(self.main)

    def __enter__(self):
        global _side_depth, _forked
        if self.on:
            _forked = True
            self.side.wait_event(self.start)
            self._ctx = torch.cuda.stream(self.side)
            self._ctx.__enter__()
            _side_depth += 1
        return self

    def __exit__(self, *exc):
        global _side_depth
        if self.on:
            _side_depth -= 1
            self._ctx.__exit__(*exc)
            self.done = torch.cuda.Event()
            self.done.record(self.side)
        return False

    def join(self, *outs):
        if self.done is not None:
            self.main.wait_event(self.done)
            for t in outs:
                if isinstance(t, torch.Tensor):
                    t.record_stream(self.main)
            self.done = None


def _arena(device) -> _TagArena:
    key = (device.type, device.index if device.index is not None else torch.cuda.current_device())
    ar = _arenas.get(key)
    if ar is None:
        ar = _arenas[key] = _TagArena(device)
    return ar


def reserve_tags(device, k: int):
    """Guarantee that the next k tag allocations on `device` do not wrap the arena (see _TagArena.reserve)."""
    _arena(device).reserve(k)


def tag_of(t: torch.Tensor):
    """The live range tag of `t`, or None.  A tag is recorded with the tensor's version counter: a torch
    in-place write (add_, mul_, slice assignment) bumps t._version and so invalidates the bound; the HIP
    kernels that write into an existing tensor raise its tag instead."""
    rec = getattr(t, "_nps_tag", None)
    if rec is None:
        return None
    tag, ver = rec
    return tag if (tag.live and ver == t._version) else None


def _attach_tag(t: torch.Tensor, tag):
    t._nps_tag = (tag, t._version)


def new_tag(t: torch.Tensor) -> int:
    """Attach a fresh (zero) tag to `t`, whose writer will raise it; returns its device pointer."""
    tag = _arena(t.device).alloc()
    _attach_tag(t, tag)
    return tag.ptr


def out_tag(t: torch.Tensor, accumulate: bool) -> int:
    """Tag pointer for a kernel that writes into the existing tensor `t`: its live tag, or a new one —
    seeded with max|t| when the kernel accumulates onto (reads) the current contents.  Otherwise the
    contents the kernel leaves unwritten must be zeros or absent (crop padding, phase outputs)."""
    tag = tag_of(t)
    if tag is not None:
        return tag.ptr
    p = new_tag(t)
    if accumulate:
        check(lib.nps_absmax_into(ptr(t), t.numel(), p, stream_ptr()), "absmax (tag seed)")  # (fresh: zero)
    return p


def share_tag(dst: torch.Tensor, src: torch.Tensor) -> torch.Tensor:
    """dst holds a subset of src's values (and zeros): it may carry src's bound."""
    tag = tag_of(src)
    if tag is not None:
        _attach_tag(dst, tag)
    return dst


def input_tag(t: torch.Tensor) -> int:
    """Tag pointer bounding |t| for a split-fp16 conv reading t (nps_absmax when t has no live tag).

    On a side stream (inside a Fork) the fresh tag is PRIVATE, not attached to t: t may be an input both
    streams read (its settled tag died in an arena wrap inside the fork), and a tag attached here would be
    raised by an absmax queued only on the side stream, which a later main-stream launch reading t could
    see before that absmax ran.  The main stream measures t itself."""
    tag = tag_of(t)
    if tag is not None:
        return tag.ptr
    p = _arena(t.device).alloc().ptr if _side_depth > 0 else new_tag(t)
    check(lib.nps_absmax_into(ptr(t), t.numel(), p, stream_ptr()), "absmax (input tag)")  # (fresh arena tag: zero)
    return p


# ------------------------------------------------------------ GroupNorm(1) moments ----
# A split-fp16 2x2/3x3 conv that writes a whole tensor can add the per-sample (sum, sum of squares) of
# the values it stores to a zeroed fp64 [B][2] buffer (nps_conv2d_t.out_stats).  The tensor then CARRIES
# its moments (attach_stats), and the GroupNorm(1) of a frame made of such tensors (ResidualBlock.norm1 /
# norm2, proc_unet_modern.py:235-236) is their sum — no statistics pass over the frame.  Sources without
# moments get them from one nps_group_norm_stats pass over that source alone, kept for later frames.
# Moments are valid while the tensor is unchanged: torch's in-place ops bump t._version, and the HIP ops
# that write into an existing tensor drop them (drop_stats).
STATS_SUB = lib.nps_stats_sub()  # NPS_STATS_SUB of the loaded library (sub-slots of a moments buffer)


_STATS_CHUNK = 1 << 15      # doubles zeroed at once; slices are handed out and never re-zeroed
_stats_chunks = {}


def new_stats(B: int, like: torch.Tensor, sub: int = STATS_SUB) -> torch.Tensor:
    """A zeroed fp64 [B][sub][2] moments buffer: sub = NPS_STATS_SUB for nps_conv2d_t.out_stats, 1 for the
    [B][G][2] statistics a GroupNorm prologue reads (G = 1).  Slices of one zero-filled chunk per device
    (one fill launch per chunk instead of one per buffer); a chunk is never reused in place — it is freed
    when its last slice is."""
    n = B * sub * 2
    d = like.device
    key = (d.type, d.index if d.index is not None else torch.cuda.current_device())
    ch = _stats_chunks.get(key)
    if n > _STATS_CHUNK // 4 or _side_depth > 0:  # (a side stream's buffers are zeroed on that stream)
        return torch.zeros((B, sub, 2), dtype=torch.float64, device=d)
    if ch is None or ch[1] + n > _STATS_CHUNK:
        ch = [torch.zeros(_STATS_CHUNK, dtype=torch.float64, device=d), 0]
        _stats_chunks[key] = ch
    v = ch[0][ch[1]:ch[1] + n].view(B, sub, 2)
    ch[1] += (n + 31) // 32 * 32
    return v


def _stats_sum(parts, B, out):
    """out[b][0] = sum of the parts' (sum, sum of squares) over their sub-slots (nps_stats_sum)."""
    p = list(parts) + [None] * (3 - len(parts))
    n = [t.shape[1] if t is not None else 0 for t in p]
    check(lib.nps_stats_sum(ptr(p[0]), n[0], ptr(p[1]), n[1], ptr(p[2]), n[2], B, ptr(out), out.shape[1],
                            stream_ptr()), "stats_sum")
    return out


def attach_stats(t: torch.Tensor, st: torch.Tensor) -> torch.Tensor:
    """Record that st holds t's GroupNorm(1) moments (every element of t was added exactly once)."""
    if not getattr(st, "_nps_incomplete", False):
        t._nps_stats = (st, t._version)
    return t


def drop_stats(t: torch.Tensor):
    if getattr(t, "_nps_stats", None) is not None:
        t._nps_stats = None


_DEBUG_STATS = os.environ.get("NPS_DEBUG_STATS") == "1"  # dev: print every GroupNorm statistics pass and its caller


def stats_of(t: torch.Tensor) -> Optional[torch.Tensor]:
    """t's live GroupNorm(1) moments, or None."""
    rec = getattr(t, "_nps_stats", None)
    if rec is None:
        return None
    st, ver = rec
    return st if ver == t._version else None


def source_stats(t: torch.Tensor) -> torch.Tensor:
    """t's GroupNorm(1) moments: carried, or one nps_group_norm_stats pass (then carried).  Read-only:
    seed a buffer of your own with copy_stats() to accumulate into."""
    st = stats_of(t)
    if st is None:
        if _DEBUG_STATS:
            import traceback
            print("nps stats pass (source)", tuple(t.shape), "".join(traceback.format_stack(limit=5)[:-1]), flush=True)
        st = new_stats(t.shape[0], t, 1)
        check(lib.nps_group_norm_stats(_c_src([Src(t)]), 1, t.shape[0], t.shape[1], t.shape[2], t.shape[3], 1,
                                       ptr(st), 0, stream_ptr()), "group_norm_stats (source)")
        attach_stats(t, st)
    return st


def copy_stats(st: torch.Tensor) -> torch.Tensor:
    """A new out_stats buffer seeded with st's moments (to accumulate a conv's changes into)."""
    return _stats_sum([st], st.shape[0], new_stats(st.shape[0], st))


def _c_src(srcs: Sequence[Src]):
    arr = (_CSrc * 3)()
    for i, s in enumerate(srcs):
        t = s.t
        if t.dtype != torch.float32 or not t.is_contiguous() or t.dim() != 4:
            raise RuntimeError(f"nps_hip: sources must be contiguous fp32 NHWC, got {t.dtype} {tuple(t.shape)}")
        arr[i].ptr = ptr(t)
        arr[i].H, arr[i].W, arr[i].C = t.shape[1], t.shape[2], t.shape[3]
        arr[i].off_y, arr[i].off_x = int(s.off_y), int(s.off_x)
    return arr


def crop_offset(cur: int, des: int) -> int:
    """Top/left zero-pad (negative = crop) that crop_Nd applies when resizing cur -> des
    (models/common.py:20-34: the ±0.001 tie-break pads the trailing side one more)."""
    return int(round((des - cur) / 2 - 0.001))


def empty_nhwc(B, H, W, C, like: torch.Tensor):
    return torch.empty((B, H, W, C), dtype=torch.float32, device=like.device)


# ----------------------------------------------------------------- weights ----
def _pack(w, Cout, Cin, KH, KW, mode, precision):
    n = lib.nps_conv2d_packed_size(Cout, Cin, KH * KW)
    out = torch.empty(n, dtype=torch.float32, device=w.device)
    fn = lib.nps_conv2d_pack_weights_x3 if precision == PREC_X3F16 else lib.nps_conv2d_pack_weights
    check(fn(ptr(w), ptr(out), Cout, Cin, KH, KW, mode, stream_ptr()), "conv2d_pack_weights")
    out.nps_precision = precision   # read back by conv2d(): the kernel must match the packing
    # how to redo it in place (_repack_stale): the source pointer and the pack arguments (split-fp16 packings only)
    out._nps_job = (w.data_ptr(), Cout, Cin, KH, KW, mode) if precision == PREC_X3F16 else None
    return out


# After an optimizer step every cached packing is stale (trainers/base.py:493 bumps every parameter's version):
# the first stale lookup repacks ALL stale split-fp16 packings of the device in one batched call
# (nps_conv2d_pack_weights_x3_batch, two launches per 48 weights) into their existing buffers, instead of two
# launches per weight and kind (~430 per U-FNO training step, launch-bound).  Dev knob NPS_PACK_BATCH=0: off.
PACK_BATCH = os.environ.get("NPS_PACK_BATCH", "1") != "0"
_PACK_OWNERS = weakref.WeakValueDictionary()  # id(parameter) -> parameter holding a pack cache


def _pack_key(w):
    return (w.data_ptr(), w._version, str(w.device), CONV_PRECISION)


def _replay_jobs(w, packed):
    """The batch jobs that redo `packed` (one tensor or the convT phase list) from w in place, or None."""
    ts = packed if isinstance(packed, list) else [packed]
    jobs = []
    for t in ts:
        j = getattr(t, "_nps_job", None)
        if j is None or j[0] != w.data_ptr():
            return None
        jobs.append(PackJob(w.data_ptr(), t.data_ptr(), *j[1:]))
    return jobs


def _repack_stale(device):
    jobs, fresh = [], []
    for p in list(_PACK_OWNERS.values()):
        if p.device != device:
            continue
        key = _pack_key(p)
        for kind, (k, packed) in list(getattr(p, "_nps_packs", {}).items()):
            if k == key or k[3] != CONV_PRECISION:
                continue
            js = _replay_jobs(p, packed)
            if js is not None:
                jobs += js
                fresh.append((p, kind, key, packed))
    if jobs:
        check(lib.nps_conv2d_pack_weights_x3_batch((PackJob * len(jobs))(*jobs), len(jobs), stream_ptr()),
              "conv2d_pack_weights_x3_batch")
    for p, kind, key, packed in fresh:
        p._nps_packs[kind] = (key, packed)


def cached_pack(w: torch.Tensor, kind, fn):
    """fn(w) — a packed copy of the parameter w — cached on w per `kind` until w changes (data pointer,
    w._version: the optimizer's in-place step bumps it) or the conv precision does.  The inference run()
    paths and the autograd functions share the cache, so a training step packs each weight once for the
    no-grad pushforward unroll and the differentiable forward together; a stale entry first triggers the batched
    repack of every stale packing on the device (_repack_stale)."""
    key = _pack_key(w)
    cache = getattr(w, "_nps_packs", None)
    if cache is None:
        cache = w._nps_packs = {}
    ent = cache.get(kind)
    if ent is not None and ent[0] != key and PACK_BATCH and ent[0][3] == CONV_PRECISION:
        _repack_stale(w.device)
        ent = cache.get(kind)
    if ent is None or ent[0] != key:
        ent = cache[kind] = (key, fn(w))
        _PACK_OWNERS[id(w)] = w
    return ent[1]


def pack_conv_weight(w: torch.Tensor, stride=1, dil=1) -> torch.Tensor:
    """nn.Conv2d weight (Cout, Cin, KH, KW) -> MFMA-fragment-packed buffer (fp32 or split-fp16 fragments,
    whichever the conv of this geometry runs in)."""
    w = w.detach().contiguous()
    Cout, Cin, KH, KW = w.shape
    return _pack(w, Cout, Cin, KH, KW, -1, conv_precision(KH, KW, stride, dil))


def pack_conv_weight_dgrad(w: torch.Tensor, dil=1) -> torch.Tensor:
    """Weight (Cout, Cin, KH, KW) of a stride-1 conv -> the packed weight of its input-gradient conv
    (Cin outputs, Cout inputs, taps flipped): the transpose + flip happen inside the pack kernel (mode -3)."""
    w = w.detach().contiguous()
    Cout, Cin, KH, KW = w.shape
    return _pack(w, Cin, Cout, KH, KW, -3, conv_precision(KH, KW, 1, dil))


def pack_conv_weight_s2d(w: torch.Tensor) -> torch.Tensor:
    """3x3 stride-2 weight (Cout, C, 3, 3) -> packed 2x2 conv over the space-to-depth input (4C channels)."""
    w = w.detach().contiguous()
    Cout, C = w.shape[0], w.shape[1]
    return _pack(w, Cout, 4 * C, 2, 2, -2, conv_precision(2, 2))


def space_to_depth(x: torch.Tensor, pad: int, Hq: int, Wq: int) -> torch.Tensor:
    B, H, W, C = x.shape
    out = torch.empty((B, Hq, Wq, 4 * C), dtype=torch.float32, device=x.device)
    check(lib.nps_space_to_depth(ptr(x), ptr(out), B, H, W, C, pad, Hq, Wq, stream_ptr()), "space_to_depth")
    return share_tag(out, x)


def pack_convT_phases(w: torch.Tensor) -> List[torch.Tensor]:
    """nn.ConvTranspose2d(k=4, s=2) weight (Cin, Cout, 4, 4) -> 4 packed 2x2 phase convs, views of ONE buffer
    (phase ph at ph * nps_phase_stride floats), so the split-fp16 kernel can run all 4 in one launch
    (nps_conv2d_t.nphase, conv2d(phases=...))."""
    w = w.detach().contiguous()
    Cin, Cout = w.shape[0], w.shape[1]
    prec = conv_precision(2, 2)
    n = lib.nps_conv2d_packed_size(Cout, Cin, 4)
    buf = torch.cat([_pack(w, Cout, Cin, 2, 2, ph, prec) for ph in range(4)])
    views = []
    for ph in range(4):
        v = buf[ph * n:(ph + 1) * n]
        v.nps_precision = prec
        v.nps_phase_stride = n
        v._nps_job = (w.data_ptr(), Cout, Cin, 2, 2, ph) if prec == PREC_X3F16 else None
        views.append(v)
    return views


def pack_spectral_weight(w1: torch.Tensor, w2: torch.Tensor, H: int) -> torch.Tensor:
    """weights1/weights2 (Cin, Cout, m1, m2) complex64 -> [R][m2][Cin][Cout] complex for frame height H."""
    w1 = w1.detach().contiguous()
    w2 = w2.detach().contiguous()
    Cin, Cout, m1, m2 = w1.shape
    R = min(H, 2 * m1)
    out = torch.empty((R, m2, Cin, Cout), dtype=torch.complex64, device=w1.device)
    check(lib.nps_spectral_pack_weights(ptr(w1), ptr(w2), ptr(out), Cin, Cout, H, m1, m2, stream_ptr()),
          "spectral_pack_weights")
    return out


# ------------------------------------------------------------------- conv -----
class GN(NamedTuple):
    stats: torch.Tensor      # (B, G, 2) float64
    gamma: torch.Tensor
    beta: torch.Tensor
    groups: int
    eps: float


def group_norm_stats(srcs: Sequence[Src], frame_hw, groups: int) -> torch.Tensor:
    """(B, groups, 2) fp64 (sum, sum of squares) of the virtual frame's groups — the moments of
    nn.GroupNorm.  GroupNorm(1) of sources that each lie wholly inside the frame (crop_Nd zero-pads them,
    it does not cut them): the sum of the sources' carried moments (source_stats)."""
    t0 = srcs[0].t
    B = t0.shape[0]
    if groups == 1 and all(0 <= s.off_y and s.off_y + s.t.shape[1] <= frame_hw[0] and
                           0 <= s.off_x and s.off_x + s.t.shape[2] <= frame_hw[1] for s in srcs):
        parts = [source_stats(s.t) for s in srcs]
        if len(parts) == 1 and parts[0].shape[1] == 1:
            return parts[0]
        return _stats_sum(parts, B, new_stats(B, t0, 1))
    Cin = sum(s.t.shape[3] for s in srcs)
    if _DEBUG_STATS:
        import traceback
        print("nps stats pass (frame)", [tuple(s.t.shape) for s in srcs], frame_hw, groups,
              "".join(traceback.format_stack(limit=5)[:-1]), flush=True)
    stats = torch.empty((B, groups, 2), dtype=torch.float64, device=t0.device)
    check(lib.nps_group_norm_stats(_c_src(srcs), len(srcs), B, frame_hw[0], frame_hw[1], Cin, groups, ptr(stats), 1,
                                   stream_ptr()), "group_norm_stats")
    return stats


def conv2d(srcs: Sequence[Src], frame_hw, wpack: torch.Tensor, bias: Optional[torch.Tensor], Cout: int, KH: int,
           KW: int, stride=1, dil=1, pad=(0, 0), circ=0, out_hw=None, gn: Optional[GN] = None, pre_act=0,
           out: Optional[torch.Tensor] = None, out_nchw=False, out_os=1, out_off=(0, 0), accumulate=False,
           addends: Sequence[torch.Tensor] = (), act=0, add_after_act=False, pad_bottom=None,
           in_scale: Optional[Union[torch.Tensor, int]] = None, out_stats: Optional[torch.Tensor] = None, phases: int = 1,
           s2d_pad: Optional[int] = None, spec: Optional[tuple] = None):
    """One fused conv launch.  `pad` = top/left zero padding (in the circularly
    extended frame), `pad_bottom` defaults to `pad`.  `out_stats`: a new_stats() buffer the launch adds
    the GroupNorm(1) moments of its stored values to (marked incomplete when this conv's kernel cannot;
    attach_stats then ignores it).  `phases` = 4: `wpack` is phase 0 of pack_convT_phases and the launch runs
    all 4 transposed-conv phases, phase (py, px) written at out_off + (py, px) (split-fp16 only).  `s2d_pad`:
    the frame (frame_hw, 4 C channels) is the space-to-depth view of the single source srcs[0] (C % 16 == 0)
    with that padding (nps_conv2d_t.s2d; the Downsample's 3x3/s2 conv as a 2x2 conv).  Returns `out`."""
    t0 = srcs[0].t
    B = t0.shape[0]
    Hin, Win = int(frame_hw[0]), int(frame_hw[1])
    Cin = sum(s.t.shape[3] for s in srcs)
    if s2d_pad is not None:
        if len(srcs) != 1 or Cin % 16 or gn is not None or pre_act or KH != 2 or KW != 2:
            raise ValueError("conv2d: the space-to-depth view takes one 16-channel-aligned source, a 2x2 kernel, "
                             "no prologue")
        Cin *= 4
    cin_alg = Cin  # algorithmic input channels (before any zero channel padding)
    x3 = getattr(wpack, "nps_precision", PREC_F32) == PREC_X3F16
    aligned = not x3 or lib.nps_conv2d_x3_sources_ok(_c_src(srcs), len(srcs))
    fused = (x3 and aligned and FUSE_PROLOGUE and (gn is not None or pre_act) and stride == 1 and dil == 1 and
             lib.nps_conv2d_x3_prologue_ok(KH, KW, Cin, gn.groups if gn is not None else 0, pre_act) and
             (KH * KW != 1 or (FUSE_PROLOGUE_1X1 and Cout <= 192 and not out_nchw and phases == 1)))
    if not fused and (((gn is not None or pre_act) and stride == 1 and dil == 1 and KH == KW and KH in (1, 2, 3))
                      or not aligned):
        # the stride-1 producer/consumer convs stage raw bytes only (the split-fp16 one from 16-channel
        # aligned sources): materialise act(GN(frame)) / the concatenation once
        srcs = [Src(frame_pack(srcs, (Hin, Win), gn, pre_act, pad4=x3))]
        gn, pre_act = None, 0
        Cin = srcs[0].t.shape[3]  # (channel padding: the packed weight is zero for ci >= the true Cin)
    pb = pad if pad_bottom is None else pad_bottom
    if out_hw is None:
        Hout = (Hin + 2 * circ + pad[0] + pb[0] - dil * (KH - 1) - 1) // stride + 1
        Wout = (Win + 2 * circ + pad[1] + pb[1] - dil * (KW - 1) - 1) // stride + 1
    else:
        Hout, Wout = out_hw
    if Hout <= 0 or Wout <= 0:
        raise RuntimeError(f"nps_hip conv2d: empty output {Hout}x{Wout} for input {Hin}x{Win} k={KH}")
    out_given = out is not None
    if out_given:
        drop_stats(out)
    if out is None:
        out = (torch.empty((B, Cout, Hout, Wout), dtype=torch.float32, device=t0.device) if out_nchw
               else empty_nhwc(B, Hout, Wout, Cout, t0))
    if out_nchw:
        oC, oH, oW = out.shape[1], out.shape[2], out.shape[3]
    else:
        oH, oW, oC = out.shape[1], out.shape[2], out.shape[3]
    a = Conv2dArgs()
    a.nsrc = len(srcs)
    a.src = _c_src(srcs)
    a.B, a.Hin, a.Win, a.Cin = B, Hin, Win, Cin
    if s2d_pad is not None:
        a.s2d, a.s2d_pad = 1, int(s2d_pad)
    if gn is not None:
        a.gn_stats, a.gn_gamma, a.gn_beta = ptr(gn.stats), ptr(gn.gamma), ptr(gn.beta)
        a.gn_groups, a.gn_eps = gn.groups, gn.eps
    a.pre_act = pre_act
    a.KH, a.KW, a.stride, a.dil = KH, KW, stride, dil
    a.pad_y, a.pad_x, a.circ = pad[0], pad[1], circ
    a.Hout, a.Wout = Hout, Wout
    a.wpack, a.bias, a.Cout = ptr(wpack), ptr(bias), Cout
    a.out, a.out_C, a.out_H, a.out_W = ptr(out), oC, oH, oW
    a.out_os, a.out_off_y, a.out_off_x = out_os, out_off[0], out_off[1]
    a.out_nchw = 1 if out_nchw else 0
    a.accumulate = 1 if accumulate else 0
    ads = list(addends)
    a.addend0 = ptr(ads[0]) if len(ads) > 0 else None
    a.addend1 = ptr(ads[1]) if len(ads) > 1 else None
    a.act, a.add_after_act = act, (1 if add_after_act else 0)
    a.precision = getattr(wpack, "nps_precision", PREC_F32)
    if spec is not None:  # (Z, m2, scale): the spectral conv's W pass added in the epilogue (spectral_fusable)
        Z, m2s, sc = spec
        if Z.dtype != torch.complex64 or not Z.is_contiguous() or tuple(Z.shape) != (B, Hout, m2s, Cout):
            raise RuntimeError("conv2d: spec Z must be contiguous complex64 (B, Hout, m2, Cout)")
        a.spec_z, a.spec_m2, a.spec_scale = ptr(Z), m2s, float(sc)
    if phases > 1:
        if a.precision != PREC_X3F16 or phases != 4 or out_os != 2:
            raise ValueError("conv2d: merged transposed-conv phases need the split-fp16 2x2 packing and out_os 2")
        a.nphase, a.phase_wstride = 4, wpack.nps_phase_stride
    reserve_tags(out.device, len(srcs) + 1)  # every tag this launch reads or writes, before any pointer
    if a.precision == PREC_X3F16:
        if in_scale is not None:  # explicit range (a tag tensor or its device pointer): overrides the sources' tags
            a.in_scale = in_scale if isinstance(in_scale, int) else ptr(in_scale)
        elif USE_IN_TAGS and not (fused and gn is not None):
            # the sources' tags (a fused GroupNorm prologue normalises the frame: its output range is not
            # the sources'; the kernel bounds it from gamma, beta and the group size, gn_prologue_scale)
            tags = [input_tag(s.t) for s in srcs] + [None, None]
            a.in_scale, a.in_tag1, a.in_tag2 = tags[0], tags[1], tags[2]
    if USE_OUT_TAGS:
        a.out_tag = out_tag(out, accumulate) if out_given else new_tag(out)
    if out_stats is not None:
        # 1x1: the LDS-weight kernel's fused epilogue (at most one addend, no accumulate) takes the moments of the
        # stored values, activation and addend included
        plain = not accumulate and len(ads) <= 1
        x1_ok = Cout <= 192 and plain
        if (a.precision == PREC_X3F16 and (KH * KW != 1 or x1_ok)
                and not out_nchw and oC % 4 == 0 and Cout % 4 == 0):
            a.out_stats = ptr(out_stats)
        else:
            out_stats._nps_incomplete = True
    if lib.nps_conv2d_plan(ctypes_byref(a)) < 0:
        raise RuntimeError("conv2d_plan failed: " + lib.nps_last_error().decode())
    if conv_probe is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        check(lib.nps_conv2d_fwd(ctypes_byref(a), stream_ptr()), "conv2d_fwd")
        e1.record()
        nph = max(phases, 1)
        nbytes = 4.0 * (sum(s.t.numel() for s in srcs) + nph * (Cout * cin_alg * KH * KW + B * Hout * Wout * Cout))
        conv_probe.append((e0, e1, 2.0 * nph * B * Hout * Wout * Cout * cin_alg * KH * KW,
                           ("x3f16" if a.precision == PREC_X3F16 else "f32", KH * KW, a.waves), nbytes))
        if conv_shape_log is not None:
            conv_shape_log.append(dict(cin=cin_alg, cout=Cout, k=(KH, KW), hw=(Hin, Win), out=(Hout, Wout), B=B,
                                       nsrc=len(srcs), acc=bool(accumulate), addends=len(ads), act=act,
                                       gn=gn is not None, pre_act=pre_act, stats=out_stats is not None))
    else:
        check(lib.nps_conv2d_fwd(ctypes_byref(a), stream_ptr()), "conv2d_fwd")
    return out


def absmax(x: torch.Tensor) -> torch.Tensor:
    """Range tag (TAG_FLOATS fp32 device tensor, value max|x|) — the input range of a split-fp16 conv
    (conv2d(in_scale=...)); tag_value() reads it back."""
    x = x.contiguous()
    out = torch.empty(TAG_FLOATS, dtype=torch.float32, device=x.device)
    check(lib.nps_absmax(ptr(x), x.numel(), ptr(out), stream_ptr()), "absmax")
    return out


def tag_value(tag) -> float:
    """Host value of a range tag (a tag tensor, or a tensor carrying a live tag) — for tests / diagnostics."""
    if isinstance(tag, torch.Tensor) and tag.numel() == TAG_FLOATS and tag_of(tag) is None:
        return float(tag.view(64, 64)[:, 0].max())
    t = tag_of(tag)
    if t is None:
        return float("nan")
    i = (t.ptr - t.arena.buf.data_ptr()) // 4
    return float(t.arena.buf[i:i + TAG_FLOATS].view(64, 64)[:, 0].max())


def frame_pack(srcs: Sequence[Src], frame_hw, gn: Optional[GN] = None, pre_act=0, pad4=False) -> torch.Tensor:
    """(B, Hin, Win, Cin) = act(GN(virtual frame)) — nps_frame_pack; pad4: channels zero-padded to a
    multiple of 4 (the split-fp16 conv stages 16-B channel groups)."""
    t0 = srcs[0].t
    B = t0.shape[0]
    Hin, Win = int(frame_hw[0]), int(frame_hw[1])
    Cin = sum(s.t.shape[3] for s in srcs)
    a = Conv2dArgs()
    a.nsrc = len(srcs)
    a.src = _c_src(srcs)
    a.B, a.Hin, a.Win, a.Cin = B, Hin, Win, Cin
    if gn is not None:
        a.gn_stats, a.gn_gamma, a.gn_beta = ptr(gn.stats), ptr(gn.gamma), ptr(gn.beta)
        a.gn_groups, a.gn_eps = gn.groups, gn.eps
    a.pre_act = pre_act
    a.out_C = (Cin + 3) // 4 * 4 if pad4 else Cin
    out = empty_nhwc(B, Hin, Win, a.out_C, t0)
    a.out_tag = new_tag(out)
    check(lib.nps_frame_pack(ctypes_byref(a), ptr(out), stream_ptr()), "frame_pack")
    return out


def ctypes_byref(x):
    import ctypes
    return ctypes.byref(x)


# --------------------------------------------------------------- spectral -----
def spectral_z(srcs: Sequence[Src], wpack: torch.Tensor, m1: int, m2: int, Cout: int) -> torch.Tensor:
    """Z (B, H, m2, Cout) complex64: the spectral conv up to its W-pass synthesis (rfft2 W and H passes on the
    retained modes, the mode mixing, the inverse H pass; proc_fno.py:257-288) — spectral_conv2d's idft_w input, or the
    spec_z a 1x1 conv's epilogue synthesises itself (conv2d(spec=...), the FNO layer fusion)."""
    t0 = srcs[0].t
    B, H, W = t0.shape[0], t0.shape[1], t0.shape[2]
    Cin = sum(s.t.shape[3] for s in srcs)
    if not (m1 <= H and m2 <= W // 2 + 1):
        raise AssertionError("modes should be at most the spatial dim (// 2 + 1 for the last spatial dimension)")
    R = min(H, 2 * m1)
    dev = t0.device
    X1 = torch.empty((B, H, m2, Cin), dtype=torch.complex64, device=dev)
    X2 = torch.empty((B, R, m2, Cin), dtype=torch.complex64, device=dev)
    Y = torch.empty((B, R, m2, Cout), dtype=torch.complex64, device=dev)
    Z = torch.empty((B, H, m2, Cout), dtype=torch.complex64, device=dev)
    s = stream_ptr()
    check(lib.nps_spectral_dft_w(_c_src(srcs), len(srcs), B, H, W, Cin, m2, ptr(X1), s), "spectral_dft_w")
    check(lib.nps_spectral_dft_h(ptr(X1), ptr(X2), B, H, m1, m2, Cin, s), "spectral_dft_h")
    check(lib.nps_spectral_mix(ptr(X2), ptr(wpack), ptr(Y), B, R, m2, Cin, Cout, s), "spectral_mix")
    check(lib.nps_spectral_idft_h(ptr(Y), ptr(Z), B, H, m1, m2, Cout, s), "spectral_idft_h")
    return Z


# the FNO layer's 1x1 `w` synthesises the spectral conv's W pass in its epilogue (nps_conv2d_t.spec_z) instead of a
# separate idft_w read-modify-write of its output (dev knob NPS_FUSE_IDFT=0: off)
FUSE_IDFT = os.environ.get("NPS_FUSE_IDFT", "1") != "0"


def spectral_fusable(W: int, m2: int, Cout: int) -> bool:
    """Whether conv2d(spec=...) can take this spectral conv's W pass (nps_conv2d_t.spec_z conditions)."""
    return (FUSE_IDFT and CONV_PRECISION == PREC_X3F16 and W % 128 == 0 and m2 <= 16
            and Cout <= 192 and Cout % 4 == 0)


def spectral_conv2d(srcs: Sequence[Src], wpack: torch.Tensor, m1: int, m2: int, Cout: int,
                    out: Optional[torch.Tensor] = None, accumulate=False, addend=None, act=0):
    """y = irfft2(P(rfft2(x))) on the retained modes (proc_fno.py:257-288), NHWC in/out."""
    t0 = srcs[0].t
    B, H, W = t0.shape[0], t0.shape[1], t0.shape[2]
    Z = spectral_z(srcs, wpack, m1, m2, Cout)
    if out is not None:
        drop_stats(out)
    if out is None:
        out = empty_nhwc(B, H, W, Cout, t0)
        accumulate = False
        tag = new_tag(out)
    else:
        tag = out_tag(out, accumulate)
    check(lib.nps_spectral_idft_w(ptr(Z), ptr(out), B, H, W, m2, Cout, 1 if accumulate else 0, ptr(addend), act,
                                  tag, stream_ptr()), "spectral_idft_w")
    return out


def pack_spectral3d_weight(ws: Sequence[torch.Tensor], D: int, H: int) -> torch.Tensor:
    """SpectralConv3d weights1..4 (Cin, Cout, m1, m2, m3) complex64 -> wpack [R1][R2][m3][Cin][Cout]."""
    w1, w2, w3, w4 = [w.detach().contiguous() for w in ws]
    Cin, Cout, m1, m2, m3 = w1.shape
    R1, R2 = min(D, 2 * m1), min(H, 2 * m2)
    out = torch.empty((R1, R2, m3, Cin, Cout), dtype=torch.complex64, device=w1.device)
    check(lib.nps_spectral3d_pack_weights(ptr(w1), ptr(w2), ptr(w3), ptr(w4), ptr(out), Cin, Cout, D, H, m1, m2, m3,
                                          stream_ptr()), "spectral3d_pack_weights")
    return out


def check_modes3d(D, H, W, m1, m2, m3):
    """proc_fno.py:134-139 for three spatial dims."""
    if not (m1 <= D and m2 <= H and m3 <= W // 2 + 1):
        raise AssertionError("modes should be at most the spatial dim (// 2 + 1 for the last spatial dimension)")


def spectral_conv3d_stages(x4: Sequence[Src], D, H, W, Cin, wpack, m1, m2, m3, Cout, out, accumulate=False,
                           addend=None, act=0):
    """The SpectralConv3d forward chain on a virtual NDHWC frame given as (B, D*H, W, C) sources.
    Returns the X3 spectrum (kept for the backward)."""
    B = x4[0].t.shape[0]
    R1, R2 = min(D, 2 * m1), min(H, 2 * m2)
    dev = x4[0].t.device
    c64 = torch.complex64
    X1 = torch.empty((B, D * H, m3, Cin), dtype=c64, device=dev)
    X2 = torch.empty((B * D, R2, m3, Cin), dtype=c64, device=dev)
    X3 = torch.empty((B, R1, R2 * m3, Cin), dtype=c64, device=dev)
    Y = torch.empty((B, R1, R2 * m3, Cout), dtype=c64, device=dev)
    Z1 = torch.empty((B, D, R2 * m3, Cout), dtype=c64, device=dev)
    Z2 = torch.empty((B * D, H, m3, Cout), dtype=c64, device=dev)
    s = stream_ptr()
    check(lib.nps_spectral_dft_w(_c_src(x4), len(x4), B, D * H, W, Cin, m3, ptr(X1), s), "spectral3d dft_w")
    check(lib.nps_spectral_dft_h(ptr(X1), ptr(X2), B * D, H, m2, m3, Cin, s), "spectral3d dft_h (H)")
    check(lib.nps_spectral_dft_h(ptr(X2), ptr(X3), B, D, m1, R2 * m3, Cin, s), "spectral3d dft_h (D)")
    check(lib.nps_spectral_mix(ptr(X3), ptr(wpack), ptr(Y), B, R1, R2 * m3, Cin, Cout, s), "spectral3d mix")
    check(lib.nps_spectral_idft_h(ptr(Y), ptr(Z1), B, D, m1, R2 * m3, Cout, s), "spectral3d idft_h (D)")
    check(lib.nps_spectral_idft_h(ptr(Z1), ptr(Z2), B * D, H, m2, m3, Cout, s), "spectral3d idft_h (H)")
    check(lib.nps_spectral_idft_w(ptr(Z2), ptr(out), B, D * H, W, m3, Cout, 1 if accumulate else 0, ptr(addend), act,
                                  out_tag(out, accumulate), s), "spectral3d idft_w")
    return X3


def spectral_conv3d(srcs: Sequence[Src], D: int, wpack: torch.Tensor, m1: int, m2: int, m3: int, Cout: int,
                    out: Optional[torch.Tensor] = None, accumulate=False, addend=None, act=0):
    """y = irfftn(P(rfftn(x))) on the 4 retained corners (proc_fno.py:334-376).  Sources are NDHWC
    tensors viewed as (B, D*H, W, C); returns (B, D*H, W, Cout) (view it as (B, D, H, W, Cout))."""
    t0 = srcs[0].t
    B, DH, W = t0.shape[0], t0.shape[1], t0.shape[2]
    H = DH // D
    Cin = sum(s.t.shape[3] for s in srcs)
    check_modes3d(D, H, W, m1, m2, m3)
    if out is not None:
        drop_stats(out)
    if out is None:
        out = empty_nhwc(B, DH, W, Cout, t0)
        accumulate = False
    spectral_conv3d_stages(srcs, D, H, W, Cin, wpack, m1, m2, m3, Cout, out, accumulate, addend, act)
    return out


# ------------------------------------------------------------------ bf16 storage (C5) -----
def _c_src_bf16(srcs: Sequence[Src]):
    arr = (_CSrc * 3)()
    for i, s in enumerate(srcs):
        t = s.t
        if t.dtype != torch.bfloat16 or not t.is_contiguous() or t.dim() != 4:
            raise RuntimeError(f"nps_hip: bf16 sources must be contiguous bf16 NHWC, got {t.dtype} {tuple(t.shape)}")
        arr[i].ptr = ptr(t)
        arr[i].H, arr[i].W, arr[i].C = t.shape[1], t.shape[2], t.shape[3]
        arr[i].off_y, arr[i].off_x = int(s.off_y), int(s.off_x)
    return arr


def to_bf16(x: torch.Tensor) -> torch.Tensor:
    """bf16 copy (round-to-nearest-even) of an fp32 (or complex64, as its (re, im) pairs) device tensor."""
    if x.dtype not in (torch.float32, torch.complex64):
        raise TypeError(f"nps_hip to_bf16: expected float32 or complex64, got {x.dtype}")
    x = x.contiguous()
    xf = torch.view_as_real(x) if x.is_complex() else x
    out = torch.empty(xf.shape, dtype=torch.bfloat16, device=x.device)
    check(lib.nps_f32_to_bf16(ptr(xf), xf.numel(), ptr(out), stream_ptr()), "f32_to_bf16")
    return out


def to_f32(x: torch.Tensor) -> torch.Tensor:
    """fp32 copy of a bf16 device tensor."""
    if x.dtype != torch.bfloat16:
        raise TypeError(f"nps_hip to_f32: expected bfloat16, got {x.dtype}")
    x = x.contiguous()
    out = torch.empty(x.shape, dtype=torch.float32, device=x.device)
    check(lib.nps_bf16_to_f32(ptr(x), x.numel(), ptr(out), stream_ptr()), "bf16_to_f32")
    return out


def pack_1x1_bf16(w: torch.Tensor) -> torch.Tensor:
    """Pointwise conv weight (Cout, Cin[, 1...]) fp32 -> the bf16 [Cout][KR] packing of nps_conv1x1_bf16."""
    w = w.detach().reshape(w.shape[0], w.shape[1]).contiguous()
    Cout, Cin = w.shape
    out = torch.empty(Cout * lib.nps_conv1x1_bf16_kr(Cin), dtype=torch.bfloat16, device=w.device)
    check(lib.nps_pack_1x1_bf16(ptr(w), ptr(out), Cout, Cin, stream_ptr()), "pack_1x1_bf16")
    return out


def conv1x1_bf16(srcs: Sequence[Src], wpack: torch.Tensor, bias: Optional[torch.Tensor], Cout: int, act=0,
                 addend: Optional[torch.Tensor] = None) -> torch.Tensor:
    """act(w x + bias [+ addend]) of a bf16 NHWC virtual frame (sources covering it) -> bf16 (B, H, W, Cout)."""
    t0 = srcs[0].t
    B, H, W = t0.shape[0], t0.shape[1], t0.shape[2]
    a = Conv2dArgs()
    a.nsrc = len(srcs)
    a.src = _c_src_bf16(srcs)
    a.B, a.Hin, a.Win, a.Cin = B, H, W, sum(s.t.shape[3] for s in srcs)
    a.KH = a.KW = a.stride = a.dil = 1
    a.Hout, a.Wout = H, W
    a.wpack, a.bias, a.Cout = ptr(wpack), ptr(bias), Cout
    out = torch.empty((B, H, W, Cout), dtype=torch.bfloat16, device=t0.device)
    a.out, a.out_C, a.out_H, a.out_W, a.out_os = ptr(out), Cout, H, W, 1
    a.addend0 = ptr(addend)
    a.act = act
    check(lib.nps_conv1x1_bf16(ctypes_byref(a), stream_ptr()), "conv1x1_bf16")
    return out


def spectral_conv3d_bf16(srcs: Sequence[Src], D: int, wpack_bf16: torch.Tensor, m1: int, m2: int, m3: int, Cout: int,
                         out: Optional[torch.Tensor] = None, accumulate=False, addend=None, act=0):
    """spectral_conv3d with bf16 activations in / out and bf16 packed weights (fp32 spectra and sums)."""
    t0 = srcs[0].t
    B, DH, W = t0.shape[0], t0.shape[1], t0.shape[2]
    H = DH // D
    Cin = sum(s.t.shape[3] for s in srcs)
    check_modes3d(D, H, W, m1, m2, m3)
    if out is not None:
        drop_stats(out)
    if out is None:
        out = torch.empty((B, DH, W, Cout), dtype=torch.bfloat16, device=t0.device)
        accumulate = False
    R1, R2 = min(D, 2 * m1), min(H, 2 * m2)
    dev = t0.device
    c64 = torch.complex64
    X1 = torch.empty((B, D * H, m3, Cin), dtype=c64, device=dev)
    X2 = torch.empty((B * D, R2, m3, Cin), dtype=c64, device=dev)
    X3 = torch.empty((B, R1, R2 * m3, Cin), dtype=c64, device=dev)
    Y = torch.empty((B, R1, R2 * m3, Cout), dtype=c64, device=dev)
    Z1 = torch.empty((B, D, R2 * m3, Cout), dtype=c64, device=dev)
    Z2 = torch.empty((B * D, H, m3, Cout), dtype=c64, device=dev)
    s = stream_ptr()
    check(lib.nps_spectral_dft_w_bf16(_c_src_bf16(srcs), len(srcs), B, D * H, W, Cin, m3, ptr(X1), s), "dft_w bf16")
    check(lib.nps_spectral_dft_h(ptr(X1), ptr(X2), B * D, H, m2, m3, Cin, s), "spectral3d dft_h (H)")
    check(lib.nps_spectral_dft_h(ptr(X2), ptr(X3), B, D, m1, R2 * m3, Cin, s), "spectral3d dft_h (D)")
    check(lib.nps_spectral_mix_bf16(ptr(X3), ptr(wpack_bf16), ptr(Y), B, R1, R2 * m3, Cin, Cout, s), "mix bf16")
    check(lib.nps_spectral_idft_h(ptr(Y), ptr(Z1), B, D, m1, R2 * m3, Cout, s), "spectral3d idft_h (D)")
    check(lib.nps_spectral_idft_h(ptr(Z1), ptr(Z2), B * D, H, m2, m3, Cout, s), "spectral3d idft_h (H)")
    check(lib.nps_spectral_idft_w_bf16(ptr(Z2), ptr(out), B, D * H, W, m3, Cout, 1 if accumulate else 0, ptr(addend),
                                       act, s), "idft_w bf16")
    return out


# ------------------------------------------------------------ 3-D U-Net (C5) -----
class Src3(NamedTuple):
    t: torch.Tensor          # (B, D, H, W, C) NDHWC contiguous, fp32 or bf16
    off_d: int = 0
    off_h: int = 0
    off_w: int = 0


def _fill_frame3(a, srcs: Sequence[Src3], frame_dhw):
    t0 = srcs[0].t
    dt = t0.dtype
    if dt not in (torch.float32, torch.bfloat16):
        raise RuntimeError(f"nps_hip conv3d: fp32 or bf16 sources, got {dt}")
    a.nsrc = len(srcs)
    for i, s in enumerate(srcs):
        t = s.t
        if t.dtype != dt or not t.is_contiguous() or t.dim() != 5 or t.shape[0] != t0.shape[0]:
            raise RuntimeError(f"nps_hip conv3d: sources must be contiguous NDHWC of one dtype / batch, got "
                               f"{t.dtype} {tuple(t.shape)}")
        a.src[i].ptr = ptr(t)
        a.src[i].D, a.src[i].H, a.src[i].W, a.src[i].C = t.shape[1], t.shape[2], t.shape[3], t.shape[4]
        a.src[i].off_d, a.src[i].off_h, a.src[i].off_w = int(s.off_d), int(s.off_h), int(s.off_w)
    a.B = t0.shape[0]
    a.Dc, a.Hc, a.Wc = (int(v) for v in frame_dhw)
    a.Cin = sum(s.t.shape[4] for s in srcs)
    a.bf16 = 1 if dt == torch.bfloat16 else 0
    return a


def pack_conv3d_weight(w: torch.Tensor, transposed=False, bf16=False) -> torch.Tensor:
    """nn.Conv3d weight (Cout, Cin, K, K, K) / nn.ConvTranspose3d weight (Cin, Cout, 4, 4, 4) -> the
    nps_conv3d packing in fp32 or bf16."""
    w = w.detach().float().contiguous()
    if transposed:
        Cin, Cout, K = w.shape[0], w.shape[1], 2
    else:
        Cout, Cin, K = w.shape[0], w.shape[1], w.shape[2]
    nbytes = lib.nps_conv3d_packed_bytes(Cout, Cin, K, 1 if transposed else 0, 1 if bf16 else 0)
    out = torch.empty(nbytes // (2 if bf16 else 4), dtype=torch.bfloat16 if bf16 else torch.float32, device=w.device)
    check(lib.nps_conv3d_pack_weights(ptr(w), ptr(out), Cout, Cin, K, 1 if transposed else 0, 1 if bf16 else 0,
                                      stream_ptr()), "conv3d_pack_weights")
    return out


def gn_stats3d(srcs: Sequence[Src3], frame_dhw, groups: int) -> torch.Tensor:
    """(B, groups, 2) fp64 (sum, sum of squares) of the virtual NDHWC frame's GroupNorm groups."""
    a = _fill_frame3(Conv3dArgs(), srcs, frame_dhw)
    st = torch.zeros((a.B, groups, 2), dtype=torch.float64, device=srcs[0].t.device)
    check(lib.nps_gn_stats3d(ctypes_byref(a), groups, ptr(st), stream_ptr()), "gn_stats3d")
    return st


# 3-D GroupNorm(1) frames take their sources' carried moments (the 3-D convs' out_stats) instead of an nps_gn_stats3d
# pass over the frame (dev knob NPS_CARRY3D=0: always the pass)
CARRY3D = os.environ.get("NPS_CARRY3D", "1") != "0"


def source_stats3d(t: torch.Tensor) -> torch.Tensor:
    """NDHWC t's GroupNorm(1) moments: carried, or one nps_gn_stats3d pass (then carried)."""
    st = stats_of(t)
    if st is None:
        st = gn_stats3d([Src3(t)], tuple(t.shape[1:4]), 1)
        attach_stats(t, st)
    return st


def group_norm_stats3d(srcs: Sequence[Src3], frame_dhw, groups: int) -> torch.Tensor:
    """gn_stats3d of a 3-D frame; GroupNorm(1) of sources that lie wholly inside the frame (crop_Nd zero-pads them,
    it does not cut them): the sum of the sources' carried moments (source_stats3d), as the 2-D group_norm_stats."""
    t0 = srcs[0].t
    if CARRY3D and groups == 1 and all(
            all(0 <= o and o + n <= f for o, n, f in zip((s.off_d, s.off_h, s.off_w), s.t.shape[1:4], frame_dhw))
            for s in srcs):
        parts = [source_stats3d(s.t) for s in srcs]
        if len(parts) == 1 and parts[0].shape[1] == 1:
            return parts[0]
        return _stats_sum(parts, t0.shape[0], new_stats(t0.shape[0], t0, 1))
    return gn_stats3d(srcs, frame_dhw, groups)


# Materialise act(GN(frame)) before a K > 1 conv whose frame needs a prologue or several / offset / unaligned
# sources (nps_frame_pack3d), so the conv runs its single-source fast path (dev knob NPS_CONV3D_PACK=0: off)
CONV3D_PACK = os.environ.get("NPS_CONV3D_PACK", "1") == "1"


def frame_pack3d(srcs: Sequence[Src3], frame_dhw, gn: Optional[GN] = None, pre_act=0) -> torch.Tensor:
    """(B, Dc, Hc, Wc, Cpad) = act(GN(virtual frame)), channels zero-padded to a multiple of 16."""
    a = _fill_frame3(Conv3dArgs(), srcs, frame_dhw)
    if gn is not None:
        a.gn_stats, a.gn_gamma, a.gn_beta = ptr(gn.stats), ptr(gn.gamma), ptr(gn.beta)
        a.gn_groups, a.gn_eps = gn.groups, gn.eps
    a.pre_act = pre_act
    cpad = (a.Cin + 15) // 16 * 16
    out = torch.empty((a.B, a.Dc, a.Hc, a.Wc, cpad), dtype=srcs[0].t.dtype, device=srcs[0].t.device)
    check(lib.nps_frame_pack3d(ctypes_byref(a), ptr(out), cpad, stream_ptr()), "frame_pack3d")
    return out


def conv3d(srcs: Sequence[Src3], frame_dhw, wpack: torch.Tensor, bias: Optional[torch.Tensor], Cout: int, K: int,
           stride=1, transposed=False, circ=0, zpad=0, gn: Optional[GN] = None, pre_act=0,
           out: Optional[torch.Tensor] = None, out_os=1, out_off=(0, 0, 0), accumulate=False,
           addend: Optional[torch.Tensor] = None, act=0, out_stats: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One nps_conv3d launch over a virtual NDHWC frame (sources at crop offsets), extended per side by
    `circ` circular then `zpad` zero voxels; valid K^3 conv (stride), or with `transposed` the 8 phase convs
    (K = 2) of a k4/s2 transposed conv written with out_os = 2.  Without `out` a tensor of the conv's
    output extent (x2 per axis when transposed) is allocated.  Returns `out`."""
    simple = (len(srcs) == 1 and gn is None and not pre_act and tuple(srcs[0].t.shape[1:4]) == tuple(frame_dhw)
              and not (srcs[0].off_d or srcs[0].off_h or srcs[0].off_w) and srcs[0].t.shape[4] % 16 == 0)
    cin_alg = sum(s.t.shape[4] for s in srcs)  # algorithmic input channels (before channel padding)
    if CONV3D_PACK and K > 1 and not simple:
        srcs, gn, pre_act = [Src3(frame_pack3d(srcs, frame_dhw, gn, pre_act))], None, 0
    a = _fill_frame3(Conv3dArgs(), srcs, frame_dhw)
    ext = 2 * (circ + zpad)
    Dout, Hout, Wout = ((n + ext - K) // stride + 1 for n in (a.Dc, a.Hc, a.Wc))
    if min(Dout, Hout, Wout) <= 0:
        raise RuntimeError(f"nps_hip conv3d: empty output for frame {tuple(frame_dhw)} K={K}")
    dt = srcs[0].t.dtype
    if (wpack.dtype == torch.bfloat16) != (dt == torch.bfloat16):
        raise RuntimeError("nps_hip conv3d: weight packing dtype must match the activations")
    if out is None:
        f = 2 if transposed else 1
        out = torch.empty((a.B, f * Dout, f * Hout, f * Wout, Cout), dtype=dt, device=srcs[0].t.device)
        if transposed:
            out_os = 2
    if out.dtype != dt or not out.is_contiguous() or out.dim() != 5:
        raise RuntimeError("nps_hip conv3d: out must be contiguous NDHWC of the sources' dtype")
    if addend is not None and (addend.shape != out.shape or addend.dtype != dt or not addend.is_contiguous()):
        raise RuntimeError("nps_hip conv3d: addend must be laid out like out")
    a.circ, a.zpad = circ, zpad
    if gn is not None:
        a.gn_stats, a.gn_gamma, a.gn_beta = ptr(gn.stats), ptr(gn.gamma), ptr(gn.beta)
        a.gn_groups, a.gn_eps = gn.groups, gn.eps
    a.pre_act = pre_act
    a.K, a.stride, a.transposed = K, stride, 1 if transposed else 0
    a.Dout, a.Hout, a.Wout = Dout, Hout, Wout
    a.out_stats = ptr(out_stats)  # (new_stats(B, ..) buffer: the stored values' GroupNorm(1) moments)
    a.wpack, a.bias, a.Cout = ptr(wpack), ptr(bias), Cout
    a.out, a.out_C, a.out_D, a.out_H, a.out_W = ptr(out), out.shape[4], out.shape[1], out.shape[2], out.shape[3]
    a.out_os, (a.out_off_d, a.out_off_h, a.out_off_w) = out_os, out_off
    a.accumulate, a.addend, a.act = 1 if accumulate else 0, ptr(addend), act
    if conv_probe is not None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        check(lib.nps_conv3d_fwd(ctypes_byref(a), stream_ptr()), "conv3d")
        e1.record()
        nph = 8 if transposed else 1
        es = 2 if a.bf16 else 4
        nbytes = es * (sum(s.t.numel() for s in srcs) + nph * Cout * cin_alg * K ** 3 + nph * a.B * Dout * Hout * Wout * Cout)
        conv_probe.append((e0, e1, 2.0 * nph * a.B * Dout * Hout * Wout * Cout * cin_alg * K ** 3,
                           ("bf16_3d" if a.bf16 else "f32_3d", K ** 3, 4), nbytes))
    else:
        check(lib.nps_conv3d_fwd(ctypes_byref(a), stream_ptr()), "conv3d")
    return out


# ------------------------------------------------------------------ data path -----
def gather_windows(u: torch.Tensor, steps, tw: int, offset: int) -> torch.Tensor:
    """out[b] = u[b][:, steps[b] + offset : steps[b] + offset + tw] for a device-resident trajectory batch
    u (B, C, T, *spatial) — DataCreator.create_data's per-sample windows (common/data_creator.py:48-78) as
    one HIP gather (nps_gather_windows)."""
    u = u.contiguous()
    B, C, T = u.shape[:3]
    HW = math.prod(u.shape[3:]) if u.dim() > 3 else 1
    if len(steps) != B:
        raise ValueError(f"gather_windows: {len(steps)} steps for a batch of {B}")
    for st in steps:
        if st + offset < 0 or st + offset + tw > T:
            raise AssertionError("this step - time window combination is not valid")
    st_dev = torch.tensor([int(v) for v in steps], dtype=torch.int32).to(u.device, non_blocking=True)
    out = torch.empty((B, C, tw) + tuple(u.shape[3:]), dtype=torch.float32, device=u.device)
    check(lib.nps_gather_windows(ptr(u), ptr(st_dev), ptr(out), B, C, T, HW, tw, offset, stream_ptr()),
          "gather_windows")
    return out


# ----------------------------------------------------------- misc kernels -----
def nchw_to_nhwc(x: torch.Tensor) -> torch.Tensor:
    x = x.contiguous()
    B, C, H, W = x.shape
    out = torch.empty((B, H, W, C), dtype=torch.float32, device=x.device)
    check(lib.nps_nchw_to_nhwc(ptr(x), ptr(out), B, C, H, W, stream_ptr()), "nchw_to_nhwc")
    return share_tag(out, x)


def nhwc_to_nchw(x: torch.Tensor) -> torch.Tensor:
    B, H, W, C = x.shape
    out = torch.empty((B, C, H, W), dtype=torch.float32, device=x.device)
    check(lib.nps_nhwc_to_nchw(ptr(x), ptr(out), B, C, H, W, stream_ptr()), "nhwc_to_nchw")
    return share_tag(out, x)


def pack_grid_input(u, pos, cond, sc, Cp):
    """-> (xin (B,H,W,Cp), vb (B,H,W,K+S) or None)."""
    B, c, tw, H, W = u.shape
    K = 0 if cond is None else cond.shape[1]
    S = 0 if sc is None else sc.shape[1]
    xin = torch.empty((B, H, W, Cp), dtype=torch.float32, device=u.device)
    vb = torch.empty((B, H, W, K + S), dtype=torch.float32, device=u.device) if K + S > 0 else None
    check(lib.nps_pack_grid_input(ptr(u), ptr(pos), ptr(cond), ptr(sc), ptr(xin), ptr(vb), B, c * tw, H, W, K, S, Cp,
                                  stream_ptr()), "pack_grid_input")
    return xin, vb


def timeconv_decode(pre, u, w1, b1, w2, b2, dtcum, mask, mask_ch, act_tanh, num_c, tw):
    B, _, _, H, W = u.shape
    out = torch.empty((B, num_c, tw, H, W), dtype=torch.float32, device=u.device)
    S = 0 if mask is None else mask.shape[1]
    check(lib.nps_timeconv_decode(ptr(pre), ptr(u), ptr(w1), ptr(b1), ptr(w2), ptr(b2), ptr(dtcum), ptr(mask), S,
                                  mask_ch, ptr(out), B, num_c, tw, H, W, 1 if act_tanh else 0, stream_ptr()),
          "timeconv_decode")
    return out


def plane_sums(base: torch.Tensor, offset: int, plane_stride: int, plane_size: int, nplanes: int) -> torch.Tensor:
    sums = torch.empty(nplanes, dtype=torch.float64, device=base.device)
    check(lib.nps_plane_sums(ptr(base) + 4 * offset, plane_stride, plane_size, nplanes, ptr(sums), stream_ptr()),
          "plane_sums")
    return sums


def volume_rescale(u, new_tot, prev_tot, mpdcum, mask, mask_ch):
    B, c, tw, H, W = u.shape
    S = 0 if mask is None else mask.shape[1]
    check(lib.nps_volume_rescale(ptr(u), ptr(new_tot), ptr(prev_tot), ptr(mpdcum), ptr(mask), S, mask_ch, B, c, tw,
                                 H, W, stream_ptr()), "volume_rescale")
    return u


def sq_err_sum(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    a = a.contiguous()
    b = b.contiguous()
    if a.shape != b.shape:
        raise RuntimeError(f"sq_err_sum: shape mismatch {tuple(a.shape)} vs {tuple(b.shape)}")
    out = torch.zeros(1, dtype=torch.float64, device=a.device)
    check(lib.nps_sq_err_sum(ptr(a), ptr(b), a.numel(), ptr(out), stream_ptr()), "sq_err_sum")
    return out[0]
