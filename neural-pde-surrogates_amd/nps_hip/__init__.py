"""ctypes binding of libnps_hip.so — the C ABI declared in include/nps.h.

This is the product's only compute path: every function here launches a
hand-written gfx950 HIP kernel on the caller's current torch stream.  There is
no CPU or torch fallback; importing this module raises if the library is
missing, and every op raises unless its tensors are fp32 on a ROCm device.

Tensors are passed as raw device pointers; PyTorch provides the memory
(caching allocator), streams and graph capture only.
"""
import ctypes
import os

import torch

__all__ = ["lib", "Src", "Conv2dArgs", "WgradArgs", "Src3", "Conv3dArgs", "PackJob", "check", "stream_ptr", "ptr", "LIB_PATH"]

LIB_PATH = os.environ.get("NPS_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)), "libnps_hip.so"))
if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"nps_hip: {LIB_PATH} not found. Build it with `python -c 'import __graft_entry__ as g; g.build()'` "
        "or `make -C neural-pde-surrogates_amd/csrc` (hipcc --offload-arch=gfx950).")
lib = ctypes.CDLL(LIB_PATH)

MAX_SRC = 3


class Src(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("C", ctypes.c_int), ("H", ctypes.c_int), ("W", ctypes.c_int),
                ("off_y", ctypes.c_int), ("off_x", ctypes.c_int)]


class Conv2dArgs(ctypes.Structure):
    _fields_ = [
        ("nsrc", ctypes.c_int), ("src", Src * MAX_SRC),
        ("B", ctypes.c_int), ("Hin", ctypes.c_int), ("Win", ctypes.c_int), ("Cin", ctypes.c_int),
        ("gn_stats", ctypes.c_void_p), ("gn_gamma", ctypes.c_void_p), ("gn_beta", ctypes.c_void_p),
        ("gn_groups", ctypes.c_int), ("gn_eps", ctypes.c_float), ("pre_act", ctypes.c_int),
        ("KH", ctypes.c_int), ("KW", ctypes.c_int), ("stride", ctypes.c_int), ("dil", ctypes.c_int),
        ("pad_y", ctypes.c_int), ("pad_x", ctypes.c_int), ("circ", ctypes.c_int),
        ("Hout", ctypes.c_int), ("Wout", ctypes.c_int),
        ("wpack", ctypes.c_void_p), ("bias", ctypes.c_void_p), ("Cout", ctypes.c_int),
        ("out", ctypes.c_void_p), ("out_C", ctypes.c_int), ("out_H", ctypes.c_int), ("out_W", ctypes.c_int),
        ("out_os", ctypes.c_int), ("out_off_y", ctypes.c_int), ("out_off_x", ctypes.c_int),
        ("out_nchw", ctypes.c_int), ("accumulate", ctypes.c_int),
        ("addend0", ctypes.c_void_p), ("addend1", ctypes.c_void_p),
        ("act", ctypes.c_int), ("add_after_act", ctypes.c_int),
        ("TH", ctypes.c_int), ("TW", ctypes.c_int), ("lattice", ctypes.c_int), ("waves", ctypes.c_int),
        ("precision", ctypes.c_int), ("in_scale", ctypes.c_void_p), ("in_tag1", ctypes.c_void_p),
        ("in_tag2", ctypes.c_void_p), ("out_tag", ctypes.c_void_p), ("out_stats", ctypes.c_void_p),
        ("nphase", ctypes.c_int), ("phase_wstride", ctypes.c_long), ("s2d", ctypes.c_int), ("s2d_pad", ctypes.c_int),
        ("spec_z", ctypes.c_void_p), ("spec_m2", ctypes.c_int), ("spec_scale", ctypes.c_float),
    ]


class WgradArgs(ctypes.Structure):
    _fields_ = [
        ("a", ctypes.c_void_p), ("B", ctypes.c_int), ("Ha", ctypes.c_int), ("Wa", ctypes.c_int), ("M", ctypes.c_int),
        ("x", ctypes.c_void_p), ("Hx", ctypes.c_int), ("Wx", ctypes.c_int), ("N", ctypes.c_int),
        ("KH", ctypes.c_int), ("KW", ctypes.c_int), ("dil", ctypes.c_int), ("pad_y", ctypes.c_int),
        ("pad_x", ctypes.c_int), ("circ", ctypes.c_int), ("g", ctypes.c_void_p), ("db", ctypes.c_void_p),
    ]


class PackJob(ctypes.Structure):
    _fields_ = [("w", ctypes.c_void_p), ("wpack", ctypes.c_void_p), ("Cout", ctypes.c_int), ("Cin", ctypes.c_int),
                ("KH", ctypes.c_int), ("KW", ctypes.c_int), ("transposed_phase", ctypes.c_int)]


class Src3(ctypes.Structure):
    _fields_ = [("ptr", ctypes.c_void_p), ("C", ctypes.c_int), ("D", ctypes.c_int), ("H", ctypes.c_int),
                ("W", ctypes.c_int), ("off_d", ctypes.c_int), ("off_h", ctypes.c_int), ("off_w", ctypes.c_int)]


class Conv3dArgs(ctypes.Structure):
    _fields_ = [
        ("nsrc", ctypes.c_int), ("src", Src3 * MAX_SRC),
        ("B", ctypes.c_int), ("Dc", ctypes.c_int), ("Hc", ctypes.c_int), ("Wc", ctypes.c_int), ("Cin", ctypes.c_int),
        ("circ", ctypes.c_int), ("zpad", ctypes.c_int),
        ("gn_stats", ctypes.c_void_p), ("gn_gamma", ctypes.c_void_p), ("gn_beta", ctypes.c_void_p),
        ("gn_groups", ctypes.c_int), ("gn_eps", ctypes.c_float), ("pre_act", ctypes.c_int),
        ("K", ctypes.c_int), ("stride", ctypes.c_int), ("transposed", ctypes.c_int),
        ("Dout", ctypes.c_int), ("Hout", ctypes.c_int), ("Wout", ctypes.c_int),
        ("wpack", ctypes.c_void_p), ("bias", ctypes.c_void_p), ("Cout", ctypes.c_int),
        ("out", ctypes.c_void_p), ("out_C", ctypes.c_int), ("out_D", ctypes.c_int), ("out_H", ctypes.c_int),
        ("out_W", ctypes.c_int), ("out_os", ctypes.c_int), ("out_off_d", ctypes.c_int), ("out_off_h", ctypes.c_int),
        ("out_off_w", ctypes.c_int), ("accumulate", ctypes.c_int), ("addend", ctypes.c_void_p), ("act", ctypes.c_int),
        ("bf16", ctypes.c_int), ("out_stats", ctypes.c_void_p),
    ]


_vp, _i, _l, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_size_t
_SIGS = {
    "nps_conv2d_packed_size": (_sz, [_i, _i, _i]),
    "nps_conv2d_pack_weights": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_conv2d_pack_weights_x3": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_conv2d_pack_weights_x3_batch": (_i, [ctypes.POINTER(PackJob), _i, _vp]),
    "nps_conv2d_x3_eligible": (_i, [_i, _i, _i, _i]),
    "nps_conv2d_x3_sources_ok": (_i, [ctypes.POINTER(Src), _i]),
    "nps_conv2d_x3_prologue_ok": (_i, [_i, _i, _i, _i, _i]),
    "nps_absmax": (_i, [_vp, _l, _vp, _vp]),
    "nps_absmax_into": (_i, [_vp, _l, _vp, _vp]),
    "nps_conv2d_plan": (_i, [ctypes.POINTER(Conv2dArgs)]),
    "nps_conv2d_x3_weight_span": (_l, [ctypes.POINTER(Conv2dArgs)]),
    "nps_conv2d_fwd": (_i, [ctypes.POINTER(Conv2dArgs), _vp]),
    "nps_frame_pack": (_i, [ctypes.POINTER(Conv2dArgs), _vp, _vp]),
    "nps_space_to_depth": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "nps_group_norm_stats": (_i, [ctypes.POINTER(Src), _i, _i, _i, _i, _i, _i, _vp, _i, _vp]),
    "nps_stats_sum": (_i, [_vp, _i, _vp, _i, _vp, _i, _i, _vp, _i, _vp]),
    "nps_stats_sub": (_i, []),
    "nps_x3_set_grid": (_i, [ctypes.c_long]),
    "nps_spectral_dft_w": (_i, [ctypes.POINTER(Src), _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "nps_spectral_dft_h": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_spectral_pack_weights": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_spectral_mix": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_spectral_idft_h": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_spectral_idft_w": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _vp, _vp]),
    "nps_pack_grid_input": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "nps_timeconv_decode": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp, _i, _i, _i, _i, _i, _i,
                                 _vp]),
    "nps_plane_sums": (_i, [_vp, _l, _i, _i, _vp, _vp]),
    "nps_volume_rescale": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "nps_sq_err_sum": (_i, [_vp, _vp, _l, _vp, _vp]),
    "nps_nchw_to_nhwc": (_i, [_vp, _vp, _i, _i, _i, _i, _vp]),
    "nps_nhwc_to_nchw": (_i, [_vp, _vp, _i, _i, _i, _i, _vp]),
    # backward (training)
    "nps_wgrad_lds_bytes": (_sz, [_i, _i]),
    "nps_conv2d_wgrad": (_i, [ctypes.POINTER(WgradArgs), _vp]),
    "nps_wgrad_x3_ws_floats": (_sz, [_i, _i, _i, _i]),
    "nps_conv2d_wgrad_x3": (_i, [ctypes.POINTER(WgradArgs), _vp, _vp, _vp, _vp]),
    "nps_conv2d_wgrad_x3_set": (_i, [ctypes.POINTER(WgradArgs), _vp, _vp, _vp, _vp]),
    "nps_channel_sums": (_i, [_vp, _l, _i, _vp, _vp]),
    "nps_frame_pack_bwd": (_i, [ctypes.POINTER(Conv2dArgs), _vp, ctypes.POINTER(ctypes.c_void_p), _vp, _vp, _vp, _vp]),
    "nps_frame_pack_bwd_tagged": (_i, [ctypes.POINTER(Conv2dArgs), _vp, ctypes.POINTER(ctypes.c_void_p),
                                       ctypes.POINTER(ctypes.c_void_p), _vp, _vp, _vp, _vp]),
    "nps_frame_pack_bwd2": (_i, [ctypes.POINTER(Conv2dArgs), _vp, _vp, ctypes.POINTER(ctypes.c_void_p),
                                 ctypes.POINTER(ctypes.c_void_p), _vp, _vp, _vp, _vp]),
    "nps_gelu": (_i, [_vp, _vp, _l, _vp]),
    "nps_gelu_bwd": (_i, [_vp, _vp, _vp, _l, _vp]),
    "nps_add_at": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "nps_add_at_copy": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "nps_circular_pad": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_circular_fold": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_scaled_diff": (_i, [_vp, _vp, _vp, _vp, _l, _vp]),
    "nps_spectral_idft_w_bwd": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_spectral_dft_w_bwd": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_spectral_mix_bwd": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_spectral_unpack_grad": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_gather_windows": (_i, [_vp, _vp, _vp, _i, _i, _i, _l, _i, _i, _vp]),
    "nps_spectral3d_pack_weights": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "nps_spectral3d_unpack_grad": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _i, _vp]),
    "nps_timeconv_decode_bwd": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _vp, _i, _i, _i, _i,
                                     _i, _i, _vp]),
    "nps_plane_dot": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "nps_volume_rescale_bwd": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    # one call per module (composites of the spectral stages)
    "nps_spectral_conv2d_workspace": (_sz, [_i] * 7),
    "nps_spectral_conv2d_fwd": (_i, [_vp] * 5 + [_i] * 9 + [_vp]),
    "nps_spectral_conv2d_bwd": (_i, [_vp] * 8 + [_i] * 7 + [_vp]),
    "nps_fno_layer2d_workspace": (_sz, [_i] * 7),
    "nps_fno_layer2d_fwd": (_i, [ctypes.POINTER(Conv2dArgs), _vp, _vp, _i, _i, _vp, _vp]),
    "nps_spectral_conv3d_workspace": (_sz, [_i] * 9),
    "nps_spectral_conv3d_fwd": (_i, [_vp] * 7 + [_i] * 11 + [_vp]),
    "nps_spectral_conv3d_bwd": (_i, [_vp] * 12 + [_i] * 9 + [_vp]),
    # bf16 storage (C5)
    "nps_spectral_dft_w_bf16": (_i, [ctypes.POINTER(Src), _i, _i, _i, _i, _i, _i, _vp, _vp]),
    "nps_spectral_mix_bf16": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_spectral_idft_w_bf16": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _i, _vp, _i, _vp]),
    "nps_f32_to_bf16": (_i, [_vp, _l, _vp, _vp]),
    "nps_bf16_to_f32": (_i, [_vp, _l, _vp, _vp]),
    "nps_conv1x1_bf16_kr": (_i, [_i]),
    "nps_pack_1x1_bf16": (_i, [_vp, _vp, _i, _i, _vp]),
    "nps_conv1x1_bf16": (_i, [ctypes.POINTER(Conv2dArgs), _vp]),
    # 3-D U-Net (C5 U-FNO 3D)
    "nps_conv3d_packed_bytes": (_sz, [_i, _i, _i, _i, _i]),
    "nps_conv3d_pack_weights": (_i, [_vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "nps_conv3d_fwd": (_i, [ctypes.POINTER(Conv3dArgs), _vp]),
    "nps_gn_stats3d": (_i, [ctypes.POINTER(Conv3dArgs), _i, _vp, _vp]),
    "nps_frame_pack3d": (_i, [ctypes.POINTER(Conv3dArgs), _vp, _i, _vp]),
    "nps_last_error": (ctypes.c_char_p, []),
    "nps_version": (ctypes.c_char_p, []),
}
for _name, (_res, _args) in _SIGS.items():
    _f = getattr(lib, _name)  # AttributeError here = the .so does not export what include/nps.h declares
    _f.restype = _res
    _f.argtypes = _args

EXPORTED = tuple(_SIGS)


def check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {lib.nps_last_error().decode()}")


def ptr(t):
    """Device pointer of an fp32/fp64/complex64/bf16 ROCm tensor (None -> NULL)."""
    if t is None:
        return None
    if not t.is_cuda:
        raise RuntimeError("nps_hip ops run on the MI355X only: tensor is on " + str(t.device))
    return t.data_ptr()


def stream_ptr():
    return torch.cuda.current_stream().cuda_stream
