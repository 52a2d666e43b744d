"""ctypes binding of libfloodgan.so (the C-ABI declared in include/floodgan.h).

The library is the product path: there is no CPU or PyTorch fallback.  Loading fails
loudly if the shared object is missing, and every entry point raises RuntimeError with the
library's own message when a call returns non-zero.
"""
import ctypes as C
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FLOODGAN_LIB", os.path.join(_HERE, "lib", "libfloodgan.so"))

FG_PAD_ZERO, FG_PAD_REFLECT = 0, 1
FG_ACT_NONE, FG_ACT_RELU, FG_ACT_LRELU = 0, 1, 2
FG_MATH_FP32, FG_MATH_FWD_X6, FG_MATH_WGRAD_X6, FG_MATH_BF16X6 = 0, 1, 2, 3
FG_MATH_FWD_F16X3, FG_MATH_WGRAD_F16X3, FG_MATH_F16X3 = 4, 8, 12
CONV_MATH = {"fp32": FG_MATH_FP32, "fwd_x6": FG_MATH_FWD_X6, "wgrad_x6": FG_MATH_WGRAD_X6, "bf16x6": FG_MATH_BF16X6,
             "fwd_f16x3": FG_MATH_FWD_F16X3, "wgrad_f16x3": FG_MATH_WGRAD_F16X3, "f16x3": FG_MATH_F16X3}


class fg_view(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("n", C.c_int), ("h", C.c_int), ("w", C.c_int),
                ("c_alloc", C.c_int), ("pad", C.c_int)]


class fg_sview(C.Structure):
    _fields_ = [("ptr", C.c_void_p), ("sn", C.c_longlong), ("sc", C.c_longlong),
                ("sy", C.c_longlong), ("sx", C.c_longlong)]


fg_wview = fg_sview   # same layout (float* + 4 strides), writable on the C side


class fg_conv_problem(C.Structure):
    _fields_ = [("x", C.c_void_p), ("w", C.c_void_p), ("bias", C.c_void_p), ("y", C.c_void_p),
                ("sxn", C.c_longlong), ("sxa", C.c_longlong), ("sxb", C.c_longlong), ("sxr", C.c_longlong),
                ("syn", C.c_longlong), ("sya", C.c_longlong), ("syb", C.c_longlong), ("syc", C.c_longlong),
                ("m_img", C.c_int), ("m_a", C.c_int), ("m_b", C.c_int),
                ("kh", C.c_int), ("j_valid", C.c_int), ("jp", C.c_int),
                ("n_out", C.c_int), ("ldw", C.c_int), ("act", C.c_int), ("accumulate", C.c_int),
                ("w_split", C.c_int), ("x_absmax", C.c_void_p), ("w_absmax", C.c_void_p), ("jc", C.c_int),
                ("in_stats", C.c_void_p), ("x_presplit", C.c_int),
                ("q_n", C.c_int), ("q_mask", C.c_int), ("q_yoff", C.c_longlong * 4), ("q_soff", C.c_longlong)]


class fg_wgrad_problem(C.Structure):
    _fields_ = [("p", C.c_void_p), ("x", C.c_void_p), ("out", C.c_void_p),
                ("spn", C.c_longlong), ("spa", C.c_longlong), ("spb", C.c_longlong),
                ("sxn", C.c_longlong), ("sxa", C.c_longlong), ("sxb", C.c_longlong), ("sxr", C.c_longlong),
                ("m_img", C.c_int), ("m_a", C.c_int), ("m_b", C.c_int),
                ("n_a", C.c_int), ("kh", C.c_int), ("j_valid", C.c_int),
                ("splits", C.c_int), ("m_chunk", C.c_int), ("p_absmax", C.c_void_p), ("x_absmax", C.c_void_p),
                ("p_presplit", C.c_int), ("x_presplit", C.c_int)]


class fg_weight_map(C.Structure):
    _fields_ = [("n_out", C.c_int), ("kh", C.c_int), ("kw", C.c_int), ("c", C.c_int),
                ("c_valid", C.c_int), ("jp", C.c_int), ("dim0_is_n", C.c_int),
                ("d0", C.c_int), ("d1", C.c_int), ("KH", C.c_int), ("KW", C.c_int),
                ("n_base", C.c_int), ("rtab", C.c_int * 8), ("stab", C.c_int * 8), ("q_n", C.c_int)]


class fg_pack_job(C.Structure):
    _fields_ = [("w", C.c_void_p), ("w_absmax", C.c_void_p), ("dst", C.c_void_p), ("map", fg_weight_map)]


FG_PACK_BATCH_MAX = 24


class fg_adam_tensor(C.Structure):
    _fields_ = [("param", C.c_void_p), ("grad", C.c_void_p), ("exp_avg", C.c_void_p),
                ("exp_avg_sq", C.c_void_p), ("numel", C.c_longlong), ("absmax", C.c_void_p)]


FG_TILE_MAX_CH = 16

# fg_set_f3_order's default (csrc/conv_f3.hip g_f3_alt): tests restore it after sweeping the bits
F3_ORDER_DEFAULT = 31


class fg_tile_batch(C.Structure):
    _fields_ = [("src", C.c_void_p), ("tile_stride", C.c_longlong),
                ("n", C.c_int), ("h_in", C.c_int), ("w_in", C.c_int), ("c_src", C.c_int),
                ("flip", C.c_void_p), ("c_out", C.c_int), ("chan", C.c_int * FG_TILE_MAX_CH),
                ("crop", C.c_void_p), ("row_lo", C.c_void_p), ("rows", C.c_int), ("out_h", C.c_int), ("out_w", C.c_int),
                ("x_idx0", C.c_void_p), ("x_w", C.c_void_p), ("x_taps", C.c_int),
                ("y_idx0", C.c_void_p), ("y_w", C.c_void_p), ("y_taps", C.c_int),
                ("tmp", C.c_void_p), ("dst", fg_wview)]


# (name, argtypes) of every exported symbol; tests check the library exports all of them
SIGNATURES = {
    "fg_last_error": [],
    "fg_last_launch": [],
    "fg_version": [],
    "fg_device_ok": [],
    "fg_timing_event_create": [C.c_int, C.POINTER(C.c_void_p)],
    "fg_timing_event_record": [C.c_void_p, C.c_void_p],
    "fg_timing_event_elapsed": [C.c_void_p, C.c_void_p, C.POINTER(C.c_float)],
    "fg_timing_event_destroy": [C.c_void_p],
    "fg_timing_arm": [C.c_void_p, C.c_void_p],
    "fg_timing_disarm": [],
    "fg_conv_fwd": [C.POINTER(fg_conv_problem), C.c_int, C.c_void_p],
    "fg_conv_stats_ok": [C.POINTER(fg_conv_problem), C.c_int],
    "fg_set_conv_math": [C.c_int],
    "fg_get_conv_math": [],
    "fg_set_fwd_tile": [C.c_int],
    "fg_set_wgrad_tile": [C.c_int],
    "fg_set_f3_tile": [C.c_int],
    "fg_set_f3_order": [C.c_int],
    "fg_set_f3_sched": [C.c_int],
    "fg_set_f3_persistent": [C.c_int],
    "fg_set_f3_fill": [C.c_int],
    "fg_set_f3_interleave": [C.c_int],
    "fg_set_wgrad_f3": [C.c_int],
    "fg_set_in_rows": [C.c_int],
    "fg_set_f3_ps_wide": [C.c_int],
    "fg_set_f3_ps_tall": [C.c_int],
    "fg_conv_wgrad": [C.POINTER(fg_wgrad_problem), C.c_void_p],
    "fg_wgrad_reduce": [C.c_void_p, C.c_int, C.POINTER(fg_weight_map), C.c_void_p, C.c_int, C.c_void_p],
    "fg_pack_weight": [C.c_void_p, C.POINTER(fg_weight_map), C.c_void_p, C.c_void_p],
    "fg_pack_weight_split": [C.c_void_p, C.POINTER(fg_weight_map), C.c_void_p, C.c_void_p],
    "fg_pack_weight_f16": [C.c_void_p, C.POINTER(fg_weight_map), C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_pack_weight_f16_batch": [C.c_void_p, C.c_int, C.c_void_p],
    "fg_absmax": [C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p],
    "fg_conv_n1_fwd": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                       C.c_int, C.c_void_p],
    "fg_conv_n1_wgrad_blocks": [C.c_int, C.c_int, C.c_int],
    "fg_conv_n1_wgrad": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int,
                         C.c_void_p, C.c_void_p],
    "fg_d0_input_grad": [fg_view, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int, C.c_int, C.c_int,
                         C.c_int, C.c_void_p],
    "fg_split_pixels": [C.c_void_p, C.c_longlong, C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_conv_win": [C.POINTER(fg_conv_problem), C.c_void_p, C.c_longlong, C.c_void_p],
    "fg_conv_wgrad_win": [C.POINTER(fg_wgrad_problem), C.c_void_p, C.c_longlong, C.c_int, C.c_int, C.c_void_p,
                          C.c_longlong, C.c_int, C.c_void_p],
    "fg_conv1x1_fwd": [fg_view, C.c_void_p, C.c_void_p, C.c_int, fg_view, C.c_void_p],
    "fg_conv1x1_dgrad": [fg_view, C.c_void_p, C.c_int, fg_view, C.c_void_p],
    "fg_conv1x1_wgrad": [fg_view, fg_view, C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p],
    "fg_conv1x1_wgrad_workspace_floats": [C.c_int],
    "fg_pack_input": [fg_sview, C.c_int, fg_sview, C.c_int, fg_view, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p],
    "fg_zero_border": [fg_view, C.c_void_p],
    "fg_fold_add": [fg_view, C.c_int, fg_view, fg_view, C.c_void_p],
    "fg_unfold_nchw": [fg_view, C.c_int, C.c_int, fg_wview, C.c_int, C.c_int, C.c_int, C.c_void_p],
    "fg_in_workspace_doubles": [C.c_int, C.c_int],
    "fg_in_stats": [fg_view, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_in_stats_partials": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_void_p, C.c_void_p,
                             C.c_void_p, C.c_void_p],
    "fg_in_partials_workspace_doubles": [C.c_int, C.c_int],
    "fg_in_apply": [fg_view, C.c_void_p, C.c_void_p, C.c_int, fg_view, fg_view, C.c_int, C.c_void_p, C.c_void_p],
    "fg_in_bwd": [fg_view, C.c_int, fg_view, fg_view, C.c_void_p, C.c_void_p, C.c_int, fg_view, C.c_void_p,
                  C.c_int, fg_view, C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_in_apply_presplit": [fg_view, C.c_void_p, C.c_void_p, C.c_int, fg_view, C.c_int, C.c_void_p, C.c_void_p],
    "fg_in_apply_splitpix": [fg_view, C.c_void_p, C.c_void_p, C.c_int, fg_view, C.c_int, C.c_void_p, C.c_void_p],
    "fg_in_apply_dual": [fg_view, C.c_void_p, C.c_void_p, C.c_int, fg_view, C.c_void_p, fg_view, C.c_int, C.c_void_p,
                         C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_in_apply_head": [fg_view, C.c_void_p, C.c_void_p, C.c_int, fg_view, C.c_int, C.c_void_p, C.c_void_p,
                         C.c_void_p, C.c_int, fg_view, C.c_void_p],
    "fg_in_bwd_head": [fg_view, C.c_void_p, C.c_int, fg_view, C.c_void_p, C.c_void_p, C.c_int, fg_view, C.c_void_p,
                       C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                       C.c_void_p],
    "fg_in_head_wgrad_workspace_floats": [C.c_int, C.c_int, C.c_int, C.c_int],
    "fg_in_bwd_presplit": [fg_view, C.c_int, fg_view, fg_view, C.c_void_p, C.c_void_p, C.c_int, fg_view, C.c_void_p,
                           C.c_int, fg_view, C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_act_bwd": [fg_view, fg_view, C.c_int, C.c_void_p, C.c_void_p],
    "fg_channel_sum": [fg_view, C.c_int, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p],
    "fg_channel_sum_workspace_doubles": [C.c_int],
    "fg_tail_fwd": [fg_view, fg_view, fg_sview, C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_tail_bwd": [fg_view, fg_view, fg_sview, fg_sview, fg_sview, fg_view, fg_view, fg_wview, C.c_void_p, C.c_void_p,
                    C.c_void_p],
    "fg_tanh_head_fwd": [fg_view, C.c_int, fg_wview, C.c_void_p],
    "fg_tanh_head_bwd": [fg_view, C.c_int, fg_sview, fg_view, C.c_void_p],
    "fg_mse_const": [C.c_void_p, C.c_longlong, C.c_float, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p,
                     C.c_void_p],
    "fg_l1": [fg_sview, fg_sview, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float, C.c_void_p,
              C.c_void_p, C.c_int, C.c_void_p, C.c_void_p],
    "fg_adam_step": [C.POINTER(fg_adam_tensor), C.c_int, C.c_double, C.c_double, C.c_double, C.c_double,
                     C.c_longlong, C.c_void_p],
    "fg_bn_workspace_doubles": [C.c_int, C.c_int],
    "fg_bn_stats": [fg_view, C.c_int, C.c_float, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                    C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_bn_eval_stats": [C.c_int, C.c_void_p, C.c_void_p, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_bn_apply": [fg_view, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_float,
                    C.c_ulonglong, C.c_int, fg_view, C.c_void_p, C.c_int, fg_view, C.c_void_p, C.c_void_p],
    "fg_bn_bwd": [fg_view, C.c_int, fg_view, C.c_int, fg_view, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                  C.c_void_p, C.c_float, C.c_ulonglong, fg_view, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                  C.c_void_p, C.c_void_p],
    "fg_dropout_mask": [C.c_ulonglong, C.c_float, C.c_longlong, C.c_void_p, C.c_void_p],
    "fg_bernoulli_mt_workspace_words": [C.c_int],
    "fg_bernoulli_mt": [C.c_void_p, C.c_longlong, C.c_longlong, C.c_void_p, C.c_int, C.c_longlong, C.c_int,
                        C.POINTER(C.c_void_p), C.POINTER(C.c_longlong), C.c_double, C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_unit_image": [fg_sview, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, fg_view, C.c_void_p],
    "fg_ssim_workspace_doubles": [C.c_int, C.c_int, C.c_int, C.c_int],
    "fg_ssim": [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_float, C.c_float,
                C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_avg_pool2": [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p],
    "fg_msssim_combine": [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_sq_err_workspace_doubles": [],
    "fg_sq_err_sum": [C.c_void_p, C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p, C.c_void_p],
    "fg_mask_confusion": [fg_view, fg_view, C.c_void_p, C.c_void_p],
    "fg_maxpool2": [fg_view, fg_view, C.c_void_p],
    "fg_tiff_probe": [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)],
    "fg_tiff_read": [C.c_char_p, C.c_void_p, C.c_longlong],
    "fg_tile_transform": [C.POINTER(fg_tile_batch), C.c_void_p],
}
RESTYPES = {"fg_bernoulli_mt_workspace_words": C.c_longlong, "fg_last_error": C.c_char_p, "fg_last_launch": C.c_char_p, "fg_in_workspace_doubles": C.c_longlong, "fg_bn_workspace_doubles": C.c_longlong,
            "fg_ssim_workspace_doubles": C.c_longlong, "fg_sq_err_workspace_doubles": C.c_longlong,
            "fg_channel_sum_workspace_doubles": C.c_longlong,
            "fg_in_partials_workspace_doubles": C.c_longlong, "fg_conv1x1_wgrad_workspace_floats": C.c_longlong}

_lib = None


def load(path=LIB_PATH):
    """Load (once) and return the ctypes handle.  Raises if the library is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"floodgan HIP library not found at {path}; run __graft_entry__.build() "
                           "(or python flood-prediction-gan_amd/floodgan/build.py) first")
    # torch must be imported first so that its HIP runtime (SONAME libamdhip64.so.7) is the
    # one this library binds to: a single runtime means torch's streams are valid here.
    lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
    for name, argt in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = argt
        fn.restype = RESTYPES.get(name, C.c_int)
    _lib = lib
    mode = os.environ.get("FLOODGAN_CONV_MATH")
    if mode:
        set_conv_math(mode)
    return lib


def set_conv_math(mode):
    """'fp32' (v_mfma_f32_32x32x2_f32) or 'bf16x6' (fp32-equivalent split-bf16 MFMA)."""
    check(load().fg_set_conv_math(CONV_MATH[mode]), "set_conv_math")


def fwd_x6():
    """True when the forward / input-gradient convs run the bf16x6 kernels (pre-split weights)."""
    return bool(load().fg_get_conv_math() & FG_MATH_FWD_X6)


def fwd_f16x3():
    """True when the forward / input-gradient convs run the f16x3 kernels."""
    return bool(load().fg_get_conv_math() & FG_MATH_FWD_F16X3)


def wgrad_f16x3():
    return bool(load().fg_get_conv_math() & FG_MATH_WGRAD_F16X3)


def set_fwd_tile(cfg):
    """Tuning hook: force a bf16x6 forward tile config (-1 = automatic)."""
    check(load().fg_set_fwd_tile(int(cfg)), "set_fwd_tile")


def set_wgrad_tile(cfg):
    """Tuning hook: force a bf16x6 weight-gradient tile config (-1 = automatic)."""
    check(load().fg_set_wgrad_tile(int(cfg)), "set_wgrad_tile")


def set_f3_tile(cfg):
    """Tuning hook of the pipelined f16x3 forward kernel: -1 automatic, -2 off, 0..12 forced."""
    check(load().fg_set_f3_tile(int(cfg)), "set_f3_tile")


_WGRAD_F3 = True


def set_wgrad_f3(mode):
    """A/B hook of the pipelined f16x3 weight-gradient kernel: 0 off, 1 stage schedule 0,
    3 stage schedule 1, 2 (default, also True) the measured choice per tile."""
    global _WGRAD_F3
    mode = 2 if mode is True else int(mode)
    check(load().fg_set_wgrad_f3(mode), "set_wgrad_f3")
    _WGRAD_F3 = mode != 0


def wgrad_f3_on():
    return _WGRAD_F3


def get_conv_math():
    inv = {v: k for k, v in CONV_MATH.items()}
    return inv[load().fg_get_conv_math()]


def check(rc, what):
    if rc != 0:
        msg = load().fg_last_error().decode(errors="replace")
        raise RuntimeError(f"floodgan {what} failed (code {rc}): {msg}")


def stream_handle(device=None):
    s = torch.cuda.current_stream(device)
    return C.c_void_p(s.cuda_stream)


def ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


def require_device(t, what="tensor"):
    if not (t.is_cuda and t.dtype == torch.float32):
        raise RuntimeError(f"floodgan: {what} must be a float32 tensor on a HIP device "
                           f"(got {t.dtype} on {t.device}); there is no CPU path")


def last_launch():
    """the kernel family the most recent fg_* call on this thread launched (fg_last_launch)"""
    return load().fg_last_launch().decode()
