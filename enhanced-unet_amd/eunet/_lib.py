"""ctypes binding of libeunet_hip.so (the C-ABI in include/eunet.h).

The product path has exactly one implementation: the HIP library.  If it is
missing or cannot be loaded, every op raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_float, c_int, c_size_t, c_void_p, c_char_p, c_int64

# EUNET_LIB overrides the in-tree library (A/B of two builds); the default is the in-tree build
LIB_PATH = os.environ.get("EUNET_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libeunet_hip.so")

EUNET_F32 = 0
EUNET_BF16 = 1


class Act(ctypes.Structure):
    """eunet_act: NHWC view (ptr, n, h, w, c, ctot, coff, dtype)."""
    _fields_ = [("ptr", c_void_p), ("n", c_int), ("h", c_int), ("w", c_int), ("c", c_int),
                ("ctot", c_int), ("coff", c_int), ("dtype", c_int)]


class PackDesc(ctypes.Structure):
    """eunet_pack_desc (include/eunet.h)."""
    _fields_ = [("w", c_void_p), ("cout", c_int), ("cin", c_int), ("flip", c_int), ("wp", c_void_p)]


PACK_MAX = 32  # EUNET_PACK_MAX


class LossParams(ctypes.Structure):
    """eunet_loss_params (include/eunet.h): the loss configuration of one combined-loss call."""
    _fields_ = [("ce_weight", c_float * 3), ("alpha", c_float * 3), ("gamma", c_float), ("ignore_index", c_int),
                ("dice_weight", c_float * 3), ("tversky_weight", c_float * 3), ("tversky_alpha", c_float),
                ("w_focal", c_float), ("w_dice", c_float), ("w_tversky", c_float), ("class_div", c_float),
                ("focal_norm", c_int)]


class OptTensor(ctypes.Structure):
    """eunet_opt_tensor (include/eunet.h): one parameter's data / grad / AdamW state / step counter."""
    _fields_ = [("param", c_void_p), ("grad", c_void_p), ("exp_avg", c_void_p), ("exp_avg_sq", c_void_p),
                ("step", c_void_p), ("numel", ctypes.c_longlong)]


_P = POINTER(Act)
_f = c_void_p  # float* / void* device pointers are passed as integers

# name -> argtypes (restype is always c_int except the two string getters)
SIGNATURES = {
    "eunet_nchw_to_nhwc": [_f, _P, c_void_p],
    "eunet_stream_wait": [c_void_p, c_void_p],
    "eunet_set_update_guard": [c_int, c_void_p],
    "eunet_conv3x3_packed_bytes": [c_int, c_int, c_int, POINTER(c_size_t)],
    "eunet_conv3x3_pack": [_f, c_int, c_int, c_int, _f, c_int, c_void_p],
    "eunet_conv3x3_pack_many": [c_void_p, c_int, c_int, c_void_p],
    "eunet_conv3x3_tiles": [_P, POINTER(c_int)],
    "eunet_conv3x3_fwd": [_P, _f, _f, c_int, _f, _f, _P, _f, c_void_p],
    "eunet_conv3x3_dgrad_bnbwd": [_P, _f, _P, _P, _f, _f, _f, _f, _f, _f, c_void_p],
    "eunet_conv3x3_dgrad": [_P, _f, _P, _f, c_void_p],
    "eunet_conv3x3_dgrad_fused": [_P, _P, _f, _P, _f, _P, _P, _f, _f, _f, _f, _f, _f, c_void_p],
    "eunet_conv3x3_wgrad_splits": [_P, c_int, c_int, POINTER(c_int)],
    "eunet_conv3x3_wgrad": [_P, _f, _f, c_int, _P, _f, _f, c_int, c_void_p],
    "eunet_wgrad_reduce": [_f, _f, c_int, c_int, c_int, c_int, _f, _f, c_void_p],
    "eunet_conv_small_fwd": [_P, _f, _f, _P, _f, c_void_p],
    "eunet_conv_small_wgrad_splits": [_P, POINTER(c_int)],
    "eunet_conv_small_wgrad": [_P, _P, _f, _f, c_int, c_void_p],
    "eunet_bn_finalize": [_f, c_int, c_int, _f, _f, c_float, c_float, _f, _f, _f, _f, _f, _f, _f, c_void_p],
    "eunet_opt_table": [c_void_p, c_int, c_void_p, POINTER(c_int)],
    "eunet_clip_adamw": [c_void_p, c_int, c_int, c_void_p, c_float, ctypes.c_double, ctypes.c_double,
                         ctypes.c_double, ctypes.c_double, ctypes.c_double, _f, _f, _f, c_void_p],
    "eunet_bn_eval_affine": [c_int, _f, _f, _f, _f, c_float, _f, _f, c_void_p],
    "eunet_bnrelu": [_P, _f, _f, _P, c_void_p],
    "eunet_bnrelu_pool": [_P, _f, _f, _P, _P, c_void_p],
    "eunet_bnrelu_upsample": [_P, _f, _f, _P, c_void_p],
    "eunet_bnrelu_conv1x1": [_P, _f, _f, _f, _f, c_int, _f, c_void_p],
    "eunet_head_workspace_bytes": [c_int, c_int, c_int, c_int, c_int, POINTER(c_size_t)],
    "eunet_head_fwd": [_f, c_int, c_int, c_int, c_int, _f, _f, _f, _f, _f, _f, c_int, c_float, c_float,
                       _f, _f, _f, _f, _f, _f, c_int, _f, c_void_p],
    "eunet_head_bwd": [_f, c_int, c_int, c_int, c_int, _f, _f, _f, _f, _f, _f, _f, _f, _f, _f,
                       _f, _f, _f, _f, _f, _f, c_int, _f, c_void_p],
    "eunet_loss_reference_params": [POINTER(LossParams)],
    "eunet_loss_sums_len": [c_int, c_int, POINTER(c_int)],
    "eunet_loss_workspace_bytes": [c_int, c_int, c_int, c_int, POINTER(c_size_t)],
    "eunet_loss_fwd": [_f, _f, c_int, c_int, c_int, c_int, POINTER(LossParams), _f, _f, _f, _f, c_void_p],
    "eunet_loss_bwd": [_f, _f, c_int, c_int, c_int, c_int, POINTER(LossParams), _f, _f, _f, c_void_p],
    "eunet_bn_bwd_tiles": [_P, POINTER(c_int)],
    "eunet_bn_bwd_reduce": [_P, _P, _f, _f, _f, _f, _f, c_void_p],
    "eunet_colsum_ws_bytes": [c_int, c_int, POINTER(c_size_t)],
    "eunet_colsum": [_f, c_int, c_int, _f, _f, c_void_p],
    "eunet_colsum_split": [_f, c_int, c_int, c_int, _f, _f, _f, c_void_p],
    "eunet_bn_bwd_apply": [_P, _P, _f, _f, _f, _f, _f, _f, _P, c_void_p],
    "eunet_bn_bwd_apply_1x1": [_P, _f, c_int, _f, _f, _f, _f, _f, _f, _f, _P, c_void_p],
    "eunet_bn_bwd_coef": [_f, _f, _f, _f, _f, _f, c_int64, c_int, _f, c_void_p],
    "eunet_bn_bwd_apply_coef": [_P, _P, _f, _P, c_void_p],
    "eunet_pool_bwd_add": [_P, _P, _P, _P, c_void_p],
    "eunet_upsample_bwd": [_P, _P, c_void_p],
    "eunet_pool_bwd_add_bnr_rows": [_P, POINTER(c_int)],
    "eunet_pool_bwd_add_bnr": [_P, _P, _P, _P, _P, _f, _f, _f, _f, _f, c_void_p],
    "eunet_bn_bwd_apply_pool": [_P, _P, _P, _f, _f, _f, _f, _f, _f, _P, c_void_p],
    "eunet_upsample_bwd_bnr_rows": [_P, POINTER(c_int)],
    "eunet_upsample_bwd_bnr": [_P, _P, _P, _f, _f, _f, _f, _f, c_void_p],
    "eunet_conv1x1_bwd_tiles": [_P, POINTER(c_int)],
    "eunet_conv1x1_bwd": [_P, _f, _f, _f, c_int, _f, _P, _f, c_void_p],
    "eunet_conv1x1_bwd_bnr": [_P, _f, _f, _f, c_int, _f, _P, _f, _f, _f, _f, c_void_p],
    "eunet_semantic_counts": [_f, _f, c_int, c_int64, _f, c_void_p],
    "eunet_binary_overlap": [_f, _f, c_int64, _f, c_void_p],
    "eunet_resize_bilinear": [_f, c_int, c_int, c_int, _f, c_int, c_int, c_float, c_float, c_int, c_int,
                              c_void_p],
    "eunet_softmax_crop": [_f, c_int, c_int, c_int, c_int, c_int, c_int, c_int, _f, c_void_p],
    "eunet_accumulate": [_f, _f, c_int64, c_int, c_float, c_void_p],
    "eunet_probs_to_mask": [_f, c_int, c_int, c_int, _f, _f, c_void_p],
    "eunet_fusion_tiles": [c_int, c_int, c_int, POINTER(c_int), POINTER(c_int)],
    "eunet_gate_fwd": [_f, _f, c_int, c_int, c_int, c_int, _f, _f, _f, _f, _f, c_void_p],
    "eunet_gate_mid_fwd": [_f, _f, c_int, c_int, c_int, c_int, _f, _f, _f, _f, _f, _f, c_void_p],
    "eunet_gate_out_fwd": [_f, _f, c_int, c_int, c_int, c_int, _f, _f, _f, _P, c_void_p],
    "eunet_fusion_out_fwd": [_f, _f, c_int, _P, _f, _f, _f, _f, _f, _f, _f, _f, _f, _f, c_void_p],
    "eunet_fusion_out_bwd": [_f, _f, c_int, c_int, c_int, c_int, _f, _f, _f, _f, _f, _f, _f, _f, c_void_p],
    "eunet_gate_bwd1": [_f, _f, c_int, _P, _f, _f, _f, _f, _f, _f, _f, _f, _f, c_void_p],
    "eunet_gate_bwd2": [c_int, c_int, c_int, c_int, _f, _f, _f, _f, _f, _f, _f, _f, _f, _f, _f, _f, _f, _f,
                        _f, c_void_p],
    "eunet_gate_bwd3": [_f, _f, c_int, c_int, c_int, c_int, _f, _f, _f, _f, _f, _f, _f, _f, _f, _f, _f, _f,
                        _f, _f, c_void_p],
    "eunet_dropout_affine": [_f, _f, _f, c_int, c_int, c_float, _f, _f, _f, c_void_p],
    "eunet_rasterize_polygons": [_f, _f, _f, c_int, c_int, c_int, _f, c_void_p],
    "eunet_rasterize_instances": [_f, _f, c_int, c_int, c_int, c_int, c_int, _f, c_void_p],
    "eunet_flip_u8": [_f, _f, c_int, c_int, c_int, c_int, c_void_p],
    "eunet_flip_mask": [_f, _f, c_int, c_int, c_int, c_void_p],
    "eunet_augment_ratio_u8": [_f, c_int64, _f, c_int, ctypes.c_double, ctypes.c_double, c_void_p],
    "eunet_augment_u8": [_f, c_int64, c_int, ctypes.c_double, ctypes.c_double, _f, _f, c_void_p],
    "eunet_to_tensor": [_f, c_int, c_int, c_int, _f, c_void_p],
    "eunet_resize_u8": [_f, c_int, c_int, c_int, _f, c_int, c_int, c_void_p],
    "eunet_rgb2lab_u8": [_f, _f, c_int64, c_void_p],
    "eunet_lab2rgb_u8": [_f, _f, c_int64, c_void_p],
    "eunet_lab_tables": [c_void_p, c_size_t],
    "eunet_rgb2gray_u8": [_f, _f, c_int64, c_void_p],
    "eunet_hsv_adjust_u8": [_f, c_int64, c_float, c_float, c_float, c_int, c_void_p],
    "eunet_clahe_u8": [_f, c_int, c_int, c_int, ctypes.c_double, c_int, c_int, _f, _f, c_void_p],
    "eunet_filter3x3_u8": [_f, _f, c_int, c_int, c_int, _f, c_void_p],
    "eunet_unsharp_u8": [_f, _f, c_int, c_int, c_int, c_void_p],
    "eunet_edge_features_workspace_bytes": [c_int, c_int, POINTER(ctypes.c_size_t)],
    "eunet_edge_features_u8": [_f, c_int, c_int, _f, _f, c_void_p],
    "eunet_live_boost_u8": [_f, _f, c_int64, c_void_p],
    "eunet_cell_mix_u8": [_f, _f, _f, _f, _f, c_int64, _f, c_void_p],
    "eunet_chw_to_u8_workspace_bytes": [c_int, c_int, c_int, POINTER(ctypes.c_size_t)],
    "eunet_chw_to_u8": [_f, c_int, c_int, c_int, _f, _f, c_void_p],
    "eunet_debug_enabled": [],
    "eunet_debug_status": [POINTER(ctypes.c_uint), POINTER(ctypes.c_uint), c_int],
    "eunet_debug_selftest": [c_void_p],
    "eunet_consistency_tiles": [c_int, c_int, POINTER(c_int)],
    "eunet_consistency_fwd": [_f, _f, _f, c_int, c_int, c_int, c_int, c_float, c_float, _f, _f, c_void_p],
    "eunet_consistency_bwd": [_f, _f, _f, c_int, c_int, c_int, c_int, c_float, c_float, _f, _f, _f, _f,
                              c_void_p],
}
STRING_FNS = ("eunet_version", "eunet_last_error")


class EunetError(RuntimeError):
    pass


_lib = None


def load(path: str = LIB_PATH):
    """Load (once) and type the library.  Raises if it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise EunetError(f"libeunet_hip.so not found at {path}: build it with "
                         f"`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    lib = ctypes.CDLL(path)
    for name in STRING_FNS:
        fn = getattr(lib, name)
        fn.restype = c_char_p
        fn.argtypes = []
    missing = []
    for name, argt in SIGNATURES.items():
        try:
            fn = getattr(lib, name)
        except AttributeError:
            missing.append(name)
            continue
        fn.restype = c_int
        fn.argtypes = argt
    if missing:
        # an older build under A/B may lack entry points, but only when asked for explicitly: a stale or
        # partial library otherwise fails here, not at its first call
        if os.environ.get("EUNET_LIB_ALLOW_PARTIAL") != "1":
            raise EunetError(f"{path} lacks {len(missing)} entry point(s) of include/eunet.h: {missing[:6]} "
                             "(stale build? rebuild, or set EUNET_LIB_ALLOW_PARTIAL=1 for an A/B of an older library)")
        import warnings
        warnings.warn(f"{path}: {len(missing)} entry point(s) unbound (EUNET_LIB_ALLOW_PARTIAL=1): {missing}")
    _lib = lib
    return lib


# kprof.BusyTimer installs itself here: every launching entry point is then bracketed by events on
# torch's current stream (the stream the C-ABI enqueues on), for the whole-step kernel-busy figure
BUSY_HOOK = None
_NO_LAUNCH = ("_tiles", "_bytes", "_splits", "_rows", "_len", "_params", "debug_", "_table", "lab_tables",
              "stream_wait")


def call(name: str, *args):
    lib = load()
    h = BUSY_HOOK
    if h is not None and not any(s in name for s in _NO_LAUNCH):
        e0 = h.begin()
        rc = getattr(lib, name)(*args)
        h.end(e0)
    else:
        rc = getattr(lib, name)(*args)
    if rc != 0:
        msg = lib.eunet_last_error().decode(errors="replace")
        raise EunetError(f"{name} failed ({rc}): {msg}")
    return rc


def exported_symbols():
    return list(SIGNATURES) + list(STRING_FNS)


def version() -> str:
    return load().eunet_version().decode()


DEBUG_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libeunet_hip_debug.so")


def debug_status(reset: bool = False):
    """(unit * 100000 + line of the first failed device check, failed-check count) of the loaded
    library; (0, 0) in the release build (eunet_debug_enabled() == 0), where checks compile away."""
    lib = load()
    line, cnt = ctypes.c_uint(0), ctypes.c_uint(0)
    call("eunet_debug_status", ctypes.byref(line), ctypes.byref(cnt), 1 if reset else 0)
    return int(line.value), int(cnt.value)


__all__ = ["Act", "LossParams", "load", "call", "EunetError", "EUNET_F32", "EUNET_BF16", "exported_symbols",
           "c_int", "c_size_t", "c_float", "c_int64"]
