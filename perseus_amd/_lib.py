"""ctypes binding of libperseus_amd.so (the C ABI in include/perseus_amd.h).

The library is the product: there is no fallback.  If it is missing or fails to
load, `lib()` raises; build it with `python -m perseus_amd.build`.
"""

from __future__ import annotations

import ctypes as C
import os

from . import build as _build

_LIB = None

c_double_p = C.POINTER(C.c_double)
c_float_p = C.POINTER(C.c_float)


class PerseusError(RuntimeError):
    pass


class TrajArgs(C.Structure):
    """Mirror of `pa_traj_args` (include/perseus_amd.h)."""

    _fields_ = [("T", C.c_int), ("L", C.c_int), ("n_kp", C.c_int), ("H", C.c_int), ("W", C.c_int),
                ("y", C.c_void_p), ("pose", C.c_void_p), ("vel", C.c_void_p), ("angvel", C.c_void_p),
                ("corners", C.c_void_p), ("K", C.c_void_p), ("tcam", C.c_void_p), ("dt", C.c_double),
                ("vel_frame", C.c_int), ("isig_proj", C.c_void_p), ("isig_dyn", C.c_void_p),
                ("isig_cv", C.c_void_p), ("r_proj", C.c_void_p), ("j_proj", C.c_void_p), ("err_proj", C.c_void_p),
                ("status", C.c_void_p), ("r_dyn", C.c_void_p), ("j_dyn0", C.c_void_p), ("j_dyn1", C.c_void_p),
                ("j_dyn2", C.c_void_p), ("j_dyn3", C.c_void_p), ("err_dyn", C.c_void_p), ("r_cv", C.c_void_p),
                ("j_cv0", C.c_void_p), ("j_cv1", C.c_void_p), ("err_cv", C.c_void_p), ("nvalid", C.c_void_p)]


# name -> (restype, argtypes)
_SIGS = {
    "pa_trajectory_linearize": (C.c_int, [C.POINTER(TrajArgs), C.c_void_p]),
    "pa_debug_trajectory_linearize": (C.c_int, [C.POINTER(TrajArgs), C.c_int, C.c_void_p, C.c_void_p]),
    "pa_last_error": (C.c_char_p, []),
    "pa_version": (C.c_char_p, []),
    "pa_detector_create": (C.c_int, [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.POINTER(C.c_void_p)]),
    "pa_detector_destroy": (None, [C.c_void_p]),
    "pa_detector_reserve": (C.c_int, [C.c_void_p, C.c_int]),
    "pa_detector_set_precision": (C.c_int, [C.c_void_p, C.c_int]),
    "pa_detector_set_split_k": (C.c_int, [C.c_void_p, C.c_int]),
    "pa_detector_forward": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]),
    "pa_detector_profile": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p,
                                      C.c_void_p, C.c_void_p, C.c_int]),
    "pa_detector_flops_per_frame": (C.c_double, [C.c_void_p]),
    "pa_detector_time_launch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int,
                                          C.c_int, C.c_void_p, C.c_void_p]),
    "pa_detector_debug_set_variant": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "pa_detector_debug_set_trace": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pa_debug_timing_variants_built": (C.c_int, []),
    "pa_preprocess_rgbd": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                     C.c_float, C.c_float, C.c_int, C.c_int, C.c_void_p, C.c_void_p]),
    "pa_keypoints_postprocess": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.c_void_p, C.c_void_p, C.c_void_p]),
    "pa_detector_forward_rgbd": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                           C.c_float, C.c_float, C.c_void_p, C.c_void_p]),
    "pa_detector_forward_rgbd_px": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                              C.c_float, C.c_float, C.c_void_p, C.c_void_p, C.c_void_p]),
    "pa_trajectory_gn_workspace": (C.c_size_t, [C.c_int, C.c_int]),
    "pa_trajectory_gn_step": (C.c_int, [C.c_int, C.c_int, C.c_int] + [C.c_void_p] * 11 + [C.c_double]
                              + [C.c_void_p] * 6 + [C.c_size_t, C.c_void_p]),
    "pa_window_advance": (C.c_int, [C.c_int, C.c_int, C.c_int] + [C.c_void_p] * 5 + [C.c_double, C.c_int,
                                                                                     C.c_void_p]),
    "pa_window_advance_n": (C.c_int, [C.c_int, C.c_int, C.c_int] + [C.c_void_p] * 6 + [C.c_double, C.c_int,
                                                                                       C.c_void_p]),
    "pa_window_retract": (C.c_int, [C.c_int, C.c_int] + [C.c_void_p] * 6),
    "pa_debug_gn_set_assemblers": (C.c_int, [C.c_int]),
    "pa_window_retract_newest": (C.c_int, [C.c_int, C.c_int] + [C.c_void_p] * 7),
    "pa_debug_gn_set_trace": (C.c_int, [C.c_void_p]),
    "pa_host_device_pointer": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p)]),
    "pa_window_pose_tick": (C.c_int, [C.POINTER(TrajArgs), C.c_void_p, C.c_double, C.c_void_p, C.c_void_p, C.c_void_p,
                                      C.c_void_p]),
    "pa_window_pose_tick_workspace": (C.c_size_t, [C.c_int, C.c_int]),
    "pa_window_pose_tick_pre": (C.c_int, [C.POINTER(TrajArgs), C.c_double, C.c_void_p, C.c_size_t, C.c_void_p]),
    "pa_window_pose_tick_post": (C.c_int, [C.POINTER(TrajArgs), C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_void_p]),
    "pa_loss_statistics_workspace": (C.c_size_t, [C.c_longlong]),
    "pa_loss_statistics": (C.c_int, [C.c_void_p, C.c_longlong, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "pa_proj_linearize": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_int,
                                    C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                    C.c_void_p, C.c_void_p]),
    "pa_dyn_linearize": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_double,
                                   C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                   C.c_void_p, C.c_void_p, C.c_void_p]),
    "pa_cv_linearize": (C.c_int, [C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_void_p, C.c_void_p, C.c_void_p]),
    # include/perseus_amd_loader.h (host pointers)
    "pa_png_info": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "pa_png_decode": (C.c_int, [C.c_void_p, C.c_size_t, C.c_int, C.c_void_p, C.c_size_t]),
    "pa_tiff_info": (C.c_int, [C.c_void_p, C.c_size_t, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "pa_tiff_decode_f32": (C.c_int, [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]),
    "pa_load_keypoint_items": (C.c_int, [C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                         C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p,
                                         C.c_void_p]),
}

PREC_FP16 = 0
PREC_FP32 = 1
PREC_FP16X3 = 2
PRECISIONS = {"fp16": PREC_FP16, "fp32": PREC_FP32, "fp16x3": PREC_FP16X3}


def precision_code(name: str) -> int:
    try:
        return PRECISIONS[name]
    except KeyError:
        raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {name!r}") from None

VEL_WORLD = 0
VEL_BODY = 1


def lib_path() -> str:
    return _build.LIB


def lib(build_if_missing: bool = True):
    """Load (and on first use, if absent and a compiler exists, build) the library."""
    global _LIB
    if _LIB is not None:
        return _LIB
    # PERSEUS_AMD_LIB_AB: another build of the library, for tools/so_ab.py's interleaved A/B of
    # two builds on one box (measurement tooling only; unset, the in-tree build is the library)
    path = os.environ.get("PERSEUS_AMD_LIB_AB") or _build.LIB
    if not os.path.exists(path) and build_if_missing and path == _build.LIB:
        _build.build()
    if not os.path.exists(path):
        raise PerseusError(f"{path} not found: run `python -m perseus_amd.build`")
    L = C.CDLL(path)
    for name, (res, args) in _SIGS.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _LIB = L
    return L


def check(rc: int, what: str = "") -> int:
    if rc < 0:
        msg = lib().pa_last_error().decode(errors="replace")
        raise PerseusError(f"{what}: {msg} (code {rc})" if what else f"{msg} (code {rc})")
    return rc


def ptr(t) -> int | None:
    """Device pointer of a torch tensor (None for None; an int is taken as a device address)."""
    if t is None or isinstance(t, int):
        return t
    return t.data_ptr()


def stream_of(device) -> int:
    import torch

    return torch.cuda.current_stream(device).cuda_stream
