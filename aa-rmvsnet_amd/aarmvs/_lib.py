"""ctypes binding of libaarmvs.so (the C ABI declared in include/aarmvs.h).

The library is built in-tree by ``make -C aa-rmvsnet_amd/csrc`` (or
``__graft_entry__.build()``).  There is no fallback: if the shared object is
missing or fails to load, every entry point raises.
"""
from __future__ import annotations

import ctypes
import os

MAX_SRC = 16
_HERE = os.path.dirname(os.path.abspath(__file__))
# AARMVS_LIB: an alternative build of the library (A/B diagnostics; tools/), else the in-tree one
LIB_PATH = os.environ.get("AARMVS_LIB") or os.path.join(_HERE, "libaarmvs.so")

c_int, c_size_t, c_void_p, c_char_p = ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_char_p


class TrainRecord(ctypes.Structure):
    """Mirror of ``aarmvs_train_record``."""
    _fields_ = [("x", c_void_p), ("state", c_void_p), ("z", c_void_p), ("u", c_void_p),
                ("stats", c_void_p), ("t1", c_void_p), ("ostats", c_void_p)]


class SweepArgs(ctypes.Structure):
    """Mirror of ``aarmvs_sweep_args``."""
    _fields_ = [
        ("B", c_int), ("C", c_int), ("H", c_int), ("W", c_int),
        ("nsrc", c_int), ("D", c_int), ("d_begin", c_int), ("d_end", c_int),
        ("ref_fea", c_void_p),
        ("src_fea", c_void_p * MAX_SRC),
        ("rel_proj", c_void_p),
        ("depth_values", c_void_p),
        ("packed_params", c_void_p),
        ("workspace", c_void_p),
        ("depth_out", c_void_p),
        ("conf_out", c_void_p),
        ("cost_out", c_void_p),
        ("slice_out", c_void_p),
        ("omega_out", c_void_p),
        ("aux_stream", c_void_p),
        ("record", ctypes.POINTER(TrainRecord)),
    ]


class BackwardArgs(ctypes.Structure):
    """Mirror of ``aarmvs_backward_args``."""
    _fields_ = [
        ("B", c_int), ("C", c_int), ("H", c_int), ("W", c_int), ("nsrc", c_int), ("D", c_int),
        ("ref_fea", c_void_p),
        ("src_fea", c_void_p * MAX_SRC),
        ("rel_proj", c_void_p),
        ("depth_values", c_void_p),
        ("packed_params", c_void_p),
        ("record", ctypes.POINTER(TrainRecord)),
        ("grad_cost", c_void_p),
        ("grad_ref", c_void_p),
        ("grad_src", c_void_p * MAX_SRC),
        ("grad_params", c_void_p),
        ("grad_x", c_void_p),
        ("workspace", c_void_p),
        ("scratch", c_void_p),
        ("regulariser_only", c_int),
    ]


MAX_FUSION_SRC = 10


def fusion_cam_floats(nsrc: int) -> int:
    return 18 + 42 * nsrc


class FusionArgs(ctypes.Structure):
    """Mirror of ``aarmvs_fusion_args``."""
    _fields_ = [
        ("H", c_int), ("W", c_int), ("nsrc", c_int),
        ("ref_depth", c_void_p),
        ("confidence", c_void_p),
        ("src_depth", c_void_p * MAX_FUSION_SRC),
        ("cams", c_void_p),
        ("photo_threshold", ctypes.c_float),
        ("photo_mask", c_void_p),
        ("geo_mask", c_void_p),
        ("final_mask", c_void_p),
        ("depth_avg", c_void_p),
    ]


# name -> (restype, argtypes)
SIGNATURES = {
    "aarmvs_last_error": (c_char_p, []),
    "aarmvs_version": (c_char_p, []),
    "aarmvs_param_count": (c_size_t, []),
    "aarmvs_packed_param_bytes": (c_size_t, []),
    "aarmvs_pack_params": (c_int, [c_void_p, c_void_p, c_void_p]),
    "aarmvs_homo_warp": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                 c_void_p, c_void_p]),
    "aarmvs_homo_warp_backward_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "aarmvs_homo_warp_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                          c_void_p, c_void_p, c_void_p]),
    "aarmvs_sweep_workspace_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "aarmvs_sweep": (c_int, [ctypes.POINTER(SweepArgs), c_void_p]),
    "aarmvs_aux_stream": (c_int, [ctypes.POINTER(c_void_p)]),
    "aarmvs_train_record_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "aarmvs_backward_scratch_bytes": (c_size_t, [c_int, c_int, c_int, c_int]),
    "aarmvs_sweep_backward": (c_int, [ctypes.POINTER(BackwardArgs), c_void_p]),
    "aarmvs_state_ptr": (c_void_p, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int]),
    "aarmvs_unet_step": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                 c_void_p, c_void_p]),
    "aarmvs_softmax_depth": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p]),
    "aarmvs_lstm_gates_forward": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p,
                                          c_void_p]),
    "aarmvs_lstm_gates_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int,
                                           c_void_p, c_void_p, c_void_p]),
    "aarmvs_group_norm_scratch_bytes": (c_size_t, [c_int, c_int, c_int]),
    "aarmvs_group_norm_forward": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int,
                                          ctypes.c_float, c_void_p, c_void_p, c_void_p, c_void_p]),
    "aarmvs_group_norm_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                           c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                           c_void_p]),
    "aarmvs_cost_slice": (c_int, [c_void_p, ctypes.POINTER(c_void_p), c_void_p, c_void_p, c_void_p,
                                  c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p,
                                  c_void_p]),
    "aarmvs_wta_update": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int,
                                  c_void_p]),
    "aarmvs_fusion_filter": (c_int, [ctypes.POINTER(FusionArgs), c_void_p]),
    "aarmvs_evidential_epilogue": (c_int, [ctypes.POINTER(c_void_p), c_void_p, c_int, c_int, c_void_p,
                                           c_void_p, c_void_p]),
    "aarmvs_evidential_epilogue_backward": (c_int, [ctypes.POINTER(c_void_p), c_void_p, c_int, c_int,
                                                    c_void_p, c_void_p, ctypes.POINTER(c_void_p),
                                                    c_void_p]),
    "aarmvs_deform_sample": (c_int, [c_void_p, c_void_p, c_void_p] + [c_int] * 8 + [c_void_p, c_void_p]),
    "aarmvs_deform_sample_backward": (c_int, [c_void_p, c_void_p, c_void_p] + [c_int] * 8
                                      + [c_void_p] * 5),
    "aarmvs_profile_enable": (None, [c_int]),
    "aarmvs_profile_reset": (None, []),
    "aarmvs_profile_kernel_count": (c_int, []),
    "aarmvs_profile_kernel_name": (c_char_p, [c_int]),
    "aarmvs_profile_read": (c_int, [c_int, ctypes.POINTER(ctypes.c_longlong),
                                    ctypes.POINTER(ctypes.c_double)]),
}

_LIB = None


class AarmvsError(RuntimeError):
    pass


def lib():
    """Load (once) and return the configured CDLL.  Raises if it is not built."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise AarmvsError(
                f"libaarmvs.so not found at {LIB_PATH}: build it with "
                "`make -C aa-rmvsnet_amd/csrc` (hipcc, gfx950). There is no CPU fallback.")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _LIB = handle
    return _LIB


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().aarmvs_last_error().decode(errors="replace")
        raise AarmvsError(f"{what} failed (status {rc}): {msg}")
