"""ctypes binding of ``libpdsc.so`` (the C ABI declared in ``include/pdsc.h``).

The library is built in-tree by ``make -C pointdsc_amd/csrc`` (or
``__graft_entry__.build()``).  There is no fallback: if the library is missing
or cannot be loaded, every entry point raises ``RuntimeError``.
"""
from __future__ import annotations

import ctypes
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# PDSC_LIB_VARIANT=<v> loads libpdsc_<v>.so (an A/B build of the same sources,
# `make -C pointdsc_amd/csrc variant V=<v> VFLAGS=...`; measurement only)
_VARIANT = os.environ.get("PDSC_LIB_VARIANT", "")
LIB_PATH = os.path.join(_HERE, f"libpdsc_{_VARIANT}.so" if _VARIANT else "libpdsc.so")

c_int32, c_size_t, c_float, c_double = ctypes.c_int32, ctypes.c_size_t, ctypes.c_float, ctypes.c_double
vp = ctypes.c_void_p


class PdscConfig(ctypes.Structure):
    """``struct pdsc_config`` (include/pdsc.h)."""
    _fields_ = [
        ("in_dim", c_int32),
        ("num_layers", c_int32),
        ("num_channels", c_int32),
        ("num_iterations", c_int32),
        ("k", c_int32),
        ("ratio", c_double),
        ("inlier_threshold", c_float),
        ("nms_radius", c_float),
        ("refine_threshold", c_float),
        ("precision", c_int32),
    ]


# enum pdsc_precision (include/pdsc.h)
PRECISIONS = {"h3": 0, "f32": 1}


def precision_code(precision) -> int:
    """'h3' (default: 3 fp16 MFMA products per fp32 product) or 'f32' (exact fp32 MFMA)."""
    if precision not in PRECISIONS:
        raise ValueError(f"precision must be one of {sorted(PRECISIONS)}, got {precision!r}")
    return PRECISIONS[precision]


CFG = ctypes.POINTER(PdscConfig)


class PdscForwardDebug(ctypes.Structure):
    """``struct pdsc_forward_debug`` (include/pdsc.h): optional stage outputs."""
    _fields_ = [("conf", vp), ("seeds", vp), ("knn", vp), ("weights", vp), ("trans_pre_refine", vp)]


# name -> (restype, argtypes)
_PROTOS = {
    "pdsc_version": (ctypes.c_char_p, []),
    "pdsc_last_error": (ctypes.c_char_p, []),
    "pdsc_param_count": (c_int32, [CFG]),
    "pdsc_param_name": (ctypes.c_char_p, [CFG, c_int32]),
    "pdsc_packed_weights_floats": (c_size_t, [CFG]),
    "pdsc_pack_weights": (c_int32, [CFG, ctypes.POINTER(vp), vp, vp]),
    "pdsc_compat_f32": (c_int32, [vp, vp, c_int32, c_int32, vp, vp, vp]),
    "pdsc_compat_packed_floats": (c_size_t, [c_int32]),
    "pdsc_compat_packed_f32": (c_int32, [vp, vp, c_int32, c_int32, vp, vp, vp]),
    "pdsc_encoder_workspace_bytes": (c_size_t, [CFG, c_int32, c_int32]),
    "pdsc_encoder_f32": (c_int32, [CFG, vp, vp, vp, c_int32, c_int32, vp, vp, vp, vp, c_size_t, vp]),
    "pdsc_attention_workspace_bytes": (c_size_t, [c_int32, c_int32, c_int32, c_int32]),
    "pdsc_attention_f32": (c_int32, [vp, vp, vp, vp, c_int32, c_int32, c_int32, c_int32, vp, vp, c_size_t, vp]),
    "pdsc_attention_layout": (c_int32, [c_int32, c_int32, c_int32, ctypes.POINTER(c_int32),
                                        ctypes.POINTER(c_int32)]),
    "pdsc_encoder_plan": (c_int32, [c_int32, c_int32, c_int32, ctypes.POINTER(c_int32)]),
    "pdsc_attention_timing": (c_int32, [ctypes.POINTER(vp), ctypes.POINTER(vp), c_int32, ctypes.POINTER(c_int32)]),
    "pdsc_forward_timing": (c_int32, [ctypes.POINTER(vp), c_int32, ctypes.POINTER(c_int32)]),
    "pdsc_diag_qkv_delay": (c_int32, [c_int32]),
    "pdsc_pick_seeds": (c_int32, [vp, vp, c_int32, c_int32, c_float, c_int32, vp, vp, vp]),
    "pdsc_seed_knn_workspace_bytes": (c_size_t, [c_int32, c_int32, c_int32]),
    "pdsc_seed_knn": (c_int32, [vp, vp, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, vp, vp, c_size_t,
                                vp]),
    "pdsc_nsm_workspace_bytes": (c_size_t, [c_int32, c_int32, c_int32, c_int32, c_int32]),
    "pdsc_nsm_weights": (c_int32, [vp, vp, vp, vp, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                                   vp, vp, vp, vp, vp, c_size_t, vp]),
    "pdsc_rigid_transform_3d": (c_int32, [vp, vp, vp, c_int32, c_int32, vp, vp]),
    "pdsc_seed_hypotheses_workspace_bytes": (c_size_t, [c_int32, c_int32]),
    "pdsc_seed_hypotheses": (c_int32, [vp, vp, vp, vp, c_int32, c_int32, c_int32, c_int32, c_float,
                                       vp, vp, vp, vp, vp, vp, c_size_t, vp]),
    "pdsc_post_refine": (c_int32, [vp, vp, vp, c_int32, c_int32, c_float, vp]),
    "pdsc_mutual_nn_workspace_bytes": (c_size_t, [c_int32, c_int32]),
    "pdsc_mutual_nn": (c_int32, [vp, vp, c_int32, c_int32, c_int32, vp, vp, vp, c_size_t, vp]),
    "pdsc_build_correspondences": (c_int32, [vp, vp, vp, vp, c_int32, c_int32, c_int32, c_int32, vp, c_double,
                                             vp, vp, vp, vp, vp, vp, vp, c_size_t, vp]),
    "pdsc_spectral_matching_workspace_bytes": (c_size_t, [c_int32]),
    "pdsc_spectral_matching": (c_int32, [vp, vp, vp, c_int32, c_double, c_double, c_int32, vp, vp, vp, vp,
                                         c_size_t, vp]),
    "pdsc_sm_matvec": (c_int32, [vp, vp, c_int32, vp, vp]),
    "pdsc_forward_workspace_bytes": (c_size_t, [CFG, c_int32, c_int32]),
    "pdsc_forward_testing": (c_int32, [CFG, vp, vp, vp, vp, c_int32, c_int32, vp, vp, vp, vp, vp,
                                       c_size_t, vp]),
    "pdsc_forward_testing_debug": (c_int32, [CFG, vp, vp, vp, vp, c_int32, c_int32, vp, vp,
                                             ctypes.POINTER(PdscForwardDebug), vp, c_size_t, vp]),
    "pdsc_forward_testing_ragged": (c_int32, [CFG, vp, vp, vp, vp, c_int32, c_int32, ctypes.POINTER(c_int32), vp, vp,
                                              ctypes.POINTER(PdscForwardDebug), vp, c_size_t, vp]),
    "pdsc_ply_read_xyz": (c_int32, [ctypes.c_char_p, vp, ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]),
    "pdsc_radius_knn_workspace_bytes": (c_size_t, [c_int32]),
    "pdsc_radius_knn": (c_int32, [vp, c_int32, c_float, c_int32, vp, vp, vp, vp, c_size_t, vp]),
    "pdsc_estimate_normals_workspace_bytes": (c_size_t, [c_int32, c_int32]),
    "pdsc_estimate_normals": (c_int32, [vp, c_int32, c_float, c_int32, c_int32, vp, vp, vp, c_size_t, vp]),
    "pdsc_voxel_down_sample_workspace_bytes": (c_size_t, [c_int32]),
    "pdsc_voxel_down_sample": (c_int32, [vp, vp, c_int32, c_float, vp, vp, vp, vp, c_size_t, vp]),
    "pdsc_compute_fpfh_workspace_bytes": (c_size_t, [c_int32, c_int32]),
    "pdsc_compute_fpfh": (c_int32, [vp, vp, c_int32, c_float, c_int32, vp, vp, vp, c_size_t, vp]),
    "pdsc_forward_training_workspace_bytes": (c_size_t, [CFG, c_int32, c_int32]),
    "pdsc_range_status": (c_int32, [vp, c_int32, ctypes.POINTER(c_int32), vp]),
    "pdsc_range_poll": (c_int32, [vp, c_int32, vp]),
    "pdsc_forward_training": (c_int32, [CFG, vp, vp, vp, vp, c_int32, c_int32, vp, vp, vp, vp, vp, c_size_t, vp]),
    "pdsc_spectral_matching_loss_workspace_bytes": (c_size_t, [c_int32, c_int32]),
    "pdsc_spectral_matching_loss": (c_int32, [vp, vp, c_int32, c_int32, c_int32, vp, vp, c_size_t, vp]),
}

EXPORTS = tuple(_PROTOS)

_lib = None
_lock = threading.Lock()


def load():
    """Load libpdsc.so once; raise RuntimeError (no fallback) if unavailable."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise RuntimeError(
                    f"pointdsc_amd: HIP library {LIB_PATH} is missing; build it with "
                    "`make -C pointdsc_amd/csrc` or `python -c 'import __graft_entry__ as g; g.build()'`. "
                    "There is no CPU fallback.")
            try:
                lib = ctypes.CDLL(LIB_PATH)
            except OSError as e:
                raise RuntimeError(f"pointdsc_amd: cannot load {LIB_PATH}: {e}") from e
            for name, (res, args) in _PROTOS.items():
                fn = getattr(lib, name)
                fn.restype, fn.argtypes = res, args
            _lib = lib
    return _lib


def check(status: int, what: str):
    if status != 0:
        msg = load().pdsc_last_error().decode(errors="replace")
        raise RuntimeError(f"{what} failed (status {status}): {msg}")


def make_config(in_dim=6, num_layers=12, num_channels=128, num_iterations=10, k=40, ratio=0.1,
                inlier_threshold=0.10, nms_radius=0.10, precision="h3") -> PdscConfig:
    """Build ``pdsc_config``; the refine threshold follows models/PointDSC.py:415-418."""
    refine = 0.10 if inlier_threshold == 0.10 else 1.2
    return PdscConfig(int(in_dim), int(num_layers), int(num_channels), int(num_iterations), int(k),
                      float(ratio), float(inlier_threshold), float(nms_radius), float(refine),
                      precision_code(precision))
