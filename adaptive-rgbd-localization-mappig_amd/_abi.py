"""ctypes view of include/odo.h (the C-ABI of libodo_hip.so).

The product path is the HIP library; this module only binds it. There is no
CPU fallback: if the shared library or a gfx950 device is missing, loading or
odo_create() fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libodo_hip.so")

P = C.c_void_p


class OrbKP(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


class DMatch(C.Structure):
    _fields_ = [("queryIdx", C.c_int32), ("trainIdx", C.c_int32), ("imgIdx", C.c_int32), ("distance", C.c_float)]


class Calib(C.Structure):
    _fields_ = [(n, C.c_float) for n in ("fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2", "k3",
                                         "depth_factor", "mbf", "th_depth")]


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class PnPRansacResult(C.Structure):
    """odo_pnp_ransac_result (include/odo_types.h)."""
    _fields_ = [("rvec", C.c_double * 3), ("tvec", C.c_double * 3), ("model_rvec", C.c_double * 3),
                ("model_tvec", C.c_double * 3), ("Tcw", C.c_float * 16), ("ok", C.c_int32),
                ("n_inliers", C.c_int32), ("best_iter", C.c_int32), ("iterations_visited", C.c_int32)]


class RansacParams(C.Structure):
    _fields_ = [("iterations", C.c_int32), ("min_inlier_th", C.c_int32), ("max_mahalanobis", C.c_float),
                ("sample_size", C.c_int32), ("check_depth", C.c_int32)]


class AdaptiveParams(C.Structure):
    _fields_ = [("grid_rows", C.c_int32), ("grid_cols", C.c_int32), ("edge_threshold", C.c_int32),
                ("max_total_keypoints", C.c_int32), ("cell_min", C.c_int32), ("cell_max", C.c_int32),
                ("escape_iters", C.c_int32), ("init_thresh", C.c_double), ("min_thresh", C.c_double),
                ("max_thresh", C.c_double), ("increase_factor", C.c_double), ("decrease_factor", C.c_double),
                ("retain_best", C.c_int32)]


class Rng(C.Structure):
    _fields_ = [("state", C.c_int32 * 31), ("fpos", C.c_int32), ("rpos", C.c_int32)]


class PairResult(C.Structure):
    _fields_ = [("T12", C.c_float * 16), ("Tcw", C.c_float * 16), ("rmse", C.c_float),
                ("n_matches", C.c_int32), ("n_good", C.c_int32), ("n_inliers", C.c_int32),
                ("ransac_ok", C.c_int32), ("pnp_inliers", C.c_int32), ("visited", C.c_int32),
                ("n_queries", C.c_int32), ("n_sweeps", C.c_int32), ("n_fit_points", C.c_int32)]


class KernelForms(C.Structure):
    """odo_kernel_forms (include/odo.h): bit-identical kernel alternatives."""
    _fields_ = [("knn", C.c_int32), ("knn_split", C.c_int32), ("ransac_lanes_min_open", C.c_int32),
                ("pyramid", C.c_int32), ("ransac_first_hyps", C.c_int32)]


class Config(C.Structure):
    _fields_ = [("struct_size", C.c_uint32), ("width", C.c_int32), ("height", C.c_int32), ("max_batch", C.c_int32),
                ("orb", OrbParams), ("calib", Calib), ("nn_ratio", C.c_float),
                ("ransac", RansacParams), ("seed", C.c_uint32), ("detector", C.c_int32),
                ("adaptive", AdaptiveParams), ("forms", KernelForms)]


KNN_FORM_FP4 = 0   # include/odo.h ODO_KNN_FORM_FP4
KNN_FORM_VALU = 1  # include/odo.h ODO_KNN_FORM_VALU
PYRAMID_FORM_AUTO = 0  # include/odo.h ODO_PYRAMID_FORM_AUTO
PYRAMID_FORM_CHAIN = 1  # include/odo.h ODO_PYRAMID_FORM_CHAIN
PYRAMID_FORM_FUSED_NOBLUR = 2  # include/odo.h ODO_PYRAMID_FORM_FUSED_NOBLUR
PYRAMID_FORM_FUSED = 3  # include/odo.h ODO_PYRAMID_FORM_FUSED


DETECTOR_ORB_SLAM2 = 0       # include/odo.h ODO_DETECTOR_ORB_SLAM2
DETECTOR_ADAPTIVE_FAST = 1   # include/odo.h ODO_DETECTOR_ADAPTIVE_FAST
DETECTOR_ADAPTIVE_ORB = 2    # include/odo.h ODO_DETECTOR_ADAPTIVE_ORB


class FoldResult(C.Structure):
    _fields_ = [("best_h", C.c_int32), ("visited", C.c_int32), ("valid", C.c_int32), ("n_inliers", C.c_int32),
                ("rmse", C.c_float), ("n_good", C.c_int32), ("pad", C.c_int32 * 2)]


HYP_DTYPE = np.dtype([("err", "<f8"), ("cnt", "<i4"), ("pad", "<i4"), ("T", "<f4", 12)])  # odo_hyp_summary
LANDMARK_DTYPE = np.dtype([("X", "<f4", 3), ("flags", "<i4"), ("desc", "u1", 32)])  # odo_landmark
LM_BAD, LM_SEEN, LM_HAS_OBS = 1, 2, 4
KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
DMATCH_DTYPE = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("imgIdx", "<i4"), ("distance", "<f4")])
PAIR_DTYPE = np.dtype([("T12", "<f4", 16), ("Tcw", "<f4", 16), ("rmse", "<f4"), ("n_matches", "<i4"),
                       ("n_good", "<i4"), ("n_inliers", "<i4"), ("ransac_ok", "<i4"), ("pnp_inliers", "<i4"),
                       ("visited", "<i4"), ("n_queries", "<i4"), ("n_sweeps", "<i4"), ("n_fit_points", "<i4")])

# Every symbol include/odo.h declares, with its ctypes signature.
SIGNATURES = {
    "odo_abi_version": (C.c_int, []),
    "odo_default_config": (None, [P, C.c_int, C.c_int, C.c_int]),
    "odo_create": (P, [P, C.c_int]),
    "odo_destroy": (None, [P]),
    "odo_last_error": (C.c_char_p, []),
    "odo_stream": (P, [P]),
    "odo_reset": (C.c_int, [P]),
    "odo_set_latch": (C.c_int, [P, C.c_double]),
    "odo_get_latch": (C.c_double, [P]),
    "odo_track_batch": (C.c_int, [P, P, P, C.c_int, P]),
    "odo_track_batch_host": (C.c_int, [P, P, P, C.c_int, P]),
    "odo_host_alloc": (P, [C.c_size_t]),
    "odo_track_batch_async": (C.c_int, [P, P, P, C.c_int, P]),
    "odo_track_batch_host_sparse_depth": (C.c_int, [P, P, P, C.c_int, P]),
    "odo_track_batch_host_async": (C.c_int, [P, P, P, C.c_int, P]),
    "odo_host_depth_query": (C.c_int, [P]),
    "odo_host_depth_wait": (C.c_int, [P]),
    "odo_seek": (C.c_int, [P, C.c_uint64, C.c_int]),
    "odo_host_free": (C.c_int, [P]),
    "odo_extract_batch": (C.c_int, [P, P, P, C.c_int]),
    "odo_synchronize": (C.c_int, [P]),
    "odo_get_frame": (C.c_int, [P, C.c_int, P, P, P, P, P, C.c_int, P]),
    "odo_get_pair": (C.c_int, [P, C.c_int, P, C.c_int, P, P, P, P, P, P]),
    "odo_extract": (C.c_int, [P, P, C.c_int, P, P, P, P, P, P, C.c_int, P]),
    "odo_knn2_hamming": (C.c_int, [P, P, C.c_int, P, C.c_int, P, P]),
    "odo_ransac": (C.c_int, [P, P, C.c_int, P, C.c_int, P, C.c_int, P, P, P, P, P, P, P, P]),
    "odo_pnp_motion_ba": (C.c_int, [P, P, P, C.c_int, P, P, P, P, P]),
    "odo_kabsch": (C.c_int, [P, P, C.c_int, P]),
    "odo_pnp_ransac": (C.c_int, [P, P, P, C.c_int, P, C.c_int, C.c_float, C.c_double, P, P, P]),
    "odo_pnp_ransac_batch": (C.c_int, [P, P, P, P, C.c_int, P, C.c_int, C.c_float, C.c_double, P, P]),
    "odo_gicp_batch": (C.c_int, [P, P, P, P, P, P, C.c_int, C.c_int, C.c_double, P, P, P, P]),
    "odo_gicp": (C.c_int, [P, P, C.c_int, P, C.c_int, P, C.c_int, C.c_double, P, P, P, P]),
    "odo_rng_seed": (None, [P, C.c_uint32]),
    "odo_rng_next": (C.c_int32, [P]),
    "odo_debug_pyramid": (C.c_int, [P, C.c_int, P, C.c_size_t]),
    "odo_debug_fast": (C.c_int, [P, C.c_int, C.c_int, P, C.c_int, P]),
    "odo_debug_octree": (C.c_int, [P, C.c_int, C.c_int, P, C.c_int, P]),
    "odo_debug_sort": (C.c_int, [P, P, C.c_int, P]),
    "odo_knn_replay_time": (C.c_int, [P, C.c_int, C.POINTER(C.c_float)]),
    "odo_set_timing": (C.c_int, [P, C.c_int]),
    "odo_kernel_timing": (C.c_int, [P, P, P]),
    "odo_step_marks": (C.c_int, [P, C.POINTER(C.c_double), C.c_int]),
    "odo_debug_blur": (C.c_int, [P, C.c_int, P, C.c_size_t]),
    "odo_last_timings": (C.c_int, [P, P, C.c_int, P]),
    "odo_debug_adaptive": (C.c_int, [P, C.c_int, P, P]),
    "odo_set_adaptive_thresholds": (C.c_int, [P, P, C.c_int]),
    "odo_debug_select": (C.c_int, [P, P, C.c_int, C.c_int, C.c_int, P, P]),
    "odo_image_bounds": (C.c_int, [P, P]),
    "odo_chain_poses": (C.c_int, [P, C.c_int, P, P]),
    "odo_write_tum_trajectory": (C.c_int, [C.c_char_p, P, P, C.c_int, C.c_int]),
    "odo_projection_match": (C.c_int, [P, P, P, C.c_int, P, P, P, C.c_int, P, C.c_float, C.c_float, P, P, P]),
    "odo_ransac_hyps": (C.c_int, [P, P, C.c_int, P, C.c_int, P, C.c_int, P, P, P, C.c_int, C.c_int, P, P]),
    "odo_ransac_fold": (C.c_int, [P, C.c_int, C.c_int, P, P]),
    "odo_ransac_hyps_finish": (C.c_int, [P, P, P, P, P, P, P, P, P]),
    "odo_ransac_hyps_dev": (C.c_int, [P, P, C.c_int, P, C.c_int, P, C.c_int, P, P, P, C.c_int, C.c_int, P, P]),
    "odo_ransac_fold_dev": (C.c_int, [P, P, C.c_int, P]),
    "odo_ransac_hyps_payload_words": (C.c_int, [P]),
    "odo_ransac_hyps_finish_dev": (C.c_int, [P, P, C.c_int, P, C.c_int]),
    "odo_ransac_hyps_result": (C.c_int, [P, P, P, P, P, P, P, P, P]),
}

_lib = None


def load(path: str = None):
    """Load libodo_hip.so and bind every C-ABI symbol. Raises if it is missing.
    ODO_LIB names an alternative build of the same library (A/B experiments)."""
    global _lib
    if _lib is not None:
        return _lib
    path = path or os.environ.get("ODO_LIB") or LIB_PATH
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not built: run __graft_entry__.build() (make -C adaptive-rgbd-localization-mappig_amd)")
    # One HIP runtime per process: torch bundles its own libamdhip64.so.7 /
    # libhsa-runtime64.so.1 under the same SONAMEs as /opt/rocm's. Loaded
    # first, this library would pull in /opt/rocm's copies and torch would then
    # bind to them and find no GPU; with torch imported first, the dynamic
    # linker resolves this library's HIP dependency to torch's copy.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    _lib = L
    return L


def ptr(a):
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(P)
    return C.cast(C.pointer(a), P) if not isinstance(a, int) else P(a)


def check(rc: int):
    if rc != 0:
        raise RuntimeError(f"odo error {rc}: {load().odo_last_error().decode()}")
    return rc
