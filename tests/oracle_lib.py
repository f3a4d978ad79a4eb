"""ctypes binding of the CPU oracle (oracle/liboracle.so) — TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "liboracle.so")

P = C.c_void_p


class OrbKP(C.Structure):
    _fields_ = [("x", C.c_float), ("y", C.c_float), ("size", C.c_float), ("angle", C.c_float),
                ("response", C.c_float), ("octave", C.c_int32), ("class_id", C.c_int32)]


LANDMARK_DTYPE = np.dtype([("X", "<f4", 3), ("flags", "<i4"), ("desc", "u1", 32)])
HYP_DTYPE = np.dtype([("err", "<f8"), ("cnt", "<i4"), ("pad", "<i4"), ("T", "<f4", 12)])
KP_DTYPE = np.dtype([("x", "<f4"), ("y", "<f4"), ("size", "<f4"), ("angle", "<f4"),
                     ("response", "<f4"), ("octave", "<i4"), ("class_id", "<i4")])
DMATCH_DTYPE = np.dtype([("queryIdx", "<i4"), ("trainIdx", "<i4"), ("imgIdx", "<i4"), ("distance", "<f4")])


class OrbParams(C.Structure):
    _fields_ = [("nfeatures", C.c_int32), ("scale_factor", C.c_float), ("nlevels", C.c_int32),
                ("ini_th_fast", C.c_int32), ("min_th_fast", C.c_int32)]


class Calib(C.Structure):
    _fields_ = [(n, C.c_float) for n in ("fx", "fy", "cx", "cy", "k1", "k2", "p1", "p2", "k3",
                                         "depth_factor", "mbf", "th_depth")]


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


def fr1_calib() -> Calib:
    # Utils/common.h:35-44, 67, 71-72
    return Calib(517.3, 516.5, 318.6, 255.3, 0.262383, -0.953104, -0.005358, 0.002628, 1.163314,
                 1.0 / 5000.0, 40.0, 40.0)


def calib_from(fx, fy, cx, cy, dist=(0.262383, -0.953104, -0.005358, 0.002628, 1.163314)) -> Calib:
    return Calib(fx, fy, cx, cy, *dist, 1.0 / 5000.0, 40.0, 40.0)


def ptr(a: np.ndarray):
    return a.ctypes.data_as(P)


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = C.CDLL(LIB_PATH)
        sig = {
            "oracle_bgr2gray": (None, [P, C.c_int, C.c_int, C.c_int, P]),
            "oracle_depth_to_f32": (None, [P, C.c_int, C.c_float, P]),
            "oracle_level_sizes": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P]),
            "oracle_umax": (C.c_int, [P]),
            "oracle_pyramid": (C.c_int, [P, C.c_int, C.c_int, P, P]),
            "oracle_fast_level": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_int]),
            "oracle_octree": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_int]),
            "oracle_blur": (None, [P, C.c_int, C.c_int, P]),
            "oracle_fast_atan2": (C.c_float, [C.c_float, C.c_float]),
            "oracle_orb_extract": (C.c_int, [P, C.c_int, C.c_int, P, P, P, C.c_int]),
            "oracle_frame_geometry": (None, [P, C.c_int, P, C.c_int, C.c_int, P, P, P, P]),
            "oracle_extract_frame": (C.c_int, [P, P, C.c_int, C.c_int, P, P, P, P, P, P, P, C.c_int]),
            "oracle_knn2": (None, [P, C.c_int, P, C.c_int, P, P]),
            "oracle_knn_match": (C.c_int, [P, C.c_int, P, C.c_int, C.c_float, P, P, P, P, P, P, P, C.c_int]),
            "oracle_sort_dmatch": (None, [P, C.c_int]),
            "oracle_vo_landmarks": (C.c_int, [P, C.c_int, C.c_float, P]),
            "oracle_rng_seed": (None, [P, C.c_uint32]),
            "oracle_rng_next": (C.c_int32, [P]),
            "oracle_libc_rand_stream": (None, [C.c_uint32, C.c_int, P]),
            "oracle_ransac": (C.c_int, [P, C.c_int, P, P, P, P, P, P, P, P, P, P, P]),
            "oracle_tfc": (None, [P, P, P, C.c_int, P]),
            "oracle_last_ransac_work": (None, [P, P]),
            "oracle_svd3": (None, [P, P, P, P]),
            "oracle_pnp": (C.c_int, [P, P, C.c_int, P, P, P, P]),
            "oracle_kabsch": (None, [P, P, C.c_int, P]),
            "oracle_track_pair": (C.c_int, [P, P, P, C.c_int, P, P, P, P, P, C.c_int, P, C.c_float, P,
                                            C.c_uint32, P, P, P, P, C.c_int, P, P]),
            "oracle_adaptive_default": (None, [P]),
            "oracle_image_bounds": (None, [P, C.c_int, C.c_int, P]),
            "oracle_projection_match": (C.c_int, [P, P, C.c_int, P, P, P, C.c_int, P, P, P, C.c_float, C.c_float,
                                                  P, P]),
            "oracle_ransac_hyps": (C.c_int, [P, C.c_int, P, P, P, P, P, C.c_int, C.c_int, P]),
            "oracle_adaptive_detect": (C.c_int, [P, C.c_int, C.c_int, P, P, P, C.c_int, P]),
            "oracle_fast_roi": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_int]),
            "oracle_adaptive_extract": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P, C.c_int, P]),
            "oracle_nth_element_score": (None, [P, C.c_int, C.c_int]),
            "oracle_retain_best_score": (C.c_int, [P, C.c_int, C.c_int]),
            "oracle_extract_frame_adaptive": (C.c_int, [P, P, C.c_int, C.c_int, P, P, P, P, P, P, P, P, C.c_int]),
            "oracle_adaptive_orb_extract": (C.c_int, [P, C.c_int, C.c_int, P, P, P, P, C.c_int, P]),
            "oracle_adaptive_orb_detect": (C.c_int, [P, C.c_int, C.c_int, P, P, P, C.c_int, P]),
            "oracle_orbcv_detect": (C.c_int, [P, C.c_int, C.c_int, C.c_int, C.c_int, P, C.c_int]),
            "oracle_harris": (C.c_float, [P, C.c_int, C.c_int, C.c_int, C.c_int]),
            "oracle_orbcv_levels": (C.c_int, [C.c_int, C.c_int, P, P, P, P]),
            "oracle_extract_frame_adaptive_orb": (C.c_int, [P, P, C.c_int, C.c_int, P, P, P, P, P, P, P, P,
                                                            C.c_int]),
            "oracle_pnp_ransac": (C.c_int, [P, P, C.c_int, P, C.c_int, C.c_float, C.c_double, P, P, P, P, P, P, P,
                                            P]),
            "oracle_cvrng_stream": (None, [C.c_uint64, C.c_int, C.c_int, C.c_int, P]),
            "oracle_ransac_update_num_iters": (C.c_int, [C.c_double, C.c_double, C.c_int, C.c_int]),
            "oracle_rodrigues": (None, [P, P, P]),
            "oracle_rodrigues_inv": (None, [P, P]),
            "oracle_epnp": (None, [P, P, C.c_int, P, P]),
            "oracle_pnp_refine": (None, [P, P, C.c_int, P, P]),
            "oracle_pnp_extrinsic_init": (C.c_int, [P, P, C.c_int, P, P]),
            "oracle_gicp": (C.c_int, [P, C.c_int, P, C.c_int, P, C.c_int, C.c_double, P, P, P, P]),
            "oracle_gicp_covariances": (None, [P, C.c_int, P]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def orb_params(nfeatures=2000, scale=1.2, nlevels=8, ini=20, mn=7) -> OrbParams:
    return OrbParams(nfeatures, scale, nlevels, ini, mn)


def ransac_params(iters=200, min_inl=20, max_mahal=3.0, sample=4, check_depth=1) -> RansacParams:
    return RansacParams(iters, min_inl, max_mahal, sample, check_depth)


def gray(bgr: np.ndarray) -> np.ndarray:
    h, w = bgr.shape[:2]
    out = np.empty((h, w), np.uint8)
    lib().oracle_bgr2gray(ptr(np.ascontiguousarray(bgr)), w, h, 3 * w, ptr(out))
    return out


def extract_frame(bgr, depth, params: OrbParams, calib: Calib, cap=None):
    h, w = bgr.shape[:2]
    cap = cap or params.nfeatures + 8 * params.nlevels + 8
    kps = np.zeros(cap, KP_DTYPE)
    desc = np.zeros((cap, 32), np.uint8)
    kun = np.zeros((cap, 2), np.float32)
    xyz = np.zeros((cap, 3), np.float32)
    ur = np.zeros(cap, np.float32)
    n = lib().oracle_extract_frame(ptr(np.ascontiguousarray(bgr)), ptr(np.ascontiguousarray(depth)), w, h,
                                   C.byref(params), C.byref(calib), ptr(kps), ptr(desc), ptr(kun),
                                   ptr(xyz), ptr(ur), cap)
    assert n <= cap
    return dict(kps=kps[:n], desc=desc[:n], kun=kun[:n], xyz=xyz[:n], ur=ur[:n])


def knn2(q: np.ndarray, t: np.ndarray):
    nq = q.shape[0]
    idx = np.zeros((nq, 2), np.int32)
    dist = np.zeros((nq, 2), np.int32)
    lib().oracle_knn2(ptr(np.ascontiguousarray(q)), nq, ptr(np.ascontiguousarray(t)), t.shape[0],
                      ptr(idx), ptr(dist))
    return idx, dist


def track_pair(f1, f2, calib: Calib, rp: RansacParams, seed: int, latch=float("nan"), ratio=0.9):
    """One pair through the oracle's Track path. Returns (PairResult, PnP
    inlier mask over F2, KnnMatch list, latch); the PairResult also carries
    `inliers`, Ransac::mvInliers as a DMATCH_DTYPE array in list order
    (ransac.cpp:240, 258)."""
    n1, n2 = len(f1["kps"]), len(f2["kps"])
    res = PairResult()
    mask = np.zeros(max(n2, 1), np.uint8)
    matches = np.zeros(max(n1, 1), DMATCH_DTYPE)
    rinl = np.zeros(max(n1, 1), DMATCH_DTYPE)
    nr = C.c_int(0)
    lat = C.c_double(latch)
    L = lib()
    nm = L.oracle_track_pair(ptr(f1["kps"]), ptr(f1["desc"]), ptr(f1["xyz"]), n1,
                             ptr(f2["kps"]), ptr(f2["desc"]), ptr(f2["kun"]), ptr(f2["xyz"]), ptr(f2["ur"]), n2,
                             C.byref(calib), ratio, C.byref(rp), seed, C.byref(lat), C.byref(res),
                             ptr(mask), ptr(matches), max(n1, 1), ptr(rinl), C.byref(nr))
    assert nr.value == res.n_inliers
    res.inliers = rinl[:nr.value]
    return res, mask[:n2], matches[:nm], lat.value


def check_ransac_inliers(gpu_pair, ref, tag):
    """The batched path's RANSAC inlier list (the good-match list masked by
    the kernel's inlier bits) equals Ransac::mvInliers entry for entry:
    queryIdx, trainIdx, imgIdx and distance, in order."""
    got = gpu_pair["good"][gpu_pair["ransac_inliers"].astype(bool)]
    exp = ref.inliers
    assert len(got) == len(exp), f"{tag}: RANSAC inlier list length {len(got)} vs {len(exp)}"
    assert np.array_equal(got, exp), (f"{tag}: RANSAC inlier list differs at "
                                      f"{np.nonzero(got != exp)[0][:8]}")


def adaptive_params() -> AdaptiveParams:
    p = AdaptiveParams()
    lib().oracle_adaptive_default(C.byref(p))
    return p


class AdaptiveExtractor:
    """Extractor(FAST, ORB, ADAPTIVE) (inner="fast") or Extractor(ORB, ORB,
    ADAPTIVE) (inner="orb", the cv::ORB cell detector): per-cell thresholds
    persist across calls."""

    def __init__(self, params: AdaptiveParams = None, inner: str = "fast"):
        assert inner in ("fast", "orb")
        self.inner = inner
        self.p = params or adaptive_params()
        self.thresh = np.full(self.p.grid_rows * self.p.grid_cols, self.p.init_thresh, np.float64)

    def extract_frame(self, bgr, depth, calib: Calib, cap=1100):
        h, w = bgr.shape[:2]
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        kun = np.zeros((cap, 2), np.float32)
        xyz = np.zeros((cap, 3), np.float32)
        ur = np.zeros(cap, np.float32)
        fn = lib().oracle_extract_frame_adaptive if self.inner == "fast" else lib().oracle_extract_frame_adaptive_orb
        n = fn(ptr(np.ascontiguousarray(bgr)), ptr(np.ascontiguousarray(depth)),
                                                w, h, C.byref(self.p), ptr(self.thresh), C.byref(calib), ptr(kps),
                                                ptr(desc), ptr(kun), ptr(xyz), ptr(ur), cap)
        assert n <= cap
        return dict(kps=kps[:n], desc=desc[:n], kun=kun[:n], xyz=xyz[:n], ur=ur[:n])

    def extract_gray(self, gray, cap=1100):
        h, w = gray.shape
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        t_used = np.zeros(self.p.grid_rows * self.p.grid_cols, np.int32)
        fn = lib().oracle_adaptive_extract if self.inner == "fast" else lib().oracle_adaptive_orb_extract
        n = fn(ptr(np.ascontiguousarray(gray)), w, h, C.byref(self.p), ptr(self.thresh),
                                          ptr(kps), ptr(desc), cap, ptr(t_used))
        return kps[:n], desc[:n], t_used


def pnp_chi2(Tcw, Xw, ob, cal):
    """g2o edge chi2 at pose Tcw (EdgeSE3ProjectXYZOnlyPose / StereoOnlyPose,
    information 1/Xw.z^2), as the oracle's PnPProblem::compute_error."""
    R = Tcw[:3, :3].astype(np.float64)
    t = Tcw[:3, 3].astype(np.float64)
    Xc = Xw.astype(np.float64) @ R.T + t
    info = (1.0 / (Xw[:, 2].astype(np.float32) * Xw[:, 2].astype(np.float32))).astype(np.float64)
    stereo = ~(ob[:, 2] < 0)
    invz32 = (np.float32(1.0) / Xc[:, 2].astype(np.float32)).astype(np.float64)
    invz = np.where(stereo, invz32, 1.0 / Xc[:, 2])
    u = Xc[:, 0] * invz * cal.fx + cal.cx
    v = Xc[:, 1] * invz * cal.fy + cal.cy
    ur = u - float(np.float32(cal.mbf)) * invz
    e0, e1 = ob[:, 0] - u, ob[:, 1] - v
    e2 = np.where(stereo, ob[:, 2] - ur, 0.0)
    return info * (e0 * e0 + e1 * e1 + e2 * e2), stereo


def check_pnp_flags(got_flags, ref_flags, f1, f2, f2_src, Tcw_ref, cal, tag):
    """PnP inlier flags must agree except within a 2 % chi2 margin of the
    classification threshold (SURVEY §7 hard part 6), and at most
    max(2, 1 % of the edges) may differ at all (a systematic shift of
    borderline edges fails); returns the number of (marginal) flags that
    differ."""
    bad = np.nonzero(got_flags != ref_flags)[0]
    if bad.size == 0:
        return 0
    cap = max(2, int(0.01 * int((np.asarray(f2_src) >= 0).sum())))
    assert bad.size <= cap, f"{tag}: {bad.size} PnP inlier flags differ (cap {cap})"
    src = f2_src[bad]
    assert (src >= 0).all(), f"{tag}: PnP flag differs on a keypoint without a landmark"
    Xw = f1["xyz"][src]
    ob = np.stack([f2["kun"][bad, 0], f2["kun"][bad, 1], f2["ur"][bad]], 1).astype(np.float64)
    chi, stereo = pnp_chi2(Tcw_ref, Xw, ob, cal)
    th = np.where(stereo, 7.815, 5.991)
    far = np.abs(chi - th) > 0.02 * th
    assert not far.any(), (f"{tag}: PnP inlier flags differ away from the chi2 threshold at keypoints "
                           f"{bad[far][:8]} (chi2 {chi[far][:8]})")
    return int(bad.size)


def pnp_ransac(Xw, uv, calib: Calib, iterations=500, reproj=3.0, confidence=0.85):
    """PnPRansac::Compute's cv::solvePnPRansac (pnpransac.cpp:34) on the oracle."""
    Xw = np.ascontiguousarray(Xw, np.float32)
    uv = np.ascontiguousarray(uv, np.float32)
    n = len(Xw)
    model = np.zeros(6)
    rt = np.zeros(6)
    T = np.zeros(16, np.float32)
    mask = np.zeros(max(n, 1), np.uint8)
    good = np.zeros(max(iterations, 1), np.int32)
    ni, bi, nit = C.c_int(), C.c_int(), C.c_int()
    ok = lib().oracle_pnp_ransac(ptr(Xw), ptr(uv), n, C.byref(calib), iterations, reproj, confidence, ptr(model),
                                 ptr(rt), ptr(T), ptr(mask), C.byref(ni), C.byref(bi), C.byref(nit), ptr(good))
    return dict(ok=ok, model=model, rt=rt, T=T.reshape(4, 4), mask=mask[:n].astype(bool), n_inliers=ni.value,
                best_iter=bi.value, niters=nit.value, good=good[:nit.value])


def gicp(src, tgt, guess=None, max_iterations=10, max_corr_dist=0.07):
    """GeneralizedICP(iters, dist)::Compute(source, target, guess) on the oracle."""
    src = np.ascontiguousarray(src, np.float32)
    tgt = np.ascontiguousarray(tgt, np.float32)
    g = np.ascontiguousarray(np.eye(4, dtype=np.float32) if guess is None else guess, np.float32)
    T = np.zeros(16, np.float32)
    conv, it, nc = C.c_int(), C.c_int(), C.c_int()
    ok = lib().oracle_gicp(ptr(src), len(src), ptr(tgt), len(tgt), ptr(g), max_iterations, max_corr_dist, ptr(T),
                           C.byref(conv), C.byref(it), C.byref(nc))
    return dict(ok=ok, T=T.reshape(4, 4), converged=conv.value, iterations=it.value, n_corr=nc.value)
