"""MI355X-native per-frame odometry hot path of Adaptive-RGBD-Localization-Mapping.

The compute path is libodo_hip.so (hand-written HIP for gfx950, C-ABI in
include/odo.h). This package is a thin Python binding used by tests and
bench.py; the reference-shaped C++ adapters (Extractor / Matcher / Ransac /
PnPSolver / Kabsch) are shown in INTEGRATION.md.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import (DETECTOR_ADAPTIVE_FAST, DETECTOR_ADAPTIVE_ORB, DETECTOR_ORB_SLAM2, KNN_FORM_FP4, KNN_FORM_VALU,
                   PYRAMID_FORM_AUTO, PYRAMID_FORM_CHAIN, PYRAMID_FORM_FUSED, PYRAMID_FORM_FUSED_NOBLUR,
                   AdaptiveParams, Calib, Config, DMatch, PnPRansacResult,
                   DMATCH_DTYPE, KP_DTYPE, OrbParams, PAIR_DTYPE, PairResult, RansacParams, Rng, check, load, ptr)

__all__ = ["Odometry", "HostFrames", "PinnedResults", "default_config", "load", "KP_DTYPE", "DMATCH_DTYPE", "PAIR_DTYPE", "rng_stream",
           "kabsch", "Calib", "OrbParams", "RansacParams", "Config", "AdaptiveParams", "DETECTOR_ORB_SLAM2",
           "DETECTOR_ADAPTIVE_FAST", "DETECTOR_ADAPTIVE_ORB", "KNN_FORM_FP4", "KNN_FORM_VALU",
           "PYRAMID_FORM_AUTO", "PYRAMID_FORM_FUSED", "PYRAMID_FORM_CHAIN",
           "PYRAMID_FORM_FUSED_NOBLUR"]


def default_config(width=640, height=480, max_batch=1, nfeatures=1000, iterations=200, seed=0x5EED0000,
                   calib=None, detector=_abi.DETECTOR_ORB_SLAM2, forms=None) -> Config:
    """Reference defaults (extractor.cpp:86, odometry.cpp:28, common.h FR1).
    detector: DETECTOR_ORB_SLAM2 (main.cpp:19-21), DETECTOR_ADAPTIVE_FAST
    (Extractor(FAST, ORB, ADAPTIVE), extractor.cpp:55-77) or
    DETECTOR_ADAPTIVE_ORB (Extractor(ORB, ORB, ADAPTIVE): the cv::ORB cell
    detector of detectoradjuster.cpp:29). forms: odo_kernel_forms fields
    (knn = KNN_FORM_FP4 / KNN_FORM_VALU, knn_split, ransac_lanes_min_open,
    pyramid = PYRAMID_FORM_AUTO / PYRAMID_FORM_FUSED / PYRAMID_FORM_CHAIN /
    PYRAMID_FORM_FUSED_NOBLUR, ransac_first_hyps)."""
    cfg = Config()
    load().odo_default_config(ptr(cfg), width, height, max_batch)
    cfg.detector = detector
    cfg.orb.nfeatures = nfeatures
    cfg.ransac.iterations = iterations
    cfg.seed = seed
    if calib is not None:
        for k, v in calib.items():
            setattr(cfg.calib, k, v)
    for k, v in (forms or {}).items():  # odo_kernel_forms: bit-identical kernel alternatives
        setattr(cfg.forms, k, v)
    return cfg


class HostFrames:
    """Page-locked host buffers for n frames of BGR8 + depth16 (odo_host_alloc):
    decode into `bgr` / `depth` (numpy views) and pass the object to
    Odometry.track_batch_host; the DMA engines read it without a staging copy."""

    def __init__(self, n: int, width: int, height: int):
        self.lib = load()
        self.n, self.w, self.h = n, width, height
        nb, nd = n * height * width * 3, n * height * width * 2
        self._pb = self.lib.odo_host_alloc(nb)
        self._pd = self.lib.odo_host_alloc(nd)
        if not self._pb or not self._pd:
            self.close()
            raise MemoryError("odo_host_alloc failed: " + self.lib.odo_last_error().decode())
        self.bgr = np.ctypeslib.as_array(C.cast(self._pb, C.POINTER(C.c_uint8)), (n, height, width, 3))
        self.depth = np.ctypeslib.as_array(C.cast(self._pd, C.POINTER(C.c_uint16)), (n, height, width))

    def close(self):
        for a in ("_pb", "_pd"):
            p = getattr(self, a, None)
            if p:
                self.lib.odo_host_free(p)
                setattr(self, a, None)
        self.bgr = self.depth = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PinnedResults:
    """Page-locked ring of result records for Odometry.track_batch_async:
    `rows` batches of `n` records each (a numpy PAIR_DTYPE view per row)."""

    def __init__(self, rows: int, n: int):
        self.lib = load()
        self.rows, self.n = rows, n
        self._p = self.lib.odo_host_alloc(rows * n * PAIR_DTYPE.itemsize)
        if not self._p:
            raise MemoryError("odo_host_alloc failed: " + self.lib.odo_last_error().decode())
        raw = np.ctypeslib.as_array(C.cast(self._p, C.POINTER(C.c_uint8)), (rows * n * PAIR_DTYPE.itemsize,))
        self.all = raw.view(PAIR_DTYPE).reshape(rows, n)

    def row_ptr(self, r: int) -> int:
        return self._p + (r % self.rows) * self.n * PAIR_DTYPE.itemsize

    def close(self):
        if getattr(self, "_p", None):
            self.lib.odo_host_free(self._p)
            self._p = None
        self.all = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Odometry:
    """One context = one HIP stream + HBM scratch + previous-frame/latch state."""

    def __init__(self, cfg: Config, device: int = 0):
        self.lib = load()
        self.cfg = cfg
        h = self.lib.odo_create(ptr(cfg), device)
        if not h:
            raise RuntimeError("odo_create failed: " + self.lib.odo_last_error().decode())
        self.h = h
        self.kp_cap = max(cfg.orb.nfeatures + 4 * cfg.orb.nlevels + 64,
                          cfg.adaptive.max_total_keypoints + 64)

    def close(self):
        if getattr(self, "h", None):
            self.lib.odo_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return self.lib.odo_stream(self.h) or 0

    def reset(self):
        check(self.lib.odo_reset(self.h))

    def set_latch(self, v: float):
        check(self.lib.odo_set_latch(self.h, v))

    @property
    def latch(self) -> float:
        return self.lib.odo_get_latch(self.h)

    def track_batch(self, bgr_ptr: int, depth_ptr: int, n: int, want_results=True):
        """Device-resident inputs (e.g. torch tensor .data_ptr())."""
        out = np.zeros(n, PAIR_DTYPE) if want_results else None
        check(self.lib.odo_track_batch(self.h, C.c_void_p(bgr_ptr), C.c_void_p(depth_ptr), n,
                                       ptr(out) if want_results else None))
        return out

    def track_batch_async(self, bgr_ptr: int, depth_ptr: int, n: int, results: PinnedResults, row: int):
        """Device-resident inputs; the n result records land in results.all[row]
        after the next synchronize() (no host sync here)."""
        check(self.lib.odo_track_batch_async(self.h, C.c_void_p(bgr_ptr), C.c_void_p(depth_ptr), n,
                                             C.c_void_p(results.row_ptr(row))))

    def seek(self, pair_index: int, keep_prev: bool = False):
        """Next batch's pair p gets global pair index pair_index + p; without
        keep_prev its first frame starts a segment (a halo frame, no pair)."""
        check(self.lib.odo_seek(self.h, int(pair_index), 1 if keep_prev else 0))

    def _host_frames(self, hf: "HostFrames", n):
        """(n, bgr pointer, depth pointer) of a HostFrames after checking that it
        holds n frames of this context's size: the C-ABI trusts n * W * H."""
        n = hf.n if n is None else int(n)
        if not 0 < n <= hf.n:
            raise ValueError(f"n = {n} frames requested from a HostFrames of {hf.n}")
        if (hf.w, hf.h) != (self.cfg.width, self.cfg.height):
            raise ValueError(f"HostFrames are {hf.w}x{hf.h}, the context tracks "
                             f"{self.cfg.width}x{self.cfg.height}")
        if hf._pb is None:
            raise ValueError("HostFrames closed")
        return n, hf._pb, hf._pd

    def track_batch_host(self, bgr, depth=None, want_results=True, n=None):
        """Host inputs: numpy arrays (pageable) or a HostFrames (pinned; then
        `n` frames of it, default all). Without results the call returns once
        the host buffers are consumed and the batch is queued (the upload
        overlaps the compute of earlier batches; the batch runs asynchronously)."""
        if isinstance(bgr, HostFrames):
            n, pb, pd = self._host_frames(bgr, n)
        else:
            bgr = np.ascontiguousarray(bgr, np.uint8)
            depth = np.ascontiguousarray(depth, np.uint16)
            W, H = self.cfg.width, self.cfg.height
            n = bgr.shape[0]
            if bgr.shape != (n, H, W, 3) or depth.shape != (n, H, W):
                raise ValueError(f"frames must be (n, {H}, {W}, 3) u8 and (n, {H}, {W}) u16, got "
                                 f"{bgr.shape} and {depth.shape}")
            pb, pd = ptr(bgr), ptr(depth)
        out = np.zeros(n, PAIR_DTYPE) if want_results else None
        check(self.lib.odo_track_batch_host(self.h, pb, pd, n, ptr(out) if want_results else None))
        return out

    def track_batch_host_async(self, hf: "HostFrames", results: "PinnedResults", row: int, n=None, first: int = 0):
        """odo_track_batch_host_async: frames [first, first + n) of a HostFrames
        uploaded and tracked, the records streamed into results.all[row] (valid
        after synchronize(); the host frames are consumed on return)."""
        n = (hf.n - first) if n is None else int(n)
        if first < 0 or not 0 < n <= hf.n - first or n > results.n:
            raise ValueError(f"frames [{first}, {first + n}) of {hf.n}, result rows of {results.n}")
        self._host_frames(hf, first + n)
        fb, fd = hf.w * hf.h * 3, hf.w * hf.h * 2
        check(self.lib.odo_track_batch_host_async(self.h, C.c_void_p(hf._pb + first * fb),
                                                  C.c_void_p(hf._pd + first * fd), n,
                                                  C.c_void_p(results.row_ptr(row))))

    def track_batch_host_sparse_depth(self, hf: "HostFrames", want_results=True, n=None):
        """odo_track_batch_host_sparse_depth: BGR uploaded, depth read in place
        from the pinned HostFrames. Until the batch has read it the depth view
        is made read-only (numpy raises on a refill): depth_wait(),
        depth_busy() == False or synchronize() release it."""
        n, pb, pd = self._host_frames(hf, n)
        out = np.zeros(n, PAIR_DTYPE) if want_results else None
        check(self.lib.odo_track_batch_host_sparse_depth(self.h, pb, pd, n, ptr(out) if want_results else None))
        if not want_results:
            hf.depth.flags.writeable = False
            self._depth_hold = getattr(self, "_depth_hold", []) + [hf]
        return out

    def _release_depth(self):
        # the event covers the last sparse batch; earlier ones ran before it
        # on the same stream
        for hf in getattr(self, "_depth_hold", []):
            if hf.depth is not None:
                hf.depth.flags.writeable = True
        self._depth_hold = []

    def depth_busy(self) -> bool:
        """odo_host_depth_query: the last sparse-depth batch may still read its depth frames."""
        r = self.lib.odo_host_depth_query(self.h)
        if r < 0:
            check(r)
        if r == 0:
            self._release_depth()
        return r == 1

    def depth_wait(self):
        """odo_host_depth_wait: block until the sparse-depth frames are released."""
        check(self.lib.odo_host_depth_wait(self.h))
        self._release_depth()

    def set_timing(self, enable, mode: int = None):
        """Timing mode: 0 off, 1 per-stage HIP events in odo_track_batch
        (serialises the streams a little; see timings()), 2 an event pair around
        the Hamming-match launch of every batch (see kernel_timing())."""
        m = mode if mode is not None else (1 if enable else 0)
        check(self.lib.odo_set_timing(self.h, m))

    def knn_replay_ms(self, reps: int = 20) -> float:
        """Mean duration of the last batch's kNN-2 launch re-run alone (measurement)."""
        ms = C.c_float(0)
        check(self.lib.odo_knn_replay_time(self.h, reps, C.byref(ms)))
        return float(ms.value)

    def kernel_timing(self):
        """(mean Hamming-match launch duration in ms, launches) since mode 2 was set."""
        avg = C.c_double(0)
        n = C.c_long(0)
        check(self.lib.odo_kernel_timing(self.h, C.byref(avg), C.byref(n)))
        return avg.value, n.value

    def step_marks(self):
        """odo_step_marks: the start (ms after set_timing mode 2) of every batch's
        kNN-2 launch since then; np.diff gives the per-step times."""
        n = self.lib.odo_step_marks(self.h, None, 0)
        if n < 0:
            check(n)
        buf = (C.c_double * max(1, n))()
        k = self.lib.odo_step_marks(self.h, buf, n)
        if k < 0:
            check(k)
        return [float(buf[i]) for i in range(min(k, n))]

    def synchronize(self):
        check(self.lib.odo_synchronize(self.h))
        self._release_depth()

    def frame(self, i: int):
        cap = self.kp_cap
        kps = np.zeros(cap, KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        kun = np.zeros((cap, 2), np.float32)
        xyz = np.zeros((cap, 3), np.float32)
        ur = np.zeros(cap, np.float32)
        n = C.c_int(0)
        check(self.lib.odo_get_frame(self.h, i, ptr(kps), ptr(desc), ptr(kun), ptr(xyz), ptr(ur), cap, C.byref(n)))
        m = n.value
        return dict(kps=kps[:m], desc=desc[:m], kun=kun[:m], xyz=xyz[:m], ur=ur[:m])

    def pair(self, i: int):
        cap = self.kp_cap
        matches = np.zeros(cap, DMATCH_DTYPE)
        good = np.zeros(cap, DMATCH_DTYPE)
        rin = np.zeros(cap, np.uint8)
        pin = np.zeros(cap, np.uint8)
        src = np.zeros(cap, np.int32)
        nm, ng = C.c_int(0), C.c_int(0)
        check(self.lib.odo_get_pair(self.h, i, ptr(matches), cap, C.byref(nm), ptr(good), C.byref(ng), ptr(rin),
                                    ptr(pin), ptr(src)))
        return dict(matches=matches[:nm.value], good=good[:ng.value], ransac_inliers=rin[:ng.value],
                    pnp_inliers=pin, f2_src=src)

    def debug_pyramid(self, i: int, total: int):
        out = np.zeros(total + 4096, np.uint8)
        n = self.lib.odo_debug_pyramid(self.h, i, ptr(out), out.size)
        if n < 0:
            check(n)
        return out[:n]

    def debug_blur(self, i: int, total: int):
        out = np.zeros(total + 4096, np.uint8)
        n = self.lib.odo_debug_blur(self.h, i, ptr(out), out.size)
        if n < 0:
            check(n)
        return out[:n]

    def debug_fast(self, i: int, level: int, cap: int = 1 << 18):
        out = np.zeros(cap, KP_DTYPE)
        n = C.c_int(0)
        check(self.lib.odo_debug_fast(self.h, i, level, ptr(out), cap, C.byref(n)))
        return out[:n.value]

    def debug_octree(self, i: int, level: int, cap: int = 1 << 14):
        out = np.zeros(cap, KP_DTYPE)
        n = C.c_int(0)
        check(self.lib.odo_debug_octree(self.h, i, level, ptr(out), cap, C.byref(n)))
        return out[:n.value]

    def adaptive_state(self, i: int = None):
        """(FAST threshold per grid cell used for frame i of the last batch or
        None, current per-cell DetectorAdjuster thresholds)."""
        nc = self.cfg.adaptive.grid_rows * self.cfg.adaptive.grid_cols
        t = np.zeros(nc, np.int32)
        th = np.zeros(nc, np.float64)
        rc = self.lib.odo_debug_adaptive(self.h, -1 if i is None else i, None if i is None else ptr(t), ptr(th))
        if rc < 0:
            check(rc)
        return (None if i is None else t), th

    def set_adaptive_thresholds(self, th):
        th = np.ascontiguousarray(th, np.float64)
        check(self.lib.odo_set_adaptive_thresholds(self.h, ptr(th), th.size))

    def select(self, keys, nth: int, mode: int = 0):
        """GPU std::nth_element (mode 0) / retainBest (mode 1) on packed keys."""
        keys = np.ascontiguousarray(keys, np.uint32)
        out = np.zeros_like(keys)
        n = C.c_int(0)
        check(self.lib.odo_debug_select(self.h, ptr(keys), keys.size, nth, mode, ptr(out), C.byref(n)))
        return out, n.value

    def pnp_ransac(self, Xw, uv, calib=None, iterations: int = 500, reproj_err: float = 3.0,
                   confidence: float = 0.85):
        """PnPRansac::Compute (pnpransac.cpp:11-51) on the GPU: cv::solvePnPRansac
        over n landmark observations. Returns (result, inlier mask, per-hypothesis
        inlier counts)."""
        Xw = np.ascontiguousarray(Xw, np.float32).reshape(-1, 3)
        uv = np.ascontiguousarray(uv, np.float32).reshape(-1, 2)
        n = Xw.shape[0]
        res = PnPRansacResult()
        mask = np.zeros(max(n, 1), np.uint8)
        good = np.zeros(max(iterations, 1), np.int32)
        cal = calib if calib is not None else self.cfg.calib
        check(self.lib.odo_pnp_ransac(self.h, ptr(Xw), ptr(uv), n, ptr(cal), iterations, reproj_err, confidence,
                                      ptr(res), ptr(mask), ptr(good)))
        return res, mask[:n].astype(bool), good

    def pnp_ransac_batch(self, problems, calib=None, iterations: int = 500, reproj_err: float = 3.0,
                         confidence: float = 0.85):
        """PnPRansac::Compute for a list of (Xw n x 3, uv n x 2) problems in one
        launch chain. Returns (results[nprob], list of inlier masks)."""
        sizes = [len(x) for x, _ in problems]
        offs = np.zeros(len(problems) + 1, np.int32)
        offs[1:] = np.cumsum(sizes)
        Xw = np.ascontiguousarray(np.concatenate([np.asarray(x, np.float32).reshape(-1, 3) for x, _ in problems])
                                  if problems else np.zeros((0, 3), np.float32))
        uv = np.ascontiguousarray(np.concatenate([np.asarray(u, np.float32).reshape(-1, 2) for _, u in problems])
                                  if problems else np.zeros((0, 2), np.float32))
        res = (PnPRansacResult * max(len(problems), 1))()
        mask = np.zeros(max(int(offs[-1]), 1), np.uint8)
        cal = calib if calib is not None else self.cfg.calib
        check(self.lib.odo_pnp_ransac_batch(self.h, ptr(Xw), ptr(uv), ptr(offs), len(problems), ptr(cal), iterations,
                                            reproj_err, confidence, C.cast(res, C.c_void_p), ptr(mask)))
        return [res[i] for i in range(len(problems))], [mask[offs[i]:offs[i + 1]].astype(bool)
                                                         for i in range(len(problems))]

    def gicp(self, src, tgt, guess=None, max_iterations: int = 10, max_corr_dist: float = 0.07):
        """GeneralizedICP(max_iterations, max_corr_dist)::Compute(source, target,
        guess) (generalizedicp.cpp:30-39, 65-89) on the GPU. Returns
        (T12 4x4, converged, iterations, n_corr)."""
        src = np.ascontiguousarray(src, np.float32).reshape(-1, 3)
        tgt = np.ascontiguousarray(tgt, np.float32).reshape(-1, 3)
        g = np.ascontiguousarray(np.eye(4, dtype=np.float32) if guess is None else guess, np.float32)
        T = np.zeros(16, np.float32)
        conv, it, nc = C.c_int(), C.c_int(), C.c_int()
        check(self.lib.odo_gicp(self.h, ptr(src), src.shape[0], ptr(tgt), tgt.shape[0], ptr(g), max_iterations,
                                max_corr_dist, ptr(T), C.byref(conv), C.byref(it), C.byref(nc)))
        return T.reshape(4, 4), conv.value, it.value, nc.value

    def gicp_batch(self, pairs, max_iterations: int = 10, max_corr_dist: float = 0.07):
        """GeneralizedICP::Compute for a list of (src n x 3, tgt m x 3, guess 4x4 or
        None) in one launch chain. Returns a list of (T12, converged, iterations,
        n_corr)."""
        P = len(pairs)
        so = np.zeros(P + 1, np.int32)
        to = np.zeros(P + 1, np.int32)
        so[1:] = np.cumsum([len(s) for s, _, _ in pairs])
        to[1:] = np.cumsum([len(t) for _, t, _ in pairs])
        cat = lambda xs: np.ascontiguousarray(np.concatenate([np.asarray(x, np.float32).reshape(-1, 3) for x in xs])
                                              if xs else np.zeros((0, 3), np.float32))
        src, tgt = cat([s for s, _, _ in pairs]), cat([t for _, t, _ in pairs])
        g = np.ascontiguousarray(np.stack([np.eye(4, dtype=np.float32) if q is None else np.asarray(q, np.float32)
                                           for _, _, q in pairs]) if P else np.zeros((1, 4, 4), np.float32))
        T = np.zeros((max(P, 1), 16), np.float32)
        conv, it, nc = (np.zeros(max(P, 1), np.int32) for _ in range(3))
        check(self.lib.odo_gicp_batch(self.h, ptr(src), ptr(so), ptr(tgt), ptr(to), ptr(g), P, max_iterations,
                                      max_corr_dist, ptr(T), ptr(conv), ptr(it), ptr(nc)))
        return [(T[p].reshape(4, 4), int(conv[p]), int(it[p]), int(nc[p])) for p in range(P)]

    def timings(self):
        ms = np.zeros(16, np.float32)
        names = (C.c_char_p * 16)()
        n = self.lib.odo_last_timings(self.h, ptr(ms), 16, C.cast(names, C.c_void_p))
        return {names[i].decode(): float(ms[i]) for i in range(n)}


def rng_stream(seed: int, n: int) -> np.ndarray:
    """glibc rand() stream as restated by the library (host helper)."""
    r = Rng()
    L = load()
    L.odo_rng_seed(ptr(r), seed)
    return np.array([L.odo_rng_next(ptr(r)) for _ in range(n)], np.int32)


def pair_seed(base: int, pair: int) -> int:
    """Per-pair RANSAC seed of the batched contract: splitmix64(base ^ pair), low 32 bits."""
    m = (1 << 64) - 1
    z = ((base ^ pair) + 0x9E3779B97F4A7C15) & m
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & m
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & m
    z ^= z >> 31
    return z & 0xFFFFFFFF


def kabsch(A: np.ndarray, B: np.ndarray) -> np.ndarray:
    A = np.ascontiguousarray(A, np.float32)
    B = np.ascontiguousarray(B, np.float32)
    T = np.zeros(16, np.float32)
    check(load().odo_kabsch(ptr(A), ptr(B), A.shape[0], ptr(T)))
    return T.reshape(4, 4)
