"""GPU parity of the ADAPTIVE extractor with the cv::ORB inner detector
(SURVEY §8(f) rank 2): Extractor(ORB, ORB, ADAPTIVE) through the C-ABI
against the oracle's restatement of detectoradjuster.cpp:29 (cv::ORB(10000,
1.2, 8, 15, 0, 2, HARRIS, 31, t)::detect per grid cell), the grid / dynamic
adapted detectors, Extract's retainBest(1000) and cv::ORB::compute with the
detector's octaves (extractor.cpp:39-50).

Bit-exact: keypoints (coordinates, size, angle, Harris response, octave,
order), descriptors, undistorted points, xyz, uR, the threshold every cell
used on every frame and the persistent thresholds; the tracked pairs as in
test_adaptive_gpu.py. OpenCV's ORB internals are restated, not linked, so
parity with the real library is unpinned.
"""
import numpy as np
import pytest

import oracle_lib as O
from conftest import load_pkg, sequence
from test_adaptive_gpu import assert_frame, cal_of

pytestmark = pytest.mark.gpu


def make(pkg, n, w=640, h=480, iters=200, seed=0x5EED000C):
    cfg = pkg.default_config(w, h, n, nfeatures=1000, iterations=iters, seed=seed,
                             detector=pkg.DETECTOR_ADAPTIVE_ORB)
    return pkg.Odometry(cfg), cfg


def test_adaptive_orb_batches_match_oracle():
    """Two batches (6 + 3 frames): frames, per-cell thresholds, persistent
    thresholds, tracked pairs."""
    pkg = load_pkg()
    bgr, dep, _ = sequence(9, seed=0x5EED000C)
    odo, cfg = make(pkg, 6, iters=300)
    cal = cal_of(cfg)
    ex = O.AdaptiveExtractor(inner="orb")
    frames, t_ref = [], []
    for i in range(9):
        img = O.gray(bgr[i])
        before = ex.thresh.copy()
        _, _, t = ex.extract_gray(img)
        ex.thresh[:] = before
        frames.append(ex.extract_frame(bgr[i], dep[i], cal))
        t_ref.append(t)
    res_a = odo.track_batch_host(bgr[:6], dep[:6])
    lists = [odo.pair(i) for i in range(6)]
    for i in range(6):
        t_used, _ = odo.adaptive_state(i)
        assert np.array_equal(t_used, t_ref[i]), f"frame {i}: cell thresholds {t_used} vs {t_ref[i]}"
        assert_frame(odo.frame(i), frames[i], f"frame {i}")
    res_b = odo.track_batch_host(bgr[6:], dep[6:])
    lists += [odo.pair(i) for i in range(3)]
    for i in range(3):
        t_used, th = odo.adaptive_state(i)
        assert np.array_equal(t_used, t_ref[6 + i]), f"frame {6 + i}: cell thresholds"
        assert_frame(odo.frame(i), frames[6 + i], f"frame {6 + i}")
    assert np.array_equal(th, ex.thresh), "persistent thresholds differ"
    rp = O.ransac_params(300)
    latch = float("nan")
    res = list(res_a) + list(res_b)
    for p in range(1, 9):
        r, mask, matches, latch = O.track_pair(frames[p - 1], frames[p], cal, rp, pkg.pair_seed(cfg.seed, p), latch)
        g = res[p]
        assert (g["n_matches"], g["n_good"], g["visited"], g["n_inliers"]) == \
            (r.n_matches, r.n_good, r.visited, r.n_inliers), f"pair {p}: counts"
        O.check_ransac_inliers(lists[p], r, f"pair {p}")
        assert np.array_equal(g["T12"], np.array(r.T12, np.float32)), f"pair {p}: T12"
        assert np.abs(g["Tcw"] - np.array(r.Tcw, np.float32)).max() < 1e-4, f"pair {p}: PnP pose"
    odo.close()


def test_adaptive_orb_noise_frames_bind_every_selection():
    """Noise frames at low start thresholds: per-level retainBest by FAST
    score (2 * quota) and by Harris response (quota) bind, every cell is 'too
    many' and keeps 113 by |response|, retainBest(1000) trims the 1017."""
    pkg = load_pkg()
    rng = np.random.default_rng(5)
    n = 3
    bgr = rng.integers(0, 256, (n, 480, 640, 3), dtype=np.uint8)
    dep = rng.integers(2000, 20000, (n, 480, 640)).astype(np.uint16)
    odo, cfg = make(pkg, n)
    cal = cal_of(cfg)
    ex = O.AdaptiveExtractor(inner="orb")
    start = np.array([2.0, 3.0, 5.0, 20.0, 2.0, 9.5, 2.0, 40.0, 2.0])
    ex.thresh[:] = start
    odo.set_adaptive_thresholds(start)
    frames = [ex.extract_frame(bgr[i], dep[i], cal) for i in range(n)]
    odo.track_batch_host(bgr, dep)
    for i in range(n):
        assert_frame(odo.frame(i), frames[i], f"noise frame {i}")
        assert len(frames[i]["kps"]) > 0
    _, th = odo.adaptive_state()
    assert np.array_equal(th, ex.thresh)
    odo.close()


@pytest.mark.parametrize("w,h", [(640, 480), (320, 240)])
def test_adaptive_orb_extract_entry_point(w, h):
    """odo_extract (one frame per call) advances the cell thresholds exactly
    as the oracle; a 320x240 image exercises small cell levels (level 7 of a
    cell is 28 px high: runByImageBorder(15) drops the whole level)."""
    pkg = load_pkg()
    bgr, dep, _ = sequence(3, w=w, h=h, seed=0x5EED000D)
    odo, cfg = make(pkg, 1, w=w, h=h)
    cal = cal_of(cfg)
    ex = O.AdaptiveExtractor(inner="orb")
    lib = pkg.load()
    cap = 1100
    for i in range(3):
        ref = ex.extract_frame(bgr[i], dep[i], cal)
        kps = np.zeros(cap, pkg.KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        kun = np.zeros((cap, 2), np.float32)
        xyz = np.zeros((cap, 3), np.float32)
        ur = np.zeros(cap, np.float32)
        nn = O.C.c_int(0)
        pkg.check(lib.odo_extract(odo.h, pkg.ptr(np.ascontiguousarray(bgr[i])), 3,
                                  pkg.ptr(np.ascontiguousarray(dep[i])), pkg.ptr(kps), pkg.ptr(desc), pkg.ptr(kun),
                                  pkg.ptr(xyz), pkg.ptr(ur), cap, O.C.byref(nn)))
        m = nn.value
        assert_frame(dict(kps=kps[:m], desc=desc[:m], kun=kun[:m], xyz=xyz[:m], ur=ur[:m]), ref, f"call {i}")
    odo.close()
