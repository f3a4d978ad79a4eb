"""GPU parity of the ADAPTIVE extractor: Extractor(FAST, ORB,
ADAPTIVE) through the C-ABI against the oracle's restatement of
extractor.cpp:39-77 + videogridadaptedfeaturedetector.cpp +
videodynamicadaptedfeaturedetector.cpp + detectoradjuster.cpp.

Bit-exact: keypoints (coordinates, response, order), descriptors, undistorted
points, xyz, uR, the FAST threshold every cell used on every frame, the
persistent per-cell thresholds after each batch, and the selection
permutations (std::nth_element / retainBest) on arbitrary inputs.
"""
import numpy as np
import pytest

import oracle_lib as O
from conftest import load_pkg, sequence

pytestmark = pytest.mark.gpu


def make(pkg, n, w=640, h=480, iters=200, seed=0x5EED000A):
    cfg = pkg.default_config(w, h, n, nfeatures=1000, iterations=iters, seed=seed,
                             detector=pkg.DETECTOR_ADAPTIVE_FAST)
    return pkg.Odometry(cfg), cfg


def cal_of(cfg):
    k = cfg.calib
    return O.Calib(k.fx, k.fy, k.cx, k.cy, k.k1, k.k2, k.p1, k.p2, k.k3, k.depth_factor, k.mbf, k.th_depth)


def assert_frame(got, ref, tag):
    assert len(got["kps"]) == len(ref["kps"]), f"{tag}: N {len(got['kps'])} vs {len(ref['kps'])}"
    for fld in ref["kps"].dtype.names:
        bad = np.nonzero(got["kps"][fld] != ref["kps"][fld])[0]
        assert bad.size == 0, (f"{tag}: kp.{fld} differs at {bad[:8]}: gpu {got['kps'][bad[:4]]} "
                               f"ref {ref['kps'][bad[:4]]}")
    bad = np.nonzero((got["desc"] != ref["desc"]).any(1))[0]
    assert bad.size == 0, f"{tag}: descriptors differ at {bad[:10]}"
    for f in ("kun", "xyz", "ur"):
        assert np.array_equal(got[f], ref[f]), f"{tag}: {f}"


@pytest.mark.parametrize("n,nth", [(1, 0), (4, 2), (5, 3), (114, 113), (300, 113), (1017, 113), (3000, 113),
                                   (9000, 113), (1017, 1000), (2000, 1999)])
@pytest.mark.parametrize("levels", [3, 40, 250])
def test_select_is_nth_element(n, nth, levels):
    pkg = load_pkg()
    odo, _ = make(pkg, 1)
    rng = np.random.default_rng(n * 7 + levels)
    score = rng.integers(3, 3 + levels, n).astype(np.uint32)
    keys = (score << 24) | (rng.integers(0, 480, n).astype(np.uint32) << 12) | rng.integers(0, 640, n).astype(np.uint32)
    if n > 100:  # sorted and reversed runs stress the median-of-3 pivots
        k = n // 3
        keys[:k] = np.sort(keys[:k])
        keys[k:2 * k] = np.sort(keys[k:2 * k])[::-1]
    ref = keys.copy()
    O.lib().oracle_nth_element_score(O.ptr(ref), n, nth)
    got, m = odo.select(keys, nth, 0)
    assert m == n and np.array_equal(got, ref), "nth_element permutation differs"
    if nth >= 1:
        ref2 = keys.copy()
        m2 = O.lib().oracle_retain_best_score(O.ptr(ref2), n, nth)
        got2, g2 = odo.select(keys, nth, 1)
        exp_m = m2 if n > nth else n
        assert g2 == exp_m and np.array_equal(got2[:g2], ref2[:exp_m]), "retainBest differs"
    odo.close()


def test_adaptive_batches_match_oracle():
    """Two batches (6 + 3 frames): frames, per-cell thresholds used on every
    frame, the persistent thresholds, and the tracked pairs."""
    pkg = load_pkg()
    bgr, dep, _ = sequence(9, seed=0x5EED000A)
    odo, cfg = make(pkg, 6, iters=300)
    cal = cal_of(cfg)
    ex = O.AdaptiveExtractor()
    frames, t_ref = [], []
    for i in range(9):
        img = O.gray(bgr[i])
        before = ex.thresh.copy()
        k, d, t = ex.extract_gray(img)
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


def test_adaptive_noise_frames_retain_best_and_big_cells():
    """Noise frames: every cell is 'too many' (thousands of FAST corners at
    the start threshold, beyond the LDS selection capacity), all nine cells
    keep 113, and retainBest(1000) trims the 1017 with its boundary ties."""
    pkg = load_pkg()
    rng = np.random.default_rng(3)
    n = 3
    bgr = rng.integers(0, 256, (n, 480, 640, 3), dtype=np.uint8)
    dep = rng.integers(2000, 20000, (n, 480, 640)).astype(np.uint16)
    odo, cfg = make(pkg, n)
    cal = cal_of(cfg)
    ex = O.AdaptiveExtractor()
    start = np.array([2.0, 3.0, 5.0, 20.0, 2.0, 9.5, 2.0, 40.0, 2.0])
    ex.thresh[:] = start
    odo.set_adaptive_thresholds(start)
    frames = [ex.extract_frame(bgr[i], dep[i], cal) for i in range(n)]
    odo.track_batch_host(bgr, dep)
    for i in range(n):
        assert_frame(odo.frame(i), frames[i], f"noise frame {i}")
    _, th = odo.adaptive_state()
    assert np.array_equal(th, ex.thresh)
    odo.close()


def test_adaptive_extract_entry_point_advances_state():
    pkg = load_pkg()
    bgr, dep, _ = sequence(3, seed=0x5EED000B)
    odo, cfg = make(pkg, 1)
    cal = cal_of(cfg)
    ex = O.AdaptiveExtractor()
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
    odo.reset()
    _, th = odo.adaptive_state()
    assert np.all(th == cfg.adaptive.init_thresh)
    odo.close()
