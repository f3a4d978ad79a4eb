"""Edge cases of the hot path (SURVEY §8 parity bar: empty and ragged inputs):
uniform frames (no FAST corner anywhere: N = 0), frames without depth (no
landmarks, no matches), a textured frame next to a blank one (N2 = 0), half
blank frames (some pyramid levels empty), and the ADAPTIVE detector on blank
frames (every cell too few: thresholds fall to the minimum). The GPU batched
path against the oracle, bit-exact as elsewhere. The reference itself would
index knnMatch's second neighbour out of bounds when F2 has < 2 descriptors
(matcher.cpp:64); here (and in the oracle) an absent neighbour is (-1, INT_MAX)."""
import numpy as np
import pytest

import oracle_lib as O
from conftest import load_pkg, sequence


def _frames():
    bgr, dep, _ = sequence(4, seed=0x5EED000C)
    bgr = bgr.copy()
    dep = dep.copy()
    bgr[1] = 128                      # uniform: N = 0
    dep[2] = 0                        # no depth: no landmark, no xyz
    bgr[3, :, 320:] = 0               # half blank
    return bgr, dep


def _oracle(bgr, dep, nf=1000, iters=200, seed_base=0x5EED0000, pkg=None):
    cal = O.fr1_calib()
    fr = [O.extract_frame(bgr[i], dep[i], O.orb_params(nf), cal) for i in range(len(bgr))]
    out, latch = [], float("nan")
    for p in range(1, len(bgr)):
        r, mask, matches, latch = O.track_pair(fr[p - 1], fr[p], cal, O.ransac_params(iters),
                                               pkg.pair_seed(seed_base, p), latch)
        out.append((r, matches))
    return fr, out


def test_oracle_handles_empty_frames():
    pkg = load_pkg()
    bgr, dep = _frames()
    fr, out = _oracle(bgr, dep, pkg=pkg)
    assert len(fr[1]["kps"]) == 0 and len(fr[0]["kps"]) > 500
    assert np.all(fr[2]["xyz"] == 0)
    for r, m in out[:2]:  # pairs touching the blank frame / the depthless frame
        assert r.n_matches == 0 and r.ransac_ok == 0


@pytest.mark.gpu
def test_gpu_empty_and_ragged_frames():
    pkg = load_pkg()
    bgr, dep = _frames()
    fr, out = _oracle(bgr, dep, pkg=pkg)
    odo = pkg.Odometry(pkg.default_config(640, 480, 4, nfeatures=1000, iterations=200))
    res = odo.track_batch_host(bgr, dep)
    for i in range(4):
        g = odo.frame(i)
        assert len(g["kps"]) == len(fr[i]["kps"]), f"frame {i}: N"
        assert np.array_equal(g["kps"], fr[i]["kps"]) and np.array_equal(g["desc"], fr[i]["desc"])
        assert np.array_equal(g["xyz"], fr[i]["xyz"])
    for p in range(1, 4):
        r, matches = out[p - 1]
        assert np.array_equal(odo.pair(p)["matches"], matches), f"pair {p}: matches"
        assert (res[p]["n_matches"], res[p]["n_good"], res[p]["ransac_ok"], res[p]["n_inliers"], res[p]["visited"]) \
            == (r.n_matches, r.n_good, r.ransac_ok, r.n_inliers, r.visited), f"pair {p}: counts"
        O.check_ransac_inliers(odo.pair(p), r, f"pair {p}")
        assert np.array_equal(res[p]["T12"], np.array(r.T12, np.float32)), f"pair {p}: T12"
        assert np.abs(res[p]["Tcw"] - np.array(r.Tcw, np.float32)).max() < 1e-4, f"pair {p}: Tcw"
    # the next batch starts from the half-blank frame
    res2 = odo.track_batch_host(bgr[:2], dep[:2])
    assert res2[1]["n_matches"] == 0
    odo.close()


@pytest.mark.gpu
def test_gpu_adaptive_blank_frames():
    pkg = load_pkg()
    bgr, dep = _frames()
    bgr = bgr[[1, 1, 0]]
    dep = dep[[1, 1, 0]]
    ex = O.AdaptiveExtractor()
    cal = O.fr1_calib()
    ref = [ex.extract_frame(bgr[i], dep[i], cal) for i in range(3)]
    cfg = pkg.default_config(640, 480, 3, nfeatures=1000, detector=pkg.DETECTOR_ADAPTIVE_FAST)
    odo = pkg.Odometry(cfg)
    odo.track_batch_host(bgr, dep)
    for i in range(3):
        g = odo.frame(i)
        assert np.array_equal(g["kps"], ref[i]["kps"]) and np.array_equal(g["desc"], ref[i]["desc"]), f"frame {i}"
    _, th = odo.adaptive_state()
    assert np.array_equal(th, ex.thresh)
    odo.close()


@pytest.mark.gpu
def test_gpu_knn_degenerate_sizes():
    pkg = load_pkg()
    odo = pkg.Odometry(pkg.default_config(640, 480, 1))
    lib = pkg.load()
    rng = np.random.default_rng(3)
    for nq, nt in ((0, 5), (5, 0), (7, 1), (1, 2), (300, 1)):
        q = rng.integers(0, 256, (max(nq, 1), 32), dtype=np.uint8)
        t = rng.integers(0, 256, (max(nt, 1), 32), dtype=np.uint8)
        ri = np.zeros((max(nq, 1), 2), np.int32)
        rd = np.zeros((max(nq, 1), 2), np.int32)
        if nq:
            O.lib().oracle_knn2(O.ptr(q), nq, O.ptr(t), nt, O.ptr(ri), O.ptr(rd))
        gi = np.zeros_like(ri)
        gd = np.zeros_like(rd)
        pkg.check(lib.odo_knn2_hamming(odo.h, pkg.ptr(q), nq, pkg.ptr(t), nt, pkg.ptr(gi), pkg.ptr(gd)))
        assert np.array_equal(gi[:nq], ri[:nq]) and np.array_equal(gd[:nq], rd[:nq]), (nq, nt)
    odo.close()


@pytest.mark.gpu
@pytest.mark.parametrize("scale", [2.0, 4.0])
def test_gpu_far_scenes_vo_landmark_sort_path(scale):
    """Scenes pushed beyond Calibration::mThDepth: fewer than 100 keypoints
    within it, so UpdateLastFrame takes the 101 nearest (k_vo_lm's sort
    path) and kNN-2 runs on those queries only. Landmark counts, matches and
    poses against the oracle."""
    pkg = load_pkg()
    bgr, dep, _ = sequence(3, seed=0x5EED0042)
    dep = np.clip(dep.astype(np.float64) * scale, 0, 65535).astype(np.uint16)
    cal = O.fr1_calib()
    fr = [O.extract_frame(bgr[i], dep[i], O.orb_params(1000), cal) for i in range(3)]
    cfg = pkg.default_config(640, 480, 3, nfeatures=1000, iterations=200)
    odo = pkg.Odometry(cfg)
    res = odo.track_batch_host(bgr, dep)
    latch = float("nan")
    for p in range(1, 3):
        r, _, matches, latch = O.track_pair(fr[p - 1], fr[p], cal, O.ransac_params(200),
                                            pkg.pair_seed(cfg.seed, p), latch)
        th = cal.mbf * cal.th_depth / cal.fx
        z = fr[p - 1]["xyz"][:, 2]
        assert np.count_nonzero((z > 0) & (z <= th)) < 100 or scale == 2.0
        assert res[p]["n_queries"] == r.n_queries, f"pair {p}: VO landmarks"
        assert np.array_equal(odo.pair(p)["matches"], matches), f"pair {p}: matches"
        assert np.array_equal(res[p]["T12"], np.array(r.T12, np.float32)), f"pair {p}: T12"
        assert np.abs(res[p]["Tcw"] - np.array(r.Tcw, np.float32)).max() < 1e-4, f"pair {p}: Tcw"
    odo.close()
