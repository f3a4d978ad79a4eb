"""CPU checks of the oracle's cv::ORB restatement (the ADAPTIVE extractor's
ORB inner detector, detectoradjuster.cpp:29; OpenCV 3.4 orb.cpp): Harris
responses against an independent numpy transcription, the pyramid sizes /
getScale / nfeaturesPerLevel tables, the level-0 keypoints against plain FAST
+ runByImageBorder, and the grid detector's invariants. Parity with the real
OpenCV is unpinned (the library is not in the image)."""
import numpy as np
import pytest

import oracle_lib as O


def harris_np(img, x0, y0):
    """HarrisResponses (orb.cpp) for one point: 7x7 block, integer sums, float32."""
    im = img.astype(np.int64)
    a = b = c = 0
    for y in range(y0 - 3, y0 + 4):
        for x in range(x0 - 3, x0 + 4):
            ix = (im[y, x + 1] - im[y, x - 1]) * 2 + (im[y - 1, x + 1] - im[y - 1, x - 1]) + \
                 (im[y + 1, x + 1] - im[y + 1, x - 1])
            iy = (im[y + 1, x] - im[y - 1, x]) * 2 + (im[y + 1, x - 1] - im[y - 1, x - 1]) + \
                 (im[y + 1, x + 1] - im[y - 1, x + 1])
            a += ix * ix
            b += iy * iy
            c += ix * iy
    f = np.float32
    scale = f(1.0) / f(4 * 7 * f(255.0))
    ssq = scale * scale * scale * scale
    fa, fb, fc = f(a), f(b), f(c)
    return (fa * fb - fc * fc - f(0.04) * (fa + fb) * (fa + fb)) * ssq


def test_harris_matches_numpy():
    rng = np.random.default_rng(1)
    img = rng.integers(0, 256, (60, 70), dtype=np.uint8)
    img[20:40, 30:50] = 255  # a corner-rich block
    for (x, y) in [(10, 10), (30, 20), (49, 39), (35, 25), (60, 50), (5, 5)]:
        got = O.lib().oracle_harris(O.ptr(img), 70, 60, x, y)
        assert np.float32(got) == harris_np(img, x, y), (x, y)


def test_orbcv_tables():
    lw, lh = np.zeros(8, np.int32), np.zeros(8, np.int32)
    sc, q = np.zeros(8, np.float32), np.zeros(8, np.int32)
    O.lib().oracle_orbcv_levels(640, 480, O.ptr(lw), O.ptr(lh), O.ptr(sc), O.ptr(q))
    s = np.array([np.float32(np.float64(np.float32(1.2)) ** l) for l in range(8)], np.float32)
    assert np.array_equal(sc, s)
    inv = (np.float32(1) / s).astype(np.float32)
    assert np.array_equal(lw, np.rint(np.float32(640) * inv).astype(np.int32))
    assert np.array_equal(lh, np.rint(np.float32(480) * inv).astype(np.int32))
    # the frame pyramid of the ORB_SLAM2 extractor has the same sizes at 640x480
    assert list(lw) == [640, 533, 444, 370, 309, 257, 214, 179]
    assert list(lh) == [480, 400, 333, 278, 231, 193, 161, 134]
    assert q.sum() == 10000 and q.min() > 113  # the GPU chain's exactness bound


def test_orbcv_level0_is_fast_inside_the_border():
    """With no level binding, cv::ORB's level-0 keypoints are FAST(t)'s in
    emission order, minus runByImageBorder(15), with Harris responses."""
    rng = np.random.default_rng(2)
    img = (rng.integers(0, 2, (12, 16)) * 200 + 20).astype(np.uint8).repeat(16, 0).repeat(16, 1)  # 192 x 256 blocks
    img = np.ascontiguousarray(img)
    h, w = img.shape
    cap = 20000
    kp = np.zeros(cap, O.KP_DTYPE)
    n = O.lib().oracle_orbcv_detect(O.ptr(img), w, h, w, 20, O.ptr(kp), cap)
    kp = kp[:n]
    assert n > 0 and np.all(np.diff(kp["octave"]) >= 0), "level-major order"
    l0 = kp[kp["octave"] == 0]
    fk = np.zeros(cap, O.KP_DTYPE)
    m = O.lib().oracle_fast_roi(O.ptr(img), w, h, w, 20, O.ptr(fk), cap)
    fk = fk[:m]
    inside = (fk["x"] >= 15) & (fk["x"] < w - 15) & (fk["y"] >= 15) & (fk["y"] < h - 15)
    fk = fk[inside]
    assert len(fk) < 2172
    assert np.array_equal(l0["x"], fk["x"]) and np.array_equal(l0["y"], fk["y"])
    for k in l0[:40]:
        assert np.float32(k["response"]) == harris_np(img, int(k["x"]), int(k["y"]))
    for l in range(8):
        sl = np.float32(np.float64(np.float32(1.2)) ** l)
        assert np.all(kp[kp["octave"] == l]["size"] == np.float32(31) * sl)


def test_adaptive_orb_grid_invariants():
    """Grid detector + retainBest(1000) + cv::ORB::compute: at most 1000
    keypoints, octave-major, inside the 31-px border, thresholds persist."""
    from conftest import sequence
    bgr, dep, _ = sequence(3, seed=0x5EED000C)
    ex = O.AdaptiveExtractor(inner="orb")
    for i in range(3):
        k, d, t = ex.extract_gray(O.gray(bgr[i]))
        assert 0 < len(k) <= 1000
        assert np.all(np.diff(k["octave"]) >= 0)
        assert np.all((k["x"] >= 31) & (k["x"] < 640 - 31) & (k["y"] >= 31) & (k["y"] < 480 - 31))
        assert np.all((t >= 2) & (t <= 255))
    assert np.all(ex.thresh >= 2) and np.all(ex.thresh <= 10000)
