"""CPU checks of the decomposition the GPU ADAPTIVE extractor is built on
(DESIGN.md §4 "ADAPTIVE grid"), against the oracle's literal restatement of
the reference (videogridadaptedfeaturedetector.cpp, videodynamicadapted…,
detectoradjuster.cpp, extractor.cpp:39-77):

* cv::FAST(roi, t, nonmax) == {p in the ROI's detection region : S(p) > t and
  S(p) >= 2 and S(p) > S(q) for every 8-neighbour q inside the region},
  response S(p) - 1,
  where S(p) = max(0, best 9-arc contrast) is threshold-free. So one S map per
  frame gives every threshold's keypoint set and count.
* the per-cell threshold chain (tooFew / tooMany / good) replayed on the
  per-cell count-above-threshold tables reproduces the oracle's thresholds
  frame after frame.
* the single-range parallel Hoare partition model of libstdc++'s introselect
  (what the GPU runs for keepStrongest / retainBest) returns exactly
  std::nth_element's permutation.
"""
import numpy as np
import pytest

import oracle_lib as O
from conftest import sequence

CIRCLE = [(0, 3), (1, 3), (2, 2), (3, 1), (3, 0), (3, -1), (2, -2), (1, -3),
          (0, -3), (-1, -3), (-2, -2), (-3, -1), (-3, 0), (-3, 1), (-2, 2), (-1, 3)]


def s_map(img):
    """S(p) for p in [3,h-3)x[3,w-3), 0 elsewhere (int32)."""
    h, w = img.shape
    v = img[3:h - 3, 3:w - 3].astype(np.int32)
    d = np.stack([v - img[3 + dy:h - 3 + dy, 3 + dx:w - 3 + dx].astype(np.int32) for dx, dy in CIRCLE])
    best = np.zeros_like(v)
    for k in range(16):
        arc = d[[(k + i) % 16 for i in range(9)]]
        best = np.maximum(best, np.maximum(arc.min(0), (-arc).min(0)))
    S = np.zeros((h, w), np.int32)
    S[3:h - 3, 3:w - 3] = best
    return S


def model_fast(S_roi, t):
    """Keypoints of cv::FAST(roi, t, nonmax) from the ROI's S map (row-major)."""
    rows, cols = S_roi.shape
    R = np.zeros_like(S_roi)
    R[3:rows - 3, 3:cols - 3] = S_roi[3:rows - 3, 3:cols - 3]  # detection region only
    P = np.pad(R, 1)
    nb = np.stack([P[1 + dy:1 + dy + rows, 1 + dx:1 + dx + cols] for dy in (-1, 0, 1) for dx in (-1, 0, 1)
                   if dy or dx]).max(0)
    keep = (R > t) & (R >= 2) & (R > nb)  # score S-1 >= 1: a 0 score never passes the NMS
    ys, xs = np.nonzero(keep)
    return xs, ys, R[ys, xs] - 1


def oracle_fast(img, y0, x0, rows, cols, t):
    w = img.shape[1]
    out = np.zeros(1 << 16, O.KP_DTYPE)
    sub = np.ascontiguousarray(img)
    n = O.lib().oracle_fast_roi(O.C.c_void_p(sub.ctypes.data + y0 * w + x0), w, rows, cols, t, O.ptr(out), out.size)
    return out[:n]


@pytest.mark.parametrize("t", [0, 2, 5, 7, 13, 20, 41, 254, 255])
def test_fast_is_thresholded_s_map(t):
    bgr, _, _ = sequence(2)
    img = O.gray(bgr[1])
    S = s_map(img)
    rng = np.random.default_rng(t)
    for _ in range(3):
        rows, cols = int(rng.integers(20, 230)), int(rng.integers(20, 280))
        y0, x0 = int(rng.integers(0, 480 - rows)), int(rng.integers(0, 640 - cols))
        ref = oracle_fast(img, y0, x0, rows, cols, t)
        # S of the full image equals S of the ROI inside the ROI's own detection region
        xs, ys, resp = model_fast(S[y0:y0 + rows, x0:x0 + cols], t)
        assert len(ref) == len(xs), (t, rows, cols)
        assert np.array_equal(ref["x"], xs.astype(np.float32)) and np.array_equal(ref["y"], ys.astype(np.float32))
        assert np.array_equal(ref["response"], resp.astype(np.float32))


def cell_geometry(w, h, p):
    cells = []
    for i in range(p.grid_rows):
        rs, re = max(i * h // p.grid_rows - p.edge_threshold, 0), min(h, (i + 1) * h // p.grid_rows + p.edge_threshold)
        for j in range(p.grid_cols):
            cs, ce = max(j * w // p.grid_cols - p.edge_threshold, 0), min(w, (j + 1) * w // p.grid_cols + p.edge_threshold)
            cells.append((rs, re, cs, ce))
    return cells


def chain_step(thresh, count_above, p):
    """VideoDynamicAdaptedFeatureDetector::detect replayed on count_above[t]."""
    it = p.escape_iters
    while True:
        t = min(max(int(thresh), 0), 255)
        n = int(count_above[t])
        if n < p.cell_min:
            thresh = max(thresh * p.decrease_factor, p.min_thresh)
        elif n > p.cell_max:
            thresh = min(thresh * p.increase_factor, p.max_thresh)
            break
        else:
            break
        it -= 1
        if not (it > 0 and p.min_thresh < thresh < p.max_thresh):
            break
    return thresh, t


def test_threshold_chain_matches_oracle():
    bgr, _, _ = sequence(6)
    ex = O.AdaptiveExtractor()
    p = ex.p
    assert (p.grid_rows, p.grid_cols, p.cell_min, p.cell_max, p.max_total_keypoints) == (3, 3, 67, 113, 1020)
    thresh = np.full(9, p.init_thresh)
    cells = cell_geometry(640, 480, p)
    for f in range(6):
        img = O.gray(bgr[f])
        S = s_map(img)
        _, _, t_ref = ex.extract_gray(img)
        for c, (rs, re, cs, ce) in enumerate(cells):
            xs, ys, resp = model_fast(S[rs:re, cs:ce], 0)
            hist = np.bincount(resp + 1, minlength=257)
            count_above = hist[::-1].cumsum()[::-1]  # count_above[t] = #{S >= t}; need S > t
            above = np.append(count_above[1:], 0)
            thresh[c], t_used = chain_step(thresh[c], above, p)
            assert t_used == t_ref[c], (f, c)
        assert np.array_equal(thresh, ex.thresh), f"frame {f}"


# ---- introselect model (single range per level, parallel Hoare partition)
def introselect_model(a, nth, key):
    a = list(a)
    n = len(a)
    if n == 0 or nth == n:
        return a
    first, last = 0, n
    depth = 2 * (n.bit_length() - 1)
    while last - first > 3:
        if depth == 0:
            raise NotImplementedError("heap_select")  # not reached by these inputs
        depth -= 1
        mid = first + (last - first) // 2
        x, y, z = first + 1, mid, last - 1
        kx, ky, kz = key(a[x]), key(a[y]), key(a[z])
        if kx < ky:
            m = y if ky < kz else (z if kx < kz else x)
        else:
            m = x if kx < kz else (z if ky < kz else y)
        a[first], a[m] = a[m], a[first]
        pk = key(a[first])
        L = [j for j in range(first + 1, last) if key(a[j]) >= pk]
        R = [j for j in range(last - 1, first, -1) if key(a[j]) <= pk]
        ks = sum(1 for k in range(min(len(L), len(R))) if L[k] < R[k])
        for k in range(ks):
            a[L[k]], a[R[k]] = a[R[k]], a[L[k]]
        cut = L[ks] if ks < len(L) else last
        if ks > 0:
            cut = min(cut, R[ks - 1])
        if cut <= nth:
            first = cut
        else:
            last = cut
    for i in range(first + 1, last):  # __insertion_sort
        v = a[i]
        if key(v) < key(a[first]):
            a[first + 1:i + 1] = a[first:i]
            a[first] = v
        else:
            j = i
            while key(v) < key(a[j - 1]):
                a[j] = a[j - 1]
                j -= 1
            a[j] = v
    return a


@pytest.mark.parametrize("seed", range(12))
def test_introselect_model_matches_nth_element(seed):
    rng = np.random.default_rng(seed)
    n = int(rng.choice([4, 5, 17, 114, 200, 1017, 3000]))
    levels = int(rng.choice([2, 5, 30, 250]))
    score = rng.integers(3, 3 + levels, n)
    a = ((score.astype(np.uint32) << 24) | np.arange(n, dtype=np.uint32)).astype(np.uint32)
    nth = int(rng.integers(0, n))
    ref = a.copy()
    O.lib().oracle_nth_element_score(O.ptr(ref), n, nth)
    got = introselect_model(a, nth, key=lambda e: 255 - (int(e) >> 24))
    assert np.array_equal(np.array(got, np.uint32), ref)
