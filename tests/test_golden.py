"""Committed golden fixtures (tests/golden/*.npz, made by make_golden.py).

CPU: the oracle reproduces every fixture (a regression pin on the checker),
and the kNN-2 fixture is cross-checked by an independent numpy brute force.
GPU (-m gpu): the HIP path, called through the C-ABI, reproduces the same
fixtures: descriptors, keypoints, kNN-2 arrays, match lists, RANSAC counts,
T12 and rmse bit-exactly, the PnP pose within 1e-4 (inlier flags within 2).
"""
import os
import sys
import zlib

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
sys.path.insert(0, GOLD)
from conftest import load_pkg  # noqa: E402
import oracle_lib as O  # noqa: E402
import make_golden as MG  # noqa: E402


def load(name):
    return np.load(os.path.join(GOLD, name))  # allow_pickle=False (default)


@pytest.fixture(scope="module")
def inputs():
    bgr, dep, crc = MG.golden_inputs()
    gold = load("frames_640x480_2000.npz")
    assert list(gold["input_crc32"]) == crc, "synthetic generator drifted from the committed fixtures"
    return bgr, dep


def _frame_equal(got, gold, i):
    for f in ("x", "y", "size", "angle", "response", "octave"):
        assert np.array_equal(got["kps"][f], gold[f"f{i}_kps"][f]), f"frame {i}: kp.{f}"
    assert np.array_equal(got["desc"], gold[f"f{i}_desc"]), f"frame {i}: descriptors"
    for k in ("kun", "xyz", "ur"):
        assert np.array_equal(got[k], gold[f"f{i}_{k}"]), f"frame {i}: {k}"


# ------------------------------------------------------------------ CPU
def test_oracle_reproduces_frame_fixture(inputs):
    bgr, dep = inputs
    gold = load("frames_640x480_2000.npz")
    for i in range(2):
        _frame_equal(O.extract_frame(bgr[i], dep[i], O.orb_params(MG.NF), O.fr1_calib()), gold, i)


def _knn2_numpy(q, t):
    """Independent brute force: popcount of xor, BFMatcher top-2 (ties keep the lower train index)."""
    x = np.unpackbits(q[:, None, :] ^ t[None, :, :], axis=2).sum(2).astype(np.int64)
    key = x * (1 << 20) + np.arange(t.shape[0])[None, :]
    order = np.argsort(key, axis=1, kind="stable")[:, :2]
    d = np.take_along_axis(x, order, 1)
    return order.astype(np.int32), d.astype(np.int32)


@pytest.mark.parametrize("n", [1000, 2000])
def test_knn2_fixture_oracle_and_numpy(n):
    g = load("knn2_hamming.npz")
    q, t = g[f"q{n}"], g[f"t{n}"]
    idx, dist = O.knn2(q, t)
    assert np.array_equal(idx, g[f"idx{n}"]) and np.array_equal(dist, g[f"dist{n}"])
    if n == 1000:  # the numpy cross-check allocates n*n*32 bytes
        ni, nd = _knn2_numpy(q, t)
        assert np.array_equal(ni, g[f"idx{n}"]) and np.array_equal(nd, g[f"dist{n}"])


def test_oracle_reproduces_pair_fixture(inputs):
    gold = load("frames_640x480_2000.npz")
    g = load("pair_ransac_pnp.npz")
    frames = [{k: gold[f"f{i}_{k}"] for k in ("kps", "desc", "kun", "xyz", "ur")} for i in range(2)]
    r, mask, matches, latch = O.track_pair(frames[0], frames[1], O.fr1_calib(), O.ransac_params(int(g["iters"][0])),
                                           int(g["seed"][0]))
    assert np.array_equal(matches, g["matches"])
    assert np.array_equal(r.inliers, g["ransac_inliers"]), "Ransac::mvInliers list"
    assert np.array_equal(mask, g["pnp_inlier_mask"])
    assert np.float32(r.rmse) == g["rmse"][0]
    assert np.array_equal(np.array(r.T12, np.float32), g["T12"])
    assert np.array_equal(np.array(r.Tcw, np.float32), g["Tcw"])
    assert [r.n_matches, r.n_good, r.n_inliers, r.ransac_ok, r.pnp_inliers, r.visited] == list(g["counts"])
    assert latch == g["latch"][0]


# ------------------------------------------------------------------ GPU
@pytest.mark.gpu
def test_hip_reproduces_frame_and_pair_fixtures(inputs):
    bgr, dep = inputs
    pkg = load_pkg()
    gold = load("frames_640x480_2000.npz")
    g = load("pair_ransac_pnp.npz")
    cfg = pkg.default_config(MG.W, MG.H, 2, nfeatures=MG.NF, iterations=int(g["iters"][0]), seed=MG.SEED_BASE)
    odo = pkg.Odometry(cfg)
    res = odo.track_batch_host(bgr, dep)
    for i in range(2):
        _frame_equal(odo.frame(i), gold, i)
    p = odo.pair(1)  # pair 1 = (frame 0, frame 1), seed pair_seed(base, 1)
    assert np.array_equal(p["matches"], g["matches"]), "match list"
    got = p["good"][p["ransac_inliers"].astype(bool)]
    assert np.array_equal(got, g["ransac_inliers"]), "RANSAC inlier list (Ransac::mvInliers)"
    assert np.array_equal(res[1]["T12"], g["T12"]), "T12 not bit-exact"
    assert res[1]["rmse"] == g["rmse"][0]
    assert np.abs(res[1]["Tcw"] - g["Tcw"]).max() < 1e-4, "PnP pose"
    # PnP inlier flags: g2o accumulation order is not reproducible (SURVEY §7 hard
    # part 6), so a flag may differ only within the chi2 margin of its threshold
    n2 = len(g["pnp_inlier_mask"])
    fr = [{k: gold[f"f{i}_{k}"] for k in ("kps", "desc", "kun", "xyz", "ur")} for i in range(2)]
    O.check_pnp_flags(p["pnp_inliers"][:n2], g["pnp_inlier_mask"], fr[0], fr[1], p["f2_src"][:n2],
                      g["Tcw"].reshape(4, 4), O.fr1_calib(), "golden pair")
    c = g["counts"]
    assert (res[1]["n_matches"], res[1]["n_good"], res[1]["n_inliers"], res[1]["visited"]) == (c[0], c[1], c[2], c[5])
    assert odo.latch == g["latch"][0]
    odo.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1000, 2000])
def test_hip_knn2_fixture(n):
    pkg = load_pkg()
    g = load("knn2_hamming.npz")
    odo = pkg.Odometry(pkg.default_config(640, 480, 1))
    q, t = g[f"q{n}"], g[f"t{n}"]
    idx = np.zeros((n, 2), np.int32)
    dist = np.zeros((n, 2), np.int32)
    pkg.check(pkg.load().odo_knn2_hamming(odo.h, pkg.ptr(q), n, pkg.ptr(t), n, pkg.ptr(idx), pkg.ptr(dist)))
    assert np.array_equal(idx, g[f"idx{n}"]) and np.array_equal(dist, g[f"dist{n}"])
    odo.close()
