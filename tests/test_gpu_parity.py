"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bit-exact for integer/byte/index work (pyramid, FAST candidates, octree,
blurred levels, keypoints, descriptors, kNN indices and distances, match
lists, std::sort order, RANSAC inlier masks) and for the float/double RANSAC
fit (same operation order); PnP pose within 1e-4 (SURVEY §8 contract) with
inlier flags compared outside a small chi2 margin.
"""
import numpy as np
import pytest

import oracle_lib as O
from conftest import load_pkg, sequence

pytestmark = pytest.mark.gpu

FR1_CAL = dict(fx=517.3, fy=516.5, cx=318.6, cy=255.3)


def make_odo(pkg, w, h, nf, iters, batch, seed=0x5EED0000, calib=None):
    cfg = pkg.default_config(w, h, batch, nfeatures=nf, iterations=iters, seed=seed, calib=calib)
    return pkg.Odometry(cfg), cfg


def oracle_calib(cfg):
    c = cfg.calib
    return O.Calib(c.fx, c.fy, c.cx, c.cy, c.k1, c.k2, c.p1, c.p2, c.k3, c.depth_factor, c.mbf, c.th_depth)


def level_geometry(nf, w, h):
    L = O.lib()
    lw = (O.C.c_int * 8)()
    lh = (O.C.c_int * 8)()
    sc = (O.C.c_float * 8)()
    q = (O.C.c_int * 8)()
    p = O.orb_params(nf)
    L.oracle_level_sizes(O.C.byref(p), w, h, lw, lh, sc, q)
    return list(lw), list(lh), list(q)


def kp_equal(a, b):
    return (np.array_equal(a["x"], b["x"]) and np.array_equal(a["y"], b["y"]) and
            np.array_equal(a["response"], b["response"]))


@pytest.fixture(scope="module")
def cfg2_run():
    """config 2 proxy: 640x480, 2000 kp, RANSAC 500, 4 frames in one batch."""
    pkg = load_pkg()
    bgr, dep, _ = sequence(4)
    odo, cfg = make_odo(pkg, 640, 480, 2000, 500, 4)
    res = odo.track_batch_host(bgr, dep)
    return pkg, odo, cfg, bgr, dep, res


def test_pyramid_and_blur_bit_exact(cfg2_run):
    pkg, odo, cfg, bgr, dep, _ = cfg2_run
    lw, lh, _ = level_geometry(2000, 640, 480)
    total = sum(a * b for a, b in zip(lw, lh))
    gray = O.gray(bgr[0])
    ref = np.zeros(total, np.uint8)
    O.lib().oracle_pyramid(O.ptr(gray), 640, 480, O.C.byref(O.orb_params(2000)), O.ptr(ref))
    got = odo.debug_pyramid(0, total)
    assert got.size == total
    assert np.array_equal(got, ref), f"pyramid mismatch at {np.nonzero(got != ref)[0][:10]}"
    blur = odo.debug_blur(0, total)
    off = 0
    for l in range(8):
        n = lw[l] * lh[l]
        rb = np.zeros(n, np.uint8)
        O.lib().oracle_blur(O.ptr(np.ascontiguousarray(ref[off:off + n])), lw[l], lh[l], O.ptr(rb))
        assert np.array_equal(blur[off:off + n], rb), f"blur level {l}"
        off += n


def test_fast_and_octree_bit_exact(cfg2_run):
    pkg, odo, cfg, bgr, dep, _ = cfg2_run
    lw, lh, quota = level_geometry(2000, 640, 480)
    total = sum(a * b for a, b in zip(lw, lh))
    gray = O.gray(bgr[1])
    pyr = np.zeros(total, np.uint8)
    O.lib().oracle_pyramid(O.ptr(gray), 640, 480, O.C.byref(O.orb_params(2000)), O.ptr(pyr))
    off = 0
    for l in range(8):
        n = lw[l] * lh[l]
        lvl = np.ascontiguousarray(pyr[off:off + n])
        off += n
        cap = 1 << 18
        ref = np.zeros(cap, O.KP_DTYPE)
        nr = O.lib().oracle_fast_level(O.ptr(lvl), lw[l], lh[l], 20, 7, O.ptr(ref), cap)
        ref = ref[:nr]
        got = odo.debug_fast(1, l)
        assert len(got) == nr, f"level {l}: FAST count {len(got)} vs {nr}"
        assert kp_equal(got, ref), f"level {l}: FAST candidates differ"
        oref = np.zeros(4096, O.KP_DTYPE)
        no = O.lib().oracle_octree(O.ptr(ref), nr, 16, lw[l] - 16, 16, lh[l] - 16, quota[l], O.ptr(oref), 4096)
        ogot = odo.debug_octree(1, l)
        assert len(ogot) == no, f"level {l}: octree count {len(ogot)} vs {no}"
        assert kp_equal(ogot, oref[:no]), f"level {l}: octree output/order differs"


def test_frame_features_bit_exact(cfg2_run):
    pkg, odo, cfg, bgr, dep, _ = cfg2_run
    cal = oracle_calib(cfg)
    for i in range(4):
        ref = O.extract_frame(bgr[i], dep[i], O.orb_params(2000), cal)
        got = odo.frame(i)
        assert len(got["kps"]) == len(ref["kps"]), f"frame {i}: N {len(got['kps'])} vs {len(ref['kps'])}"
        for f in ("x", "y", "size", "angle", "response", "octave"):
            assert np.array_equal(got["kps"][f], ref["kps"][f]), f"frame {i}: kp.{f} differs"
        bad = np.nonzero((got["desc"] != ref["desc"]).any(1))[0]
        assert bad.size == 0, f"frame {i}: descriptors differ at {bad[:10]}"
        assert np.array_equal(got["kun"], ref["kun"]), f"frame {i}: undistorted kps differ"
        assert np.array_equal(got["xyz"], ref["xyz"]), f"frame {i}: xyz differ"
        assert np.array_equal(got["ur"], ref["ur"]), f"frame {i}: uR differ"


def test_pairs_match_ransac_pnp(cfg2_run):
    pkg, odo, cfg, bgr, dep, res = cfg2_run
    cal = oracle_calib(cfg)
    rp = O.ransac_params(500)
    frames = [O.extract_frame(bgr[i], dep[i], O.orb_params(2000), cal) for i in range(4)]
    latch = float("nan")
    assert res[0]["n_matches"] == 0  # first frame of a sequence has no predecessor
    for p in range(1, 4):
        seed = pkg.pair_seed(cfg.seed, p)
        r, mask, matches, latch = O.track_pair(frames[p - 1], frames[p], cal, rp, seed, latch)
        g = odo.pair(p)
        print(f"pair {p}: matches {r.n_matches} good {r.n_good} visited {r.visited} inliers {r.n_inliers} "
              f"rmse {r.rmse:.4f} pnp {r.pnp_inliers} | gpu pnp {res[p]['pnp_inliers']}")
        assert np.array_equal(g["matches"], matches), f"pair {p}: match list differs"
        assert res[p]["n_matches"] == r.n_matches
        assert res[p]["n_good"] == r.n_good
        assert res[p]["visited"] == r.visited, f"pair {p}: visited {res[p]['visited']} vs {r.visited}"
        assert res[p]["n_inliers"] == r.n_inliers
        assert res[p]["ransac_ok"] == r.ransac_ok
        assert np.array_equal(res[p]["T12"], np.array(r.T12, np.float32)), f"pair {p}: T12 not bit-exact"
        assert res[p]["rmse"] == np.float32(r.rmse)
        T_gpu = res[p]["Tcw"].reshape(4, 4)
        T_ref = np.array(r.Tcw, np.float32).reshape(4, 4)
        assert np.abs(T_gpu - T_ref).max() < 1e-4, f"pair {p}: PnP pose differs {np.abs(T_gpu - T_ref).max()}"
        assert abs(int(res[p]["pnp_inliers"]) - r.pnp_inliers) <= 2
        n2 = len(frames[p]["kps"])
        assert (g["pnp_inliers"][:n2] != mask).sum() <= 2
    assert abs(odo.latch - latch) == 0


def test_knn2_entry_point(pkg):
    rng = np.random.default_rng(7)
    q = rng.integers(0, 256, (777, 32), dtype=np.uint8)
    t = rng.integers(0, 256, (1025, 32), dtype=np.uint8)
    t[100] = t[5]  # exact ties
    q[3] = t[5]
    ri, rd = O.knn2(q, t)
    odo, _ = make_odo(pkg, 640, 480, 1000, 200, 1)
    lib = pkg.load()
    gi = np.zeros((777, 2), np.int32)
    gd = np.zeros((777, 2), np.int32)
    pkg.check(lib.odo_knn2_hamming(odo.h, pkg.ptr(q), 777, pkg.ptr(t), 1025, pkg.ptr(gi), pkg.ptr(gd)))
    assert np.array_equal(gi, ri) and np.array_equal(gd, rd)
