"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle.

Bit-exact for integer/byte/index work (pyramid, FAST candidates, octree,
blurred levels, keypoints, descriptors, kNN indices and distances, match
lists, std::sort order, RANSAC inlier masks) and for the float/double RANSAC
fit (same operation order); PnP pose within 1e-4 (SURVEY §8 contract) with
inlier flags compared outside a small chi2 margin (oracle_lib.check_pnp_flags:
a flag may differ only where the edge's chi2 at the oracle pose is within 2 %
of the 5.991 / 7.815 threshold).
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
        O.check_ransac_inliers(g, r, f"pair {p}")
        assert res[p]["ransac_ok"] == r.ransac_ok
        assert (res[p]["n_sweeps"], res[p]["n_fit_points"]) == (r.n_sweeps, r.n_fit_points), f"pair {p}: work"
        assert np.array_equal(res[p]["T12"], np.array(r.T12, np.float32)), f"pair {p}: T12 not bit-exact"
        assert res[p]["rmse"] == np.float32(r.rmse)
        T_gpu = res[p]["Tcw"].reshape(4, 4)
        T_ref = np.array(r.Tcw, np.float32).reshape(4, 4)
        assert np.abs(T_gpu - T_ref).max() < 1e-4, f"pair {p}: PnP pose differs {np.abs(T_gpu - T_ref).max()}"
        n2 = len(frames[p]["kps"])
        nb = O.check_pnp_flags(g["pnp_inliers"][:n2], mask, frames[p - 1], frames[p], g["f2_src"][:n2], T_ref, cal,
                               f"pair {p}")
        assert abs(int(res[p]["pnp_inliers"]) - r.pnp_inliers) <= nb, f"pair {p}: PnP inlier count"
    assert abs(odo.latch - latch) == 0


def test_pipelined_batches_roll_and_seeds():
    """Batches queued back to back (extraction of one overlapping the pair and
    PnP stages of the two before it, frame sets used round robin and wrapping):
    the last batch's pair 0 links the previous batch's last frame, seeds follow
    the global pair index and the latch from the first valid pair carries over."""
    pkg = load_pkg()
    bgr, dep, _ = sequence(11)
    odo, cfg = make_odo(pkg, 640, 480, 1000, 300, 3)
    cal = oracle_calib(cfg)
    cuts = [0, 3, 5, 7, 9, 11]
    for a, b in zip(cuts[:-2], cuts[1:-1]):
        odo.track_batch_host(bgr[a:b], dep[a:b], want_results=False)
    res = odo.track_batch_host(bgr[9:11], dep[9:11])
    frames = [O.extract_frame(bgr[i], dep[i], O.orb_params(1000), cal) for i in range(11)]
    for i in range(2):
        got = odo.frame(i)
        assert np.array_equal(got["desc"], frames[9 + i]["desc"]), f"frame {9 + i} descriptors"
    rp = O.ransac_params(300)
    latch = float("nan")
    refs = {}
    for f in range(1, 11):  # the oracle walks the whole sequence (latch set by pair 1)
        refs[f] = O.track_pair(frames[f - 1], frames[f], cal, rp, pkg.pair_seed(cfg.seed, f), latch)
        latch = refs[f][3]
    for p, f in ((0, 9), (1, 10)):
        r, mask, matches, _ = refs[f]
        g = odo.pair(p)
        assert np.array_equal(g["matches"], matches), f"frame {f}: match list differs"
        assert res[p]["visited"] == r.visited and res[p]["n_inliers"] == r.n_inliers
        O.check_ransac_inliers(g, r, f"frame {f}")
        assert np.array_equal(res[p]["T12"], np.array(r.T12, np.float32)), f"frame {f}: T12 not bit-exact"
        T_gpu = res[p]["Tcw"].reshape(4, 4)
        assert np.abs(T_gpu - np.array(r.Tcw, np.float32).reshape(4, 4)).max() < 1e-4
    assert odo.latch == latch


@pytest.mark.parametrize("n,levels", [(1, 3), (15, 4), (16, 3), (17, 5), (100, 2), (613, 40), (777, 256),
                                      (2048, 30), (4099, 7), (8192, 200)])
def test_good_match_sort_is_std_sort(pkg, n, levels):
    """The pair stage's workgroup-parallel introsort returns exactly
    libstdc++'s std::sort permutation (ties included: Hamming distances take
    few values), against the oracle's std::sort on the same DMatch array."""
    rng = np.random.default_rng(n * 31 + levels)
    m = np.zeros(n, O.DMATCH_DTYPE)
    m["queryIdx"] = np.arange(n)
    m["trainIdx"] = rng.integers(0, 5000, n)
    m["distance"] = rng.integers(0, levels, n).astype(np.float32)
    if n > 100:  # presorted and reversed runs stress the median-of-3 / depth limit
        k = n // 3
        m["distance"][:k] = np.sort(m["distance"][:k])
        m["distance"][k:2 * k] = np.sort(m["distance"][k:2 * k])[::-1]
    ref = m.copy()
    O.lib().oracle_sort_dmatch(O.ptr(ref), n)
    got = np.zeros(n, O.DMATCH_DTYPE)
    odo, _ = make_odo(pkg, 640, 480, 1000, 10, 1)
    pkg.check(pkg.load().odo_debug_sort(odo.h, pkg.ptr(m), n, pkg.ptr(got)))
    assert np.array_equal(got["queryIdx"], ref["queryIdx"]), "permutation differs from std::sort"


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


def _frames_cfg1():
    bgr, dep, _ = sequence(3, seed=0x5EED0001)
    cal = O.fr1_calib()
    return bgr, dep, cal, [O.extract_frame(bgr[i], dep[i], O.orb_params(1000), cal) for i in range(3)]


def test_extract_entry_point_bgr_and_gray(pkg):
    bgr, dep, cal, frames = _frames_cfg1()
    odo, _ = make_odo(pkg, 640, 480, 1000, 200, 1)
    lib = pkg.load()
    cap = 1100
    for channels in (3, 1):
        img = np.ascontiguousarray(bgr[0] if channels == 3 else O.gray(bgr[0]))
        kps = np.zeros(cap, pkg.KP_DTYPE)
        desc = np.zeros((cap, 32), np.uint8)
        kun = np.zeros((cap, 2), np.float32)
        xyz = np.zeros((cap, 3), np.float32)
        ur = np.zeros(cap, np.float32)
        n = O.C.c_int(0)
        pkg.check(lib.odo_extract(odo.h, pkg.ptr(img), channels, pkg.ptr(np.ascontiguousarray(dep[0])), pkg.ptr(kps),
                                  pkg.ptr(desc), pkg.ptr(kun), pkg.ptr(xyz), pkg.ptr(ur), cap, O.C.byref(n)))
        ref = frames[0]
        assert n.value == len(ref["kps"])
        assert np.array_equal(kps[:n.value], ref["kps"]) and np.array_equal(desc[:n.value], ref["desc"])
        assert np.array_equal(xyz[:n.value], ref["xyz"])


@pytest.mark.parametrize("iters,corrupt", [(1, 0.0), (200, 0.0), (500, 0.0), (500, 0.3), (500, 0.55),
                                           (1200, 0.5), (40, 0.7),
                                           (4096, 0.6), (8192, 0.75)])
def test_ransac_entry_point_stream_and_latch(pkg, iters, corrupt):
    """odo_ransac == Ransac::Iterate: bit-exact T12/rmse/inliers, rand() stream
    advanced by exactly the visited draws, latch set on first call. `corrupt`
    re-targets that fraction of the matches at random keypoints so the inlier
    ratio stays under the 80% break and later rounds (side-stream samples,
    several 512-hypothesis rounds) are exercised."""
    bgr, dep, cal, frames = _frames_cfg1()
    f1, f2 = frames[0], frames[1]
    n1, n2 = len(f1["kps"]), len(f2["kps"])
    has = np.zeros(n1, np.uint8)
    O.lib().oracle_vo_landmarks(O.ptr(f1["xyz"]), n1, 40 * 40 / 517.3, O.ptr(has))
    obs2 = np.full(n2, -1, np.int32)
    src2 = np.full(n2, -1, np.int32)
    out2 = np.zeros(n2, np.uint8)
    m = np.zeros(n1, O.DMATCH_DTYPE)
    nm = O.lib().oracle_knn_match(O.ptr(f1["desc"]), n1, O.ptr(f2["desc"]), n2, 0.9, O.ptr(has),
                                  O.ptr(np.zeros(n1, np.uint8)), O.ptr(np.zeros(n1, np.int32)), O.ptr(obs2),
                                  O.ptr(src2), O.ptr(out2), O.ptr(m), n1)
    m = m[:nm]
    if corrupt > 0:
        rs = np.random.default_rng(int(corrupt * 1000) + iters)
        sel = rs.random(nm) < corrupt
        m["trainIdx"][sel] = rs.integers(0, n2, int(sel.sum()))
    rp = O.ransac_params(iters)
    odo, _ = make_odo(pkg, 640, 480, 1000, iters, 1)
    lib = pkg.load()
    for trial in range(2):
        r_ref, r_gpu = O.Rng(), pkg.Rng()
        O.lib().oracle_rng_seed(O.C.byref(r_ref), 777 + trial)
        lib.odo_rng_seed(pkg.ptr(r_gpu), 777 + trial)
        lat_ref = O.C.c_double(float("nan") if trial == 0 else 1e-3)
        lat_gpu = O.C.c_double(lat_ref.value)
        T_ref = np.zeros(16, np.float32)
        rmse_ref = O.C.c_float(0)
        inl_ref = np.zeros(nm, O.DMATCH_DTYPE)
        ni_ref, vis, ng = O.C.c_int(0), O.C.c_int(0), O.C.c_int(0)
        ok_ref = O.lib().oracle_ransac(O.ptr(m), nm, O.ptr(f1["xyz"]), O.ptr(f2["xyz"]), O.C.byref(rp),
                                       O.C.byref(r_ref), O.C.byref(lat_ref), O.ptr(T_ref), O.C.byref(rmse_ref),
                                       O.ptr(inl_ref), O.C.byref(ni_ref), O.C.byref(vis), O.C.byref(ng))
        T = np.zeros(16, np.float32)
        rmse = O.C.c_float(0)
        inl = np.zeros(nm, O.DMATCH_DTYPE)
        ni, ok = O.C.c_int(0), O.C.c_int(0)
        rpg = pkg.RansacParams(iters, 20, 3.0, 4, 1)
        pkg.check(lib.odo_ransac(odo.h, pkg.ptr(m), nm, pkg.ptr(f1["xyz"]), n1, pkg.ptr(f2["xyz"]), n2,
                                 pkg.ptr(rpg), pkg.ptr(r_gpu), O.C.byref(lat_gpu), pkg.ptr(T), O.C.byref(rmse),
                                 pkg.ptr(inl), O.C.byref(ni), O.C.byref(ok)))
        print(f"iters {iters} corrupt {corrupt}: good {ng.value} visited {vis.value} inliers {ni_ref.value}")
        assert ok.value == ok_ref and ni.value == ni_ref.value
        assert np.array_equal(T, T_ref) and rmse.value == rmse_ref.value
        assert np.array_equal(inl[:ni.value], inl_ref[:ni_ref.value])
        assert lat_gpu.value == lat_ref.value
        assert list(r_gpu.state) == list(r_ref.state) and (r_gpu.fpos, r_gpu.rpos) == (r_ref.fpos, r_ref.rpos)


def test_pnp_entry_point(pkg):
    rng = np.random.default_rng(5)
    from test_oracle import _pnp_problem
    R, t, Xw, obs = _pnp_problem(rng, n=300)
    obs[:15, 1] += 30
    Tinit = np.eye(4, dtype=np.float32)
    Tinit[:3, 3] = t + 0.01
    T_ref = np.zeros(16, np.float32)
    out_ref = np.zeros(300, np.uint8)
    n_ref = O.lib().oracle_pnp(O.ptr(Xw), O.ptr(obs), 300, O.C.byref(O.fr1_calib()), O.ptr(Tinit.ravel()),
                               O.ptr(T_ref), O.ptr(out_ref))
    odo, cfg = make_odo(pkg, 640, 480, 1000, 200, 1)
    T = np.zeros(16, np.float32)
    out = np.zeros(300, np.uint8)
    n = O.C.c_int(0)
    pkg.check(pkg.load().odo_pnp_motion_ba(odo.h, pkg.ptr(Xw), pkg.ptr(obs), 300, pkg.ptr(cfg.calib),
                                           pkg.ptr(Tinit.ravel()), pkg.ptr(T), pkg.ptr(out), O.C.byref(n)))
    assert np.abs(T - T_ref).max() < 1e-4
    assert n.value == n_ref and np.array_equal(out, out_ref)
    assert np.abs(T.reshape(4, 4)[:3, 3] - t).max() < 1e-4


def test_kabsch_entry_point(pkg):
    rng = np.random.default_rng(9)
    from test_oracle import _rand_rigid
    R, t = _rand_rigid(rng)
    A = (rng.random((500, 3)) * 2 - 1).astype(np.float32)
    B = (A @ R.T + t + rng.normal(size=(500, 3)) * 1e-3).astype(np.float32)
    K_ref = np.zeros(16, np.float32)
    O.lib().oracle_kabsch(O.ptr(A), O.ptr(B), 500, O.ptr(K_ref))
    K = pkg.kabsch(A, B)
    assert np.abs(K.ravel() - K_ref).max() < 1e-4
