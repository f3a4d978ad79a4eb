"""PnPRansac::Compute (Odometry/pnpransac.cpp:11-51):
cv::solvePnPRansac(v3D, v2D, mK, noDist, r, t, false, 500, 3.0f, 0.85, inliers).

CPU: the oracle's restatement (oracle/pnpransac_ref.cpp) checked piecewise —
cv::RNG and RANSACUpdateNumIters against independent Python transcriptions,
cvRodrigues2 against scipy and finite differences, EPnP on exact minimal sets,
the whole RANSAC + Levenberg-Marquardt path recovering known poses. OpenCV is
absent, so parity with the real library is UNPINNED.

GPU: odo_pnp_ransac (k_pnpransac.hip) against the oracle on the same inputs:
every visited hypothesis' inlier count, the winning hypothesis, the iterations
run and the inlier mask exactly; the RANSAC model within 1e-9 and the refined
pose within 1e-7 (the device libm's cos/sin/acos are the only non-IEEE steps;
the refinement's J^T J is reduced in a different order). The refinement
starts where solvePnP(useExtrinsicGuess = false) starts (pnpransac.cpp:34):
cvFindExtrinsicCameraParams2's DLT, or its homography branch for coplanar
landmarks (test_gpu_parity_planar).
"""
import math

import numpy as np
import pytest
from scipy.spatial.transform import Rotation

import oracle_lib as O
from conftest import load_pkg, sequence


def _problem(seed, n, outlier_frac, noise=0.5, planar=False):
    rng = np.random.default_rng(seed)
    cal = O.fr1_calib()
    Xc = np.c_[rng.uniform(-2, 2, n), rng.uniform(-1.5, 1.5, n), rng.uniform(1, 5, n)]
    if planar:
        Xc[:, 2] = 3.0 + 0.2 * Xc[:, 0]
    rv = rng.normal(0, 0.2, 3)
    t = rng.normal(0, 0.3, 3)
    R = Rotation.from_rotvec(rv).as_matrix()
    Xw = (Xc - t) @ R  # Xc = R Xw + t
    uv = np.c_[cal.fx * Xc[:, 0] / Xc[:, 2] + cal.cx, cal.fy * Xc[:, 1] / Xc[:, 2] + cal.cy]
    uv += rng.normal(0, noise, uv.shape)
    out = rng.random(n) < outlier_frac
    uv[out] += rng.uniform(-80, 80, (out.sum(), 2))
    return Xw.astype(np.float32), uv.astype(np.float32), cal, rv, t, out


def _frames_problem(nf=1000):
    """Landmarks = frame-1 camera points, observations = frame-2 undistorted
    keypoints matched by kNN-2 + ratio 0.9 (mismatches are the outliers)."""
    bgr, dep, poses = sequence(3, seed=0x5EED0011)
    cal = O.fr1_calib()
    f1 = O.extract_frame(bgr[0], dep[0], O.orb_params(nf), cal)
    f2 = O.extract_frame(bgr[2], dep[2], O.orb_params(nf), cal)
    idx, dist = O.knn2(f1["desc"], f2["desc"])
    keep = (dist[:, 0] < 0.9 * dist[:, 1]) & (f1["xyz"][:, 2] > 0)
    q = np.nonzero(keep)[0]
    Xw = f1["xyz"][q].astype(np.float32)
    uv = f2["kun"][idx[q, 0]].astype(np.float32)
    return Xw, uv, cal


# ----------------------------------------------------------------- CPU
def _cvrng_py(state, a, b, n):
    out = []
    for _ in range(n):
        state = ((state & 0xFFFFFFFF) * 4164903690 + (state >> 32)) & ((1 << 64) - 1)
        out.append(a + (state & 0xFFFFFFFF) % (b - a))
    return out


def test_cvrng_stream():
    got = np.zeros(64, np.int32)
    O.lib().oracle_cvrng_stream((1 << 64) - 1, 0, 97, 64, O.ptr(got))
    assert got.tolist() == _cvrng_py((1 << 64) - 1, 0, 97, 64)


def _update_py(p, ep, m, maxit):
    p = min(max(p, 0.0), 1.0)
    ep = min(max(ep, 0.0), 1.0)
    num = max(1.0 - p, 2.2250738585072014e-308)
    denom = 1.0 - (1.0 - ep) ** m
    if denom < 2.2250738585072014e-308:
        return 0
    num, denom = math.log(num), math.log(denom)
    return maxit if denom >= 0 or -num >= maxit * (-denom) else int(round(num / denom))


@pytest.mark.parametrize("ep", [0.0, 0.05, 0.3, 0.5, 0.7, 0.9, 0.99, 1.0])
def test_update_num_iters(ep):
    for maxit in (1, 34, 500, 4096):
        got = O.lib().oracle_ransac_update_num_iters(0.85, ep, 5, maxit)
        assert got == _update_py(0.85, ep, 5, maxit), (ep, maxit)
    # a known value: p 0.99, half outliers, 5 points -> log(0.01)/log(1-1/32) = 145.0
    assert O.lib().oracle_ransac_update_num_iters(0.99, 0.5, 5, 1000) == 145


def test_rodrigues():
    rng = np.random.default_rng(3)
    for _ in range(20):
        r = rng.normal(0, 1.0, 3)
        R = np.zeros(9)
        J = np.zeros(27)
        O.lib().oracle_rodrigues(O.ptr(r), O.ptr(R), O.ptr(J))
        np.testing.assert_allclose(R.reshape(3, 3), Rotation.from_rotvec(r).as_matrix(), atol=1e-13)
        back = np.zeros(3)
        O.lib().oracle_rodrigues_inv(O.ptr(R), O.ptr(back))
        np.testing.assert_allclose(back, r if np.linalg.norm(r) < np.pi else back, atol=1e-12)
        for i in range(3):  # dR/dr_i by central differences
            h = 1e-6
            rp, rm = r.copy(), r.copy()
            rp[i] += h
            rm[i] -= h
            Rp, Rm = np.zeros(9), np.zeros(9)
            O.lib().oracle_rodrigues(O.ptr(rp), O.ptr(Rp), None)
            O.lib().oracle_rodrigues(O.ptr(rm), O.ptr(Rm), None)
            np.testing.assert_allclose(J[9 * i:9 * i + 9], (Rp - Rm) / (2 * h), atol=1e-8)
    # theta = 0 and theta = pi branches
    R = np.eye(3).ravel().copy()
    back = np.zeros(3)
    O.lib().oracle_rodrigues_inv(O.ptr(R), O.ptr(back))
    assert np.all(back == 0)
    Rpi = Rotation.from_rotvec([0, np.pi, 0]).as_matrix().ravel().copy()
    O.lib().oracle_rodrigues_inv(O.ptr(Rpi), O.ptr(back))
    np.testing.assert_allclose(np.abs(back), [0, np.pi, 0], atol=1e-7)


@pytest.mark.parametrize("n", [5, 6, 12, 50])
def test_epnp_exact(n):
    Xw, uv, cal, rv, t, _ = _problem(7 + n, n, 0.0, noise=0.0)
    K = np.array([cal.fx, cal.fy, cal.cx, cal.cy], np.float64)
    model = np.zeros(6)
    O.lib().oracle_epnp(O.ptr(Xw.astype(np.float64)), O.ptr(uv.astype(np.float64)), n, O.ptr(K), O.ptr(model))
    # float32 inputs: exact up to the input rounding
    np.testing.assert_allclose(model[:3], rv, atol=2e-4)
    np.testing.assert_allclose(model[3:], t, atol=2e-4)


@pytest.mark.parametrize("seed,n,outl", [(1, 400, 0.4), (2, 150, 0.1), (3, 1200, 0.6), (4, 60, 0.0)])
def test_oracle_recovers_pose(seed, n, outl):
    Xw, uv, cal, rv, t, out = _problem(seed, n, outl)
    r = O.pnp_ransac(Xw, uv, cal)
    assert r["ok"] == 1
    np.testing.assert_allclose(r["rt"][:3], rv, atol=5e-3)
    np.testing.assert_allclose(r["rt"][3:], t, atol=2e-2)
    # gross outliers (|offset| up to 80 px) are rejected, true points mostly kept
    assert (r["mask"] & out).sum() <= max(2, 0.02 * out.sum())
    assert r["mask"][~out].mean() > 0.75  # the mask is the RANSAC model's (confidence 0.85 stops early)
    assert r["n_inliers"] == r["mask"].sum()
    assert r["good"][r["best_iter"]] == r["n_inliers"]
    T = r["T"]
    np.testing.assert_allclose(T[:3, :3], Rotation.from_rotvec(r["rt"][:3]).as_matrix(), atol=1e-6)
    # refinement never worsens the inlier reprojection error of the RANSAC model
    def rms(rt):
        R = Rotation.from_rotvec(rt[:3]).as_matrix()
        Xc = Xw[r["mask"]].astype(np.float64) @ R.T + rt[3:]
        p = np.c_[cal.fx * Xc[:, 0] / Xc[:, 2] + cal.cx, cal.fy * Xc[:, 1] / Xc[:, 2] + cal.cy]
        return np.sqrt(((p - uv[r["mask"]]) ** 2).sum(1).mean())
    assert rms(r["rt"]) <= rms(r["model"]) + 1e-9


@pytest.mark.parametrize("planar", [False, True], ids=["dlt", "homography"])
@pytest.mark.parametrize("n", [6, 40, 300])
def test_extrinsic_init_exact(planar, n):
    """cvFindExtrinsicCameraParams2's start without a guess (the final
    solvePnP of solvePnPRansac: pnpransac.cpp:34 passes useExtrinsicGuess =
    false): the DLT (non-planar points) and the homography decomposition
    (coplanar points) recover a noise-free pose on their own, and CvLevMarq
    from that start lands on it."""
    Xw, uv, cal, rv, t, _ = _problem(40 + n, n, 0.0, noise=0.0, planar=planar)
    K = np.array([cal.fx, cal.fy, cal.cx, cal.cy], np.float64)
    M, m = Xw.astype(np.float64), uv.astype(np.float64)
    p = np.zeros(6)
    O.lib().oracle_pnp_extrinsic_init(O.ptr(M), O.ptr(m), n, O.ptr(K), O.ptr(p))
    np.testing.assert_allclose(p[:3], rv, atol=2e-3)
    np.testing.assert_allclose(p[3:], t, atol=5e-3)
    O.lib().oracle_pnp_refine(O.ptr(M), O.ptr(m), n, O.ptr(K), O.ptr(p))
    np.testing.assert_allclose(p[:3], rv, atol=1e-4)
    np.testing.assert_allclose(p[3:], t, atol=1e-4)


def _five_inliers(seed):
    """12 observations, 5 exact and 7 moved 40-120 px: the best RANSAC model
    has exactly 5 inliers (goodCount > modelPoints - 1 accepts it)."""
    Xw, uv, cal, *_ = _problem(seed, 12, 0.0, noise=0.0)
    rng = np.random.default_rng(seed + 1000)
    ang = rng.uniform(0, 2 * np.pi, 7)
    uv[5:] += (np.c_[np.cos(ang), np.sin(ang)] * rng.uniform(40, 120, (7, 1))).astype(np.float32)
    return Xw, uv, cal


def test_oracle_five_inliers_dlt_asserts():
    """with exactly 5 non-planar inliers the final solvePnP's
    cvFindExtrinsicCameraParams2 takes its DLT branch, which asserts count >= 6
    (OpenCV throws, PnPRansac::Compute does not catch): the oracle reports -1
    with the RANSAC model, mask and count and no pose. A 5-point set that is
    planar (seed 61) takes the homography branch and refines normally."""
    Xw, uv, cal = _five_inliers(62)
    r = O.pnp_ransac(Xw, uv, cal, 4096)
    assert r["ok"] == -1 and r["n_inliers"] == 5 and r["mask"].sum() == 5
    assert np.all(r["T"] == 0) and np.all(r["rt"] == 0) and np.any(r["model"] != 0)
    Xw, uv, cal = _five_inliers(61)
    r = O.pnp_ransac(Xw, uv, cal, 4096)
    assert r["ok"] == 1 and r["n_inliers"] == 5
    # the DLT start alone: 5 non-planar points fail, 6 succeed
    Xw, uv, cal, *_ = _problem(45, 6, 0.0, noise=0.0)
    K = np.array([cal.fx, cal.fy, cal.cx, cal.cy], np.float64)
    M, m, p = Xw.astype(np.float64), uv.astype(np.float64), np.zeros(6)
    assert O.lib().oracle_pnp_extrinsic_init(O.ptr(M[:5].copy()), O.ptr(m[:5].copy()), 5, O.ptr(K), O.ptr(p)) == 0
    assert O.lib().oracle_pnp_extrinsic_init(O.ptr(M), O.ptr(m), 6, O.ptr(K), O.ptr(p)) == 1


def test_oracle_too_few_points():
    Xw, uv, cal, *_ = _problem(5, 9, 0.0)
    r = O.pnp_ransac(Xw, uv, cal)
    assert r["ok"] == 0 and r["n_inliers"] == 0


def test_oracle_frames_problem():
    Xw, uv, cal = _frames_problem()
    r = O.pnp_ransac(Xw, uv, cal)
    assert r["ok"] == 1 and r["n_inliers"] > 0.5 * len(Xw)


# ----------------------------------------------------------------- GPU
def _check_gpu(odo, Xw, uv, cal, iterations=500, reproj=3.0, conf=0.85):
    ref = O.pnp_ransac(Xw, uv, cal, iterations, reproj, conf)
    res, mask, good = odo.pnp_ransac(Xw, uv, None, iterations, reproj, conf)
    assert res.ok == ref["ok"]
    if not ref["ok"] and len(Xw) < 10:
        return ref, res
    assert res.iterations_visited == ref["niters"]
    v = ref["niters"]
    np.testing.assert_array_equal(good[:v], ref["good"][:v])
    assert res.best_iter == ref["best_iter"]
    if not ref["ok"]:
        return ref, res
    assert res.n_inliers == ref["n_inliers"]
    np.testing.assert_array_equal(mask, ref["mask"])
    np.testing.assert_allclose(np.r_[res.model_rvec[:], res.model_tvec[:]], ref["model"], rtol=0, atol=1e-9)
    np.testing.assert_allclose(np.r_[res.rvec[:], res.tvec[:]], ref["rt"], rtol=0, atol=1e-7)
    np.testing.assert_allclose(np.array(res.Tcw[:]).reshape(4, 4), ref["T"], rtol=0, atol=1e-5)
    return ref, res


@pytest.fixture(scope="module")
def odo():
    pkg = load_pkg()
    cfg = pkg.default_config(640, 480, 1, nfeatures=1000, iterations=200)
    o = pkg.Odometry(cfg)
    yield o
    o.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,outl", [(1, 400, 0.4), (2, 150, 0.1), (3, 1200, 0.6), (4, 60, 0.0),
                                         (5, 3000, 0.3), (6, 20, 0.25), (8, 800, 0.75)])
def test_gpu_parity_synthetic(odo, seed, n, outl):
    Xw, uv, cal, *_ = _problem(seed, n, outl)
    _check_gpu(odo, Xw, uv, cal)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,outl", [(31, 300, 0.3), (32, 40, 0.0), (33, 900, 0.5)])
def test_gpu_parity_planar(odo, seed, n, outl):
    """Coplanar landmarks: the final solvePnP's unseeded start takes
    cvFindExtrinsicCameraParams2's homography branch (findHomography + its
    LMSolver polish on lane 0) instead of the DLT."""
    Xw, uv, cal, rv, t, _ = _problem(seed, n, outl, planar=True)
    ref, res = _check_gpu(odo, Xw, uv, cal)
    assert res.ok == 1
    np.testing.assert_allclose(np.r_[res.rvec[:]], rv, atol=5e-3)


@pytest.mark.gpu
def test_gpu_parity_frames_problem(odo):
    Xw, uv, cal = _frames_problem()
    ref, res = _check_gpu(odo, Xw, uv, cal)
    assert res.ok == 1


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [60, 61, 62])
def test_gpu_parity_five_inliers(odo, seed):
    """Best model with exactly 5 inliers: non-planar -> ok = -1 on
    both sides (the DLT's count >= 6 assertion), same model, mask, visited
    hypotheses; seed 61's inliers are planar -> refined pose as usual."""
    Xw, uv, cal = _five_inliers(seed)
    ref, res = _check_gpu(odo, Xw, uv, cal, 4096)
    assert res.ok == (1 if seed == 61 else -1) and res.n_inliers == 5


@pytest.mark.gpu
@pytest.mark.parametrize("iters,reproj,conf", [(1, 3.0, 0.85), (4096, 3.0, 0.85), (500, 1.0, 0.99), (64, 8.0, 0.5)])
def test_gpu_parity_params(odo, iters, reproj, conf):
    Xw, uv, cal, *_ = _problem(11, 700, 0.5)
    _check_gpu(odo, Xw, uv, cal, iters, reproj, conf)


@pytest.mark.gpu
def test_gpu_edge_cases(odo):
    # fewer than 10 observations: PnPRansac::Compute returns 0 before solvePnPRansac
    Xw, uv, cal, *_ = _problem(12, 9, 0.0)
    res, mask, _ = odo.pnp_ransac(Xw, uv)
    assert res.ok == 0 and res.n_inliers == 0 and not mask.any()
    # pure noise: no hypothesis reaches 5 inliers -> bOK false, same as the oracle
    rng = np.random.default_rng(13)
    Xw = rng.uniform(-2, 2, (200, 3)).astype(np.float32) + np.float32([0, 0, 4])
    uv = rng.uniform(0, 640, (200, 2)).astype(np.float32)
    _check_gpu(odo, Xw, uv, O.fr1_calib())
    # exact, noise-free data: every point an inlier
    Xw, uv, cal, *_ = _problem(14, 300, 0.0, noise=0.0)
    ref, res = _check_gpu(odo, Xw, uv, cal)
    assert res.n_inliers == 300
    # bad confidence is rejected like ptsetreg.cpp's CV_Assert
    pkg = load_pkg()
    with pytest.raises(RuntimeError):
        odo.pnp_ransac(Xw, uv, None, 500, 3.0, 1.0)
    assert pkg is not None


@pytest.mark.gpu
def test_gpu_batch_matches_oracle(odo):
    """odo_pnp_ransac_batch: every problem of a ragged batch (incl. < 10
    observations, pure noise, large) equals the oracle and the one-call API."""
    probs = []
    for seed, n, outl in [(21, 400, 0.4), (22, 9, 0.0), (23, 1200, 0.6), (24, 60, 0.0), (25, 0, 0.0),
                          (26, 800, 0.75), (27, 30, 0.2)]:
        Xw, uv, cal, *_ = _problem(seed, max(n, 1), outl)
        probs.append((Xw[:n], uv[:n]))
    rng = np.random.default_rng(28)
    probs.append((rng.uniform(-2, 2, (200, 3)).astype(np.float32) + np.float32([0, 0, 4]),
                  rng.uniform(0, 640, (200, 2)).astype(np.float32)))
    probs.append(_frames_problem())
    cal = O.fr1_calib()
    res, masks = odo.pnp_ransac_batch([(x, u) for x, u, *_ in probs])
    for (Xw, uv, *_), r, m in zip(probs, res, masks):
        ref = O.pnp_ransac(Xw, uv, cal)
        one, mask1, _ = odo.pnp_ransac(Xw, uv)
        assert r.ok == ref["ok"] == one.ok
        if len(Xw) < 10:
            assert r.best_iter == -1 and not m.any()
            continue
        assert r.iterations_visited == ref["niters"] == one.iterations_visited
        assert r.best_iter == ref["best_iter"]
        if not ref["ok"]:
            continue
        assert r.n_inliers == ref["n_inliers"]
        np.testing.assert_array_equal(m, ref["mask"])
        np.testing.assert_array_equal(m, mask1)
        np.testing.assert_allclose(np.r_[r.rvec[:], r.tvec[:]], ref["rt"], rtol=0, atol=1e-7)
        assert np.array_equal(np.array(r.Tcw[:]), np.array(one.Tcw[:]))
