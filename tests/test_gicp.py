"""GeneralizedICP::Compute(source, target, guess) (Odometry/generalizedicp.cpp:
30-39, 65-89): the PCL GICP refinement of Odometry::Compute's ADAPTIVE_RICP mode
(odometry.cpp:46-78), built with GeneralizedICP(10, 0.07).

CPU: the oracle's restatement (oracle/gicp_ref.cpp) recovers known rigid
motions of planar synthetic scenes, its covariances have the (1, 1, 1e-3)
spectrum, and the early exits follow generalizedicp.cpp (< 20 points) and PCL
(< 4 correspondences: not converged, identity). PCL is absent, so parity with the
library is UNPINNED.

GPU: odo_gicp (k_gicp.hip) against the oracle on the same clouds: converged
flag, ICP iterations and correspondence count exactly; T12 within 1e-5 (the
device's double cos / sin in the gradient are the only non-IEEE steps; every
sum over correspondences uses the same 256-thread association on both sides).
"""
import numpy as np
import pytest
from scipy.spatial.transform import Rotation

import oracle_lib as O
from conftest import load_pkg, sequence


def _scene(seed, n=400, noise=0.002, rv=(0.01, -0.02, 0.015), t=(0.02, -0.01, 0.03), outl=0.0):
    rng = np.random.default_rng(seed)
    k = n // 3
    P = np.r_[np.c_[rng.uniform(-1, 1, k), rng.uniform(-1, 1, k), np.full(k, 3.0)],
              np.c_[np.full(k, -1.0), rng.uniform(-1, 1, k), rng.uniform(2, 4, k)],
              np.c_[rng.uniform(-1, 1, n - 2 * k), np.full(n - 2 * k, 1.0), rng.uniform(2, 4, n - 2 * k)]]
    P += rng.normal(0, noise, P.shape)
    R = Rotation.from_rotvec(rv).as_matrix()
    Q = P @ R.T + np.asarray(t)
    if outl:
        m = rng.random(n) < outl
        Q[m] += rng.uniform(-0.3, 0.3, (m.sum(), 3))
    T = np.eye(4)
    T[:3, :3] = R
    T[:3, 3] = t
    return P.astype(np.float32), Q.astype(np.float32), T


def _frames_clouds():
    """Ransac::Iterate's mpSourceCloud / mpTargetCloud (ransac.cpp:175-189) of a
    synthetic pair: the kNN-2 + ratio matches with valid depth on both sides."""
    bgr, dep, _ = sequence(3, seed=0x5EED0012)
    cal = O.fr1_calib()
    f1 = O.extract_frame(bgr[0], dep[0], O.orb_params(1000), cal)
    f2 = O.extract_frame(bgr[1], dep[1], O.orb_params(1000), cal)
    idx, dist = O.knn2(f1["desc"], f2["desc"])
    keep = dist[:, 0] < 0.9 * dist[:, 1]
    q = np.nonzero(keep)[0]
    tr = idx[q, 0]
    ok = (f1["xyz"][q, 2] > 0) & (f2["xyz"][tr, 2] > 0)
    return f1["xyz"][q[ok]].astype(np.float32), f2["xyz"][tr[ok]].astype(np.float32)


# ----------------------------------------------------------------- CPU
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_oracle_recovers_motion(seed):
    P, Q, T = _scene(seed)
    r = O.gicp(P, Q)
    assert r["ok"] == 1 and r["converged"] == 1
    assert 1 <= r["iterations"] <= 10
    np.testing.assert_allclose(r["T"], T, atol=2e-3)


def test_oracle_covariances():
    P, _, _ = _scene(4, n=200)
    C = np.zeros((200, 9))
    O.lib().oracle_gicp_covariances(O.ptr(P), 200, O.ptr(C))
    for c in C.reshape(-1, 3, 3):
        np.testing.assert_allclose(c, c.T, atol=1e-15)
        np.testing.assert_allclose(np.linalg.eigvalsh(c), [1e-3, 1.0, 1.0], atol=1e-9)


def test_oracle_early_exits():
    P, Q, _ = _scene(5, n=19)
    r = O.gicp(P, Q)
    assert r["converged"] == 0 and np.array_equal(r["T"], np.eye(4, dtype=np.float32))
    P, Q, _ = _scene(6, n=100, t=(3.0, 0.0, 0.0))  # nothing within 0.07 m
    r = O.gicp(P, Q)
    assert r["converged"] == 0 and r["n_corr"] < 4 and np.array_equal(r["T"], np.eye(4, dtype=np.float32))


def test_oracle_guess_composes():
    P, Q, T = _scene(7, t=(0.08, -0.05, 0.1))
    guess = T.astype(np.float32).copy()
    guess[:3, 3] += np.float32([0.01, -0.01, 0.005])
    r = O.gicp(P, Q, guess)
    assert r["converged"] == 1
    np.testing.assert_allclose(r["T"], T, atol=3e-3)


# ----------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def odo():
    pkg = load_pkg()
    o = pkg.Odometry(pkg.default_config(640, 480, 1))
    yield o
    o.close()


def _check(odo, P, Q, guess=None, iters=10, dist=0.07):
    ref = O.gicp(P, Q, guess, iters, dist)
    T, conv, it, nc = odo.gicp(P, Q, guess, iters, dist)
    assert conv == ref["converged"]
    assert it == ref["iterations"]
    assert nc == ref["n_corr"]
    np.testing.assert_allclose(T, ref["T"], rtol=0, atol=1e-5)
    return ref


@pytest.mark.gpu
@pytest.mark.parametrize("seed,n,outl", [(1, 400, 0.0), (2, 150, 0.0), (3, 1500, 0.1), (8, 60, 0.3)])
def test_gpu_parity_scenes(odo, seed, n, outl):
    P, Q, _ = _scene(seed, n=n, outl=outl)
    ref = _check(odo, P, Q)
    assert ref["converged"] == 1


@pytest.mark.gpu
def test_gpu_parity_guess_and_params(odo):
    P, Q, T = _scene(9, t=(0.08, -0.05, 0.1))
    guess = T.astype(np.float32).copy()
    guess[:3, 3] += np.float32([0.01, -0.01, 0.005])
    _check(odo, P, Q, guess)
    _check(odo, P, Q, None, iters=3, dist=0.2)
    _check(odo, P, Q, None, iters=20, dist=0.05)


@pytest.mark.gpu
def test_gpu_parity_frames_clouds(odo):
    P, Q = _frames_clouds()
    assert len(P) >= 20
    _check(odo, P, Q)


@pytest.mark.gpu
def test_gpu_edge_cases(odo):
    P, Q, _ = _scene(5, n=19)
    T, conv, it, nc = odo.gicp(P, Q)
    assert conv == 0 and it == 0 and np.array_equal(T, np.eye(4, dtype=np.float32))
    P, Q, _ = _scene(6, n=100, t=(3.0, 0.0, 0.0))
    ref = _check(odo, P, Q)
    assert ref["converged"] == 0


@pytest.mark.gpu
def test_gpu_batch_matches_oracle(odo):
    """odo_gicp_batch: every pair of a ragged batch (incl. < 20 points and no
    correspondences) equals the oracle and the one-call API."""
    pairs = []
    for seed, n, outl, t in [(31, 400, 0.0, (0.02, -0.01, 0.03)), (32, 19, 0.0, (0.0, 0.0, 0.0)),
                             (33, 1500, 0.1, (0.02, -0.01, 0.03)), (34, 100, 0.0, (3.0, 0.0, 0.0)),
                             (35, 60, 0.3, (0.02, -0.01, 0.03))]:
        P, Q, _ = _scene(seed, n=n, outl=outl, t=t)
        pairs.append((P, Q, None))
    P, Q, T = _scene(36, t=(0.08, -0.05, 0.1))
    guess = T.astype(np.float32).copy()
    guess[:3, 3] += np.float32([0.01, -0.01, 0.005])
    pairs.append((P, Q, guess))
    pairs.append((*_frames_clouds(), None))
    out = odo.gicp_batch(pairs)
    for (P, Q, g), (T, conv, it, nc) in zip(pairs, out):
        ref = O.gicp(P, Q, g)
        T1, conv1, it1, nc1 = odo.gicp(P, Q, g)
        assert conv == ref["converged"] == conv1
        assert it == ref["iterations"] == it1
        assert nc == ref["n_corr"] == nc1
        np.testing.assert_allclose(T, ref["T"], rtol=0, atol=1e-5)
        assert np.array_equal(T, T1)
