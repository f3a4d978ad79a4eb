"""Tracking::SearchLocalLMs / Matcher::ProjectionMatch:
Frame::isInFrustum + GetFeaturesInArea + the stable best/second-best with the
same-level ratio test, in landmark order, skipping slots that hold a landmark
with observations (including those taken earlier in the same call).

CPU: the oracle's C restatement against an independent pure-Python transcription
of matcher.cpp:90-145 / frame.cpp:100-133, 258-274 (parity unpinned against the
reference itself: OpenCV/ORB-SLAM2 cannot be built here). GPU: the HIP path
(odo_projection_match) against the oracle, bit-exact (slot assignments,
projections, match count), including windows with more than 16 candidates.
"""
import math

import numpy as np
import pytest

import oracle_lib as O
from conftest import load_pkg, sequence


def _frames(n_frames=3, nf=1000):
    bgr, dep, poses = sequence(n_frames, seed=0x5EED0007)
    cal = O.fr1_calib()
    fr = [O.extract_frame(bgr[i], dep[i], O.orb_params(nf), cal) for i in range(n_frames)]
    return fr, poses, cal


def make_problem(seed=1, dup=60, th=8.0):
    """Landmarks from frame 1 (world = its camera pose), the current frame is
    frame 2 at its true pose; flags, taken slots and near-duplicate landmarks
    (conflicts over one slot) drawn at random."""
    fr, poses, cal = _frames()
    rng = np.random.default_rng(seed)
    f1, f2 = fr[1], fr[2]
    ok = f1["xyz"][:, 2] > 0
    Xc = f1["xyz"][ok].astype(np.float64)
    Twc1 = poses[1]
    Xw = (Xc @ Twc1[:3, :3].T + Twc1[:3, 3]).astype(np.float32)
    d1 = f1["desc"][ok]
    nL = len(Xw) + dup
    lms = np.zeros(nL, O.LANDMARK_DTYPE)
    lms["X"][:len(Xw)] = Xw
    lms["desc"][:len(Xw)] = d1
    pick = rng.integers(0, len(Xw), dup)
    lms["X"][len(Xw):] = Xw[pick] + rng.normal(0, 0.002, (dup, 3)).astype(np.float32)
    lms["desc"][len(Xw):] = d1[pick] ^ (rng.random((dup, 32)) < 0.03).astype(np.uint8)
    order = rng.permutation(nL)
    lms = lms[order]
    fl = np.where(rng.random(nL) < 0.7, O.C.c_int(4).value, 0)
    fl |= np.where(rng.random(nL) < 0.04, 1, 0)
    fl |= np.where(rng.random(nL) < 0.04, 2, 0)
    lms["flags"] = fl
    Tcw = np.linalg.inv(poses[2]).astype(np.float32)
    n = len(f2["kps"])
    taken = (rng.random(n) < 0.1).astype(np.uint8)
    return dict(lms=lms, Tcw=Tcw, kun=np.ascontiguousarray(f2["kun"]), octave=np.ascontiguousarray(f2["kps"]["octave"]),
                desc=np.ascontiguousarray(f2["desc"]), taken=taken, cal=cal, th=th)


def oracle_run(P):
    n, nL = len(P["kun"]), len(P["lms"])
    b = np.zeros(4, np.float32)
    O.lib().oracle_image_bounds(O.C.byref(P["cal"]), 640, 480, O.ptr(b))
    sl = np.zeros(n, np.int32)
    proj = np.zeros((nL, 3), np.float32)
    nm = O.lib().oracle_projection_match(O.ptr(P["Tcw"].ravel()), O.ptr(P["lms"]), nL, O.ptr(P["kun"]),
                                         O.ptr(P["octave"]), O.ptr(P["desc"]), n, O.ptr(P["taken"]),
                                         O.C.byref(P["cal"]), O.ptr(b), P["th"], 0.8, O.ptr(sl), O.ptr(proj))
    return sl, proj, nm, b


def python_reference(P, b):
    """Direct transcription of the reference loops (float32 where the reference is float)."""
    f32 = np.float32
    T, lms, kun = P["Tcw"], P["lms"], P["kun"]
    c = P["cal"]
    nL, n = len(lms), len(kun)
    taken = P["taken"].astype(bool).copy()
    sl = np.full(n, -1, np.int32)
    inview = np.zeros(nL, bool)
    uv = np.zeros((nL, 2), np.float32)
    for i in range(nL):
        if lms["flags"][i] & 3:
            continue
        X = lms["X"][i]
        Pc = [f32(((float(T[k, 0]) * float(X[0]) + float(T[k, 1]) * float(X[1])) + float(T[k, 2]) * float(X[2]))
                  + float(T[k, 3])) for k in range(3)]
        if Pc[2] < f32(0):
            continue
        invz = f32(1) / Pc[2]
        u = f32(f32(f32(c.fx) * Pc[0]) * invz) + f32(c.cx)
        v = f32(f32(f32(c.fy) * Pc[1]) * invz) + f32(c.cy)
        if u < b[0] or u > b[1] or v < b[2] or v > b[3]:
            continue
        inview[i] = True
        uv[i] = (u, v)
    th = f32(P["th"])
    nm = 0
    for i in range(nL):
        if not inview[i] or lms["flags"][i] & 1:
            continue
        u, v = uv[i]
        idx = [j for j in range(n) if abs(f32(kun[j, 0] - u)) < th and abs(f32(kun[j, 1] - v)) < th]
        if not idx:
            continue
        b1 = b2 = math.inf
        l1 = l2 = -1
        bi = -1
        for j in idx:
            if taken[j]:
                continue
            d = float(np.unpackbits(lms["desc"][i] ^ P["desc"][j]).sum())
            if d < b1:
                b2, b1, l2, l1, bi = b1, d, l1, int(P["octave"][j]), j
            elif d < b2:
                l2, b2 = int(P["octave"][j]), d
        if b1 <= 100.0:
            if l1 == l2 and b1 > float(np.float32(0.8)) * b2:
                continue
            sl[bi] = i
            taken[bi] = bool(lms["flags"][i] & 4)
            nm += 1
    return sl, nm, inview, uv


def test_oracle_matches_python_transcription():
    P = make_problem()
    sl, proj, nm, b = oracle_run(P)
    ref_sl, ref_nm, inview, uv = python_reference(P, b)
    assert nm == ref_nm and nm > 50
    assert np.array_equal(sl, ref_sl)
    assert np.array_equal(~np.isnan(proj[:, 0]), inview)
    assert np.array_equal(proj[inview, :2], uv[inview])


@pytest.mark.gpu
@pytest.mark.parametrize("seed,th", [(1, 8.0), (2, 8.0), (3, 40.0), (4, 3.0)])
def test_gpu_projection_match(seed, th):
    pkg = load_pkg()
    P = make_problem(seed, th=th)
    sl_ref, proj_ref, nm_ref, b_ref = oracle_run(P)
    odo = pkg.Odometry(pkg.default_config(640, 480, 1, nfeatures=1000))
    lib = pkg.load()
    b = np.zeros(4, np.float32)
    pkg.check(lib.odo_image_bounds(odo.h, pkg.ptr(b)))
    assert np.array_equal(b, b_ref)
    n, nL = len(P["kun"]), len(P["lms"])
    sl = np.zeros(n, np.int32)
    proj = np.zeros((nL, 3), np.float32)
    nm = O.C.c_int(0)
    pkg.check(lib.odo_projection_match(odo.h, pkg.ptr(P["Tcw"].ravel()), pkg.ptr(P["lms"]), nL, pkg.ptr(P["kun"]),
                                       pkg.ptr(P["octave"]), pkg.ptr(P["desc"]), n, pkg.ptr(P["taken"]), th, 0.8,
                                       pkg.ptr(sl), pkg.ptr(proj), O.C.byref(nm)))
    print(f"seed {seed} th {th}: landmarks {nL} in view {int((~np.isnan(proj_ref[:, 0])).sum())} matches {nm_ref}")
    assert nm.value == nm_ref
    assert np.array_equal(sl, sl_ref), f"slot assignments differ at {np.nonzero(sl != sl_ref)[0][:10]}"
    assert np.array_equal(proj.view(np.uint32), proj_ref.view(np.uint32)), "projections differ"
    odo.close()


@pytest.mark.gpu
def test_gpu_track_local_map_second_pnp():
    """TrackLocalMap (tracking.cpp:228-255): ProjectionMatch, then the second
    PnPSolver::Compute over every slot holding a landmark, from a perturbed
    pose; the HIP PnP against the oracle PnP on the same edges (pose < 1e-4)."""
    pkg = load_pkg()
    P = make_problem(5)
    fr, poses, cal = _frames()
    f2 = fr[2]
    sl_ref, _, _, _ = oracle_run(P)
    slots = np.nonzero(sl_ref >= 0)[0]
    Xw = np.ascontiguousarray(P["lms"]["X"][sl_ref[slots]], np.float32)
    obs = np.ascontiguousarray(np.stack([f2["kun"][slots, 0], f2["kun"][slots, 1], f2["ur"][slots]], 1), np.float32)
    T0 = P["Tcw"].copy()
    T0[:3, 3] += np.float32(0.01)
    T_ref = np.zeros(16, np.float32)
    out_ref = np.zeros(len(slots), np.uint8)
    n_ref = O.lib().oracle_pnp(O.ptr(Xw), O.ptr(obs), len(slots), O.C.byref(cal), O.ptr(T0.ravel()), O.ptr(T_ref),
                               O.ptr(out_ref))
    odo = pkg.Odometry(pkg.default_config(640, 480, 1, nfeatures=1000))
    T = np.zeros(16, np.float32)
    out = np.zeros(len(slots), np.uint8)
    n = O.C.c_int(0)
    pkg.check(pkg.load().odo_pnp_motion_ba(odo.h, pkg.ptr(Xw), pkg.ptr(obs), len(slots), pkg.ptr(odo.cfg.calib),
                                           pkg.ptr(T0.ravel()), pkg.ptr(T), pkg.ptr(out), O.C.byref(n)))
    assert np.abs(T - T_ref).max() < 1e-4
    assert abs(n.value - n_ref) <= 2
    # the refined pose is the frame's true pose (synthetic ground truth)
    assert np.abs(T.reshape(4, 4)[:3, 3] - P["Tcw"][:3, 3]).max() < 0.01
    odo.close()
