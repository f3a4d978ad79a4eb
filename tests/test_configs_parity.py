"""GPU parity at BASELINE.json configs 3-5, single GPU.

* cfg3 "fr2/desk": 640x480, FR2 intrinsics with the FR1 distortion the
  reference keeps (common.h:47-50, App. B.16), 4000 kp, RANSAC 4096.
* cfg4 "ICL living_room": 640x480, K=(481.2, -480.0, 319.5, 239.5), no
  distortion (undistortPoints short-circuits, frame.cpp:288), 2000 kp, RANSAC 500.
* cfg5 synthetic 1280x960, K = 2x FR1, no distortion, 8000 kp, RANSAC 8192.

Same bar as test_gpu_parity: features, match lists, RANSAC outputs bit-exact;
PnP pose within 1e-4. Three frames per config (two pairs) keep the oracle to
seconds; the whole batched path (odo_track_batch) runs on the GPU.
"""
import numpy as np
import pytest

import oracle_lib as O
from conftest import load_pkg, sequence

pytestmark = pytest.mark.gpu

FR1 = dict(fx=517.3, fy=516.5, cx=318.6, cy=255.3)
FR2 = dict(fx=520.9, fy=521.0, cx=325.1, cy=249.7)
ICL = dict(fx=481.2, fy=-480.0, cx=319.5, cy=239.5)
NODIST = dict(k1=0.0, k2=0.0, p1=0.0, p2=0.0, k3=0.0)

CONFIGS = {
    "cfg3_fr2_4000": dict(w=640, h=480, nf=4000, iters=4096, intr=FR2, calib=dict(FR2), seed=0x5EED0003),
    "cfg4_icl_2000": dict(w=640, h=480, nf=2000, iters=500, intr=ICL, calib=dict(ICL, **NODIST), seed=0x5EED0004),
    "cfg5_1280_8000": dict(w=1280, h=960, nf=8000, iters=8192, intr=FR1,
                           calib=dict(fx=2 * FR1["fx"], fy=2 * FR1["fy"], cx=2 * FR1["cx"], cy=2 * FR1["cy"],
                                      **NODIST), seed=0x5EED0005),
}


@pytest.mark.parametrize("name", list(CONFIGS))
def test_config_path_parity(name):
    c = CONFIGS[name]
    pkg = load_pkg()
    bgr, dep, _ = sequence(3, c["w"], c["h"], intrinsics=c["intr"], seed=c["seed"])
    cfg = pkg.default_config(c["w"], c["h"], 3, nfeatures=c["nf"], iterations=c["iters"], seed=c["seed"],
                             calib=c["calib"])
    odo = pkg.Odometry(cfg)
    res = odo.track_batch_host(bgr, dep)
    k = cfg.calib
    cal = O.Calib(k.fx, k.fy, k.cx, k.cy, k.k1, k.k2, k.p1, k.p2, k.k3, k.depth_factor, k.mbf, k.th_depth)
    op = O.orb_params(c["nf"])
    frames = [O.extract_frame(bgr[i], dep[i], op, cal) for i in range(3)]
    for i in range(3):
        got, ref = odo.frame(i), frames[i]
        assert len(got["kps"]) == len(ref["kps"]), f"{name} frame {i}: N"
        assert np.array_equal(got["kps"], ref["kps"]), f"{name} frame {i}: keypoints"
        assert np.array_equal(got["desc"], ref["desc"]), f"{name} frame {i}: descriptors"
        for f in ("kun", "xyz", "ur"):
            assert np.array_equal(got[f], ref[f]), f"{name} frame {i}: {f}"
    rp = O.ransac_params(c["iters"])
    latch = float("nan")
    for p in (1, 2):
        r, mask, matches, latch = O.track_pair(frames[p - 1], frames[p], cal, rp, pkg.pair_seed(cfg.seed, p), latch)
        g = odo.pair(p)
        print(f"{name} pair {p}: N={len(frames[p]['kps'])} matches {r.n_matches} good {r.n_good} "
              f"visited {r.visited} inliers {r.n_inliers} pnp {r.pnp_inliers}")
        assert np.array_equal(g["matches"], matches), f"{name} pair {p}: match list"
        assert (res[p]["n_good"], res[p]["visited"], res[p]["n_inliers"], res[p]["ransac_ok"]) == \
            (r.n_good, r.visited, r.n_inliers, r.ransac_ok), f"{name} pair {p}: RANSAC counts"
        O.check_ransac_inliers(g, r, f"{name} pair {p}")
        assert np.array_equal(res[p]["T12"], np.array(r.T12, np.float32)), f"{name} pair {p}: T12"
        assert res[p]["rmse"] == np.float32(r.rmse)
        assert (res[p]["n_sweeps"], res[p]["n_fit_points"]) == (r.n_sweeps, r.n_fit_points), f"{name} pair {p}: work"
        dT = np.abs(res[p]["Tcw"] - np.array(r.Tcw, np.float32)).max()
        assert dT < 1e-4, f"{name} pair {p}: PnP pose differs by {dT}"
        n2 = len(frames[p]["kps"])
        nb = O.check_pnp_flags(g["pnp_inliers"][:n2], mask, frames[p - 1], frames[p], g["f2_src"][:n2],
                               np.array(r.Tcw, np.float32).reshape(4, 4), cal, f"{name} pair {p}")
        assert abs(int(res[p]["pnp_inliers"]) - r.pnp_inliers) <= nb, f"{name} pair {p}: PnP inlier count"
    assert odo.latch == latch
    odo.close()
