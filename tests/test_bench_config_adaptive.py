"""GPU parity of the ADAPTIVE bench legs (bench.py --detector adaptive /
adaptive-orb) in their pipelined configuration: device-resident batches back
to back with the default schedule (two pair streams taking alternate batches,
four frame sets in flight, the kNN-2 grid and RANSAC work list), five batches
so every frame set is reused. The per-cell detector thresholds carry from
frame to frame across all batches, so the oracle extracts every frame of the
run in order (extractor.cpp:39-77, videodynamicadaptedfeaturedetector.cpp:24-44)
and the last batch is compared:

* every frame's keypoints, descriptors, kun, xyz, uR and every cell's
  threshold: bit-exact; the persistent thresholds after the run: exact;
* every pair's match list, n_queries, RANSAC counts / T12 / rmse / inlier
  count: bit-exact; PnP pose within 1e-4; PnP flags as in
  test_bench_config_parity.py; the DepthCovariance latch: exact.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle_lib as O
from conftest import load_pkg, sequence
from test_adaptive_gpu import cal_of

pytestmark = pytest.mark.gpu

B, NB, L = 64, 5, 64


@pytest.mark.parametrize("inner", ["fast", "orb"])
def test_bench_configuration_adaptive(inner):
    import torch
    pkg = load_pkg()
    bgr, dep, _ = sequence(L, 640, 480, seed=0x5EED0002, closed_loop=True)
    det = pkg.DETECTOR_ADAPTIVE_ORB if inner == "orb" else pkg.DETECTOR_ADAPTIVE_FAST
    cfg = pkg.default_config(640, 480, B, nfeatures=1000, iterations=500, seed=0x5EED0000, detector=det)
    odo = pkg.Odometry(cfg)
    idx = np.arange(B) % L
    d_bgr = torch.from_numpy(np.ascontiguousarray(bgr[idx])).to("cuda")
    d_dep = torch.from_numpy(np.ascontiguousarray(dep[idx]).view(np.int16)).to("cuda")
    torch.cuda.synchronize()
    try:
        for _ in range(NB - 1):
            odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=False)
        res = odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=True)
        odo.synchronize()
        cal = cal_of(cfg)
        ex = O.AdaptiveExtractor(inner=inner)
        g0 = (NB - 1) * B
        frames, t_used = {}, {}
        for g in range(NB * B):
            if g >= g0:
                before = ex.thresh.copy()
                _, _, t = ex.extract_gray(O.gray(bgr[g % L]))
                ex.thresh[:] = before
                t_used[g] = t
            f = ex.extract_frame(bgr[g % L], dep[g % L], cal)
            if g <= 1 or g >= g0 - 1:
                frames[g] = f
        for i in range(B):
            got, ref = odo.frame(i), frames[g0 + i]
            tag = f"{inner} frame {g0 + i}"
            assert np.array_equal(odo.adaptive_state(i)[0], t_used[g0 + i]), f"{tag}: cell thresholds"
            assert len(got["kps"]) == len(ref["kps"]), f"{tag}: N"
            assert np.array_equal(got["kps"], ref["kps"]), f"{tag}: keypoints"
            assert np.array_equal(got["desc"], ref["desc"]), f"{tag}: descriptors"
            for fld in ("kun", "xyz", "ur"):
                assert np.array_equal(got[fld], ref[fld]), f"{tag}: {fld}"
        assert np.array_equal(odo.adaptive_state()[1], ex.thresh), f"{inner}: persistent thresholds"
        rp = O.ransac_params(500)
        _, _, _, latch = O.track_pair(frames[0], frames[1], cal, rp, pkg.pair_seed(cfg.seed, 1), float("nan"))

        def pair(p):
            g = g0 + p
            return O.track_pair(frames[g - 1], frames[g], cal, rp, pkg.pair_seed(cfg.seed, g), latch)

        with ThreadPoolExecutor(16) as pool:
            pairs = list(pool.map(pair, range(B)))
        for p in range(B):
            r, mask, matches, _ = pairs[p]
            g = odo.pair(p)
            tag = f"{inner} pair {p} (global {g0 + p})"
            assert np.array_equal(g["matches"], matches), f"{tag}: match list"
            assert res[p]["n_queries"] == r.n_queries, f"{tag}: kNN-2 query count"
            assert (res[p]["n_matches"], res[p]["n_good"], res[p]["visited"], res[p]["n_inliers"],
                    res[p]["ransac_ok"]) == (r.n_matches, r.n_good, r.visited, r.n_inliers, r.ransac_ok), \
                f"{tag}: RANSAC counts"
            O.check_ransac_inliers(g, r, tag)
            assert np.array_equal(res[p]["T12"], np.array(r.T12, np.float32)), f"{tag}: T12"
            assert res[p]["rmse"] == np.float32(r.rmse), f"{tag}: rmse"
            Tref = np.array(r.Tcw, np.float32).reshape(4, 4)
            assert np.abs(res[p]["Tcw"].reshape(4, 4) - Tref).max() < 1e-4, f"{tag}: PnP pose"
            f1, f2 = frames[g0 + p - 1], frames[g0 + p]
            n2 = len(f2["kps"])
            O.check_pnp_flags(g["pnp_inliers"][:n2], mask, f1, f2, g["f2_src"][:n2], Tref, cal, tag)
        assert odo.latch == latch, f"{inner}: latch"
    finally:
        odo.close()
