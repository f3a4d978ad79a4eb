"""Regenerate the committed golden fixtures (tests/golden/*.npz).

The reference ships no golden vectors, so these are made
by the CPU restatement (oracle/, the checker) on a seeded synthetic RGB-D pair
(adaptive-rgbd-localization-mappig_amd/synth.py, deterministic) and committed
as data: inputs are identified by their CRC32 and regenerated from the seed.
Run from the repo root:  python tests/golden/make_golden.py
"""
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from conftest import load_pkg, load_synth  # noqa: E402
import oracle_lib as O  # noqa: E402

SCENE_SEED = 0x5EED0002
W, H, NF, ITERS = 640, 480, 2000, 500
SEED_BASE = 0x5EED0000


def golden_inputs():
    bgr, dep, _ = load_synth().make_sequence(2, W, H, seed=SCENE_SEED)
    crc = [zlib.crc32(np.ascontiguousarray(bgr).tobytes()), zlib.crc32(np.ascontiguousarray(dep).tobytes())]
    return bgr, dep, crc


def main():
    pkg = load_pkg()
    bgr, dep, crc = golden_inputs()
    cal = O.fr1_calib()
    frames = [O.extract_frame(bgr[i], dep[i], O.orb_params(NF), cal) for i in range(2)]
    fx = {"input_crc32": np.array(crc, np.uint32), "params": np.array([W, H, NF, SCENE_SEED], np.int64)}
    for i, f in enumerate(frames):
        for k, v in f.items():
            fx[f"f{i}_{k}"] = v
    np.savez_compressed(os.path.join(HERE, "frames_640x480_2000.npz"), **fx)

    kx = {}
    for n in (1000, 2000):
        q, t = frames[0]["desc"][:n], frames[1]["desc"][:n]
        idx, dist = O.knn2(q, t)
        kx[f"q{n}"], kx[f"t{n}"], kx[f"idx{n}"], kx[f"dist{n}"] = q, t, idx, dist
    np.savez_compressed(os.path.join(HERE, "knn2_hamming.npz"), **kx)

    seed = pkg.pair_seed(SEED_BASE, 1)
    r, mask, matches, latch = O.track_pair(frames[0], frames[1], cal, O.ransac_params(ITERS), seed)
    np.savez_compressed(os.path.join(HERE, "pair_ransac_pnp.npz"), seed=np.array([seed], np.uint32),
                        iters=np.array([ITERS], np.int32), matches=matches, pnp_inlier_mask=mask,
                        T12=np.array(r.T12, np.float32), Tcw=np.array(r.Tcw, np.float32),
                        rmse=np.array([r.rmse], np.float32), ransac_inliers=r.inliers,
                        counts=np.array([r.n_matches, r.n_good, r.n_inliers, r.ransac_ok, r.pnp_inliers, r.visited],
                                        np.int32),
                        latch=np.array([latch], np.float64))
    print("written", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
