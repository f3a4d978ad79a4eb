"""Per-pair RANSAC/PnP statistics of the bench workload (second batch, so
pair 0 links the previous batch's last frame)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    pkg, synth = bench.load_pkg(), bench.load_synth()
    if len(sys.argv) > 1:
        pkg._abi.load(sys.argv[1])  # e.g. an instrumented build
    B = 64
    bgr, dep, _ = synth.make_sequence(B, 640, 480, seed=bench.shard_seed(0), closed_loop=True)
    cfg = pkg.default_config(640, 480, B, nfeatures=2000, iterations=500, seed=0x5EED0000)
    odo = pkg.Odometry(cfg, device=0)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(dep.view(np.int16)).cuda()
    odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=True)
    res = odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=True)
    for p in range(B):
        r = res[p]
        print(f"pair {p:2d} matches {r['n_matches']:4d} good {r['n_good']:4d} visited {r['visited']:3d} "
              f"inl {r['n_inliers']:4d} ({r['n_inliers'] / max(r['n_good'], 1):.2f}) pnp {r['pnp_inliers']:4d}")
    v = res["visited"]
    print("visited: mean", v.mean(), "max", v.max(), "hist", np.histogram(v, [0, 2, 4, 8, 16, 32, 64, 128, 501])[0])


if __name__ == "__main__":
    main()
