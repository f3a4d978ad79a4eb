"""FAST candidates and octree survivors per pyramid level of one bench frame."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    import torch
    pkg, synth = bench.load_pkg(), bench.load_synth()
    B = 4
    bgr, dep, _ = synth.make_sequence(B, 640, 480, seed=bench.shard_seed(0), closed_loop=True)
    cfg = pkg.default_config(640, 480, B, nfeatures=2000, iterations=500, seed=0x5EED0000)
    odo = pkg.Odometry(cfg, device=0)
    d_bgr = torch.from_numpy(bgr).cuda()
    d_dep = torch.from_numpy(dep.view(np.int16)).cuda()
    odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=True)
    for i in range(B):
        fast = [len(odo.debug_fast(i, l)) for l in range(8)]
        octo = [len(odo.debug_octree(i, l)) for l in range(8)]
        print(f"frame {i}: fast {fast} total {sum(fast)}; octree {octo} total {sum(octo)}")


if __name__ == "__main__":
    main()
