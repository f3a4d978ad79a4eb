"""Phase times of k_pnp on a few pairs (a -DODO_PNP_PROFILE build named by
ODO_LIB prints build / solve / chi / classify ticks per pair), at the latency
path's 1000 features and the batch path's 2000. Usage: ODO_LIB=... python
tools/pnp_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_pkg, load_synth  # noqa: E402


def main():
    pkg = load_pkg()
    synth = load_synth()
    nfr = int(os.environ.get("PNP_PROBE_FRAMES", "4"))
    bgr, dep, _ = synth.make_sequence(nfr, 640, 480, seed=0x5EED0002, closed_loop=True)
    for nf in (1000, 2000):
        cfg = pkg.default_config(640, 480, nfr, nfeatures=nf, iterations=500)
        odo = pkg.Odometry(cfg)
        print(f"nfeatures {nf}", flush=True)
        res = odo.track_batch_host(bgr, dep)
        odo.synchronize()
        print("pnp_inliers", [int(r["pnp_inliers"]) for r in res], flush=True)
        odo.close()


if __name__ == "__main__":
    main()
