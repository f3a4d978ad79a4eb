"""Per-wave timeline of k_ransac_lanes on the hard workload (a
-DODO_LANES_PROFILE build named by ODO_LIB): rounds, active lanes, TFC /
sweep / fold time per wave of the last launch. Usage: ODO_LIB=... python
tools/lanes_probe.py [batches]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_pkg, load_synth  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    pkg = load_pkg()
    synth = load_synth()
    bgr, dep, _ = synth.make_sequence(64, 640, 480, seed=0x5EED0002, closed_loop=True, hard=True)
    B = 256
    bgr = np.ascontiguousarray(np.tile(bgr, (B // 64, 1, 1, 1)))
    dep = np.ascontiguousarray(np.tile(dep, (B // 64, 1, 1)))
    cfg = pkg.default_config(640, 480, B, nfeatures=2000, iterations=500)
    odo = pkg.Odometry(cfg)
    for _ in range(nb):
        res = odo.track_batch_host(bgr, dep)
    lib = pkg.load()
    import ctypes as C
    rec = np.zeros((4096, 10), np.uint64)
    f = lib.odo_lanes_prof_read
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_int]
    n = f(rec.ctypes.data, 4096)
    ok = rec[:, 1] > 0
    r = rec[ok].astype(np.float64)
    t0 = r[:, 0].min()
    dur = (r[:, 1] - r[:, 0]) / 100.0
    out = {"waves": int(ok.sum()), "span_us": float((r[:, 1].max() - t0) / 100.0),
           "start_us": np.percentile((r[:, 0] - t0) / 100.0, [0, 50, 100]).round(1).tolist(),
           "dur_us_p": np.percentile(dur, [0, 10, 50, 90, 100]).round(1).tolist(),
           "rounds_p": np.percentile(r[:, 2], [0, 50, 90, 100]).tolist(),
           "mean_active_per_round": float((r[:, 3] / np.maximum(r[:, 2], 1)).mean()),
           "tfc_us_mean": float((r[:, 4] / 100.0).mean()), "sweep_us_mean": float((r[:, 5] / 100.0).mean()),
           "sweep_inner_us_mean": float((r[:, 6] / 100.0).mean()),
           "sweep_sum_us_mean": float((r[:, 7] / 100.0).mean()),
           # LN_COMPACT builds: pairs tested by the shortcut, pairs fully evaluated
           "shortcut_pairs": float(r[:, 8].sum()), "full_evals": float(r[:, 9].sum()),
           "visited_mean": float(np.mean(res["visited"][1:])), "sweeps_mean": float(np.mean(res["n_sweeps"][1:]))}
    # the slowest waves
    idx = np.argsort(-dur)[:8]
    out["slowest"] = [{"dur_us": round(float(dur[i]), 1), "rounds": int(r[i, 2]), "act": int(r[i, 3]),
                       "tfc_us": round(float(r[i, 4] / 100), 1), "sweep_us": round(float(r[i, 5] / 100), 1),
                       "inner_us": round(float(r[i, 6] / 100), 1), "sum_us": round(float(r[i, 7] / 100), 1)}
                      for i in idx]
    print(json.dumps(out, indent=1))
    odo.close()


if __name__ == "__main__":
    main()
