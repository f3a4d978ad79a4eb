"""Per-level timeline of k_pyramid (a -DODO_PYR_PROFILE build named by
ODO_LIB): for every frame workgroup of the last launch, the ticks at its
start, after gray, after each level's barrier and at its end. Prints the
per-phase durations (mean / p10 / p50 / p90 over the frames), the workgroups'
start spread and the launch span. Usage: ODO_LIB=... python tools/pyr_probe.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import load_pkg, load_synth  # noqa: E402


def main():
    import ctypes as C

    import torch
    pkg = load_pkg()
    synth = load_synth()
    B = 256
    bgr, dep, _ = synth.make_sequence(64, 640, 480, seed=0x5EED0002, closed_loop=True)
    idx = np.arange(B) % 64
    d_bgr = torch.from_numpy(np.ascontiguousarray(bgr[idx])).to("cuda")
    d_dep = torch.from_numpy(np.ascontiguousarray(dep[idx]).view(np.int16)).to("cuda")
    odo = pkg.Odometry(pkg.default_config(640, 480, B, nfeatures=2000, iterations=500))
    for _ in range(4):
        odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=False)
    odo.synchronize()
    lib = pkg.load()
    f = lib.odo_pyr_prof_read
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_int]
    rec = np.zeros((1024, 20), np.uint64)
    n = f(rec.ctypes.data, 1024)
    nl = 8
    r = rec[:B, :nl + 2].astype(np.float64) / 100.0  # us
    t0 = r[:, 0].min()
    phases = {"gray": r[:, 1] - r[:, 0]}
    for l in range(1, nl):
        phases[f"blur{l - 1}+resize{l}"] = r[:, l + 1] - r[:, l]
    phases[f"blur{nl - 1}"] = r[:, nl + 1] - r[:, nl]
    out = {"frames": int(n), "span_us": round(float(r[:, nl + 1].max() - t0), 1),
           "start_us_p": np.percentile(r[:, 0] - t0, [0, 50, 100]).round(1).tolist(),
           "frame_us_p": np.percentile(r[:, nl + 1] - r[:, 0], [0, 10, 50, 90, 100]).round(1).tolist(),
           "phase_us": {k: {"mean": round(float(v.mean()), 2),
                            "p10_50_90": np.percentile(v, [10, 50, 90]).round(2).tolist()} for k, v in phases.items()}}
    print(json.dumps(out, indent=1))
    odo.close()


if __name__ == "__main__":
    main()
