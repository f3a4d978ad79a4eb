"""Runs odo_ransac on a hard (corrupted-match) pair, optionally with an
instrumented library build (argv[1]); used to time RANSAC phases on the GPU."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_lib as O  # noqa: E402
from conftest import load_pkg  # noqa: E402
import test_gpu_parity as T  # noqa: E402


def main():
    pkg = load_pkg()
    lib = pkg._abi.load(sys.argv[1]) if len(sys.argv) > 1 else pkg.load()
    bgr, dep, cal, frames = T._frames_cfg1()
    f1, f2 = frames[0], frames[1]
    n1, n2 = len(f1["kps"]), len(f2["kps"])
    has = np.zeros(n1, np.uint8)
    O.lib().oracle_vo_landmarks(O.ptr(f1["xyz"]), n1, 40 * 40 / 517.3, O.ptr(has))
    m0 = np.zeros(n1, O.DMATCH_DTYPE)
    nm = O.lib().oracle_knn_match(O.ptr(f1["desc"]), n1, O.ptr(f2["desc"]), n2, 0.9, O.ptr(has),
                                  O.ptr(np.zeros(n1, np.uint8)), O.ptr(np.zeros(n1, np.int32)),
                                  O.ptr(np.full(n2, -1, np.int32)), O.ptr(np.full(n2, -1, np.int32)),
                                  O.ptr(np.zeros(n2, np.uint8)), O.ptr(m0), n1)
    odo, _ = T.make_odo(pkg, 640, 480, 1000, 500, 1)
    for corrupt in (0.3, 0.5):
        m = m0[:nm].copy()
        rs = np.random.default_rng(1)
        sel = rs.random(nm) < corrupt
        m["trainIdx"][sel] = rs.integers(0, n2, int(sel.sum()))
        r = pkg.Rng()
        lib.odo_rng_seed(pkg.ptr(r), 777)
        lat = O.C.c_double(float("nan"))
        Tm = np.zeros(16, np.float32)
        rmse = O.C.c_float(0)
        inl = np.zeros(nm, O.DMATCH_DTYPE)
        ni, ok = O.C.c_int(0), O.C.c_int(0)
        rp = pkg.RansacParams(500, 20, 3.0, 4, 1)
        pkg.check(lib.odo_ransac(odo.h, pkg.ptr(m), nm, pkg.ptr(f1["xyz"]), n1, pkg.ptr(f2["xyz"]), n2,
                                 pkg.ptr(rp), pkg.ptr(r), O.C.byref(lat), pkg.ptr(Tm), O.C.byref(rmse),
                                 pkg.ptr(inl), O.C.byref(ni), O.C.byref(ok)))
        print(f"corrupt {corrupt}: inliers {ni.value} ok {ok.value}", flush=True)


if __name__ == "__main__":
    main()
