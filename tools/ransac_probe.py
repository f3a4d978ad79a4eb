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
    for corrupt in (0.0, 0.2, 0.3, 0.5):
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
        print(f"corrupt {corrupt}: matches {nm} inliers {ni.value} ok {ok.value}", flush=True)
        if hasattr(lib, "odo_ransac_prof_read"):
            timeline(lib)


def timeline(lib):
    """Per-hypothesis records of a -DODO_RANSAC_PROFILE build (10 ns ticks)."""
    rec = np.zeros((500, 8), np.uint64)
    done = np.zeros(1, np.uint64)
    lib.odo_ransac_prof_read.restype = O.C.c_int
    lib.odo_ransac_prof_read(rec.ctypes.data_as(O.C.c_void_p), 500, done.ctypes.data_as(O.C.c_void_p))
    ok = rec[:, 0] > 0
    t0 = int(rec[ok, 0].min())
    us = lambda t: (int(t) - t0) / 100.0  # noqa: E731
    info = rec[:, 2]
    ab = (info >> np.uint64(8)) & np.uint64(1)
    print(f"  fold done at {us(done[0]):.1f} us; last end {us(rec[ok, 1].max()):.1f} us; "
          f"last exit {us(rec[ok, 7].max()):.1f} us; aborted {int(ab[ok].sum())} of {int(ok.sum())}")
    for h in range(min(32, 500)):
        if not ok[h]:
            continue
        r = rec[h]
        print(f"  h{h:3d} ab{int(ab[h])} nref{int(r[2]) & 255:2d} inl{(int(r[2]) >> 16) & 0xffffff:4d} "
              f"start {us(r[0]):6.1f} end {us(r[1]):6.1f} tfc {int(r[3]) / 100:6.1f} get {int(r[4]) / 100:5.1f} "
              f"sweep {int(r[5]) / 100:6.1f}")


if __name__ == "__main__":
    main()
