"""Trajectory of the batched odometry.

* chain_poses: relative poses of odo_track_batch -> absolute Tcw per frame
  (odo_chain_poses, the batched contract's host prefix product,
  Odometry::Compute's Tcw2 = T12 * Tcw1, odometry.cpp:110-112);
* write_tum: Tracking::SaveTrajectory's TUM line format
  (odo_write_tum_trajectory, tracking.cpp:544-582);
* ate_rmse: absolute trajectory error as the TUM benchmark's evaluate_ate
  defines it (rigid Horn/Umeyama alignment of the camera centres, RMSE of the
  translational residuals), for checking the GPU path against ground truth.
"""
from __future__ import annotations

import numpy as np

from ._abi import PAIR_DTYPE, check, load, ptr


def chain_poses(results: np.ndarray, Tcw_prev=None) -> np.ndarray:
    res = np.ascontiguousarray(results, PAIR_DTYPE)
    out = np.zeros((res.size, 16), np.float32)
    prev = None if Tcw_prev is None else np.ascontiguousarray(np.asarray(Tcw_prev, np.float32).ravel())
    check(load().odo_chain_poses(ptr(res), res.size, ptr(prev) if prev is not None else None, ptr(out)))
    return out.reshape(-1, 4, 4)


def write_tum(path: str, timestamps, Tcw: np.ndarray, append: bool = False):
    ts = np.ascontiguousarray(timestamps, np.float64)
    T = np.ascontiguousarray(np.asarray(Tcw, np.float32).reshape(-1, 16))
    check(load().odo_write_tum_trajectory(path.encode(), ptr(ts), ptr(T), ts.size, 1 if append else 0))


def camera_centres(Tcw: np.ndarray) -> np.ndarray:
    T = np.asarray(Tcw, np.float64).reshape(-1, 4, 4)
    return -np.einsum("nji,nj->ni", T[:, :3, :3], T[:, :3, 3])


def ate_rmse(est_xyz: np.ndarray, gt_xyz: np.ndarray) -> float:
    """RMSE after the rigid alignment gt ~ R est + t (Horn / Umeyama, no scale)."""
    a = np.asarray(est_xyz, np.float64)
    b = np.asarray(gt_xyz, np.float64)
    ma, mb = a.mean(0), b.mean(0)
    H = (a - ma).T @ (b - mb)
    U, _, Vt = np.linalg.svd(H)
    S = np.eye(3)
    if np.linalg.det(Vt.T @ U.T) < 0:
        S[2, 2] = -1
    R = Vt.T @ S @ U.T
    t = mb - R @ ma
    r = b - (a @ R.T + t)
    return float(np.sqrt((r * r).sum(1).mean()))
