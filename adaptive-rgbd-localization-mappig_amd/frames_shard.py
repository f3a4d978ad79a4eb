"""Frames mode of the batched path over ranks.

One sequence, T frames per step. Rank r of R tracks the contiguous chunk
[s_r, e_r) of every step, s_r = step*T + T*r//R, plus a one-frame halo: it
also extracts frame s_r - 1 (cheaper than shipping its descriptors over xGMI),
so its pairs are (s_r - 1, s_r) ... (e_r - 2, e_r - 1). Every pair of the
sequence is tracked by exactly one rank, with its global pair index as its
RANSAC seed index (odo_seek), so the pair results do not depend on R.

The reference's cross-frame state, made explicit:

* DepthCovariance latch (ransac.cpp:416-421): taken from the first valid pair
  of the sequence (global pair 1, frames 0 and 1, on rank 0) and broadcast
  once before the first step (prime_latch);
* pose chain (odometry.cpp:108-112, Tcw2 = T12 * Tcw1): PnP is solved in the
  previous camera frame, each rank chains its chunk's relative poses, and an
  all_gather of the chunk products (64 B per rank and step) plus a prefix
  product gives every frame's absolute Tcw (stitch).

The ADAPTIVE detector's per-cell thresholds carry from frame to frame, so that
mode is not frame-shardable (replicas or per-sequence sharding only).
"""
from __future__ import annotations

import numpy as np


def chunk(step: int, frames_per_step: int, rank: int, world: int):
    """Global frame range [s, e) of one rank in one step."""
    base = step * frames_per_step
    return base + frames_per_step * rank // world, base + frames_per_step * (rank + 1) // world


def batch_of(step: int, frames_per_step: int, rank: int, world: int):
    """(first global frame, frame count, halo) of the rank's batch: the halo is
    the frame before the chunk (extracted, no pair); global frame 0 has none."""
    s, e = chunk(step, frames_per_step, rank, world)
    if s == 0:
        return 0, e - s, False
    return s - 1, e - s + 1, True


def chunk_relative_poses(results: np.ndarray, first: int, halo: bool) -> np.ndarray:
    """Relative Tcw (previous camera -> this camera) of every frame of the chunk
    from the batch's result records; global frame 0 gets the identity."""
    rel = results["Tcw"].reshape(-1, 4, 4).astype(np.float64)
    if halo:
        return rel[1:]
    out = rel.copy()
    if first == 0:
        out[0] = np.eye(4)
    return out


def local_chain(rel: np.ndarray) -> np.ndarray:
    """Local(f) = rel(f) * Local(f-1), Local(s-1) = I (double)."""
    out = np.empty_like(rel)
    T = np.eye(4)
    for i in range(rel.shape[0]):
        T = rel[i] @ T
        out[i] = T
    return out


def prefix_poses(chunk_products: np.ndarray, G_start: np.ndarray) -> np.ndarray:
    """chunk_products [steps, world, 4, 4] (every rank's chunk product L, in
    chunk order) -> the absolute pose of the frame before each chunk,
    [steps, world, 4, 4]: G_before(k, r) = L(k, r-1) ... L(k, 0) G_end(k-1)."""
    K, R = chunk_products.shape[:2]
    out = np.empty_like(chunk_products)
    G = np.asarray(G_start, np.float64)
    for k in range(K):
        for r in range(R):
            out[k, r] = G
            G = chunk_products[k, r] @ G
    return out


class FramesShard:
    """Drives one rank's Odometry context in frames mode."""

    def __init__(self, odo, dist, rank: int, world: int, frames_per_step: int, device: str = "cuda"):
        self.odo, self.dist, self.rank, self.world = odo, dist, rank, world
        self.T, self.device = frames_per_step, device

    def prime_latch(self, bgr01_ptr: int, dep01_ptr: int) -> float:
        """Rank 0 tracks global frames 0 and 1 (device pointers to the two
        frames back to back) for the latch; every rank receives it."""
        import torch
        v = float("nan")
        if self.rank == 0:
            self.odo.seek(0, keep_prev=False)
            self.odo.track_batch(bgr01_ptr, dep01_ptr, 2, want_results=True)
            v = self.odo.latch
        if self.world > 1:
            t = torch.tensor([v], dtype=torch.float64, device=self.device)
            self.dist.broadcast(t, 0)
            v = float(t.item())
        self.odo.set_latch(v)
        return v

    def track_step(self, step: int, bgr_ptr: int, dep_ptr: int, frame_bytes: tuple, results=None, row: int = 0):
        """Queue this rank's batch of the step. bgr_ptr / dep_ptr point at the
        halo frame followed by the chunk's frames; without a halo (global frame
        0) the chunk starts one frame later. Returns (first, n, halo)."""
        first, n, halo = batch_of(step, self.T, self.rank, self.world)
        if not halo:
            bgr_ptr += frame_bytes[0]
            dep_ptr += frame_bytes[1]
        self.odo.seek(first, keep_prev=False)
        if results is not None:
            self.odo.track_batch_async(bgr_ptr, dep_ptr, n, results, row)
        else:
            self.odo.track_batch(bgr_ptr, dep_ptr, n, want_results=False)
        return first, n, halo

    def track_step_host(self, step: int, hf, results, row: int):
        """track_step from pinned host memory (SURVEY §8(d)'s unit): hf is a
        HostFrames holding the halo frame followed by the chunk's frames (as
        track_step's pointers); this rank uploads them over its own PCIe link
        (odo_track_batch_host_async) and the records stream to results.all[row].
        Returns (first, n, halo)."""
        first, n, halo = batch_of(step, self.T, self.rank, self.world)
        self.odo.seek(first, keep_prev=False)
        self.odo.track_batch_host_async(hf, results, row, n=n, first=0 if halo else 1)
        return first, n, halo

    def stitch(self, step_results: list, steps: list, G_start=None) -> list:
        """Absolute Tcw of this rank's frames for each of `steps` (their result
        records in step_results): local chains, one all_gather of the chunk
        products (K x 16 doubles), prefix product. Returns [K][C, 4, 4] float32."""
        import torch
        locs, prods = [], np.zeros((len(steps), 16), np.float64)
        for i, (k, res) in enumerate(zip(steps, step_results)):
            first, n, halo = batch_of(k, self.T, self.rank, self.world)
            L = local_chain(chunk_relative_poses(res[:n], first, halo))
            locs.append(L)
            prods[i] = L[-1].ravel()
        if self.world > 1:
            t = torch.from_numpy(prods).to(self.device)
            outs = [torch.empty_like(t) for _ in range(self.world)]
            self.dist.all_gather(outs, t)
            allp = np.stack([o.cpu().numpy() for o in outs], 1)  # [K, R, 16]
        else:
            allp = prods[:, None, :]
        G0 = np.eye(4) if G_start is None else np.asarray(G_start, np.float64)
        before = prefix_poses(allp.reshape(len(steps), self.world, 4, 4), G0)
        return [(L @ before[i, self.rank]).astype(np.float32) for i, L in enumerate(locs)]
