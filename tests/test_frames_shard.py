"""Frames mode host logic on CPU: chunk / halo coverage, the
latch broadcast and the cross-rank pose stitch over two gloo ranks.

The GPU half (two processes tracking one sequence, bit-equal to one rank) is
tests/test_frames_shard_gpu.py.
"""
import importlib.util
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "adaptive-rgbd-localization-mappig_amd")


def _fs():
    spec = importlib.util.spec_from_file_location("arlm_frames_shard", os.path.join(PKG_DIR, "frames_shard.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


PAIR_DTYPE = np.dtype([("T12", "<f4", 16), ("Tcw", "<f4", 16), ("rmse", "<f4"), ("n_matches", "<i4"),
                       ("n_good", "<i4"), ("n_inliers", "<i4"), ("ransac_ok", "<i4"), ("pnp_inliers", "<i4"),
                       ("visited", "<i4"), ("n_queries", "<i4"), ("n_sweeps", "<i4"), ("n_fit_points", "<i4")])


def _rel_poses(n, seed=3):
    """Random small SE(3) steps (relative Tcw per frame; frame 0 = I)."""
    rng = np.random.default_rng(seed)
    out = np.zeros((n, 4, 4))
    for i in range(n):
        w = rng.normal(size=3) * 0.02
        th = np.linalg.norm(w)
        K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
        R = np.eye(3) + np.sin(th) / th * K + (1 - np.cos(th)) / th ** 2 * K @ K
        out[i] = np.eye(4)
        out[i, :3, :3] = R
        out[i, :3, 3] = rng.normal(size=3) * 0.01
    out[0] = np.eye(4)
    return out.astype(np.float32)


@pytest.mark.parametrize("T,world,steps", [(8, 2, 3), (12, 3, 2), (256, 8, 2), (7, 2, 2)])
def test_chunks_cover_every_pair_once(T, world, steps):
    fs = _fs()
    pairs = []
    for k in range(steps):
        ends = []
        for r in range(world):
            first, n, halo = fs.batch_of(k, T, r, world)
            s, e = fs.chunk(k, T, r, world)
            ends.append((s, e))
            assert halo == (s > 0) and first == (s - 1 if halo else 0) and n == e - first
            # batch pair p is (first + p - 1, first + p): pairs of a halo batch start at p = 1
            pairs += [first + p for p in range(1 if halo else 1, n)]
        assert ends[0][0] == k * T and ends[-1][1] == (k + 1) * T
        assert all(ends[i][1] == ends[i + 1][0] for i in range(world - 1))
    assert sorted(pairs) == list(range(1, T * steps)), "every pair (f-1, f) tracked exactly once"


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _FakeOdo:
    """Duck-typed Odometry for the host logic: latch and seek only."""

    def __init__(self, rank):
        self.rank, self.latch, self.seeks = rank, float("nan"), []

    def seek(self, i, keep_prev=False):
        self.seeks.append((i, keep_prev))

    def track_batch(self, a, b, n, want_results=True):
        self.latch = 1.25e-4 if self.rank == 0 else 9.0  # only rank 0 tracks the priming pair

    def set_latch(self, v):
        self.latch = v


def _worker(rank, world, port, T, steps, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        fs = _fs()
        odo = _FakeOdo(rank)
        sh = fs.FramesShard(odo, dist, rank, world, T, device="cpu")
        latch = sh.prime_latch(0, 0)
        rel = _rel_poses(T * steps)
        step_res = []
        for k in range(steps):
            first, n, halo = fs.batch_of(k, T, rank, world)
            res = np.zeros(n, PAIR_DTYPE)
            # batch frame i is global frame first + i; its record holds the pair
            # (first + i - 1, first + i): relative pose rel[first + i]
            res["Tcw"] = rel[first:first + n].reshape(n, 16)
            step_res.append(res)
        G = sh.stitch(step_res, list(range(steps)))
        out.put((rank, latch, odo.latch, [g.copy() for g in G]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,T,steps", [(2, 8, 3), (3, 12, 2)])
def test_latch_broadcast_and_pose_stitch(world, T, steps):
    fs = _fs()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, T, steps, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # sequential chain over the whole sequence (Tcw(f) = rel(f) Tcw(f-1), float64)
    rel = _rel_poses(T * steps).astype(np.float64)
    seq = np.zeros_like(rel)
    G = np.eye(4)
    for f in range(T * steps):
        G = rel[f] @ G
        seq[f] = G
    for rank, latch, odo_latch, Gs in got:
        assert latch == 1.25e-4 and odo_latch == 1.25e-4, "every rank uses rank 0's latch"
        for k in range(steps):
            s, e = fs.chunk(k, T, rank, world)
            assert Gs[k].shape == (e - s, 4, 4)
            assert np.abs(Gs[k] - seq[s:e]).max() < 1e-6, f"rank {rank} step {k}: stitched poses"
