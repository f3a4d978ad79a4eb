"""Frames mode on the GPU: two processes (gloo for the exchange,
both on cuda:0) track one sequence as rank chunks with a one-frame halo, the
latch taken from global pair 1 and broadcast, the poses stitched with an
all_gather of the chunk products. Every pair record must equal the one-rank
batched run of the same frames bit for bit (matches, RANSAC, PnP, counts); the
stitched absolute poses match the one-rank pose chain within 1e-5. The
from-host form (each rank uploads its chunk + halo from pinned host memory,
odo_track_batch_host_async, as bench.py's from_host leg) is held to the same
bar.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_pkg, sequence

pytestmark = pytest.mark.gpu

T, STEPS, NF, ITERS, SEED = 8, 2, 1000, 300, 0x5EED0E00


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _device_frames(bgr, dep):
    import torch
    return (torch.from_numpy(np.ascontiguousarray(bgr)).to("cuda"),
            torch.from_numpy(np.ascontiguousarray(dep).view(np.int16)).to("cuda"))


def _worker(rank, world, port, out, host):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import torch
        pkg = load_pkg()
        from arlm_amd import frames_shard as fs
        bgr, dep, _ = sequence(T * STEPS, seed=0x5EED0002)
        C = T // world
        cfg = pkg.default_config(640, 480, C + 1, nfeatures=NF, iterations=ITERS, seed=SEED)
        odo = pkg.Odometry(cfg)
        sh = fs.FramesShard(odo, dist, rank, world, T, device="cpu")
        b01, d01 = _device_frames(bgr[:2], dep[:2])
        torch.cuda.synchronize()
        latch = sh.prime_latch(b01.data_ptr(), d01.data_ptr())
        ring = pkg.PinnedResults(STEPS, C + 1)
        bufs, recs = [], []
        fb = (640 * 480 * 3, 640 * 480 * 2)
        for k in range(STEPS):
            first, n, halo = fs.batch_of(k, T, rank, world)
            lo = first if halo else 0
            fb_ = bgr[lo:lo + n] if halo else np.concatenate([bgr[:1], bgr[:n]])
            fd_ = dep[lo:lo + n] if halo else np.concatenate([dep[:1], dep[:n]])
            if host:
                hf = pkg.HostFrames(fb_.shape[0], 640, 480)
                hf.bgr[:], hf.depth[:] = fb_, fd_
                bufs.append(hf)
                sh.track_step_host(k, hf, ring, k)
                continue
            b, d = _device_frames(fb_, fd_)
            torch.cuda.synchronize()
            bufs.append((b, d))
            sh.track_step(k, b.data_ptr(), d.data_ptr(), fb, results=ring, row=k)
        odo.synchronize()
        for k in range(STEPS):
            first, n, halo = fs.batch_of(k, T, rank, world)
            recs.append((first, halo, ring.all[k][:n].copy()))
        G = sh.stitch([r[2] for r in recs], list(range(STEPS)))
        out.put((rank, latch, recs, [g.copy() for g in G]))
        ring.close()
        odo.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("host", [False, True], ids=["device_inputs", "host_inputs"])
def test_two_ranks_equal_one_rank(host):
    pkg = load_pkg()
    import torch
    from arlm_amd import trajectory as tj
    bgr, dep, _ = sequence(T * STEPS, seed=0x5EED0002)
    # one rank: the whole sequence as one batch (pair f = (f-1, f), seed index f)
    cfg = pkg.default_config(640, 480, T * STEPS, nfeatures=NF, iterations=ITERS, seed=SEED)
    odo = pkg.Odometry(cfg)
    b, d = _device_frames(bgr, dep)
    torch.cuda.synchronize()
    ref = odo.track_batch(b.data_ptr(), d.data_ptr(), T * STEPS, want_results=True)
    ref_latch = odo.latch
    ref_G = tj.chain_poses(ref)
    odo.close()

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, host)) for r in range(world)]
    for p in procs:
        p.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    from arlm_amd import frames_shard as fs
    seen = set()
    for rank, latch, recs, Gs in got:
        assert latch == ref_latch, f"rank {rank}: latch {latch} vs {ref_latch}"
        for k, (first, halo, res) in enumerate(recs):
            s, e = fs.chunk(k, T, rank, world)
            for i in range(1 if halo else 1, len(res)):
                f = first + i  # pair (f - 1, f)
                seen.add(f)
                for fld in ("T12", "Tcw", "rmse", "n_matches", "n_good", "n_inliers", "ransac_ok", "pnp_inliers",
                            "visited", "n_queries", "n_sweeps", "n_fit_points"):
                    assert np.array_equal(res[i][fld], ref[f][fld]), f"rank {rank} pair {f}: {fld}"
            dG = np.abs(Gs[k] - ref_G[s:e]).max()
            assert dG < 1e-5, f"rank {rank} step {k}: stitched pose off by {dG}"
    assert seen == set(range(1, T * STEPS)), "every pair tracked once"
