"""The N>1 path of bench.py on CPU: two ranks over gloo (127.0.0.1).

bench.py shards whole sequences across ranks (frames mode, weak scaling): each
rank tracks its own scene with its own RANSAC seed stream, there is no
data-path collective, and the only cross-rank step is the MAX of the timed
region. These tests run that host logic in two processes with the gloo
backend (the GPU box uses RCCL through the same calls).
"""
import importlib.util
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load_bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bench = _load_bench()
        pkg = bench.load_pkg()
        synth = bench.load_synth()
        scene_seed, pair_seed = bench.rank_seeds(rank)
        # each rank's shard: its own small sequence and its own per-pair seed stream
        bgr, dep, _ = synth.make_sequence(2, 160, 120, seed=scene_seed, closed_loop=True)
        digest = float(np.asarray(bgr, np.float64).sum() + np.asarray(dep, np.float64).sum())
        seeds = [pkg.pair_seed(pair_seed, p) for p in range(4)]
        # the job clock: the slowest rank's timed region
        elapsed = bench.max_over_ranks(1.0 + 0.5 * rank, dist, world, device="cpu")
        value = bench.job_throughput(64, 10, world, elapsed)
        gathered = [None] * world
        dist.all_gather_object(gathered, {"rank": rank, "scene": scene_seed, "digest": digest, "seeds": seeds,
                                          "elapsed": elapsed, "value": value})
        if rank == 0:
            out.put(gathered)
    finally:
        dist.destroy_process_group()


@pytest.fixture(scope="module")
def two_ranks():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def test_ranks_track_disjoint_shards(two_ranks):
    a, b = two_ranks
    assert a["scene"] != b["scene"], "each rank must track its own sequence"
    assert a["digest"] != b["digest"], "the rank shards hold different frames"
    assert not set(a["seeds"]) & set(b["seeds"]), "RANSAC seed streams must not collide across ranks"


def test_job_time_is_max_over_ranks(two_ranks):
    for r in two_ranks:
        assert r["elapsed"] == pytest.approx(1.5), "every rank sees the slowest rank's time"
        # whole-job throughput: 64 frames x 10 steps x 2 ranks over the slowest rank's time
        assert r["value"] == pytest.approx(64 * 10 * 2 / 1.5)


def test_single_rank_needs_no_collective():
    bench = _load_bench()
    assert bench.max_over_ranks(2.5, None, 1) == 2.5
    assert bench.job_throughput(64, 40, 1, 2.0) == pytest.approx(1280.0)
