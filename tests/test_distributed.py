"""The N>1 host logic of bench.py on CPU: two ranks over gloo (127.0.0.1).

bench.py's default N > 1 mode is SURVEY §8(e) frames mode (frames_shard.py,
tested in test_frames_shard*.py): one sequence split into per-rank chunks,
with a latch broadcast before the first step and one pose all_gather per run.
`--shard independent` gives every rank its own scene and RANSAC seed stream
with no data-path exchange. In both, the job clock is the MAX over ranks of
the timed region. These tests run that host logic in two processes with the
gloo backend (the GPU box uses RCCL through the same calls), and check the
launcher that `bench.py --gpus N` uses when no WORLD_SIZE is set.
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


def test_rank_envs_distinct_local_ranks():
    """--gpus N without a launcher: N workers, each with its own RANK /
    LOCAL_RANK (= its device) and the same WORLD_SIZE and rendezvous."""
    bench = _load_bench()
    envs = bench.rank_envs(4, 29555, base={"PATH": "/usr/bin"})
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert {e["WORLD_SIZE"] for e in envs} == {"4"}
    assert {(e["MASTER_ADDR"], e["MASTER_PORT"]) for e in envs} == {("127.0.0.1", "29555")}
    assert all(e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/usr/bin" for e in envs)


def test_launch_ranks_runs_n_workers(tmp_path):
    """launch_ranks starts N child processes (no exec) that rendezvous over
    gloo and see distinct ranks; a failing rank's exit code is returned."""
    bench = _load_bench()
    out = tmp_path / "ranks"
    out.mkdir()
    script = tmp_path / "worker.py"
    script.write_text(
        "import os, sys\n"
        "import torch.distributed as dist\n"
        "dist.init_process_group('gloo')\n"
        "r = dist.get_rank()\n"
        "open(os.path.join(sys.argv[1], str(r)), 'w').write(os.environ['LOCAL_RANK'] + ' ' + str(dist.get_world_size()))\n"
        "dist.barrier()\n"
        "dist.destroy_process_group()\n")
    assert bench.launch_ranks(3, [str(out)], script=str(script)) == 0
    got = sorted(p.read_text() for p in out.iterdir())
    assert got == ["0 3", "1 3", "2 3"]
    bad = tmp_path / "bad.py"
    bad.write_text("import os, sys\nsys.exit(3 if os.environ['RANK'] == '1' else 0)\n")
    assert bench.launch_ranks(2, [], script=str(bad)) == 3


def test_launch_ranks_stdout_is_the_json_line(tmp_path, capfd):
    """Only rank 0's JSON line reaches stdout; other output of any rank (a
    process group's connection notices, ...) goes to stderr."""
    bench = _load_bench()
    script = tmp_path / "noisy.py"
    script.write_text(
        "import os\n"
        "r = os.environ['RANK']\n"
        "print('[notice] rank', r, 'connected', flush=True)\n"
        "if r == '0':\n"
        "    print('{\"metric\": \"m\", \"value\": 1}', flush=True)\n")
    assert bench.launch_ranks(2, [], script=str(script)) == 0
    out, err = capfd.readouterr()
    assert out.strip().splitlines() == ['{"metric": "m", "value": 1}']
    assert err.count("[notice] rank") == 2
