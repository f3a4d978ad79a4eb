"""Hypotheses mode on the GPU: odo_ransac_hyps over disjoint
hypothesis ranges + the ordered fold + odo_ransac_hyps_finish reproduce
odo_ransac (= Ransac::Iterate) bit for bit: T12, rmse, inlier list, ok, and
the rand() state after exactly the visited draws on every rank. Ranks are
separate contexts in one process, and two processes on the box's GPU that
exchange summaries over gloo through hyp_shard.sharded_ransac.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O
from conftest import load_pkg
from test_hyp_shard import _problem

pytestmark = pytest.mark.gpu


def _reference(pkg, odo, m, x1, x2, iters, seed):
    lib = pkg.load()
    rng = pkg.Rng()
    lib.odo_rng_seed(pkg.ptr(rng), seed)
    lat = O.C.c_double(float("nan"))
    T = np.zeros(16, np.float32)
    rmse = O.C.c_float(0)
    inl = np.zeros(max(m.size, 1), pkg.DMATCH_DTYPE)
    ni, ok = O.C.c_int(0), O.C.c_int(0)
    pkg.check(lib.odo_ransac(odo.h, pkg.ptr(m), m.size, pkg.ptr(x1), x1.shape[0], pkg.ptr(x2), x2.shape[0],
                             pkg.ptr(pkg.RansacParams(iters, 20, 3.0, 4, 1)), pkg.ptr(rng), O.C.byref(lat),
                             pkg.ptr(T), O.C.byref(rmse), pkg.ptr(inl), O.C.byref(ni), O.C.byref(ok)))
    return dict(T=T, rmse=rmse.value, inliers=inl[:ni.value], ok=ok.value, rng=bytes(rng), latch=lat.value)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("corrupt,iters", [(0.0, 500), (0.5, 4096), (0.75, 1000)])
def test_virtual_ranks_reproduce_iterate(world, corrupt, iters):
    pkg = load_pkg()
    from arlm_amd import hyp_shard
    lib = pkg.load()
    m, x1, x2, _ = _problem(corrupt, iters)
    x1 = np.ascontiguousarray(x1)
    x2 = np.ascontiguousarray(x2)
    ctxs = [pkg.Odometry(pkg.default_config(640, 480, 1, nfeatures=1000, iterations=iters)) for _ in range(world)]
    ref = _reference(pkg, ctxs[0], m, x1, x2, iters, 99)
    params = pkg.RansacParams(iters, 20, 3.0, 4, 1)
    allh = np.zeros(iters, pkg._abi.HYP_DTYPE)
    ng = O.C.c_int(0)
    for r, odo in enumerate(ctxs):
        h0, h1 = hyp_shard.shard_range(iters, r, world)
        rng = pkg.Rng()
        lib.odo_rng_seed(pkg.ptr(rng), 99)
        lat = O.C.c_double(float("nan"))
        loc = np.zeros(max(h1 - h0, 1), pkg._abi.HYP_DTYPE)
        pkg.check(lib.odo_ransac_hyps(odo.h, pkg.ptr(m), m.size, pkg.ptr(x1), x1.shape[0], pkg.ptr(x2), x2.shape[0],
                                      pkg.ptr(params), pkg.ptr(rng), O.C.byref(lat), h0, h1, pkg.ptr(loc),
                                      O.C.byref(ng)))
        assert lat.value == ref["latch"]
        allh[h0:h1] = loc[:h1 - h0]
    fr = hyp_shard.fold(allh, ng.value, params)
    owners = 0
    for r, odo in enumerate(ctxs):
        rng = pkg.Rng()
        lib.odo_rng_seed(pkg.ptr(rng), 99)
        T = np.zeros(16, np.float32)
        rmse, ni, ok, own = O.C.c_float(0), O.C.c_int(0), O.C.c_int(0), O.C.c_int(0)
        inl = np.zeros(max(m.size, 1), pkg.DMATCH_DTYPE)
        pkg.check(lib.odo_ransac_hyps_finish(odo.h, pkg.ptr(fr), pkg.ptr(rng), pkg.ptr(T), O.C.byref(rmse),
                                             pkg.ptr(inl), O.C.byref(ni), O.C.byref(ok), O.C.byref(own)))
        assert bytes(rng) == ref["rng"], f"rank {r}: rand() state after the visited draws"
        if own.value:
            owners += 1
            assert np.array_equal(T, ref["T"]) and rmse.value == ref["rmse"] and ok.value == ref["ok"]
            assert np.array_equal(inl[:ni.value], ref["inliers"]), "inlier list"
    assert owners == (1 if fr.best_h >= 0 else world)
    for odo in ctxs:
        odo.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, corrupt, iters, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = load_pkg()
        from arlm_amd import hyp_shard
        m, x1, x2, _ = _problem(corrupt, iters)
        odo = pkg.Odometry(pkg.default_config(640, 480, 1, nfeatures=1000, iterations=iters))
        rng = pkg.Rng()
        pkg.load().odo_rng_seed(pkg.ptr(rng), 5)
        ex = hyp_shard.Exchange(dist, world, rank, device="cpu")
        T, rmse, inl, ok, visited, lat = hyp_shard.sharded_ransac(odo, ex, m, x1, x2,
                                                                  pkg.RansacParams(iters, 20, 3.0, 4, 1), rng,
                                                                  float("nan"))
        res = dict(T=T, rmse=rmse, inl=inl, ok=ok, rng=bytes(rng), lat=lat)
        if rank == 0:
            res["ref"] = _reference(pkg, odo, m, np.ascontiguousarray(x1), np.ascontiguousarray(x2), iters, 5)
        odo.close()
        gathered = [None] * world
        dist.all_gather_object(gathered, res)
        if rank == 0:
            out.put(gathered)
    finally:
        dist.destroy_process_group()


def test_two_processes_sharded_ransac():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, 0.55, 2048, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = res[0]["ref"]
    for r in res:
        assert np.array_equal(r["T"].ravel(), ref["T"]) and np.float32(r["rmse"]) == np.float32(ref["rmse"])
        assert r["ok"] == ref["ok"] and np.array_equal(r["inl"], ref["inliers"])
        assert r["rng"] == ref["rng"] and r["lat"] == ref["latch"]


# ---------------------------------------------------------------- exchange in HBM
def _device_run(pkg, ctxs, m, x1, x2, iters, seed):
    """The device protocol with the collectives simulated in one process:
    every rank's block into a device tensor, the blocks concatenated (what
    all_gather_into_tensor delivers), the fold and the payloads on each rank,
    the payloads summed (the int32 SUM all_reduce)."""
    import torch
    from arlm_amd import hyp_shard
    lib = pkg.load()
    world = len(ctxs)
    params = pkg.RansacParams(iters, 20, 3.0, 4, 1)
    blocks, ngs = [], []
    for r, odo in enumerate(ctxs):
        h0, h1, per = hyp_shard.device_range(iters, r, world)
        rng = pkg.Rng()
        lib.odo_rng_seed(pkg.ptr(rng), seed)
        lat = O.C.c_double(float("nan"))
        ng = O.C.c_int(0)
        blk = torch.full((max(per, 1) * 64,), 0x5A, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()  # the fill runs on torch's stream, the library on its own
        pkg.check(lib.odo_ransac_hyps_dev(odo.h, pkg.ptr(m), m.size, pkg.ptr(x1), x1.shape[0], pkg.ptr(x2),
                                          x2.shape[0], pkg.ptr(params), pkg.ptr(rng), O.C.byref(lat), h0, h1,
                                          O.C.c_void_p(blk.data_ptr()), O.C.byref(ng)))
        torch.cuda.synchronize()
        blocks.append(blk)
        ngs.append(ng.value)
    allh = torch.cat(blocks)
    folds, payloads = [], []
    for r, odo in enumerate(ctxs):
        rec = torch.zeros(32, dtype=torch.uint8, device="cuda")
        pkg.check(lib.odo_ransac_fold_dev(odo.h, O.C.c_void_p(allh.data_ptr()), iters, O.C.c_void_p(rec.data_ptr())))
        words = lib.odo_ransac_hyps_payload_words(odo.h)
        pl = torch.full((words,), 7, dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        pkg.check(lib.odo_ransac_hyps_finish_dev(odo.h, O.C.c_void_p(rec.data_ptr()), 1 if r == 0 else 0,
                                                 O.C.c_void_p(pl.data_ptr()), words))
        torch.cuda.synchronize()
        folds.append(rec.cpu().numpy())
        payloads.append(pl)
    total = torch.stack(payloads).sum(0, dtype=torch.int32)
    outs = []
    for odo in ctxs:
        rng = pkg.Rng()
        lib.odo_rng_seed(pkg.ptr(rng), seed)
        T = np.zeros(16, np.float32)
        rmse, ni, ok, vis = O.C.c_float(0), O.C.c_int(0), O.C.c_int(0), O.C.c_int(0)
        inl = np.zeros(max(m.size, 1), pkg.DMATCH_DTYPE)
        pkg.check(lib.odo_ransac_hyps_result(odo.h, O.C.c_void_p(total.data_ptr()), pkg.ptr(rng), pkg.ptr(T),
                                             O.C.byref(rmse), pkg.ptr(inl), O.C.byref(ni), O.C.byref(ok),
                                             O.C.byref(vis)))
        outs.append(dict(T=T, rmse=rmse.value, inliers=inl[:ni.value], ok=ok.value, rng=bytes(rng), visited=vis.value))
    # the GPU fold equals the host fold over the same summaries
    allh_np = np.frombuffer(allh.cpu().numpy().tobytes(), pkg._abi.HYP_DTYPE)[:iters]
    fr = hyp_shard.fold(allh_np, ngs[0], params)
    for rec in folds:
        got = np.frombuffer(rec.tobytes(), np.int32)
        assert (got[0], got[1], got[2], got[3]) == (fr.best_h, fr.visited, fr.valid, fr.n_inliers)
        assert np.frombuffer(rec.tobytes()[16:20], np.float32)[0] == np.float32(fr.rmse)
    return outs, fr


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("corrupt,iters", [(0.0, 500), (0.5, 4096), (0.75, 1000), (1.0, 300)])
def test_device_exchange_reproduces_iterate(world, corrupt, iters):
    """the exchange on the device (summaries exported to
    HBM, the fold on the GPU, the owner's payload sum-reduced) gives every
    rank odo_ransac's T12, rmse, ok, inlier list and rand() state bit for bit
    — incl. the identity fallback / no valid hypothesis (corrupt 1.0)."""
    pkg = load_pkg()
    m, x1, x2, _ = _problem(corrupt, iters)
    x1, x2 = np.ascontiguousarray(x1), np.ascontiguousarray(x2)
    ctxs = [pkg.Odometry(pkg.default_config(640, 480, 1, nfeatures=1000, iterations=iters)) for _ in range(world)]
    try:
        ref = _reference(pkg, ctxs[0], m, x1, x2, iters, 77)
        outs, fr = _device_run(pkg, ctxs, m, x1, x2, iters, 77)
        for r, o in enumerate(outs):
            assert np.array_equal(o["T"], ref["T"]) and o["rmse"] == ref["rmse"] and o["ok"] == ref["ok"], f"rank {r}"
            assert np.array_equal(o["inliers"], ref["inliers"]), f"rank {r}: inlier list"
            assert o["rng"] == ref["rng"], f"rank {r}: rand() state after the visited draws"
            assert o["visited"] == fr.visited
    finally:
        for odo in ctxs:
            odo.close()


def test_device_exchange_too_few_matches():
    """A pair that never samples (fewer good matches than minInliers): rank 0
    reports Iterate's reset outputs, the rand() state is untouched."""
    pkg = load_pkg()
    m, x1, x2, _ = _problem(0.0, 200)
    m = np.ascontiguousarray(m[:12])
    x1, x2 = np.ascontiguousarray(x1), np.ascontiguousarray(x2)
    ctxs = [pkg.Odometry(pkg.default_config(640, 480, 1, nfeatures=1000, iterations=200)) for _ in range(2)]
    try:
        ref = _reference(pkg, ctxs[0], m, x1, x2, 200, 3)
        outs, _ = _device_run(pkg, ctxs, m, x1, x2, 200, 3)
        for o in outs:
            assert np.array_equal(o["T"], ref["T"]) and o["ok"] == 0 == ref["ok"] and o["rng"] == ref["rng"]
            assert o["rmse"] == ref["rmse"] and len(o["inliers"]) == 0
    finally:
        for odo in ctxs:
            odo.close()


def _worker_dev(rank, world, port, corrupt, iters, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = load_pkg()
        from arlm_amd import hyp_shard
        m, x1, x2, _ = _problem(corrupt, iters)
        odo = pkg.Odometry(pkg.default_config(640, 480, 1, nfeatures=1000, iterations=iters))
        rng = pkg.Rng()
        pkg.load().odo_rng_seed(pkg.ptr(rng), 5)
        ex = hyp_shard.DeviceExchange(dist, world, rank, odo.stream)
        T, rmse, inl, ok, visited, lat = hyp_shard.sharded_ransac_device(odo, ex, m, x1, x2,
                                                                         pkg.RansacParams(iters, 20, 3.0, 4, 1), rng,
                                                                         float("nan"))
        res = dict(T=T, rmse=rmse, inl=inl, ok=ok, rng=bytes(rng), lat=lat)
        if rank == 0:
            res["ref"] = _reference(pkg, odo, m, np.ascontiguousarray(x1), np.ascontiguousarray(x2), iters, 5)
        odo.close()
        gathered = [None] * world
        dist.all_gather_object(gathered, res)
        if rank == 0:
            out.put(gathered)
    finally:
        dist.destroy_process_group()


def test_two_processes_device_exchange():
    """hyp_shard.sharded_ransac_device between two processes (gloo stages the
    device tensors through the host; RCCL takes them directly)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_dev, args=(r, 2, port, 0.55, 2048, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = res[0]["ref"]
    for r in res:
        assert np.array_equal(r["T"].ravel(), ref["T"]) and np.float32(r["rmse"]) == np.float32(ref["rmse"])
        assert r["ok"] == ref["ok"] and np.array_equal(r["inl"], ref["inliers"])
        assert r["rng"] == ref["rng"] and r["lat"] == ref["latch"]
