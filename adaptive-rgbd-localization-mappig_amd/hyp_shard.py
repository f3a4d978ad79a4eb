"""Hypotheses mode of Ransac::Iterate over ranks.

The hypotheses of ONE pair are split across the ranks of a torch.distributed
group (RCCL over xGMI on the GPU box, gloo in the CPU tests):

1. every rank runs odo_ransac_hyps on its hypothesis range [H*r/R, H*(r+1)/R)
   — the same rand() stream everywhere, so hypothesis j is the same sample
   on every rank;
2. all_gather of the 64-byte per-hypothesis summaries (256 KB at H=4096);
3. every rank replays the reference's ORDERED running-best fold
   (odo_ransac_fold, ransac.cpp:233-249 — not an argmax: later equal
   hypotheses win, accepted hypotheses skip n += 10 and break above 80 %);
4. the rank whose range holds the winner (rank 0 for the identity fallback)
   broadcasts T12, rmse, ok and the inlier list; every rank advances its
   rand() state by exactly the visited draws (odo_ransac_hyps_finish).

The result on every rank equals odo_ransac / Ransac::Iterate bit for bit.

`sharded_ransac_device` is the same protocol with the exchange in HBM: the
summaries are exported into a device tensor (odo_ransac_hyps_dev), gathered
with all_gather_into_tensor (RCCL when the ranks hold distinct GPUs), folded
on the GPU (odo_ransac_fold_dev), and the winner's owner writes its payload
while every other rank writes zeros, so one int32 SUM all_reduce replaces the
broadcast and no rank needs to know the owner on the host. All of it is
queued on the context's stream; the host reads the outputs once at the end.
With gloo (CPU tensors only) DeviceExchange stages through host memory.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._abi import DMATCH_DTYPE, HYP_DTYPE, FoldResult, RansacParams, Rng, check, load, ptr


def shard_range(H: int, rank: int, world: int):
    """Hypothesis indices [h0, h1) of one rank."""
    return H * rank // world, H * (rank + 1) // world


def owner_of(h: int, H: int, world: int) -> int:
    """Rank whose range holds hypothesis h (rank 0 when h < 0: identity fallback)."""
    if h < 0:
        return 0
    for r in range(world):
        a, b = shard_range(H, r, world)
        if a <= h < b:
            return r
    raise ValueError(f"hypothesis {h} outside [0, {H})")


def fold(all_summaries: np.ndarray, n_good: int, params: RansacParams) -> FoldResult:
    """The ordered fold over all H summaries (host function of libodo_hip.so)."""
    a = np.ascontiguousarray(all_summaries, HYP_DTYPE)
    r = FoldResult()
    check(load().odo_ransac_fold(ptr(a), a.size, n_good, ptr(params), ptr(r)))
    return r


class Exchange:
    """Fixed-size byte collectives on a torch.distributed group."""

    def __init__(self, dist, world: int, rank: int, device: str = "cuda"):
        self.dist, self.world, self.rank, self.device = dist, world, rank, device

    def all_gather(self, local: np.ndarray, block: int) -> list:
        import torch
        buf = np.zeros(block, np.uint8)
        raw = np.frombuffer(np.ascontiguousarray(local).tobytes(), np.uint8)
        buf[:raw.size] = raw
        t = torch.from_numpy(buf).to(self.device)
        outs = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(outs, t)
        return [o.cpu().numpy() for o in outs]

    def broadcast(self, buf: np.ndarray, src: int) -> np.ndarray:
        import torch
        t = torch.from_numpy(np.ascontiguousarray(buf).view(np.uint8).copy()).to(self.device)
        self.dist.broadcast(t, src)
        return t.cpu().numpy()


def gather_summaries(local: np.ndarray, H: int, ex: Exchange) -> np.ndarray:
    """All ranks' summaries in hypothesis order (rank blocks are contiguous)."""
    per = -(-H // ex.world)  # ceil: every block padded to the largest range
    blocks = ex.all_gather(local.astype(HYP_DTYPE, copy=False), per * HYP_DTYPE.itemsize)
    out = np.zeros(H, HYP_DTYPE)
    for r, b in enumerate(blocks):
        a, e = shard_range(H, r, ex.world)
        out[a:e] = np.frombuffer(b.tobytes(), HYP_DTYPE, count=e - a)
    return out


def sharded_ransac(odo, ex: Exchange, m12: np.ndarray, xyz1: np.ndarray, xyz2: np.ndarray,
                   params: RansacParams, rng: Rng, latch: float):
    """Ransac::Iterate with its hypotheses sharded over the group.
    Returns (T12 4x4, rmse, inliers DMatch array, ok, visited, latch); rng is
    advanced in place, as the reference's rand() stream would be."""
    lib = load()
    m12 = np.ascontiguousarray(m12, DMATCH_DTYPE)
    xyz1 = np.ascontiguousarray(xyz1, np.float32)
    xyz2 = np.ascontiguousarray(xyz2, np.float32)
    H = max(params.iterations, 0)
    h0, h1 = shard_range(H, ex.rank, ex.world)
    local = np.zeros(max(h1 - h0, 1), HYP_DTYPE)
    lat = C.c_double(latch)
    ng = C.c_int(0)
    check(lib.odo_ransac_hyps(odo.h, ptr(m12), m12.size, ptr(xyz1), xyz1.shape[0], ptr(xyz2), xyz2.shape[0],
                              ptr(params), ptr(rng), C.byref(lat), h0, h1, ptr(local), C.byref(ng)))
    allh = gather_summaries(local[:h1 - h0], H, ex)
    fr = fold(allh, ng.value, params)
    T = np.zeros(16, np.float32)
    rmse, nin, ok, own = C.c_float(0), C.c_int(0), C.c_int(0), C.c_int(0)
    inl = np.zeros(max(ng.value, 1), DMATCH_DTYPE)
    check(lib.odo_ransac_hyps_finish(odo.h, ptr(fr), ptr(rng), ptr(T), C.byref(rmse), ptr(inl), C.byref(nin),
                                     C.byref(ok), C.byref(own)))
    src = owner_of(fr.best_h, H, ex.world)
    # owner -> all: header (T12, rmse, ok, n_inliers) + the inlier list padded to n_good
    hdr = np.zeros(16 + 3, np.float32)
    hdr[:16] = T
    hdr[16] = rmse.value
    hdr[17:19] = np.array([ok.value, nin.value], np.int32).view(np.float32)
    payload = np.concatenate([hdr.view(np.uint8), inl.view(np.uint8)])
    got = ex.broadcast(payload, src)
    hdr = got[:hdr.nbytes].view(np.float32)
    n_inl = int(hdr[17:19].view(np.int32)[1])
    inliers = got[19 * 4:].view(DMATCH_DTYPE)[:n_inl].copy()
    return (hdr[:16].reshape(4, 4).copy(), float(hdr[16]), inliers, int(hdr[17:19].view(np.int32)[0]),
            fr.visited, lat.value)


def device_range(H: int, rank: int, world: int):
    """[h0, h1) of one rank in the device protocol: contiguous blocks of
    ceil(H / world), so the gathered blocks are already in hypothesis order."""
    per = -(-H // world) if H else 0
    return min(H, rank * per), min(H, (rank + 1) * per), per


class DeviceExchange:
    """Collectives on device tensors: RCCL (nccl backend) directly; gloo, which
    takes CPU tensors only, through host copies (tests with ranks sharing one
    GPU). Issued on `stream` (the odometry context's stream), so they are
    ordered after the kernels that produce their inputs and before the ones
    that consume them."""

    def __init__(self, dist, world: int, rank: int, stream_ptr: int):
        import torch
        self.dist, self.world, self.rank = dist, world, rank
        self.nccl = world > 1 and dist.get_backend() == "nccl"
        self.stream = torch.cuda.ExternalStream(stream_ptr)

    def all_gather(self, block):
        import torch
        with torch.cuda.stream(self.stream):
            if self.world == 1:
                return block
            if self.nccl:
                out = torch.empty(self.world * block.numel(), dtype=block.dtype, device=block.device)
                self.dist.all_gather_into_tensor(out, block)
                return out
            host = block.cpu()
            parts = [torch.empty_like(host) for _ in range(self.world)]
            self.dist.all_gather(parts, host)
            return torch.cat(parts).to(block.device)

    def all_reduce_sum(self, t):
        import torch
        with torch.cuda.stream(self.stream):
            if self.world == 1:
                return t
            if self.nccl:
                self.dist.all_reduce(t)
                return t
            host = t.cpu()
            self.dist.all_reduce(host)
            t.copy_(host)
            return t


def sharded_ransac_device(odo, ex: DeviceExchange, m12: np.ndarray, xyz1: np.ndarray, xyz2: np.ndarray,
                          params: RansacParams, rng: Rng, latch: float, timing: dict = None):
    """sharded_ransac with the exchange in device memory (see the module
    docstring). Same return value; rng is advanced in place. timing (optional
    dict): the host-clock split of one call (evaluation, exchange, fold +
    finish), each phase synchronised — measurement only."""
    import time

    import torch
    lib = load()
    m12 = np.ascontiguousarray(m12, DMATCH_DTYPE)
    xyz1 = np.ascontiguousarray(xyz1, np.float32)
    xyz2 = np.ascontiguousarray(xyz2, np.float32)
    H = max(params.iterations, 0)
    h0, h1, per = device_range(H, ex.rank, ex.world)
    dev = torch.device("cuda", torch.cuda.current_device())
    # every tensor the library writes is allocated on the context's stream (its
    # non-blocking odometry stream), so the caching allocator orders its reuse
    # there; torch.empty: the padding and the fold record are written before
    # they are read, so there is no fill to race with the library's writes
    with torch.cuda.stream(ex.stream):
        block = torch.empty(max(per, 1) * HYP_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        fold_rec = torch.empty(32, dtype=torch.uint8, device=dev)
    lat = C.c_double(latch)
    ng = C.c_int(0)
    sync = (lambda: torch.cuda.synchronize()) if timing is not None else (lambda: None)
    t0 = time.perf_counter()
    check(lib.odo_ransac_hyps_dev(odo.h, ptr(m12), m12.size, ptr(xyz1), xyz1.shape[0], ptr(xyz2), xyz2.shape[0],
                                  ptr(params), ptr(rng), C.byref(lat), h0, h1, C.c_void_p(block.data_ptr()),
                                  C.byref(ng)))
    sync()
    t1 = time.perf_counter()
    allh = ex.all_gather(block)
    sync()
    t2 = time.perf_counter()
    check(lib.odo_ransac_fold_dev(odo.h, C.c_void_p(allh.data_ptr()), H, C.c_void_p(fold_rec.data_ptr())))
    words = lib.odo_ransac_hyps_payload_words(odo.h)
    if words < 0:
        check(words)
    with torch.cuda.stream(ex.stream):
        payload = torch.empty(words, dtype=torch.int32, device=dev)
    check(lib.odo_ransac_hyps_finish_dev(odo.h, C.c_void_p(fold_rec.data_ptr()), 1 if ex.rank == 0 else 0,
                                         C.c_void_p(payload.data_ptr()), words))
    sync()
    t3 = time.perf_counter()
    ex.all_reduce_sum(payload)
    sync()
    t4 = time.perf_counter()
    T = np.zeros(16, np.float32)
    rmse, nin, ok, vis = C.c_float(0), C.c_int(0), C.c_int(0), C.c_int(0)
    inl = np.zeros(max(ng.value, 1), DMATCH_DTYPE)
    check(lib.odo_ransac_hyps_result(odo.h, C.c_void_p(payload.data_ptr()), ptr(rng), ptr(T), C.byref(rmse),
                                     ptr(inl), C.byref(nin), C.byref(ok), C.byref(vis)))
    t5 = time.perf_counter()
    if timing is not None:
        timing.update(evaluate=t1 - t0, all_gather=t2 - t1, fold_finish=t3 - t2, all_reduce=t4 - t3,
                      readback=t5 - t4, total=t5 - t0)
    return T.reshape(4, 4), float(rmse.value), inl[:nin.value].copy(), int(ok.value), int(vis.value), lat.value
