#!/usr/bin/env python3
"""bench.py — frames/sec of the per-frame odometry hot path on MI355X.

Metric (BASELINE.json): frames/sec (extract + match + RANSAC-PnP) at 640x480,
2000 ORB keypoints. Workload = config 2 ("TUM fr1/desk proxy": 640x480, FR1
intrinsics + distortion, 2000 kp, RANSAC 500 hypotheses) on a synthetic
closed-loop RGB-D sequence (no datasets offline). One step = one batch of
`--batch` frames through Tracking::Track's hot path (extract every frame,
kNN-2 + ratio match against its predecessor, Ransac::Iterate, PnPSolver).

`value` is timed with the inputs already resident in HBM (the measurement
contract); `from_host` is the same path timed from BGR8 + depth16 in pinned
host memory (SURVEY §8(d)'s unit, PCIe-inclusive), with its own kernel
timing. Multi-GPU (N > 1): SURVEY §8(e) frames mode by default — ONE
sequence, each step's frames split into per-rank chunks with a one-frame
halo, the DepthCovariance latch broadcast once, the poses stitched with one
all_gather per run (frames_shard.py); each rank uploads its own chunk over
its own PCIe link in the from-host leg. `--shard independent` gives every
rank its own sequence instead (no exchange).

Prints ONE JSON line on rank 0.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np

# HIP runtime dispatch mode for this process: commands go to the runtime's
# worker thread instead of being written to the hardware queues by the
# calling thread (direct dispatch, HIP's default). The batched pipeline's
# steady state is 1.81-1.88 vs 1.92-2.03 ms per step with it on the same
# boxes (profiles/r05_w, r05_x, r05_z; DESIGN §4 Pipelining). An
# AMD_DIRECT_DISPATCH already in the environment is kept. It has to be set
# before the HIP runtime initialises (torch is imported later). The
# one-frame latency leg runs in its own process with direct dispatch (its
# synchronous per-stage calls: p50 0.87 vs 0.91-0.95 ms, profiles/r05_zb).
# The single-call latency modes (--mode pnpransac / gicp / hyp: one
# synchronous call at a time, nothing to pipeline) keep HIP's direct
# dispatch: the worker thread's hand-off is pure latency there.
DIRECT_DISPATCH_FROM_ENV = "AMD_DIRECT_DISPATCH" in os.environ
_MODE = next((sys.argv[i + 1] for i, a in enumerate(sys.argv[:-1]) if a == "--mode"),
             next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--mode=")), "track"))
os.environ.setdefault("AMD_DIRECT_DISPATCH", "1" if _MODE in ("pnpransac", "gicp", "hyp") else "0")

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "adaptive-rgbd-localization-mappig_amd")

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP64_PEAK_TFLOPS = 78.6      # MI355X_MICROARCH.md: FP64 vector spec
VALU_PEAK_TOPS = 78.6        # MI355X_MICROARCH.md: 256 CU x 4 SIMD-32 x 32 lanes x 2.4 GHz int32 lane-ops
F4_MFMA_PEAK_TOPS = 10066.3  # dense FP4 (block-scaled f8f6f4, e2m1): 4x the BF16 rate per clock
# the algorithmic Hamming work is 16 int32 lane-ops per (query,
# train) comparison (8 v_xor_b32 + 8 v_bcnt_u32_b32 over the 256-bit
# descriptors; the top-2 update is excluded)
KNN_OPS_PER_CMP = 16
# SURVEY §8(d) RANSAC work: ~120 FP64 flops per non-shortcut ErrorFunction2
# evaluation (E = sweeps x good matches) and ~40 FP32 flops per point added to
# a TransformationFromCorrespondences fit (F)
RANSAC_FLOPS_PER_EVAL = 120
RANSAC_FLOPS_PER_FIT_POINT = 40
# PMC memory-side bytes of k_knn2_f4 per launch, measured on this round's
# kernel build (tools/pmc_merge.py --traffic); absent -> roofline.traffic null.
# Kept outside profiles/ (which gpurun does not ship) so it is there when the
# bench runs on a GPU box
KNN_F4_TRAFFIC = os.path.join(ROOT, "measurements", "r04_knn2_f4_traffic.json")
# on-box peak microbenchmarks (tools/ubench_peak.hip); the fallbacks are the
# r02 measurements
UBENCH = os.path.join(ROOT, "profiles", "r02_ubench_peak.jsonl")
UBENCH_FALLBACK = {"valu_xor_bcnt": 50.213, "fp64_fma": 61.22, "hbm_read": 6946.7, "hbm_copy": 4867.8,
                   "mfma_i32_16x16x64_i8": 3484.73, "mfma_scale_f32_16x16x128_f4": 6073.79, "knn_f4_mix": 3930.16}


def measured_peaks(path=UBENCH):
    """Best rate of each instruction mix / access pattern in the committed
    microbenchmark output (Top/s, TFLOP/s or GB/s)."""
    peaks = dict(UBENCH_FALLBACK)
    if os.path.exists(path):
        best = {}
        with open(path) as f:
            for line in f:
                try:
                    r = json.loads(line)
                except ValueError:
                    continue
                b = r.get("bench")
                v = r.get("tops", r.get("tflops", r.get("gbs")))
                if b and v is not None:
                    best[b] = max(best.get(b, 0.0), float(v))
        peaks.update(best)
    return peaks


def load_module(name, path, pkg_dir=None):
    if name in sys.modules:
        return sys.modules[name]
    spec = importlib.util.spec_from_file_location(name, path, submodule_search_locations=pkg_dir)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def load_pkg():
    return load_module("arlm_amd", os.path.join(PKG_DIR, "__init__.py"), [PKG_DIR])


def load_synth():
    return load_module("arlm_amd_synth", os.path.join(PKG_DIR, "synth.py"))


def shard_seed(rank: int) -> int:
    """Scene seed of a rank's sequence: rank 0's is the cfg2 sequence (frames
    mode: every rank tracks chunks of that one sequence; --shard independent:
    rank r tracks its own sequence with this seed)."""
    return 0x5EED0002 + 7919 * rank


def rank_seeds(rank: int):
    """(scene seed, RANSAC/pair seed base) of one rank's sequence (rank 0 in
    frames mode, where the pair seeds come from global pair indices)."""
    return shard_seed(rank), 0x5EED0000 + 1000003 * rank


def max_over_ranks(x: float, dist=None, world: int = 1, device: str = "cuda") -> float:
    """Job time = the slowest rank's time (all_reduce MAX; RCCL on GPUs, gloo in tests)."""
    if world <= 1:
        return x
    import torch
    t = torch.tensor([x], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def job_throughput(frames_per_step: int, steps: int, world: int, elapsed_max: float) -> float:
    """Whole-job frames/s: every rank tracks frames_per_step frames per step."""
    return frames_per_step * steps * world / elapsed_max


def usable_cores() -> int:
    """CPUs this process may run on: the affinity mask, capped by a cgroup CPU
    quota when one is set (the GPU box shows the whole machine's CPUs to
    nproc, but grants each GPU a share)."""
    n = len(os.sched_getaffinity(0))
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", lambda t: [t.strip(), open(
                            "/sys/fs/cgroup/cpu/cpu.cfs_period_us").read().strip()])):
        try:
            with open(path) as f:
                q, per = parse(f.read())
            if q not in ("max", "-1"):
                n = min(n, max(1, -(-int(q) // int(per))))
            break
        except (OSError, ValueError):
            continue
    return n


def host_info():
    """nproc, usable cores and CPU model of this host (the GPU box's when run there)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity_cores": len(os.sched_getaffinity(0)),
            "usable_cores": usable_cores(), "model": model}


ORACLE_V3 = os.path.join(ROOT, "oracle", "liboracle_v3.so")


def oracle_for_baseline():
    """The oracle build the CPU baselines time: liboracle_v3.so (the same
    sources for x86-64-v3: AVX2 / FMA / BMI2 / POPCNT, FP contraction off, so
    the results are identical) when the host CPU has those features, else the
    x86-64 build. Returns (oracle_lib module, build description)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    try:
        flags = set(open("/proc/cpuinfo").read().split("flags")[1].split("\n")[0].split())
    except (OSError, IndexError):
        flags = set()
    need = {"avx2", "fma", "bmi2", "popcnt", "movbe", "f16c"}
    if os.path.exists(ORACLE_V3) and need <= flags:
        if O.LIB_PATH != ORACLE_V3:
            O.LIB_PATH, O._lib = ORACLE_V3, None
        return O, "g++ -O3 -march=x86-64-v3 -ffp-contract=off (oracle/liboracle_v3.so)"
    return O, "g++ -O3 -ffp-contract=off, baseline x86-64 (oracle/liboracle.so)"


def cpu_baseline(bgr, dep, nfeat, iters, n_frames, reps, adaptive=False, threads=None, inner="fast"):
    """The C++ oracle on the first n_frames frames of the same sequence.

    Single thread: this thread pinned to one core (taskset -c equivalent),
    one warm-up pass, then `reps` timed passes; per-stage medians (extraction
    per frame, match + RANSAC + PnP per pair). All cores: the same frames with
    a thread pool (ctypes releases the GIL inside the oracle) extracting frames
    and tracking pairs in parallel, the latch taken from pair 1 as in the
    batched contract (ADAPTIVE extraction stays sequential: its thresholds
    carry from frame to frame)."""
    from concurrent.futures import ThreadPoolExecutor
    O, build = oracle_for_baseline()
    cal = O.fr1_calib()
    p = O.orb_params(nfeat)
    rp = O.ransac_params(iters)
    pkg = load_pkg()
    n = len(bgr)

    def extract(ex, i):
        return ex.extract_frame(bgr[i % n], dep[i % n], cal) if ex is not None else \
            O.extract_frame(bgr[i % n], dep[i % n], p, cal)

    def run_pass():
        ex = O.AdaptiveExtractor(inner=inner) if adaptive else None
        te = tt = 0.0
        prev, latch = None, float("nan")
        for i in range(n_frames):
            t0 = time.perf_counter()
            f = extract(ex, i)
            t1 = time.perf_counter()
            if prev is not None:
                _, _, _, latch = O.track_pair(prev, f, cal, rp, pkg.pair_seed(0x5EED0000, i), latch)
            tt += time.perf_counter() - t1
            te += t1 - t0
            prev = f
        return te, tt

    aff = os.sched_getaffinity(0)
    core = min(aff)
    os.sched_setaffinity(0, {core})
    try:
        run_pass()  # warm-up
        passes = [run_pass() for _ in range(reps)]
    finally:
        os.sched_setaffinity(0, aff)
    tot = sorted(te + tt for te, tt in passes)
    med = tot[len(tot) // 2]
    ext_ms = sorted(te for te, _ in passes)[len(passes) // 2] / n_frames * 1e3
    trk_ms = sorted(tt for _, tt in passes)[len(passes) // 2] / max(1, n_frames - 1) * 1e3

    # all usable cores (affinity mask capped by the cgroup CPU quota)
    nthr = max(1, min(threads or usable_cores(), len(aff)))
    nf_all = max(n_frames * 4, 2 * nthr)

    def all_cores_pass():
        t0 = time.perf_counter()
        with ThreadPoolExecutor(nthr) as pool:
            if adaptive:
                ex = O.AdaptiveExtractor(inner=inner)
                frames = [extract(ex, i) for i in range(nf_all)]
            else:
                frames = list(pool.map(lambda i: extract(None, i), range(nf_all)))
            _, _, _, latch = O.track_pair(frames[0], frames[1], cal, rp, pkg.pair_seed(0x5EED0000, 1))
            list(pool.map(lambda i: O.track_pair(frames[i - 1], frames[i], cal, rp,
                                                 pkg.pair_seed(0x5EED0000, i), latch), range(2, nf_all)))
        return time.perf_counter() - t0

    all_cores_pass()
    ta = sorted(all_cores_pass() for _ in range(3))[1]
    return {"fps": n_frames / med, "seconds": med, "reps": reps, "core": core, "build": build,
            "stage_ms": {"extract_per_frame": round(ext_ms, 3), "match_ransac_pnp_per_pair": round(trk_ms, 3)},
            "all_cores": {"fps": nf_all / ta, "threads": nthr, "frames": nf_all}}


def timed_leg(odo, submit, steps, warmup, world, dist, coll_dev, kernel_timing=True, inside=None, marks_out=None):
    """The bench contract for one leg: `warmup` untimed steps, then exactly
    `steps` timed steps bracketed by a barrier + device synchronize on both
    sides, the wall time taken as the max over ranks. submit(i) queues step i;
    inside() runs inside the timed region after the last step (frames mode:
    the pose stitch). With kernel_timing, an event pair brackets every kNN-2
    launch of the timed steps (on the stream that runs it, odo timing mode 2),
    and marks_out (a list) receives each timed batch's kNN-2 start (ms,
    odo_step_marks), whose differences are the per-step times.
    Returns (elapsed s, host submit s, (kNN-2 mean ms, launches))."""
    import torch
    for i in range(warmup):
        submit(i)
    odo.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    if kernel_timing:
        odo.set_timing(None, mode=2)
    t0 = time.perf_counter()
    for i in range(steps):
        submit(warmup + i)
    sub = time.perf_counter() - t0
    odo.synchronize()
    if inside is not None:
        inside()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = max_over_ranks(time.perf_counter() - t0, dist, world, device=coll_dev)
    kt = (None, 0)
    if kernel_timing:
        kt = odo.kernel_timing()
        if marks_out is not None:
            marks_out.extend(odo.step_marks())
        odo.set_timing(False)
    return el, sub, kt


def step_stats(marks):
    """Per-step time distribution of a timed leg from its step marks (ms): one
    step = the interval between consecutive batches' kNN-2 starts, which
    follow each batch's extraction (the pipeline's critical stream)."""
    d = np.diff(np.asarray(marks, dtype=np.float64))
    if d.size == 0:
        return None
    med = float(np.median(d))
    return {"min": round(float(d.min()), 4), "median": round(med, 4), "p90": round(float(np.percentile(d, 90)), 4),
            "max": round(float(d.max()), 4), "mean": round(float(d.mean()), 4), "n": int(d.size),
            "max_over_median": round(float(d.max()) / med, 4) if med > 0 else None,
            "argmax": int(np.argmax(d)), "intervals": [round(float(x), 3) for x in d],
            "source": "differences of consecutive batches' kNN-2 start events (odo_step_marks, rank 0)"}


def raw_h2d_gbs(nbytes: int) -> float:
    """Pinned host -> HBM copy rate of nbytes with no compute (the PCIe bound)."""
    import torch
    hsrc = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    ddst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    ddst.copy_(hsrc, non_blocking=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(3):
        ddst.copy_(hsrc, non_blocking=True)
    torch.cuda.synchronize()
    raw = 3 * nbytes / (time.perf_counter() - t1) / 1e9
    del hsrc, ddst
    return raw


class LocalExchange:
    """hyp_shard.Exchange for a single rank (no process group)."""
    world, rank = 1, 0

    def all_gather(self, local, block):
        buf = np.zeros(block, np.uint8)
        raw = np.frombuffer(np.ascontiguousarray(local).tobytes(), np.uint8)
        buf[:raw.size] = raw
        return [buf]

    def broadcast(self, buf, src):
        return np.ascontiguousarray(buf).view(np.uint8).copy()


def hyp_mode(args, rank, world, local_rank, dist):
    """SURVEY §8(e) hypotheses mode on config 3: one hard pair's RANSAC
    (H = 4096) with its hypotheses sharded over the ranks (hyp_shard.py:
    per-rank odo_ransac_hyps, all_gather of the 64-B summaries, the ordered
    fold, broadcast of the winner). A latency metric: ms per pair."""
    import torch
    pkg = load_pkg()
    synth = load_synth()
    from importlib import import_module
    hs = import_module("arlm_amd.hyp_shard")
    fr2 = dict(fx=520.9, fy=521.0, cx=325.1, cy=249.7)  # common.h:47-50 (FR1 distortion kept, App. B.16)
    bgr, dep, _ = synth.make_sequence(2, 640, 480, intrinsics=fr2, seed=0x5EED0003)
    H_ = args.iters if args.iters != 500 else 4096
    cfg = pkg.default_config(640, 480, 2, nfeatures=4000, iterations=H_, seed=0x5EED0003, calib=fr2)
    odo = pkg.Odometry(cfg, device=local_rank % max(1, torch.cuda.device_count()))
    odo.track_batch_host(bgr, dep)
    m = odo.pair(1)["matches"].copy()
    x1, x2 = odo.frame(0)["xyz"], odo.frame(1)["xyz"]
    # a hard pair: half the matches re-targeted at random keypoints, so the
    # > 80 % early exit never fires and RANSAC visits many hypotheses
    rs = np.random.default_rng(3)
    sel = rs.random(m.size) < args.hyp_outliers
    m["trainIdx"][sel] = rs.integers(0, x2.shape[0], int(sel.sum()))
    params = pkg.RansacParams(H_, 20, 3.0, 4, 1)
    backend = dist.get_backend() if world > 1 else None
    ex_host = hs.Exchange(dist, world, rank, device="cuda" if backend == "nccl" else "cpu") if world > 1 \
        else LocalExchange()
    ex_dev = hs.DeviceExchange(dist, world, rank, odo.stream)

    def once(device=True, timing=None):
        rng = pkg.Rng()
        pkg.load().odo_rng_seed(pkg.ptr(rng), 12345)
        if device:
            return hs.sharded_ransac_device(odo, ex_dev, m, x1, x2, params, rng, float("nan"), timing)
        return hs.sharded_ransac(odo, ex_host, m, x1, x2, params, rng, float("nan"))

    def timed(device):
        for _ in range(2):
            out = once(device)
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = once(device)
        if world > 1:
            dist.barrier()
        dt = max_over_ranks(time.perf_counter() - t0, dist, world, device="cuda" if backend == "nccl" else "cpu")
        return dt / args.steps * 1e3, out

    ms_dev, out = timed(True)
    ms_host, out_h = timed(False)
    # the phase split of one call (each phase synchronised; measurement only)
    split = {}
    once(True, split)
    T, rmse, inl, ok, visited, _ = out
    same = bool(np.array_equal(T, out_h[0]) and rmse == out_h[1] and np.array_equal(inl, out_h[2]))
    if rank == 0:
        ex_ms = (split["all_gather"] + split["all_reduce"]) * 1e3
        print(json.dumps({
            "metric": f"RANSAC latency of one hard pair, hypotheses sharded (cfg3 fr2/desk proxy, H={H_})",
            "value": round(ms_dev, 4), "unit": "ms/pair", "n_gpus": world, "steps": args.steps,
            "higher_is_better": False, "scaling": "strong",
            "host_exchange_ms": round(ms_host, 4),
            "phase_ms": {k: round(v * 1e3, 4) for k, v in split.items()},
            "exchange_share": round(ex_ms / (split["total"] * 1e3), 4),
            "device_equals_host_protocol": same,
            "config": {"workload": f"cfg3 640x480 FR2 K + FR1 distortion, 4000 kp, H={H_}, "
                                   f"{int(100 * args.hyp_outliers)}% of the matches re-targeted",
                       "n_matches": int(m.size), "visited": int(visited), "n_inliers": int(len(inl)),
                       "ok": int(ok), "backend": backend or "single rank",
                       "exchange": "device: summaries exported to HBM, all_gather_into_tensor, ordered fold on the "
                                   "GPU, owner payload + int32 SUM all_reduce (value); host: 64-B summaries staged "
                                   "through host memory, host fold, owner broadcast (host_exchange_ms)"}}),
              flush=True)
    odo.close()


def hard_leg(pkg, synth, args, B, W, H, device):
    """The hard workload (synth.make_sequence(hard=True): image noise, depth
    noise ~ z^2, two independently moving cuboids, repeated texture, twice the
    inter-frame motion), same batched path and contract as the headline: the
    RANSAC of every pair runs most of its hypotheses."""
    import torch
    from importlib import import_module
    tj = import_module("arlm_amd.trajectory")
    L = min(args.seq_len, B)
    bgr, dep, gt = synth.make_sequence(L, W, H, seed=shard_seed(0), closed_loop=True, hard=True)
    idx = np.arange(B) % L
    d_bgr = torch.from_numpy(np.ascontiguousarray(bgr[idx])).to("cuda")
    d_dep = torch.from_numpy(np.ascontiguousarray(dep[idx]).view(np.int16)).to("cuda")
    cfg = pkg.default_config(W, H, B, nfeatures=args.nfeatures, iterations=args.iters, seed=rank_seeds(0)[1])
    odo = pkg.Odometry(cfg, device=device)
    torch.cuda.synchronize()
    res = odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=True)
    for _ in range(2):
        odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=False)
    res_q = odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=True)
    odo.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.hard_steps):
        odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=False)
    odo.synchronize()
    dt = time.perf_counter() - t0
    # SURVEY 8(d) RANSAC roofline on this workload: the stage time of one
    # untimed step with stage events (one stream) and the step's exact count
    # of Mahalanobis evaluations
    odo.set_timing(True)
    res_t = odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=True)
    odo.synchronize()
    tm = odo.timings()
    odo.set_timing(False)
    Tcw = tj.chain_poses(res[:L], np.linalg.inv(gt[0]).astype(np.float32))
    ate = 1000.0 * tj.ate_rmse(tj.camera_centres(Tcw), gt[:L, :3, 3])
    odo.close()
    ratio = res_q["n_inliers"] / np.maximum(res_q["n_good"], 1)
    rl = None
    if tm.get("ransac", 0) > 0:
        E = float(sum(int(r["n_sweeps"]) * int(r["n_good"]) for r in res_t))
        tr = tm["ransac"] * 1e-3
        rl = {"bound": "fp64", "achieved": round(E * RANSAC_FLOPS_PER_EVAL / tr / 1e12, 4), "peak": FP64_PEAK_TFLOPS,
              "unit": "TFLOP/s", "frac": round(E * RANSAC_FLOPS_PER_EVAL / tr / 1e12 / FP64_PEAK_TFLOPS, 5),
              "ms": round(tm["ransac"], 4), "evaluations": int(E),
              "work": f"E = sum(n_sweeps x n_good) x {RANSAC_FLOPS_PER_EVAL} FP64 flops (one stream, stage events)"}
    return {"value": round(B * args.hard_steps / dt, 2), "unit": "frames/s",
            "ms_per_step": round(dt / args.hard_steps * 1e3, 3), "steps": args.hard_steps,
            "workload": f"cfg2 {W}x{H}, {args.nfeatures} kp, RANSAC {args.iters}; image noise sigma 3, depth noise "
                        "1.425e-3 z^2, 2 moving cuboids, repeated floor/ceiling texture, 2x motion",
            "mean_matches": round(float(np.mean(res_q["n_matches"])), 1),
            "mean_inlier_ratio": round(float(np.mean(ratio)), 3),
            "mean_ransac_visited": round(float(np.mean(res_q["visited"])), 1),
            "mean_ransac_sweeps": round(float(np.mean(res_q["n_sweeps"])), 1),
            "mean_pnp_inliers": round(float(np.mean(res_q["pnp_inliers"])), 1),
            "ate_mm": round(ate, 3), "ransac_roofline": rl}


def pnpransac_mode(args):
    """PnPRansac::Compute (pnpransac.cpp:11-51), the
    cv::solvePnPRansac back-end, on one cfg2 pair: landmarks = frame 0's camera
    points of the KnnMatch matches, observations = frame 1's undistorted
    keypoints (a third of them re-targeted at random keypoints as outliers),
    500 iterations, 3 px, confidence 0.85. A latency metric: ms per call of
    odo_pnp_ransac (host arrays in and out); per-kernel times come from
    rocprofv3 of the same command."""
    import torch
    pkg = load_pkg()
    synth = load_synth()
    bgr, dep, _ = synth.make_sequence(2, args.width, args.height, seed=0x5EED0002)
    cfg = pkg.default_config(args.width, args.height, 2, nfeatures=args.nfeatures, iterations=200,
                             seed=0x5EED0002)
    odo = pkg.Odometry(cfg)
    odo.track_batch_host(bgr, dep)
    m = odo.pair(1)["matches"]
    f0, f1 = odo.frame(0), odo.frame(1)
    ok = f0["xyz"][m["queryIdx"], 2] > 0
    m = m[ok]
    Xw = np.ascontiguousarray(f0["xyz"][m["queryIdx"]])
    uv = np.ascontiguousarray(f1["kun"][m["trainIdx"]])
    rs = np.random.default_rng(5)
    sel = rs.random(len(uv)) < 1.0 / 3.0
    uv[sel] = f1["kun"][rs.integers(0, len(f1["kun"]), int(sel.sum()))]
    for _ in range(3):
        res, mask, _ = odo.pnp_ransac(Xw, uv, None, args.iters)
    torch.cuda.synchronize()
    ts = []
    for _ in range(max(args.steps, 5)):
        t0 = time.perf_counter()
        res, mask, _ = odo.pnp_ransac(Xw, uv, None, args.iters)
        ts.append((time.perf_counter() - t0) * 1e3)
    # the batched contract: B such problems (the same observations, outliers
    # re-drawn per problem) in one odo_pnp_ransac_batch launch chain
    B = 256
    probs = []
    for b in range(B):
        u2 = np.ascontiguousarray(f1["kun"][m["trainIdx"]])
        s2 = np.random.default_rng(100 + b).random(len(u2)) < 1.0 / 3.0
        u2[s2] = f1["kun"][np.random.default_rng(200 + b).integers(0, len(f1["kun"]), int(s2.sum()))]
        probs.append((Xw, u2))
    odo.pnp_ransac_batch(probs, None, args.iters)
    torch.cuda.synchronize()
    tb = []
    for _ in range(5):
        t0 = time.perf_counter()
        bres, _ = odo.pnp_ransac_batch(probs, None, args.iters)
        tb.append((time.perf_counter() - t0) * 1e3)
    bok = sum(int(r.ok == 1) for r in bres)
    odo.close()
    out = {"metric": "PnPRansac::Compute latency (cv::solvePnPRansac on the GPU, one call)",
           "value": round(float(np.median(ts)), 4), "unit": "ms/call (p50)", "n_gpus": 1, "steps": len(ts),
           "higher_is_better": False, "p90_ms": round(float(np.percentile(ts, 90)), 4),
           "observations": int(len(Xw)), "outliers_injected": int(sel.sum()), "ok": int(res.ok),
           "n_inliers": int(res.n_inliers), "iterations_visited": int(res.iterations_visited),
           "best_iter": int(res.best_iter),
           "batch": {"problems": B, "ms_per_batch": round(float(np.median(tb)), 3),
                     "problems_per_s": round(B / (float(np.median(tb)) / 1e3), 1), "ok": bok,
                     "api": "odo_pnp_ransac_batch (host arrays in and out)"},
           "config": {"workload": f"cfg2 pair {args.width}x{args.height}, {args.nfeatures} kp, "
                                  f"iterations {args.iters}, 3 px, confidence 0.85"}}
    if not args.no_cpu_baseline:
        O, build = oracle_for_baseline()
        c = cfg.calib
        cal = O.Calib(c.fx, c.fy, c.cx, c.cy, c.k1, c.k2, c.p1, c.p2, c.k3, c.depth_factor, c.mbf, c.th_depth)
        cts = []
        for _ in range(5):
            t0 = time.perf_counter()
            O.pnp_ransac(Xw, uv, cal, args.iters)
            cts.append((time.perf_counter() - t0) * 1e3)
        out["cpu_baseline"] = {"value": round(float(np.median(cts)), 3), "unit": "ms/call (median of 5)", "cores": 1,
                               "kind": "port", "sample": "the same call on oracle/pnpransac_ref.cpp", "build": build}
    print(json.dumps(out), flush=True)


def gicp_mode(args):
    """GeneralizedICP(10, 0.07)::Compute(source, target,
    T12) of Odometry::Compute's ADAPTIVE_RICP mode (odometry.cpp:46-78) on one
    cfg2 pair: Ransac::Iterate's matched clouds (depth-valid KnnMatch pairs,
    ransac.cpp:175-189) and the RANSAC T12 as the guess (odometry.cpp:61). A
    latency metric: ms per odo_gicp call (host clouds in, T12 out)."""
    import torch
    pkg = load_pkg()
    synth = load_synth()
    bgr, dep, _ = synth.make_sequence(2, args.width, args.height, seed=0x5EED0002)
    cfg = pkg.default_config(args.width, args.height, 2, nfeatures=args.nfeatures, iterations=200,
                             seed=0x5EED0002)
    odo = pkg.Odometry(cfg)
    res = odo.track_batch_host(bgr, dep)
    m = odo.pair(1)["matches"]
    f0, f1 = odo.frame(0), odo.frame(1)
    src, tgt = f0["xyz"][m["queryIdx"]], f1["xyz"][m["trainIdx"]]
    ok = (src[:, 2] > 0) & (tgt[:, 2] > 0)
    src, tgt = np.ascontiguousarray(src[ok]), np.ascontiguousarray(tgt[ok])
    guess = np.ascontiguousarray(np.asarray(res[1]["T12"], np.float32).reshape(4, 4))
    for _ in range(2):
        T, conv, it, nc = odo.gicp(src, tgt, guess, 10, 0.07)
    torch.cuda.synchronize()
    ts = []
    for _ in range(max(args.steps, 5)):
        t0 = time.perf_counter()
        T, conv, it, nc = odo.gicp(src, tgt, guess, 10, 0.07)
        ts.append((time.perf_counter() - t0) * 1e3)
    # 256 such pairs (guesses perturbed per pair) in one odo_gicp_batch chain
    B = 256
    rs = np.random.default_rng(7)
    pairs = []
    for b in range(B):
        g = guess.copy()
        g[:3, 3] += rs.normal(0, 0.005, 3).astype(np.float32)
        pairs.append((src, tgt, g))
    odo.gicp_batch(pairs, 10, 0.07)
    torch.cuda.synchronize()
    tb = []
    for _ in range(5):
        t0 = time.perf_counter()
        bout = odo.gicp_batch(pairs, 10, 0.07)
        tb.append((time.perf_counter() - t0) * 1e3)
    odo.close()
    out = {"metric": "GeneralizedICP::Compute latency (PCL GICP on the GPU, one call)",
           "value": round(float(np.median(ts)), 4), "unit": "ms/call (p50)", "n_gpus": 1, "steps": len(ts),
           "higher_is_better": False, "p90_ms": round(float(np.percentile(ts, 90)), 4),
           "points": [int(len(src)), int(len(tgt))], "converged": int(conv), "iterations": int(it),
           "correspondences": int(nc),
           "batch": {"pairs": B, "ms_per_batch": round(float(np.median(tb)), 3),
                     "pairs_per_s": round(B / (float(np.median(tb)) / 1e3), 1),
                     "converged": sum(o[1] for o in bout), "api": "odo_gicp_batch (host arrays in and out)"},
           "config": {"workload": f"cfg2 pair {args.width}x{args.height}, {args.nfeatures} kp: RANSAC's matched "
                                  "clouds, guess = RANSAC T12, GeneralizedICP(10, 0.07)"}}
    if not args.no_cpu_baseline:
        O, build = oracle_for_baseline()
        cts = []
        for _ in range(3):
            t0 = time.perf_counter()
            O.gicp(src, tgt, guess, 10, 0.07)
            cts.append((time.perf_counter() - t0) * 1e3)
        out["cpu_baseline"] = {"value": round(float(np.median(cts)), 3), "unit": "ms/call (median of 3)", "cores": 1,
                               "kind": "port", "sample": "the same call on oracle/gicp_ref.cpp", "build": build}
    print(json.dumps(out), flush=True)


def latency_mode(args):
    """Per-frame latency of the drop-in path alone (also the `latency` field of
    the track line): p50 / p99 ms per frame and per-stage medians."""
    W, H = args.width, args.height
    r = run_latency(args, W, H, max(args.steps, 16) + 8)
    print(json.dumps({"metric": "per-frame latency of the drop-in path (Tracking::Track order, one frame at a time)",
                      "value": r["p50_ms"], "unit": "ms/frame (p50)", "n_gpus": 1, "steps": r["frames"],
                      "warmup": r["warmup"], "higher_is_better": False, "p99_ms": r["p99_ms"], "p90_ms": r["p90_ms"],
                      "mean_ms": r["mean_ms"], "max_ms": r["max_ms"], "stage_median_ms": r["stage_median_ms"],
                      "config": {"workload": f"fr1/desk proxy {W}x{H}, 1000 kp (the reference's nFeatures, "
                                             f"common.h:77, as odo_frontend.hpp's Extractor uses it), "
                                             f"RANSAC {args.iters}",
                                 "mean_matches": r["mean_matches"], "mean_ransac_inliers": r["mean_ransac_inliers"],
                                 "path": "include/odo_frontend.hpp classes over the per-stage C-ABI"}}), flush=True)


def device_record(rank: int, dev: int):
    """This rank's GPU: index, name, arch and PCI address (domain:bus:device)."""
    import torch
    p = torch.cuda.get_device_properties(dev)
    return {"rank": rank, "device": dev, "name": p.name, "arch": p.gcnArchName.split(":")[0],
            "pci": f"{p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x}",
            "uuid": str(getattr(p, "uuid", ""))}


def gather_devices(rank: int, world: int, dev: int, dist=None):
    """Every rank's device_record on every rank (all_gather_object over the
    process group; the list alone for one rank)."""
    mine = device_record(rank, dev)
    if world <= 1:
        return [mine]
    out = [None] * world
    dist.all_gather_object(out, mine)
    return out


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def rank_envs(n: int, port: int, base=None):
    """Environment of each of n local ranks (one process per GPU): RANK =
    LOCAL_RANK = r, WORLD_SIZE = n, rendezvous on 127.0.0.1:port."""
    base = dict(os.environ if base is None else base)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC for RCCL on this host driver
    out = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        out.append(e)
    return out


def launch_ranks(n: int, argv, script=None) -> int:
    """`bench.py --gpus N` without a launcher: start N child processes of this
    script, one per GPU (rank r on device r), and wait for them. Runs before
    this process imports torch or touches a GPU, and starts children (never
    execs). Rank 0 prints the JSON line; the exit code is the first failing
    rank's (the others are terminated)."""
    import subprocess
    import threading
    envs = rank_envs(n, free_port())
    script = script or os.path.abspath(__file__)
    # stdout carries rank 0's JSON line only: whatever else a rank prints there
    # (the process-group library's connection notices, ...) goes to stderr
    procs = [subprocess.Popen([sys.executable, script] + list(argv), env=e,
                              stdout=subprocess.PIPE if r == 0 else 2, text=True)
             for r, e in enumerate(envs)]

    def relay(stream):
        for line in stream:
            (sys.stdout if line.lstrip().startswith("{") else sys.stderr).write(line)
            sys.stdout.flush()

    relay_t = threading.Thread(target=relay, args=(procs[0].stdout,), daemon=True)
    relay_t.start()
    rc = 0
    try:
        pending = set(range(n))
        while pending:
            for r in sorted(pending):
                c = procs[r].poll()
                if c is None:
                    continue
                pending.discard(r)
                if c != 0 and rc == 0:
                    rc = c
                    for q in pending:
                        procs[q].terminate()
            time.sleep(0.05)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
        relay_t.join(timeout=5)
    return rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256,
                    help="frames per step (the latency-bound pair stages see more pairs per launch at larger batches)")
    ap.add_argument("--seq-len", type=int, default=64, help="frames in the closed-loop sequence (motion per frame)")
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--iters", type=int, default=500, help="RANSAC hypotheses (mIterations)")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--cpu-frames", type=int, default=24, help="oracle sample (frames per timed pass)")
    ap.add_argument("--cpu-reps", type=int, default=5, help="timed oracle passes (median reported)")
    ap.add_argument("--host-steps", type=int, default=1, help="0: skip the from-host legs (they run --steps steps)")
    ap.add_argument("--latency-frames", type=int, default=120,
                    help="frames of the per-frame latency leg (odo_frontend.hpp path; 0: skip it)")
    ap.add_argument("--hard-steps", type=int, default=20, help="steps of the hard-workload leg (0: skip it)")
    ap.add_argument("--tum", default=None, help="a TUM RGB-D sequence directory with associations.txt "
                    "(utils.cpp:16-38 format): its frames replace the synthetic loop")
    ap.add_argument("--workload", choices=["default", "hard"], default="default",
                    help="main leg's sequence: the cfg2 proxy or the hard variant (synth hard=True)")
    ap.add_argument("--no-kernel-timing", action="store_true", help="no events around the kNN-2 launches")
    ap.add_argument("--no-direct-dispatch-leg", action="store_true",
                    help="skip the headline leg re-run with AMD_DIRECT_DISPATCH=1 (child process)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mode", choices=["track", "hyp", "latency", "pnpransac", "gicp"], default="track",
                    help="track: the frames/s metric; hyp: SURVEY 8(e) hypotheses mode latency (cfg3, H=4096); "
                         "latency: per-frame ms of the drop-in path through include/odo_frontend.hpp; "
                         "pnpransac / gicp: SURVEY 8(f) rank 4 back-end latency on a cfg2 pair")
    ap.add_argument("--hyp-outliers", type=float, default=0.5, help="hyp mode: fraction of matches re-targeted")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process group backend for N > 1 (gloo: several ranks sharing one GPU)")
    ap.add_argument("--shard", choices=["sequence", "independent"], default="sequence",
                    help="N > 1: 'sequence' = SURVEY 8(e) frames mode (one sequence, per-rank chunks + 1-frame "
                         "halo, latch broadcast, pose stitch); 'independent' = one sequence per rank")
    ap.add_argument("--detector", choices=["orb_slam2", "adaptive", "adaptive-orb"], default="orb_slam2",
                    help="orb_slam2: ORBextractor (the metric's config); adaptive: Extractor(FAST, ORB, ADAPTIVE); "
                         "adaptive-orb: Extractor(ORB, ORB, ADAPTIVE) (cv::ORB cell detector)")
    args = ap.parse_args()

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU, launched here (torch.distributed.run sets
        # WORLD_SIZE itself and lands in the branch below)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if "WORLD_SIZE" in os.environ and int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}")
    if args.mode == "latency":
        latency_mode(args)
        return
    if args.mode == "pnpransac":
        pnpransac_mode(args)
        return
    if args.mode == "gicp":
        gicp_mode(args)
        return
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank % max(1, torch.cuda.device_count()))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    if args.mode == "hyp":
        hyp_mode(args, rank, world, local_rank, dist)
        if world > 1:
            dist.destroy_process_group()
        return

    track_mode(args, rank, world, local_rank, dist)
    if world > 1:
        dist.destroy_process_group()


def knn_roofline(cmp: int, hbm_alg: float, knn_ms, launches, peaks, traffic, alone_ms=None, host_leg=None):
    """Roofline of the Hamming-match kernel (k_knn2_f4).

    Primary (round 5): the pipe the kernel runs on. Every (query, train)
    comparison is an exact sign-vector product on the matrix cores — 512 FP4
    MFMA ops (v_mfma_scale_f32_16x16x128_f8f6f4, e2m1 signs, K = 256) —
    so bound "mfma", achieved = 512 x comparisons / the kernel's mean duration
    over the timed region, peak = the dense FP4 spec (10.07 P ops/s). Beside
    it, `issue_ceiling`: the measured rate of the kernel's own per-tile
    instruction mix issued from registers (tools/ubench_peak.hip knn_f4_mix),
    the most this MFMA + top-2 epilogue form can reach.

    Secondary: SURVEY §8(d)'s VALU accounting (16 int32 lane-ops per
    comparison: 8 v_xor + 8 v_bcnt) as a rate, with the VALU spec beside it.
    The kernel does not execute those ops, so that rate is an equivalence, not
    a utilisation, and carries no fraction (alone it exceeds the VALU spec).
    kernel_ms = the live mean over the timed region (HIP events on the pair
    stream that runs the kernel)."""
    if not knn_ms:
        return None
    ops16 = float(KNN_OPS_PER_CMP) * cmp
    mops = 512.0 * cmp

    def fr(ms):
        a = mops / (ms * 1e-3) / 1e12
        d = {"kernel_ms": round(ms, 4), "achieved": round(a, 1), "frac": round(a / F4_MFMA_PEAK_TOPS, 4)}
        if "knn_f4_mix" in peaks:
            d["frac_of_issue_ceiling"] = round(a / peaks["knn_f4_mix"], 4)
        return d

    ach = mops / (knn_ms * 1e-3) / 1e12
    r = {"bound": "mfma", "achieved": round(ach, 1), "peak": F4_MFMA_PEAK_TOPS, "unit": "Top/s",
         "frac": round(ach / F4_MFMA_PEAK_TOPS, 4), "traffic": traffic, "kernel": "k_knn2_f4",
         "kernel_ms": round(knn_ms, 4), "launches": launches,
         "work": f"{cmp} descriptor comparisons x 512 FP4 MFMA ops (v_mfma_scale_f32_16x16x128_f8f6f4, "
                 "e2m1 sign vectors, K = 256: 2 k-steps of 128)",
         "peak_source": "MI355X_MICROARCH.md dense FP4 MFMA (no sparsity): 4x the dense BF16 rate per clock",
         "primary": "mfma_fp4 (the pipe the kernel executes on)",
         "issue_ceiling": {"achieved_peak": round(peaks.get("knn_f4_mix", float("nan")), 1),
                           "frac": round(ach / peaks["knn_f4_mix"], 4) if "knn_f4_mix" in peaks else None,
                           "source": "tools/ubench_peak.hip knn_f4_mix: the kernel's per-tile MFMA + top-2 mix "
                                     "from registers, 3 waves per SIMD"},
         "survey_8d_valu_equivalent": {
             "achieved": round(ops16 / (knn_ms * 1e-3) / 1e12, 2), "unit": "Top/s",
             "work": f"{cmp} comparisons x {KNN_OPS_PER_CMP} int32 lane-ops (8 v_xor + 8 v_bcnt, SURVEY 8(d))",
             "valu_spec": VALU_PEAK_TOPS, "measured_xor_bcnt_peak": round(peaks["valu_xor_bcnt"], 2),
             "note": "the comparisons run on the matrix cores, not as these VALU ops: an equivalent rate, "
                     "not a utilisation (no fraction)"},
         "hbm_gbs": round(hbm_alg / (knn_ms * 1e-3) / 1e9, 1)}
    if alone_ms:
        r["alone"] = fr(alone_ms)
    if host_leg:
        r["from_host_leg"] = fr(host_leg)
    return r


def run_latency(args, W, H, nframes):
    """tools/build/frontend_latency: one Tracking::Track frame at a time through
    include/odo_frontend.hpp (Extract -> KnnMatch -> Ransac::Iterate ->
    PnPSolver::Compute, each a synchronous C-ABI call) on the cfg2 sequence."""
    import subprocess
    import tempfile
    synth = load_synth()
    bgr, dep, _ = synth.make_sequence(64, W, H, seed=0x5EED0002, closed_loop=True)
    idx = np.arange(nframes) % 64
    exe = os.path.join(ROOT, "tools", "build", "frontend_latency")
    if not os.path.exists(exe):
        raise SystemExit("tools/build/frontend_latency missing: run make -C tools (done by __graft_entry__.build)")
    with tempfile.NamedTemporaryFile(suffix=".bin", dir=os.environ.get("TMPDIR", "/tmp")) as f:
        f.write(np.ascontiguousarray(bgr[idx]).tobytes())
        f.write(np.ascontiguousarray(dep[idx]).tobytes())
        f.flush()
        env = dict(os.environ)
        if not DIRECT_DISPATCH_FROM_ENV:
            env["AMD_DIRECT_DISPATCH"] = "1"
        out = subprocess.run([exe, f.name, str(W), str(H), str(nframes), str(args.iters), "8"], check=True,
                             capture_output=True, text=True, timeout=300, env=env).stdout
    rec = json.loads(out.strip().splitlines()[-1])
    rec["amd_direct_dispatch"] = env["AMD_DIRECT_DISPATCH"]
    return rec


def run_direct_dispatch(args):
    """The headline leg again in a child process with the HIP runtime's
    default direct dispatch (AMD_DIRECT_DISPATCH=1: the calling thread writes
    the packets), which is what a caller gets without setting anything; the
    headline runs with the worker-thread dispatch (DESIGN §4 Pipelining)."""
    import subprocess
    env = dict(os.environ)
    env["AMD_DIRECT_DISPATCH"] = "1"
    cmd = [sys.executable, os.path.abspath(__file__), "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--batch", str(args.batch), "--no-cpu-baseline", "--host-steps", "0", "--hard-steps", "0",
           "--latency-frames", "0", "--no-direct-dispatch-leg"]
    out = subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300, env=env).stdout
    d = json.loads(out.strip().splitlines()[-1])
    return {"value": d["value"], "unit": d["unit"], "ms_per_step": d["ms_per_step"], "step_ms": d.get("step_ms"),
            "amd_direct_dispatch": "1",
            "what": "the headline leg in a child process with HIP's default direct dispatch"}


def track_mode(args, rank, world, local_rank, dist):
    import torch
    from importlib import import_module
    ranks = gather_devices(rank, world, local_rank % max(1, torch.cuda.device_count()), dist)
    pkg = load_pkg()
    synth = load_synth()
    tj = import_module("arlm_amd.trajectory")
    B, W, H = args.batch, args.width, args.height
    # N > 1: SURVEY §8(e) frames mode by default: ONE sequence, each step's
    # B x N frames split into per-rank chunks with a one-frame halo, the latch
    # broadcast from rank 0, the poses stitched with an all_gather ("sequence");
    # "independent" gives every rank its own sequence (no exchange at all)
    seq_mode = world > 1 and args.shard == "sequence"
    scene_seed, pair_seed = rank_seeds(0 if seq_mode else rank)
    # a closed loop of --seq-len distinct frames (fixed inter-frame motion);
    # a batch of B frames walks it cyclically, so every pair is a genuine
    # consecutive pair whatever B is
    L = min(args.seq_len, B)
    if B % L:
        raise SystemExit(f"--batch {B} must be a multiple of --seq-len {L} (pair 0 links frame B-1 to frame 0)")
    if args.tum:
        # a real TUM sequence (associations.txt, utils.cpp:16-38): its first L
        # frames, cycled through the batch like the synthetic loop (the wrap
        # pair jumps back; no ground truth, so no ATE)
        tum = load_module("arlm_amd_tum", os.path.join(PKG_DIR, "tum.py"))
        bgr_loop, dep_loop, _ = tum.load_sequence(args.tum, L)
        if bgr_loop.shape[0] < L or bgr_loop.shape[1:3] != (H, W):
            raise SystemExit(f"--tum: need {L} frames of {W}x{H}, got {bgr_loop.shape}")
        gt_poses = None
    else:
        bgr_loop, dep_loop, gt_poses = synth.make_sequence(L, W, H, seed=scene_seed, closed_loop=True,
                                                           hard=args.workload == "hard")
    bgr, dep = bgr_loop[np.arange(B) % L], dep_loop[np.arange(B) % L]
    adaptive = args.detector in ("adaptive", "adaptive-orb")
    inner = "orb" if args.detector == "adaptive-orb" else "fast"
    if adaptive:
        args.nfeatures = 1000  # Extract's retainBest(nFeatures), common.h:77
        if seq_mode:
            raise SystemExit("ADAPTIVE thresholds carry from frame to frame: not frame-shardable (--shard independent)")
    fb = (W * H * 3, W * H * 2)
    # the rank's input frames; frames mode: every chunk starts at a multiple of
    # L, so its halo is loop frame L - 1, followed by the chunk's B frames
    hb = np.concatenate([bgr_loop[L - 1:], bgr]) if seq_mode else bgr
    hd = np.concatenate([dep_loop[L - 1:], dep]) if seq_mode else dep
    nb = hb.shape[0]
    d_bgr = torch.from_numpy(hb).to("cuda")                # HBM-resident leg
    d_dep = torch.from_numpy(hd.view(np.int16)).to("cuda")
    hf = pkg.HostFrames(nb, W, H)                           # from-host legs (pinned)
    hf.bgr[:] = hb
    hf.depth[:] = hd
    cfg = pkg.default_config(W, H, nb, nfeatures=args.nfeatures, iterations=args.iters, seed=pair_seed,
                             detector=(pkg.DETECTOR_ORB_SLAM2 if not adaptive else
                                       pkg.DETECTOR_ADAPTIVE_ORB if inner == "orb" else pkg.DETECTOR_ADAPTIVE_FAST))
    odo = pkg.Odometry(cfg, device=local_rank % max(1, torch.cuda.device_count()))
    torch.cuda.synchronize()
    coll_dev = "cuda" if args.backend == "nccl" else "cpu"  # where the exchanges' tensors live
    ktime = not args.no_kernel_timing
    K, Wm = args.steps, args.warmup
    head_marks = []  # the headline leg's per-batch step marks (kernel timing on)

    if seq_mode:
        fsm = import_module("arlm_amd.frames_shard")
        T = B * world
        shard = fsm.FramesShard(odo, dist, rank, world, T, device=coll_dev)
        # the DepthCovariance latch of global pair 1 (loop frames 0, 1), broadcast
        shard.prime_latch(d_bgr.data_ptr() + fb[0], d_dep.data_ptr() + fb[1])
        rows = max(K, Wm, 2) + 1
        ring = pkg.PinnedResults(rows, B + 1)
        kstep = [0]  # global step counter across legs (frames repeat every step)
        timed_steps = []

        def step(host, keep=None):
            k = kstep[0]
            kstep[0] += 1
            row = k % rows
            if host:
                shard.track_step_host(k, hf, ring, row)
            else:
                shard.track_step(k, d_bgr.data_ptr(), d_dep.data_ptr(), fb, results=ring, row=row)
            if keep is not None:
                keep.append(k)

        def stitch_timed():
            ks = timed_steps[-K:]
            shard.stitch([ring.all[k % rows][:fsm.batch_of(k, T, rank, world)[1]] for k in ks], ks)

        # untimed: steps 0 and 1 with results for the statistics and the ATE
        step(False)
        step(False)
        odo.synchronize()
        recs = [ring.all[k][:fsm.batch_of(k, T, rank, world)[1]].copy() for k in range(2)]
        G = shard.stitch(recs, [0, 1], G_start=np.linalg.inv(gt_poses[0]) if gt_poses is not None else None)
        # ATE over rank 0's first loop (global frames 0 .. L-1 of step 0)
        ate_mm = 1000.0 * tj.ate_rmse(tj.camera_centres(G[0][:L]), gt_poses[:L, :3, 3]) \
            if rank == 0 and gt_poses is not None else None
        res_q = recs[-1][1:]  # a halo step: B genuine pairs, record p+1 = pair (frame p, frame p+1)
        pair_frame0 = 1       # batch frame of record 0 of res_q

        def leg(host, marks_out=None):
            return timed_leg(odo, lambda i: step(host, timed_steps if i >= Wm else None), K, Wm, world, dist,
                             coll_dev, ktime, inside=stitch_timed, marks_out=marks_out)

        # the headline: inputs resident in HBM
        elapsed, submit, (knn_ms, knn_launches) = leg(False, head_marks)
        # from host memory: every rank uploads its chunk + halo over its own link
        h_el, h_sub, (h_knn_ms, _) = leg(True) if args.host_steps > 0 else (None, None, (None, 0))
        sd = None
        odo.set_timing(True)
        step(False)
        odo.synchronize()
        timings = odo.timings()
        odo.set_timing(False)
        ring.close()
        frames_per_rank = B  # pairs (= new frames) per rank per step
    else:
        # untimed: one batch with results for the sanity summary
        res = odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=True)
        # untimed: a batch whose pair 0 links to the previous batch, as in the timed
        # steps, for the kNN-2 query counts (F1 keypoints holding a VO landmark)
        res_q = odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=True)
        pair_frame0 = 0
        odo.synchronize()
        # quality sanity: the untimed first batch's chained poses against the
        # sequence's ground truth (absolute trajectory error, TUM definition)
        ate_mm = None
        if gt_poses is not None:
            Tcw = tj.chain_poses(res[:L], np.linalg.inv(gt_poses[0]).astype(np.float32))
            ate_mm = 1000.0 * tj.ate_rmse(tj.camera_centres(Tcw), gt_poses[:L, :3, 3])
        # the headline: inputs resident in HBM; every batch's pair records
        # (poses, counts) stream back into a pinned ring inside the timed
        # region, as Track hands each frame's pose to its caller
        rows = K + Wm
        ring = pkg.PinnedResults(rows, B)
        # ODO_BENCH_PACE_MS (measurement only): the host waits this long after
        # queueing each batch (does the pipeline state depend on how far the
        # host runs ahead?)
        pace = float(os.environ.get("ODO_BENCH_PACE_MS", "0")) * 1e-3

        def head_step(i):
            odo.track_batch_async(d_bgr.data_ptr(), d_dep.data_ptr(), B, ring, i % rows)
            if pace > 0:
                t_end = time.perf_counter() + pace
                while time.perf_counter() < t_end:
                    pass

        elapsed, submit, (knn_ms, knn_launches) = timed_leg(odo, head_step, K, Wm, world, dist, coll_dev, ktime,
                                                            marks_out=head_marks)
        # the last timed batch's records arrived: its match and query counts
        # equal any batch's after the first (every batch cycles the same loop;
        # the RANSAC outcome differs, each pair's seed is its global index)
        last = ring.all[(K + Wm - 1) % rows][:B]
        # (ADAPTIVE detectors: the per-cell thresholds carry from frame to
        # frame over every batch, so the same loop frames extract differently
        # from batch to batch and only a sanity check applies; their parity
        # is tests/test_bench_config_adaptive.py)
        for f in ("n_matches", "n_queries"):
            if adaptive:
                if int(np.count_nonzero(last[f])) < B // 2:
                    raise SystemExit(f"timed leg: streamed pair records mostly empty ({f})")
            elif not np.array_equal(last[f], res_q[f]):
                raise SystemExit(f"timed leg: streamed pair records differ from the untimed batch ({f})")
        ring.close()
        h_el = sd = None
        h_knn_ms = None
        if args.host_steps > 0:
            # from pinned host memory: one upload per batch on the copy stream
            h_el, h_sub, (h_knn_ms, _) = timed_leg(odo, lambda i: odo.track_batch_host(hf, want_results=False),
                                                   K, Wm, world, dist, coll_dev, ktime)
            # the same with the depth frames read in place (keypoint pixels only)
            sd_el, _, _ = timed_leg(odo, lambda i: odo.track_batch_host_sparse_depth(hf, want_results=False),
                                    K, Wm, world, dist, coll_dev, False)
            sd = {"value": round(job_throughput(B, K, world, sd_el), 2), "unit": "frames/s",
                  "ms_per_step": round(sd_el / K * 1e3, 3),
                  "api": "odo_track_batch_host_sparse_depth: BGR uploaded, depth read in place "
                         "(keypoint pixels only) from the pinned host frames"}
        # per-stage times: one extra (untimed) step with the stage events on
        odo.set_timing(True)
        odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=False)
        odo.synchronize()
        timings = odo.timings()
        odo.set_timing(False)
        frames_per_rank = B
    value = job_throughput(frames_per_rank, K, world, elapsed)
    ms_per_step = elapsed / K * 1e3

    from_host = None
    if h_el is not None:
        nbytes_frame = fb[0] + fb[1]
        fps = job_throughput(frames_per_rank, K, world, h_el)
        raw = raw_h2d_gbs(nb * nbytes_frame)
        from_host = {"value": round(fps, 2), "unit": "frames/s", "ms_per_step": round(h_el / K * 1e3, 3),
                     "steps": K, "warmup": Wm, "bytes_per_frame": nbytes_frame,
                     "h2d_gbs_per_gpu": round(nb * nbytes_frame * K / h_el / 1e9, 2),
                     "raw_pinned_h2d_gbs": round(raw, 2),
                     "pcie_bound_fps_per_gpu": round(raw * 1e9 / nbytes_frame * frames_per_rank / nb, 1),
                     "inputs": ("pinned host buffers (odo_host_alloc), each rank uploading its chunk + halo "
                                "(odo_track_batch_host_async)" if seq_mode else
                                "pinned host buffers (odo_host_alloc), one upload per batch on the copy stream "
                                "(odo_track_batch_host)"),
                     "sparse_depth": sd}
    hf.close()

    # keypoints of the frames the statistics' pairs match against (every batch
    # holds the same cycled frames): pair record i's train frame
    nkp = [len(odo.frame(pair_frame0 + i)["kps"]) for i in range(B)]
    nkp_mean = float(np.mean(nkp))
    peaks = measured_peaks()
    # result i = pair (frame i-1, frame i): kNN-2 compares the query frame's
    # landmark keypoints (n_queries) with every keypoint of frame i
    nq = res_q["n_queries"]
    cmp = int(sum(int(nq[i]) * nkp[i] for i in range(B)))
    hbm_alg = sum(32 * int(nq[i]) + 32 * nkp[i] + 16 * int(nq[i]) for i in range(B))
    traffic = traffic_src = None
    if os.path.exists(KNN_F4_TRAFFIC):
        with open(KNN_F4_TRAFFIC) as fh:
            tr4 = json.load(fh)
        # PMC HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, gfx950
        # correction), scaled per pair when the batch differs
        traffic = tr4["hbm_bytes_per_launch"] if tr4.get("batch") == B else tr4["hbm_bytes_per_pair"] * B
        traffic_src = {"file": os.path.relpath(KNN_F4_TRAFFIC, ROOT), "build": tr4.get("build"),
                       "per_launch_of_batch": tr4.get("batch")}
    alone = odo.knn_replay_ms(20) if knn_ms else None
    roofline = knn_roofline(cmp, hbm_alg, knn_ms, knn_launches, peaks, traffic, alone, h_knn_ms) \
        if cfg.forms.knn == pkg.KNN_FORM_FP4 else None
    if roofline is not None:
        roofline["traffic_source"] = traffic_src
        roofline["traffic_algorithmic"] = int(hbm_alg)

    # the other SURVEY §8(d) legs, from the per-stage (one stream, events
    # between stages) times of the untimed timing step
    ext_stages = [k for k in ("gray+pyramid", "gray", "smap+cand", "fast", "octree", "chain+select", "blur", "finalize")
                  if k in timings]
    ext_ms = sum(timings[k] for k in ext_stages)
    comp_bytes = B * (5 * W * H + 84 * nkp_mean)  # compulsory I/O per frame: 5WH + 84N
    legs = {"extraction": {"bound": "hbm", "achieved": round(comp_bytes / (ext_ms * 1e-3) / 1e9, 1),
                           "peak": HBM_PEAK_GBS, "unit": "GB/s",
                           "frac": round(comp_bytes / (ext_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                           "measured_peak_read": peaks["hbm_read"], "ms": round(ext_ms, 4),
                           "work": f"compulsory bytes 5WH + 84N per frame x {B} frames", "stages": ext_stages}}
    ok_res = res_q[1:] if len(res_q) > 1 else res_q
    E = float(sum(int(r["n_sweeps"]) * int(r["n_good"]) for r in res_q))
    F = float(sum(int(r["n_fit_points"]) for r in res_q))
    if "ransac" in timings and timings["ransac"] > 0:
        t = timings["ransac"] * 1e-3
        legs["ransac"] = {"bound": "fp64", "achieved": round(E * RANSAC_FLOPS_PER_EVAL / t / 1e12, 4),
                          "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                          "frac": round(E * RANSAC_FLOPS_PER_EVAL / t / 1e12 / FP64_PEAK_TFLOPS, 5),
                          "measured_peak_fma": peaks["fp64_fma"], "ms": round(timings["ransac"], 4),
                          "evaluations": int(E), "fit_points": int(F),
                          "fp32_fit_tflops": round(F * RANSAC_FLOPS_PER_FIT_POINT / t / 1e12, 5),
                          "mean_sweeps_per_pair": round(float(np.mean(ok_res["n_sweeps"])), 2),
                          "work": f"E = sum(n_sweeps x n_good) x {RANSAC_FLOPS_PER_EVAL} FP64 flops"}
    if "pnp" in timings:
        legs["pnp"] = {"bound": "latency", "ms": round(timings["pnp"], 4)}
    odo.close()
    del d_bgr, d_dep

    hard = None
    if args.hard_steps > 0 and world == 1 and not adaptive:
        hard = hard_leg(pkg, synth, args, B, W, H, local_rank % max(1, torch.cuda.device_count()))

    latency = None
    if args.latency_frames > 0 and world == 1 and not adaptive and rank == 0:
        r = run_latency(args, W, H, args.latency_frames + 8)
        latency = {"p50_ms": r["p50_ms"], "p90_ms": r["p90_ms"], "p99_ms": r["p99_ms"], "mean_ms": r["mean_ms"],
                   "max_ms": r["max_ms"], "frames": r["frames"], "warmup": r["warmup"],
                   "stage_median_ms": r["stage_median_ms"],
                   "workload": f"fr1/desk proxy {W}x{H}, 1000 kp (the reference's nFeatures, common.h:77), "
                               f"RANSAC {args.iters}, one frame at a time",
                   "path": "include/odo_frontend.hpp Extractor / Matcher / Ransac / PnPSolver over the per-stage "
                           "C-ABI (tools/frontend_latency.cpp), Tracking::Track order"}

    direct = None
    if rank == 0 and world == 1 and not args.no_direct_dispatch_leg and not adaptive and args.workload == "default" \
            and not args.tum:
        direct = run_direct_dispatch(args)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        nf = args.cpu_frames
        cb = cpu_baseline(bgr, dep, args.nfeatures, args.iters, nf, args.cpu_reps, adaptive, inner=inner)
        hi = host_info()
        cpu = {"value": round(cb["fps"], 3), "unit": "frames/s", "cores": 1, "kind": "port",
               "sample": f"{nf} frames of the rank-0 {L}-frame closed loop through the C++ oracle's extract + "
                         f"match + RANSAC + PnP, one thread pinned to core {cb['core']}, median of {cb['reps']} "
                         f"passes after a warm-up ({cb['seconds']:.2f} s per pass)",
               "stage_ms": cb["stage_ms"], "host": hi, "build": cb["build"],
               "all_cores": {"value": round(cb["all_cores"]["fps"], 2), "unit": "frames/s",
                             "cores": cb["all_cores"]["threads"],
                             "sample": f"{cb['all_cores']['frames']} frames, frames-parallel thread pool "
                                       f"(extraction and pairs) over every usable core, median of 3 passes"}}

    if rank == 0:
        ok = res_q
        out = {
            "metric": "frames/sec (extract+match+RANSAC-PnP) @640x480, 2000 kp" if not adaptive else
                      f"frames/sec (ADAPTIVE {'cv::ORB' if inner == 'orb' else 'FAST'} grid + ORB, match, "
                      f"RANSAC-PnP) @640x480, <=1000 kp",
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": K,
            "warmup": Wm,
            "ms_per_step": round(ms_per_step, 3),
            "step_ms": step_stats(head_marks),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/i32 (extract, match), f32+f64 (ransac, pnp)",
            "data": (f"TUM sequence {args.tum} (first {L} frames, cycled)" if args.tum else
                     "synthetic (ray-cast textured room, closed-loop trajectory; no dataset offline)"),
            "inputs": "resident in HBM when the timed region starts (from_host: the same path from pinned host memory)",
            "config": {"workload": (f"cfg2 fr1/desk proxy {W}x{H}, {args.nfeatures} kp, RANSAC {args.iters}"
                                    + (" (hard variant)" if args.workload == "hard" else "")
                                    if not adaptive else
                                    f"fr1/desk proxy {W}x{H}, ADAPTIVE 3x3 {'cv::ORB' if inner == 'orb' else 'FAST'} "
                                    f"grid + ORB (<=1000 kp), "
                                    f"RANSAC {args.iters}"),
                       "frames_per_step": B, "global_batch": B * world,
                       "parallelism": (f"sequence chunks x{world} (+1-frame halo, latch broadcast, pose stitch)"
                                       if seq_mode else f"frames x{world}"),
                       "world_size": world,
                       "backend": dist.get_backend() if world > 1 else None,
                       "distinct_devices": len({r["pci"] for r in ranks}),
                       "ranks": ranks,
                       "mean_keypoints": round(nkp_mean, 1),
                       "mean_knn_queries": round(float(np.mean(res_q["n_queries"])), 1),
                       "mean_matches": round(float(np.mean(ok["n_matches"])), 1),
                       "mean_ransac_inliers": round(float(np.mean(ok["n_inliers"])), 1),
                       "mean_ransac_visited": round(float(np.mean(ok["visited"])), 1),
                       "ate_mm": round(ate_mm, 3) if ate_mm is not None else None},
            "stage_ms": {k: round(v, 4) for k, v in timings.items()},
            "host_submit_ms_per_step": round(submit / K * 1e3, 3),
            "hip_runtime": {"AMD_DIRECT_DISPATCH": os.environ.get("AMD_DIRECT_DISPATCH"),
                            "dispatch": "worker thread" if os.environ.get("AMD_DIRECT_DISPATCH") == "0" else "direct",
                            "direct_dispatch_leg": direct},
            "from_host": from_host,
            "hard_workload": hard,
            "latency": latency,
            "roofline": roofline,
            "roofline_legs": legs,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
