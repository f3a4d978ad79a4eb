#!/usr/bin/env python3
"""bench.py — frames/sec of the per-frame odometry hot path on MI355X.

Metric (BASELINE.json): frames/sec (extract + match + RANSAC-PnP) at 640x480,
2000 ORB keypoints. Workload = config 2 ("TUM fr1/desk proxy": 640x480, FR1
intrinsics + distortion, 2000 kp, RANSAC 500 hypotheses) on a synthetic
closed-loop RGB-D sequence (no datasets offline). One step = one batch of
`--batch` frames through Tracking::Track's hot path (extract every frame,
kNN-2 + ratio match against its predecessor, Ransac::Iterate, PnPSolver),
inputs resident in HBM. Multi-GPU: one process per GPU, each tracking its
own sequence (frames mode, weak scaling, no data-path collective).

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

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG_DIR = os.path.join(ROOT, "adaptive-rgbd-localization-mappig_amd")

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# int32 VALU lane-ops: 256 CU x 4 SIMD x 16 lanes/clk (a wave64 VALU op issues
# every 4 clk, MI355X_MICROARCH.md cycle constants) x 2.4 GHz
INT_VALU_PEAK_TOPS = 256 * 4 * 16 * 2.4e9 / 1e12
# Hamming-match work per (query, train) comparison: 8 xor + 8 popcount over the
# 256-bit descriptors, key formation, and the top-2 update (min + med3)
KNN_OPS_PER_CMP = 19
KNN_TRAFFIC = os.path.join(ROOT, "profiles", "r01_knn2_traffic.json")


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
    """Each rank tracks its own sequence (independent scene seed)."""
    return 0x5EED0002 + 7919 * rank


def rank_seeds(rank: int):
    """(scene seed, RANSAC/pair seed base) of one rank: ranks shard the frames
    (each tracks its own sequence), no data-path collective."""
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


def level_pixels(w, h, nlevels=8, scale=1.2):
    s, tot, lv = 1.0, 0, []
    for l in range(nlevels):
        inv = np.float32(1.0) / np.float32(s)
        lw, lh = int(np.rint(np.float32(w) * inv)), int(np.rint(np.float32(h) * inv))
        lv.append((lw, lh))
        tot += lw * lh
        s = float(np.float32(np.float64(np.float32(s)) * np.float64(np.float32(scale))))
    return tot, lv


def stage_model(stage, ms, B, w, h, nkp_mean):
    """Algorithmic work per launch of a stage -> (bound, achieved, peak, unit, work)."""
    pyr_px, lv = level_pixels(w, h)
    if stage == "gray+pyramid":
        byts = B * (3 * w * h + w * h + sum(2 * a * b for a, b in lv[1:]) + sum(a * b for a, b in lv[:-1]))
        return "hbm", byts / (ms * 1e-3) / 1e9, HBM_PEAK_GBS, "GB/s", byts
    if stage == "blur":
        byts = B * 2 * pyr_px
        return "hbm", byts / (ms * 1e-3) / 1e9, HBM_PEAK_GBS, "GB/s", byts
    if stage == "fast":
        byts = B * pyr_px
        return "hbm", byts / (ms * 1e-3) / 1e9, HBM_PEAK_GBS, "GB/s", byts
    if stage == "knn2":
        ops = B * float(KNN_OPS_PER_CMP) * nkp_mean * nkp_mean
        return "valu", ops / (ms * 1e-3) / 1e12, INT_VALU_PEAK_TOPS, "Top/s", ops
    byts = B * (5 * w * h + 84 * nkp_mean)
    return "hbm", byts / (ms * 1e-3) / 1e9, HBM_PEAK_GBS, "GB/s", byts


def cpu_baseline(bgr, dep, nfeat, iters, n_frames, adaptive=False):
    """The C++ oracle (single thread) on the first n_frames frames of the same sequence."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    cal = O.fr1_calib()
    p = O.orb_params(nfeat)
    rp = O.ransac_params(iters)
    pkg = load_pkg()
    ex = O.AdaptiveExtractor() if adaptive else None
    t0 = time.perf_counter()
    prev = None
    latch = float("nan")
    for i in range(n_frames):
        if ex is not None:
            f = ex.extract_frame(bgr[i % len(bgr)], dep[i % len(dep)], cal)
        else:
            f = O.extract_frame(bgr[i % len(bgr)], dep[i % len(dep)], p, cal)
        if prev is not None:
            _, _, _, latch = O.track_pair(prev, f, cal, rp, pkg.pair_seed(0x5EED0000, i), latch)
        prev = f
    dt = time.perf_counter() - t0
    return n_frames / dt, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256,
                    help="frames per step (MI355X: 45.7k / 52.9k / 56.8k / 57.0k frames/s at 64 / 128 / 192 / 256: "
                         "the latency-bound pair stages see more pairs per launch)")
    ap.add_argument("--seq-len", type=int, default=64, help="frames in the closed-loop sequence (motion per frame)")
    ap.add_argument("--nfeatures", type=int, default=2000)
    ap.add_argument("--iters", type=int, default=500, help="RANSAC hypotheses (mIterations)")
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--cpu-frames", type=int, default=192, help="oracle sample size (frames, ~10 s)")
    ap.add_argument("--no-kernel-timing", action="store_true", help="no events around the kNN-2 launches")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--detector", choices=["orb_slam2", "adaptive"], default="orb_slam2",
                    help="orb_slam2: ORBextractor (the metric's config); adaptive: Extractor(FAST, ORB, ADAPTIVE)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))

    pkg = load_pkg()
    synth = load_synth()
    B, W, H = args.batch, args.width, args.height
    scene_seed, pair_seed = rank_seeds(rank)
    # a closed loop of --seq-len distinct frames (fixed inter-frame motion);
    # a batch of B frames walks it cyclically, so every pair is a genuine
    # consecutive pair whatever B is
    L = min(args.seq_len, B)
    if B % L:
        raise SystemExit(f"--batch {B} must be a multiple of --seq-len {L} (pair 0 links frame B-1 to frame 0)")
    bgr, dep, gt_poses = synth.make_sequence(L, W, H, seed=scene_seed, closed_loop=True)
    if B != L:
        bgr, dep = bgr[np.arange(B) % L], dep[np.arange(B) % L]
    d_bgr = torch.from_numpy(bgr).to("cuda")
    d_dep = torch.from_numpy(dep.view(np.int16)).to("cuda")
    adaptive = args.detector == "adaptive"
    if adaptive:
        args.nfeatures = 1000  # Extract's retainBest(nFeatures), common.h:77
    cfg = pkg.default_config(W, H, B, nfeatures=args.nfeatures, iterations=args.iters, seed=pair_seed,
                             detector=pkg.DETECTOR_ADAPTIVE_FAST if adaptive else pkg.DETECTOR_ORB_SLAM2)
    odo = pkg.Odometry(cfg, device=local_rank)
    torch.cuda.synchronize()

    # untimed: one batch with results for the sanity summary
    res = odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=True)
    for _ in range(args.warmup):
        odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=False)
    # untimed: a batch whose pair 0 links to the previous batch, as in the timed
    # steps, for the kNN-2 query counts (F1 keypoints holding a VO landmark)
    res_q = odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=True)
    odo.synchronize()
    torch.cuda.synchronize()

    if world > 1:
        dist.barrier()
    # Hamming-match (kNN-2) launches are bracketed by HIP events on the stream
    # that runs them (a pair stream by default) inside the timed region (odo
    # timing mode 2)
    if not args.no_kernel_timing:
        odo.set_timing(None, mode=2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=False)
    submit = time.perf_counter() - t0  # host time to queue the K steps (asynchronous)
    odo.synchronize()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = max_over_ranks(time.perf_counter() - t0, dist, world)
    knn_ms, knn_launches = odo.kernel_timing() if not args.no_kernel_timing else (None, 0)

    # per-stage times: one extra (untimed) step with the stage events on
    odo.set_timing(True)
    odo.track_batch(d_bgr.data_ptr(), d_dep.data_ptr(), B, want_results=False)
    odo.synchronize()
    timings = odo.timings()
    odo.set_timing(False)
    value = job_throughput(B, args.steps, world, elapsed)
    ms_per_step = elapsed / args.steps * 1e3

    nkp = [len(odo.frame(i)["kps"]) for i in range(B)]
    # quality sanity: the untimed first batch's chained poses against the
    # sequence's ground truth (absolute trajectory error, TUM definition)
    from importlib import import_module
    tj = import_module("arlm_amd.trajectory")
    Tcw = tj.chain_poses(res[:L], np.linalg.inv(gt_poses[0]).astype(np.float32))
    ate_mm = 1000.0 * tj.ate_rmse(tj.camera_centres(Tcw), gt_poses[:L, :3, 3])
    nkp_mean = float(np.mean(nkp))
    # Roofline of the Hamming-match kernel (k_knn2), the kernel the north star
    # names. Brute-force kNN-2 re-reads each 32-byte descriptor ~2000 times from
    # LDS, so it is bound by the integer VALU issue rate, not by HBM: achieved =
    # algorithmic lane-ops of one launch / its live mean duration.
    roofline = None
    if knn_ms:
        # result i = pair (frame i-1, frame i); frame -1 is the previous batch's
        # last frame (the same sequence is tracked every step). kNN-2 compares
        # the query frame's landmark keypoints (n_queries) with every keypoint
        # of frame i: Matcher::KnnMatch drops the other queries' matches
        nq = res_q["n_queries"]
        cmp = int(sum(int(nq[i]) * nkp[i] for i in range(B)))
        ops = float(KNN_OPS_PER_CMP) * cmp
        ach = ops / (knn_ms * 1e-3) / 1e12
        traffic = None
        if os.path.exists(KNN_TRAFFIC):
            with open(KNN_TRAFFIC) as f:
                tr = json.load(f)
            # PMC-measured HBM bytes (FETCH_SIZE x2 + WRITE_SIZE) per launch;
            # scaled per pair when this run's batch differs from the profiled one
            traffic = tr.get("hbm_bytes_per_launch") if tr.get("batch") == B else \
                (tr["hbm_bytes_per_pair"] * B if "hbm_bytes_per_pair" in tr else None)
        roofline = {"bound": "valu", "achieved": round(ach, 3), "peak": round(INT_VALU_PEAK_TOPS, 2),
                    "unit": "Top/s", "frac": round(ach / INT_VALU_PEAK_TOPS, 4), "traffic": traffic,
                    "kernel": "k_knn2", "kernel_ms": round(knn_ms, 4), "launches": knn_launches,
                    "work": f"{cmp} descriptor comparisons x {KNN_OPS_PER_CMP} int32 lane-ops",
                    # algorithmic HBM bytes: every descriptor read once, 16 B of top-2 out per query
                    "hbm_gbs": round(sum(32 * int(nq[i]) + 32 * nkp[i] + 16 * int(nq[i]) for i in range(B)) /
                                     (knn_ms * 1e-3) / 1e9, 1)}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        nf = args.cpu_frames
        fps, dt = cpu_baseline(bgr, dep, args.nfeatures, args.iters, nf, adaptive)
        cpu = {"value": round(fps, 3), "unit": "frames/s", "cores": 1, "kind": "port",
               "sample": f"{nf} frames (the rank-0 {L}-frame closed loop, cycled) through the C++ oracle's "
                         f"extract + match + RANSAC + PnP, single thread ({dt:.1f} s)"}

    if rank == 0:
        ok = res[1:]
        out = {
            "metric": "frames/sec (extract+match+RANSAC-PnP) @640x480, 2000 kp" if not adaptive else
                      "frames/sec (ADAPTIVE FAST grid + ORB, match, RANSAC-PnP) @640x480, <=1000 kp",
            "value": round(value, 2),
            "unit": "frames/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8/i32 (extract, match), f32+f64 (ransac, pnp)",
            "data": "synthetic (ray-cast textured room, closed-loop trajectory; no dataset offline)",
            "config": {"workload": (f"cfg2 fr1/desk proxy {W}x{H}, {args.nfeatures} kp, RANSAC {args.iters}"
                                    if not adaptive else
                                    f"fr1/desk proxy {W}x{H}, ADAPTIVE 3x3 FAST grid + ORB (<=1000 kp), "
                                    f"RANSAC {args.iters}"),
                       "frames_per_step": B, "global_batch": B * world, "parallelism": f"frames x{world}",
                       "mean_keypoints": round(nkp_mean, 1),
                       "mean_knn_queries": round(float(np.mean(res_q["n_queries"])), 1),
                       "mean_matches": round(float(np.mean(ok["n_matches"])), 1),
                       "mean_ransac_inliers": round(float(np.mean(ok["n_inliers"])), 1),
                       "mean_ransac_visited": round(float(np.mean(ok["visited"])), 1),
                       "ate_mm": round(ate_mm, 3)},
            "stage_ms": {k: round(v, 4) for k, v in timings.items()},
            "host_submit_ms_per_step": round(submit / args.steps * 1e3, 3),
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out), flush=True)
    odo.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
