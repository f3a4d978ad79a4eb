"""Per-kernel statistics of exactly the timed region of a `bench.py` run from
its rocprofv3 kernel trace (the roofline must recompute
from a rocprof summary of the timed region).

bench.py (track mode, one GPU) launches one k_gray (or, with the one-launch
pyramid, one k_pyramid) per batch: 2 untimed
statistics batches, W warm-up steps, then the K timed steps of the
HBM-resident leg; then W + K steps of each from-host leg. The timed region of
a leg is every kernel that starts between the leg's first timed k_gray and the
next leg's first k_gray (the legs are separated by a device synchronize).

Usage: python tools/rocprof_timed_region.py TRACE.csv BENCH.json OUT.json [W K]
Writes OUT.json (per-leg, per-kernel count / mean / total us, and the kNN-2
mean set against the bench line's event-timed kernel_ms) and prints it."""
import csv
import json
import sys
from collections import defaultdict

trace, bench, out_path = sys.argv[1], sys.argv[2], sys.argv[3]
b = json.load(open(bench))
W = int(sys.argv[4]) if len(sys.argv) > 4 else b["warmup"]
K = int(sys.argv[5]) if len(sys.argv) > 5 else b["steps"]
rows = list(csv.DictReader(open(trace)))
for r in rows:
    r["s"], r["e"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
gray = [r["s"] for r in rows if r["Kernel_Name"].split("(")[0].endswith("k_gray") or "k_pyramid" in r["Kernel_Name"]]


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("odo::", "")


def window(lo, hi):
    ks = [r for r in rows if lo <= r["s"] < hi]
    st = defaultdict(list)
    for r in ks:
        st[short(r["Kernel_Name"])].append((r["e"] - r["s"]) / 1e3)
    t0, t1 = min(r["s"] for r in ks), max(r["e"] for r in ks)
    return {"wall_ms": round((t1 - t0) / 1e6, 4),
            "kernels": {k: {"count": len(v), "mean_us": round(sum(v) / len(v), 2), "total_us": round(sum(v), 1)}
                        for k, v in sorted(st.items(), key=lambda kv: -sum(kv[1]))}}


legs = {}
first = 2 + W  # statistics batches + warm-up
if len(gray) >= first + K:
    legs["hbm_resident"] = window(gray[first], gray[first + K] if len(gray) > first + K else 1 << 62)
nxt = first + K + W
if len(gray) >= nxt + K:
    legs["from_host"] = window(gray[nxt], gray[nxt + K] if len(gray) > nxt + K else 1 << 62)
res = {"source": f"rocprofv3 --kernel-trace of the bench command ({trace})", "warmup": W, "steps": K,
       "legs": legs}
for leg, key in (("hbm_resident", "kernel_ms"), ("from_host", None)):
    kn = legs.get(leg, {}).get("kernels", {}).get("k_knn2_f4")
    if not kn:
        continue
    line = b.get("roofline") or {}
    ev = line.get("kernel_ms") if key else (line.get("from_host_leg") or {}).get("kernel_ms")
    cmp = int(line["work"].split()[0]) if line.get("work") else None
    kn["bench_event_ms"] = ev
    if cmp:
        # the line's primary roofline: 512 FP4 MFMA ops per comparison against
        # the dense FP4 spec; the SURVEY 8(d) 16-op VALU equivalent beside it
        a = 512.0 * cmp / (kn["mean_us"] * 1e-6) / 1e12
        kn["mfma_fp4_achieved_tops"] = round(a, 1)
        kn["mfma_fp4_frac_of_10066T"] = round(a / 10066.3, 4)
        kn["valu16_equivalent_tops"] = round(16.0 * cmp / (kn["mean_us"] * 1e-6) / 1e12, 2)
with open(out_path, "w") as f:
    json.dump(res, f, indent=1)
print(json.dumps(res, indent=1))
