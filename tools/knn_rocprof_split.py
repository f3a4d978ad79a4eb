"""Split the k_knn2_f4 launches of a rocprofv3 kernel trace of `bench.py`
into its phases (warm-up, the timed steps, the rest) and compare the timed
mean with the bench line's event-timed kernel_ms.
Usage: python tools/knn_rocprof_split.py TRACE.csv BENCH.json [warmup] [steps]"""
import csv
import json
import sys

trace, bench = sys.argv[1], sys.argv[2]
W = int(sys.argv[3]) if len(sys.argv) > 3 else 5
K = int(sys.argv[4]) if len(sys.argv) > 4 else 40
rows = [r for r in csv.DictReader(open(trace)) if "k_knn2_f4" in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
b = json.load(open(bench))
timed = dur[W:W + K]
out = {
    "source": f"rocprofv3 --kernel-trace of the bench command ({trace})",
    "k_knn2_f4_launches_total": len(dur),
    "mean_all_us": round(sum(dur) / len(dur), 1),
    "warmup_launches": W,
    "timed_region_launches": len(timed),
    "timed_region_mean_us": round(sum(timed) / max(1, len(timed)), 1),
    "bench_line": {"kernel_ms": b["roofline"]["kernel_ms"], "alone_ms": b["roofline"]["alone"]["kernel_ms"]},
}
print(json.dumps(out, indent=1))
