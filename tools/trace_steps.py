"""Per-stream timeline of the last steps of a rocprofv3 kernel trace (CSV).

  python tools/trace_steps.py RUN_kernel_trace.csv [steps] [anchor-kernel] [first]

Prints, for `steps` steps from the anchor's launch number `first` (default:
the last `steps` steps) (a step starts at each launch of the anchor
kernel, default the pyramid), every kernel with its stream (queue), start
offset and duration in µs, then the per-stream busy time of those steps: which
stream is the critical path, and what runs beside what."""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.split("(")[0].replace("odo::", "").replace("void ", "").strip()
    return n


def main(path, nsteps=2, anchor="k_pyramid", first=None):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if "rocclr" in r["Kernel_Name"]:
                continue
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], short(r["Kernel_Name"])))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[3].startswith(anchor)]
    if len(starts) < nsteps + 1:
        raise SystemExit(f"fewer than {nsteps + 1} launches of {anchor}")
    if first is None:
        i0, i1 = starts[-1 - nsteps], starts[-1]
    else:
        i0, i1 = starts[first], starts[first + nsteps]
    t0 = rows[i0][0]
    busy = defaultdict(int)
    for s, e, q, n in rows[i0:i1]:
        print(f"{n[:24]:24s} q{q:>3s} +{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}  end {(e - t0) / 1e3:9.1f}")
        busy[q] += e - s
    span = rows[i1][0] - t0
    print(f"steps: {nsteps}, span {span / 1e3:.1f} us ({span / 1e3 / nsteps:.1f} per step)")
    for q, b in sorted(busy.items()):
        print(f"  queue {q}: kernels {b / 1e3:.1f} us ({b / span:.2f} of the span, summed durations)")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2, sys.argv[3] if len(sys.argv) > 3 else "k_pyramid",
         int(sys.argv[4]) if len(sys.argv) > 4 else None)
