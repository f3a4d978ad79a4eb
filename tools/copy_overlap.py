"""Copy / compute overlap of the host-input path from a rocprofv3 run with
--kernel-trace --memory-copy-trace --output-format csv.

For every host-to-device copy of at least --min-mb: its duration, its rate,
and the fraction of its interval during which at least one kernel of this
process was executing. Usage: copy_overlap.py <prefix> (e.g. dir/run)."""
import argparse
import csv


def intervals(path, kind_filter=None):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if kind_filter and not kind_filter(r):
                continue
            out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r))
    return out


def merge(iv):
    iv = sorted((a, b) for a, b, _ in iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def covered(a, b, merged):
    t = 0
    for x, y in merged:
        if y <= a:
            continue
        if x >= b:
            break
        t += min(b, y) - max(a, x)
    return t


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("prefix")
    ap.add_argument("--min-mb", type=float, default=64.0)
    a = ap.parse_args()
    kern = merge([k for k in intervals(a.prefix + "_kernel_trace.csv")
                  if "rocclr" not in k[2]["Kernel_Name"]])
    copies = intervals(a.prefix + "_memory_copy_trace.csv",
                       lambda r: r["Direction"] == "MEMORY_COPY_HOST_TO_DEVICE")
    # sizes are not in the trace: pair each large copy with the bench's
    # per-batch sizes by duration (BGR 3 B/px, depth 2 B/px of 256 frames)
    big = [c for c in copies if c[1] - c[0] > 1e6]
    tot_t = tot_cov = 0
    print(f"{'copy':>4} {'start_ms':>9} {'dur_ms':>7} {'kernel_overlap':>14}")
    t0 = big[0][0] if big else 0
    for i, (s, e, _) in enumerate(big):
        cov = covered(s, e, kern)
        tot_t += e - s
        tot_cov += cov
        print(f"{i:4d} {(s - t0) / 1e6:9.3f} {(e - s) / 1e6:7.3f} {cov / (e - s):14.3f}")
    if big:
        print(f"large H2D copies: {len(big)}, {tot_t / 1e6:.2f} ms, kernels active during "
              f"{100.0 * tot_cov / tot_t:.1f}% of the copy time")


if __name__ == "__main__":
    main()
