"""Per-kernel table (calls, mean us, share) of a rocprofv3 kernel_stats.csv."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(f'{r["Name"].split("(")[0][:44]:44s} {r["Calls"]:>5s} {float(r["AverageNs"]) / 1e3:9.1f} us '
          f'{float(r["TotalDurationNs"]) / tot * 100:5.1f}%')
