"""Per-kernel mean of each PMC counter per dispatch, from a rocprofv3 run
(SQLite results .db or counter_collection.csv); optional kernel-name filter.
Adds per-wave instruction counts when SQ_WAVES was collected."""
import csv
import sqlite3
import sys
from collections import defaultdict


def rows(path):
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, cn, v, did in c.execute("select kernel_name, counter_name, value, dispatch_id from counters_collection"):
            yield name, cn, float(v), did
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                yield r["Kernel_Name"], r["Counter_Name"], float(r["Counter_Value"]), r["Dispatch_Id"]


def main(path, filt=None):
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for name, cn, v, did in rows(path):
        k = name.split("(")[0].replace("odo::", "")
        if filt and filt not in k:
            continue
        acc[k][cn][did] += v  # sum over dimensions (XCD/SE) of one dispatch
    for k, cs in sorted(acc.items()):
        print(k)
        mean = {c: sum(d.values()) / len(d) for c, d in cs.items()}
        waves = mean.get("SQ_WAVES")
        for c, m in sorted(mean.items()):
            extra = f"   per wave {m / waves:10.1f}" if waves and c.startswith("SQ_INSTS") else ""
            print(f"   {c:28s} {m:16.1f}{extra}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
