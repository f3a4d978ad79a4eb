"""One-line summary of a bench.py track line (value, from_host, hard, latency)."""
import json
import sys

for p in sys.argv[1:]:
    d = json.loads(open(p).read().strip().splitlines()[-1])
    lat = d.get("latency") or {}
    st = lat.get("stage_median_ms", {})
    print(p, "value", d["value"], "ms", d["ms_per_step"], "host", (d.get("from_host") or {}).get("value"),
          "hard", (d.get("hard_workload") or {}).get("value"), "lat p50", lat.get("p50_ms"), "p99", lat.get("p99_ms"),
          " ".join(f"{k}={v}" for k, v in st.items()), "knn frac", (d.get("roofline") or {}).get("frac"),
          "steps", {k: (d.get("step_ms") or {}).get(k) for k in ("min", "median", "p90", "max")},
          "stages", d.get("stage_ms"))
