"""Merge the PMC passes of one tools/gpu.sh `pmc=` / `pmch=` step (sq1, sq2,
tcc, tccw: one rocprofv3 --pmc run per counter group, serial streams) into one
per-kernel table: the mean of every counter per dispatch, per-wave
instruction counts, VALU / MFMA busy fractions and the memory-side traffic
with the gfx950 corrections of MI355X_MICROARCH.md (FETCH_SIZE counts half
the bytes of 16-B-per-lane reads: fetch bytes = 2 x FETCH_SIZE x 1024;
WRITE_SIZE x 1024 exact for 16-B stores; both include Infinity Cache hits).

  python tools/pmc_merge.py PMC_DIR OUT.json [--traffic KERNEL TRAFFIC.json BATCH]

--traffic also writes the file bench.py reads for roofline.traffic (the named
kernel's bytes per launch and per pair, with the build it was measured on)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(dirpath):
    acc = defaultdict(lambda: defaultdict(lambda: defaultdict(float)))
    for path in glob.glob(os.path.join(dirpath, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].split("(")[0].replace("odo::", "").replace("void ", "").strip()
                acc[k][r["Counter_Name"]][(path, r["Dispatch_Id"])] += float(r["Counter_Value"])
    return acc


N_SIMD = 1024   # 256 CUs x 4 SIMDs
CLK_GHZ = 2.4


def durations(dirpath):
    """Mean dispatch duration (ns) per kernel from the kernel-trace pass."""
    acc = defaultdict(list)
    for path in glob.glob(os.path.join(dirpath, "**", "*kernel_trace.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].split("(")[0].replace("odo::", "").replace("void ", "").strip()
                acc[k].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    pdir, out = sys.argv[1], sys.argv[2]
    durs = durations(os.path.join(pdir, "kt"))
    acc = defaultdict(dict)
    for sub in ("sq1", "sq2", "tcc", "tccw"):
        for k, cs in load(os.path.join(pdir, sub)).items():
            for c, d in cs.items():
                acc[k][c] = {"mean": sum(d.values()) / len(d), "dispatches": len(d)}
    table = {}
    for k, cs in sorted(acc.items()):
        m = {c: v["mean"] for c, v in cs.items()}
        row = {c: round(v, 1) for c, v in m.items()}
        w = m.get("SQ_WAVES")
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD"):
                if c in m:
                    row[c + "_per_wave"] = round(m[c] / w, 1)
        if m.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in m:
                    row[c + "_frac_of_wave_cycles"] = round(m[c] / m["SQ_WAVE_CYCLES"], 3)
        # SQ_VALU_MFMA_BUSY_CYCLES counts shader cycles summed over the SIMDs
        # (16 per 16x16x128 FP4 MFMA: SQ_INSTS_MFMA x 16 reproduces it), so the
        # fraction is over the chip's SIMD-cycles during the dispatch: 1024
        # SIMDs x the kernel's mean duration (the kt pass of the same
        # directory) x 2.4 GHz. SQ_BUSY_CYCLES is a per-SE count and is not a
        # denominator for it (round 4 divided by it: 13.1, not a fraction).
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and k in durs:
            row["mean_duration_us"] = round(durs[k] / 1e3, 2)
            row["mfma_busy_frac"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (N_SIMD * durs[k] * CLK_GHZ), 4)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("SQ_BUSY_CU_CYCLES"):
            # SQ_BUSY_CU_CYCLES: cycles each CU had work, summed over the CUs
            row["mfma_busy_frac_of_busy_cu"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (4 * m["SQ_BUSY_CU_CYCLES"]), 4)
        fb = 2 * m["FETCH_SIZE"] * 1024 if "FETCH_SIZE" in m else None
        wb = m["WRITE_SIZE"] * 1024 if "WRITE_SIZE" in m else None
        if fb is not None and wb is not None:
            row["hbm_bytes_corrected"] = round(fb + wb)
        table[k] = row
    doc = {"source": pdir, "passes": ["sq1", "sq2", "tcc", "tccw"],
           "correction": "fetch bytes = 2 x FETCH_SIZE x 1024 (gfx950, MI355X_MICROARCH.md); write bytes = "
                         "WRITE_SIZE x 1024; memory-side L2 requests incl. Infinity Cache hits",
           "kernels": table}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps({k: {c: v for c, v in r.items() if c.endswith(("per_wave", "frac_of_wave_cycles", "corrected"))}
                      for k, r in table.items()}, indent=1))
    if len(sys.argv) > 3 and sys.argv[3] == "--traffic":
        kern, tout, batch = sys.argv[4], sys.argv[5], int(sys.argv[6])
        r = next(v for k, v in table.items() if kern in k)
        tb = r["hbm_bytes_corrected"]
        with open(tout, "w") as f:
            json.dump({"kernel": kern, "batch": batch, "source": os.path.relpath(out),
                       "fetch_size_kb_raw": r.get("FETCH_SIZE"), "write_size_kb_raw": r.get("WRITE_SIZE"),
                       "correction": doc["correction"], "hbm_bytes_per_launch": tb,
                       "hbm_bytes_per_pair": round(tb / batch),
                       "build": os.environ.get("PMC_BUILD", "")}, f, indent=1)


if __name__ == "__main__":
    main()
