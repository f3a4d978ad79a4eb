"""Copy the judged summaries of a GPU session from gpurun_out/ (scratch) into
profiles/ (tracked):

  python tools/save_profile.py RUN [RUN ...]      e.g. r05_f r05_h

Per run directory gpurun_out/RUN -> profiles/RUN:
  * *.json, *.log, and the stderr of bench-style runs (*.err, only the lines
    that are not progress noise),
  * SUB/run_kernel_stats.csv of every rocprofv3 output dir as SUB_kernel_stats.csv
    (the full kernel traces stay in scratch),
  * for a kernel trace of the headline bench (kt/), the step timeline of two
    mid-run steps (tools/trace_steps.py) as kt_step_timeline.txt,
  * every PMC directory (pmc_*, pmch_*) merged by tools/pmc_merge.py into
    pmc_*.json, plus its kernel-trace stats."""
import glob
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def save(run):
    src = os.path.join(ROOT, "gpurun_out", run)
    dst = os.path.join(ROOT, "profiles", run)
    if not os.path.isdir(src):
        raise SystemExit(f"no {src}")
    os.makedirs(dst, exist_ok=True)
    n = 0
    for f in sorted(os.listdir(src)):
        p = os.path.join(src, f)
        if os.path.isfile(p) and f.endswith((".json", ".log", ".txt")):
            shutil.copy(p, os.path.join(dst, f))
            n += 1
        elif os.path.isfile(p) and f.endswith(".err"):
            keep = [l for l in open(p, errors="replace") if l.strip() and "it/s]" not in l]
            if keep:
                with open(os.path.join(dst, f), "w") as o:
                    o.writelines(keep[-200:])
                n += 1
        elif os.path.isdir(p):
            if f.startswith(("pmc_", "pmch_")):
                out = os.path.join(dst, f + ".json")
                subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_merge.py"), p, out], check=True,
                               stdout=subprocess.DEVNULL)
                n += 1
                for ks in glob.glob(os.path.join(p, "kt", "**", "*kernel_stats.csv"), recursive=True):
                    shutil.copy(ks, os.path.join(dst, f + "_kernel_stats.csv"))
                continue
            for ks in glob.glob(os.path.join(p, "**", "*kernel_stats.csv"), recursive=True):
                shutil.copy(ks, os.path.join(dst, f + "_kernel_stats.csv"))
                n += 1
            if f == "kt":
                tr = glob.glob(os.path.join(p, "**", "*kernel_trace.csv"), recursive=True)
                if tr:
                    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "trace_steps.py"), tr[0], "2",
                                        "k_pyramid", "20"], capture_output=True, text=True)
                    if r.returncode == 0:
                        with open(os.path.join(dst, "kt_step_timeline.txt"), "w") as o:
                            o.write(r.stdout)
                        n += 1
    print(f"{run}: {n} files -> profiles/{run}")


if __name__ == "__main__":
    for run in sys.argv[1:]:
        save(run)
