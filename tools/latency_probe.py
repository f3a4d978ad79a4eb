"""Writes bench.py's latency-leg frames (cfg2 fr1/desk proxy) and runs
tools/build/frontend_latency on them with stdout to argv[1] (for the
instrumented builds: copy the variant over libodo_hip.so first on the box)."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    out, n = sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 16
    synth = bench.load_synth()
    bgr, dep, _ = synth.make_sequence(64, 640, 480, seed=0x5EED0002, closed_loop=True)
    idx = np.arange(n) % 64
    path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "latency_probe.bin")
    with open(path, "wb") as f:
        f.write(np.ascontiguousarray(bgr[idx]).tobytes())
        f.write(np.ascontiguousarray(dep[idx]).tobytes())
    exe = os.path.join(ROOT, "tools", "build", "frontend_latency")
    with open(out, "w") as fo:
        subprocess.run([exe, path, "640", "480", str(n), "500", "4"], check=True, stdout=fo, timeout=300)


if __name__ == "__main__":
    main()
