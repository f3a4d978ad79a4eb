# rocprofv3 kernel trace of the per-frame drop-in path (tools/build/frontend_latency)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-lt}; mkdir -p $O; cd $R
python3 - <<'PY'
import os, sys, numpy as np
sys.path.insert(0, "tests")
from conftest import load_synth
bgr, dep, _ = load_synth().make_sequence(64, 640, 480, seed=0x5EED0002, closed_loop=True)
idx = np.arange(40) % 64
with open("/tmp/lat_frames.bin", "wb") as f:
    f.write(np.ascontiguousarray(bgr[idx]).tobytes()); f.write(np.ascontiguousarray(dep[idx]).tobytes())
PY
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --memory-copy-trace -d $O/kt -o run --output-format csv -- $R/tools/build/frontend_latency /tmp/lat_frames.bin 640 480 40 500 8 > $O/lat.json 2> $O/lat.err
echo trace ok
