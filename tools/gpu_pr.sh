# PnPRansac (unseeded final solvePnP + round-robin Jacobi) parity and latency,
# plus the PnP phase profile of the instrumented build.
# Usage: tools/gpu_pr.sh OUTDIR
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pr}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_pnpransac.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
timeout -k 10 300 python bench.py --mode pnpransac --steps 50 > $O/bench_pnpransac.json 2> $O/bench_pnpransac.err
echo bench ok
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt_pr -o run --output-format csv -- python3 $R/bench.py --mode pnpransac --steps 20 --no-cpu-baseline > $O/kt_pr.log 2>&1
echo kt ok
cd $R
timeout -k 10 120 python tools/pair_stats.py adaptive-rgbd-localization-mappig_amd/build_prof/libodo_hip.so > $O/pnp_prof.txt 2>&1
echo prof ok
