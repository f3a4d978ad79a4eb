# SURVEY 8(f) rank 4 back-ends: PnPRansac and GICP GPU parity tests, their
# bench latency legs and rocprofv3 kernel stats of both legs.
# Usage: tools/gpu_pose_backends.sh OUTDIR
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pb}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gicp.py tests/test_pnpransac.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
timeout -k 10 300 python bench.py --mode gicp --steps 30 > $O/bench_gicp.json 2> $O/bench_gicp.err
timeout -k 10 300 python bench.py --mode pnpransac --steps 50 > $O/bench_pnpransac.json 2> $O/bench_pnpransac.err
echo bench ok
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt_gicp -o run --output-format csv -- python3 $R/bench.py --mode gicp --steps 30 --no-cpu-baseline > $O/kt_gicp.log 2>&1
echo kt ok
