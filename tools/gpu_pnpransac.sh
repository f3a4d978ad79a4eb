# PnPRansac: GPU parity tests, the bench latency leg and
# its rocprofv3 kernel stats, in one call. Usage: tools/gpu_pnpransac.sh OUTDIR
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pr}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_pnpransac.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
timeout -k 10 300 python bench.py --mode pnpransac --steps 50 > $O/bench.json 2> $O/bench.err
echo bench ok
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --mode pnpransac --steps 50 --no-cpu-baseline > $O/kt.log 2>&1
echo kt ok
