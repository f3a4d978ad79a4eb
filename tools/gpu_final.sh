# Round-end evidence: GPU tests, smoke(), the default bench line (all legs), the
# SURVEY 8(f) rank 4 back-end legs, and the rocprofv3 kernel stats of the
# default bench command. Usage: tools/gpu_final.sh OUTDIR
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-final}; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke ok
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err
echo bench ok
timeout -k 10 300 python bench.py --mode gicp --steps 30 > $O/bench_gicp.json 2> $O/bench_gicp.err
timeout -k 10 300 python bench.py --mode pnpransac --steps 50 > $O/bench_pnpransac.json 2> $O/bench_pnpransac.err
echo legs ok
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline > $O/kt.log 2>&1
echo kt ok
