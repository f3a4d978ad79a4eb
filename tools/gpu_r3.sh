# Round-3 GPU session: the parity tests of what changed first, the bench line,
# the rocprofv3 kernel trace of the same bench command (timed-region split by
# tools/rocprof_timed_region.py), then the whole GPU suite.
# Usage: tools/gpu_r3.sh OUTDIR [quick]
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-r3}; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_bench_config_parity.py tests/test_host_path.py tests/test_frames_shard_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_changed.log 2>&1
echo pytest changed ok
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
echo bench ok
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --hard-steps 0 --latency-frames 0 > $O/kt_bench.json 2> $O/kt.err
echo kt ok
cd $R
if [ "$2" != quick ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest all ok
fi
