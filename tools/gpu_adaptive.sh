# Both ADAPTIVE paths: their GPU tests, the bench lines of both detectors and
# a serial-stream kernel trace of the cv::ORB one, in one call.
# Usage: tools/gpu_adaptive.sh OUTDIR_NAME   (results under gpurun_out/OUTDIR_NAME)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-adapt}; mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests/test_adaptive_orb_gpu.py tests/test_adaptive_gpu.py tests/test_sizes_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
timeout -k 10 300 python bench.py --detector adaptive --host-steps 0 --hard-steps 0 --no-cpu-baseline > $O/bench_fast.json 2> $O/bench_fast.err
echo bench fast ok
bash tools/bench_adaptive_orb.sh ${1:-adapt}
