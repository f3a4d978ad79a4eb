# RANSAC: lanes-kernel chunk prefetch + eval-kernel Markstein quotients vs
# HEAD (build_bp0); parity of every RANSAC path first, then the probe, the
# latency leg and the headline / hard legs
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab8}; mkdir -p $O; cd $R
P=adaptive-rgbd-localization-mappig_amd
timeout -k 10 900 python -u -m pytest tests/test_bench_config_parity.py tests/test_gpu_parity.py tests/test_hyp_shard_gpu.py tests/test_golden.py tests/test_configs_parity.py tests/test_frontend_cpp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
ODO_LIB=$P/build_lprof/libodo_hip.so timeout -k 10 300 python tools/lanes_probe.py 6 > $O/probe.json 2> $O/probe.err
timeout -k 10 300 python bench.py --mode latency > $O/latency.json 2> $O/latency.err
echo probe latency ok
for i in 1 2; do
  for v in bp0 tuning; do
    ODO_LIB=$P/build_$v/libodo_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --latency-frames 0 > $O/${v}_$i.json 2> $O/${v}_$i.err
    echo $v $i ok
  done
done
