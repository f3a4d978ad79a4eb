# k_pnp A/B (build_bp0 = the build without the change under test): parity of every PnP path, the
# phase probe, the latency leg, the headline A/B against the pivoted build
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab9}; mkdir -p $O; cd $R
P=adaptive-rgbd-localization-mappig_amd
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_config_parity.py tests/test_golden.py tests/test_configs_parity.py tests/test_frontend_cpp.py tests/test_sizes_gpu.py tests/test_projection.py tests/test_host_path.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
ODO_LIB=$P/build_pnpprof/libodo_hip.so timeout -k 10 200 python tools/pnp_probe.py > $O/pnp_probe.txt 2>&1
timeout -k 10 300 python bench.py --mode latency > $O/latency.json 2> $O/latency.err
echo probe latency ok
for i in 1 2; do
  for v in bp0 tuning; do
    ODO_LIB=$P/build_$v/libodo_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --latency-frames 0 --hard-steps 0 > $O/${v}_$i.json 2> $O/${v}_$i.err
    echo $v $i ok
  done
done
