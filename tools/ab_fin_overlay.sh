# A/B of the finalize LDS overlay: rBRIEF window over the IC disc (fov1) vs both patches (fov0)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_fov; mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden.py tests/test_configs_parity.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1
echo pytest ok
for rep in 1 2; do
  for v in fov1 fov0; do
    ODO_LIB=adaptive-rgbd-localization-mappig_amd/build/libodo_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
    echo $v $rep ok
  done
done
