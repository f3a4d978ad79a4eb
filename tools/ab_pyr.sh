# A/B of the pyramid paths: ODO_PYR_FUSED=0 (k_gray + k_resize per level),
# 1 (k_gray + fused k_pyramid), 2 (gray inside k_pyramid), band heights.
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_pyr; mkdir -p $O
cd $R
ODO_PYR_FUSED=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
ODO_PYR_FUSED=2 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_bench_config_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_fused_gray.log 2>&1
echo pytest2 ok
cd /tmp && export TMPDIR=/tmp
run() {
  local name=$1; shift
  env "$@" ODO_SERIAL_STREAMS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/$name -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/$name.log 2>&1
  echo $name ok
}
run m1r16 ODO_PYR_FUSED=1 ODO_PYR_ROWS=16 ODO_PYR_LDS_KB=32
run m1r48 ODO_PYR_FUSED=1 ODO_PYR_ROWS=48
run m1r24 ODO_PYR_FUSED=1 ODO_PYR_ROWS=24 ODO_PYR_LDS_KB=40
run m2r48 ODO_PYR_FUSED=2 ODO_PYR_ROWS=48
run m2r16 ODO_PYR_FUSED=2 ODO_PYR_ROWS=16 ODO_PYR_LDS_KB=32
