# The fused gray + level-1 launch (k_gray_l1): GPU tests, then bench lines
# alternating ODO_GRAY_L1=1 / 0 on one box, then a serial kernel trace.
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_gl1; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
for rep in 1 2; do
  for v in 1 0; do
    ODO_GRAY_L1=$v timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
    echo $v $rep ok
  done
done
cd /tmp && export TMPDIR=/tmp
ODO_SERIAL_STREAMS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/kt.log 2>&1
echo kt ok
