# A/B of the finalize kernels (ODO_FIN_LDS=1 staged patches, 0 per-lane gathers)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_fin; mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
timeout -k 10 600 python bench.py --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/bench.json 2> $O/bench.err
echo bench ok
cd /tmp && export TMPDIR=/tmp
for m in 2 1; do
  ODO_FIN_LDS=$m ODO_SERIAL_STREAMS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/kt$m -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/kt$m.log 2>&1
  echo kt$m ok
done
