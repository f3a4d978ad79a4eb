# A/B of the kNN-2 kernel forms (ODO_KNN_MFMA=1 int8, 2 FP4): the GPU tests on
# the FP4 form, the bench on both, and serial-stream kernel traces of both.
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_knn; mkdir -p $O
cd $R
ODO_KNN_MFMA=2 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
for f in 1 2; do
  ODO_KNN_MFMA=$f timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/bench_fmt$f.json 2> $O/bench_fmt$f.err
  echo bench $f ok
done
cd /tmp && export TMPDIR=/tmp
for f in 1 2; do
  ODO_KNN_MFMA=$f ODO_SERIAL_STREAMS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/kt$f -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/kt$f.log 2>&1
  echo kt $f ok
done
