# sweep compaction (product: LN_COMPACT=1) vs every lane through the LLT (nc): GPU tests, then A/B
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab19}; mkdir -p $O; cd $R
P=adaptive-rgbd-localization-mappig_amd
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
for i in 1 2; do
  for v in default nc; do
    L=$P/build_$v/libodo_hip.so; [ $v = default ] && L=$P/libodo_hip.so
    ODO_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --latency-frames 0 > $O/${v}_$i.json 2> $O/${v}_$i.err
    echo $v $i ok
  done
done
