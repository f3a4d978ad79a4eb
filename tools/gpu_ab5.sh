# k_ransac_lanes: two Mahalanobis chains per lane (branch-free ErrorFunction2)
# and branch-free TFC adds. Parity (bench configurations incl. the hard
# workload and the lanes-forced run), the per-wave probe before / after, and
# the hard leg A/B.
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab5}; mkdir -p $O; cd $R
P=adaptive-rgbd-localization-mappig_amd
timeout -k 10 600 python -u -m pytest tests/test_bench_config_parity.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
ODO_LIB=$P/build_lprof/libodo_hip.so timeout -k 10 300 python tools/lanes_probe.py 6 > $O/probe_new.json 2> $O/probe_new.err
ODO_LIB=$P/build_lprof0/libodo_hip.so timeout -k 10 300 python tools/lanes_probe.py 6 > $O/probe_old.json 2> $O/probe_old.err
echo probe ok
for i in 1 2; do
  for v in lbase tuning; do
    ODO_LIB=$P/build_$v/libodo_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --latency-frames 0 > $O/${v}_$i.json 2> $O/${v}_$i.err
    echo $v $i ok
  done
done
