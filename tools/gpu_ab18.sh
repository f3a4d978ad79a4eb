# kNN wave priority 3 (kp3) / 1 (kp1) vs the default 2 (product library)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab18}; mkdir -p $O; cd $R
P=adaptive-rgbd-localization-mappig_amd
for i in 1 2 3; do
  for v in default kp3 kp1; do
    L=$P/build_$v/libodo_hip.so; [ $v = default ] && L=$P/libodo_hip.so
    ODO_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --latency-frames 0 --hard-steps 0 > $O/${v}_$i.json 2> $O/${v}_$i.err
    echo $v $i ok
  done
done
