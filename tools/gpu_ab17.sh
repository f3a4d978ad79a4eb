# octree grid (frames, levels): every level 0 first (lpt) vs (levels, frames)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab15}; mkdir -p $O; cd $R
P=adaptive-rgbd-localization-mappig_amd
for i in 1 2 3; do
  for v in tuning lpt; do
    ODO_LIB=$P/build_$v/libodo_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --latency-frames 0 --hard-steps 0 > $O/${v}_$i.json 2> $O/${v}_$i.err
    echo $v $i ok
  done
done
