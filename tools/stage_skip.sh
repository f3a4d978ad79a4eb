# Step time with pair stages skipped (ODO_SKIP bits: 1 PnP, 16 RANSAC, 8 kNN-2, 4 all pair stages); measurement only
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-skip2}; mkdir -p $O
cd $R
for s in 0 1 16 8 4; do
  ODO_LIB=${ODO_LIB:-adaptive-rgbd-localization-mappig_amd/build_tuning/libodo_hip.so} ODO_SKIP=$s timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --hard-steps 0 --latency-frames 0 --no-kernel-timing > $O/skip_$s.json 2> $O/skip_$s.err
  echo skip $s ok
done
