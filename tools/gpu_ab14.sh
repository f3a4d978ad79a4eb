# k_ransac_eval_list grid (four-wave workgroups; default 512) on the headline leg
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab14}; mkdir -p $O; cd $R
P=adaptive-rgbd-localization-mappig_amd
for i in 1 2; do
  for g in 512 128 256 64; do
    ODO_LIB=$P/build_tuning/libodo_hip.so ODO_EV2_LIST=$g timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --latency-frames 0 --hard-steps 0 > $O/g${g}_$i.json 2> $O/g${g}_$i.err
    echo $g $i ok
  done
done
