# Priorities: extraction stream at the highest stream priority; extraction
# kernels' wave priority 2; pair kernels' wave priority 1 (instead of 3)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab4}; mkdir -p $O; cd $R
P=adaptive-rgbd-localization-mappig_amd
for i in 1 2; do
  bash tools/ab_knobs.sh ${1:-ab4} "base_$i|$P/build_tuning/libodo_hip.so|X=0" "xsp_$i|$P/build_tuning/libodo_hip.so|ODO_EXTRACT_STREAM_PRIO=1" "xp2_$i|$P/build_xprio2/libodo_hip.so|X=0" "wp1_$i|$P/build_wprio1/libodo_hip.so|X=0"
done
