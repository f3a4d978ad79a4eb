# Parity of the blur-edge fold and the fused pyramid (+ blur), then A/B:
# base (blur edges as their own launch) / blur folded / fused pyramid + blur /
# fused pyramid, blur separate, and the kNN gate / occupancy knobs
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab1}; mkdir -p $O; cd $R
timeout -k 10 500 python -u -m pytest tests/test_sizes_gpu.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
P=adaptive-rgbd-localization-mappig_amd
for i in 1 2; do
  bash tools/ab_knobs.sh ${1:-ab1} "base_$i|$P/build_base/libodo_hip.so|X=0" "blur_$i|$P/build_tuning/libodo_hip.so|X=0" "fused_$i|$P/build_fused/libodo_hip.so|X=0" "fnob_$i|$P/build_fused/libodo_hip.so|ODO_PYRAMID_FORM=2" "fgate_$i|$P/build_fused/libodo_hip.so|ODO_KNN_GATE=1" "fwg2_$i|$P/build_fused/libodo_hip.so|ODO_KNN_WG_PER_CU=2"
done
