# FAST cells per workgroup (1 / 2 / 4): parity of the 4-cell build, latency leg
# of the production build (AUTO pyramid form: the chain for one frame), A/B
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab3}; mkdir -p $O; cd $R
P=adaptive-rgbd-localization-mappig_amd
timeout -k 10 300 env ODO_LIB=$P/build_cpw4/libodo_hip.so python -u -m pytest tests/test_gpu_parity.py tests/test_sizes_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_cpw4.log 2>&1
echo pytest ok
timeout -k 10 300 python bench.py --mode latency > $O/latency.json 2> $O/latency.err
echo latency ok
for i in 1 2; do
  bash tools/ab_knobs.sh ${1:-ab3} "cpw1_$i|$P/build_tuning/libodo_hip.so|X=0" "cpw2_$i|$P/build_cpw2/libodo_hip.so|X=0" "cpw4_$i|$P/build_cpw4/libodo_hip.so|X=0"
done
