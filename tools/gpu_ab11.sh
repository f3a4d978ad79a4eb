# PnPRansac: subsets from the precomputed cv::RNG table vs one lane running the
# generator (build_bp0); parity of the back-ends, then the pnpransac leg A/B
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab11}; mkdir -p $O; cd $R
P=adaptive-rgbd-localization-mappig_amd
timeout -k 10 600 python -u -m pytest tests/test_pnpransac.py tests/test_frontend_cpp.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
for i in 1 2; do
  for v in bp0 tuning; do
    ODO_LIB=$P/build_$v/libodo_hip.so timeout -k 10 300 python bench.py --mode pnpransac --steps 50 --no-cpu-baseline > $O/${v}_$i.json 2> $O/${v}_$i.err
    echo $v $i ok
  done
done
