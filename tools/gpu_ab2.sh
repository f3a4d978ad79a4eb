# k_pyramid variants: resize rows / gray quads in flight, gray as its own
# launch; then the per-kernel times alone (serial streams) of the fused build
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab2}; mkdir -p $O; cd $R
P=adaptive-rgbd-localization-mappig_amd
timeout -k 10 300 env ODO_LIB=$P/build_pru4/libodo_hip.so python -u -m pytest tests/test_sizes_gpu.py -k pyramid_forms -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
for i in 1 2; do
  bash tools/ab_knobs.sh ${1:-ab2} "fused_$i|$P/build_fused/libodo_hip.so|X=0" "fgray_$i|$P/build_fused/libodo_hip.so|ODO_PYR_GRAY=1" "pru4_$i|$P/build_pru4/libodo_hip.so|X=0" "pgray_$i|$P/build_pru4/libodo_hip.so|ODO_PYR_GRAY=1"
done
cd /tmp && export TMPDIR=/tmp
ODO_LIB=$R/$P/build_fused/libodo_hip.so ODO_SERIAL_STREAMS=1 timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt_serial -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --host-steps 0 --hard-steps 0 --latency-frames 0 --steps 10 > $O/kt_serial.log 2>&1
echo kt ok
