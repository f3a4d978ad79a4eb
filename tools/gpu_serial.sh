# Per-kernel times alone (every stage on one stream) at HEAD: default and hard workloads
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-serial}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
export ODO_SERIAL_STREAMS=1 ODO_LIB=$R/adaptive-rgbd-localization-mappig_amd/build_tuning/libodo_hip.so
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --host-steps 0 --hard-steps 0 --latency-frames 0 --steps 10 > $O/kt.log 2>&1
echo default ok
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kth -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --host-steps 0 --latency-frames 0 --steps 2 --workload hard > $O/kth.log 2>&1
echo hard ok
