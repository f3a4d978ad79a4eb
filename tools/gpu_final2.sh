# Round-end evidence + the k_pnp phase probe (profile build)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-final}; mkdir -p $O
cd $R
ODO_LIB=adaptive-rgbd-localization-mappig_amd/build_pnpprof/libodo_hip.so timeout -k 10 200 python tools/pnp_probe.py > $O/pnp_probe.txt 2>&1 || true
echo pnp probe done
bash tools/gpu_final.sh ${1:-final}
cd $R
timeout -k 10 300 python bench.py --detector adaptive --no-cpu-baseline --host-steps 0 --hard-steps 0 --latency-frames 0 > $O/bench_adaptive.json 2> $O/bench_adaptive.err
timeout -k 10 300 python bench.py --detector adaptive-orb --no-cpu-baseline --host-steps 0 --hard-steps 0 --latency-frames 0 > $O/bench_adaptive_orb.json 2> $O/bench_adaptive_orb.err
echo adaptive ok
