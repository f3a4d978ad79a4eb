# k_ransac_lanes: per-wave sub-phase probe (new / old forms) and SQ counters
# of the lanes kernel run alone (serial streams) on the hard workload
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-lp2}; mkdir -p $O; cd $R
P=adaptive-rgbd-localization-mappig_amd
ODO_LIB=$P/build_lprof/libodo_hip.so timeout -k 10 300 python tools/lanes_probe.py 6 > $O/probe_new.json 2> $O/probe_new.err
ODO_LIB=$P/build_lprof0/libodo_hip.so timeout -k 10 300 python tools/lanes_probe.py 6 > $O/probe_old.json 2> $O/probe_old.err
echo probe ok
cd /tmp && export TMPDIR=/tmp
export ODO_SERIAL_STREAMS=1 ODO_LIB=$R/$P/build_tuning/libodo_hip.so
ARGS="$R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --host-steps 0 --hard-steps 3 --latency-frames 0"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --kernel-include-regex k_ransac_lanes -d $O/sq1 -o run --output-format csv -- python3 $ARGS > $O/sq1.log 2>&1
echo sq1 ok
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_BUSY_CU_CYCLES SQ_ACTIVE_INST_SCA --kernel-include-regex k_ransac_lanes -d $O/sq2 -o run --output-format csv -- python3 $ARGS > $O/sq2.log 2>&1
echo sq2 ok
