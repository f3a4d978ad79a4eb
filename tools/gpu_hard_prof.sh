# Kernel trace + SQ counters of the hard workload (RANSAC-bound) bench leg.
# Usage: tools/gpu_hard_prof.sh OUTDIR
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-hp}; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
CMD="python3 $R/bench.py --workload hard --steps 10 --warmup 2 --host-steps 0 --hard-steps 0 --latency-frames 0 --no-cpu-baseline"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- $CMD > $O/kt.json 2> $O/kt.err
echo kt ok
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU_FP64 -d $O/pmc1 -o run --output-format csv -- $CMD > $O/pmc1.log 2>&1
echo pmc1 ok
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY -d $O/pmc2 -o run --output-format csv -- $CMD > $O/pmc2.log 2>&1
echo pmc2 ok
