#!/bin/bash
# PMC passes over one kernel of the default bench workload, streams serialised
# (ODO_SERIAL_STREAMS=1) so the counters of a dispatch are that kernel's own.
# One rocprofv3 run per counter group (the hardware's per-block limits), each
# under its own kill timer. Usage: tools/pmc_knn.sh KERNEL_REGEX OUTDIR
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
K=${1:-k_knn2_mx}
OUT=${2:-$R/gpurun_out/pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
export ODO_SERIAL_STREAMS=1
ARGS="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 --hard-steps 0"
pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex "$K" -d "$OUT/$name" -o run \
    --output-format csv -- python3 $ARGS > "$OUT/$name.log" 2>&1
  echo "pass $name done"
}
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU
pass sq2 SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_BUSY_CU_CYCLES
pass tcc FETCH_SIZE
pass tccw WRITE_SIZE
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d "$OUT/kt" -o run --output-format csv -- python3 $ARGS > "$OUT/kt.log" 2>&1
echo "kernel trace done"
