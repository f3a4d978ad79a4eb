#!/bin/bash
# The one launcher for GPU sessions (run it under gpurun):
#
#   tools/gpu.sh OUTDIR STEP [STEP ...]
#
# Steps run in order; each has its own time limit and the first failure ends
# the call (set -e), so nothing runs on the GPU after a fault or a timeout.
#
#   tests               pytest -m gpu, the whole suite
#   tests=F1,F2         pytest -m gpu over the named test files (tests/F1 ...)
#   smoke               __graft_entry__.smoke()
#   bench               python bench.py (the driver's default line)      -> bench.json
#   bench=NAME:ARGS     python bench.py ARGS (ARGS with '+' for spaces)  -> NAME.json
#   benchenv=NAME:ENV:ARGS  the full bench line with VAR=VAL (joined by '/') in the environment
#   multi               bench.py --gpus 2 --backend gloo: two ranks sharing the GPU
#   kt                  rocprofv3 kernel trace of the headline command (+ timed-region split)
#   ktn=NAME            the A/B bench command under a kernel trace (NAME.json, NAME/)
#   ktv=V               the A/B bench command under a kernel trace, variant build_V
#   kth                 rocprofv3 kernel trace of the hard workload's pipelined main leg
#   serial              per-kernel times alone (tuning build, ODO_SERIAL_STREAMS=1),
#                       default and hard workloads
#   pmc=REGEX           PMC passes over the kernels matching REGEX (tuning build,
#                       serial streams), one counter group per rocprofv3 run
#   pmch=REGEX          the same on the hard workload
#   vpmch=V:REGEX       pmch= with variant build_V (a tuning-flagged build)
#   vserial=V           per-kernel times alone of variant build_V (built with -DODO_TUNING)
#   vtests=V:F1,F2      pytest -m gpu over the named files against variant build_V
#   probe=V:SCRIPT      python tools/SCRIPT.py with ODO_LIB = variant build_V (probe builds)
#   vpmc=V:REGEX        pmc= with variant build_V (a tuning-flagged build)
#   pmcx=NAME:REGEX:C1,C2   one PMC pass with the named counters (pmcx_NAME/)
#   vpmcx=V:NAME:REGEX:C1,C2  pmcx with variant build_V
#   listctr             rocprofv3 -L (the box's counter names) -> counters.txt
#   envbench=NAME:ENV:ARGS  bench.py on the tuning build with knobs in the environment
#                       (ENV: VAR=VAL joined by '/'; ARGS with '+' for spaces)
#   ab=N:V1,V2,...      A/B of library builds on the bench (N alternations); Vi is
#                       "default" (libodo_hip.so) or a variant name (build_Vi/);
#                       bench arguments from $AB_ARGS
set -e
R=${GRAFT_REPO_ROOT:-/root/repo}
O=$R/gpurun_out/${1:?outdir}; shift
mkdir -p "$O"
P=$R/adaptive-rgbd-localization-mappig_amd
TUNING=$P/build_tuning/libodo_hip.so
QUICK="--no-cpu-baseline --no-direct-dispatch-leg --host-steps 0 --hard-steps 0 --latency-frames 0"
export TMPDIR=/tmp

lib_of() { if [ "$1" = default ]; then echo "$P/libodo_hip.so"; else echo "$P/build_$1/libodo_hip.so"; fi; }

pmc_passes() {  # REGEX OUTDIR BENCH_ARGS...  (library: $PMC_LIB, default the tuning build)
  local K=$1 D=$2; shift 2
  local LIB=${PMC_LIB:-$TUNING}
  mkdir -p "$D"
  cd /tmp
  for spec in \
    "sq1:SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU" \
    "sq2:SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_BUSY_CU_CYCLES" \
    "tcc:FETCH_SIZE" "tccw:WRITE_SIZE"; do
    local name=${spec%%:*} ctr=${spec#*:}
    ODO_SERIAL_STREAMS=1 ODO_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$K" \
      -d "$D/$name" -o run --output-format csv -- python3 $R/bench.py "$@" > "$D/$name.log" 2>&1
    echo "pmc $K $name ok"
  done
  ODO_SERIAL_STREAMS=1 ODO_LIB=$LIB timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$D/kt" -o run \
    --output-format csv -- python3 $R/bench.py "$@" > "$D/kt.log" 2>&1
  echo "pmc $K kernel trace ok"
  cd $R
}

for step in "$@"; do
  cd $R
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
      tail -1 $O/pytest.log ;;
    tests=*)
      files=$(echo ${step#tests=} | tr ',' '\n' | sed 's|^|tests/|' | tr '\n' ' ')
      timeout -k 10 900 python -u -m pytest $files -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_part.log 2>&1
      tail -1 $O/pytest_part.log ;;
    vtests=*)
      spec=${step#vtests=}; v=${spec%%:*}
      files=$(echo ${spec#*:} | tr ',' '\n' | sed 's|^|tests/|' | tr '\n' ' ')
      ODO_LIB=$(lib_of $v) timeout -k 10 900 python -u -m pytest $files -m gpu -x -q --timeout 300 \
        --timeout-method thread > $O/pytest_$v.log 2>&1
      tail -1 $O/pytest_$v.log ;;
    probe=*)
      spec=${step#probe=}; v=${spec%%:*}; sc=${spec#*:}
      ODO_LIB=$(lib_of $v) timeout -k 10 300 python tools/$sc.py > $O/probe_${v}_$sc.json 2> $O/probe_${v}_$sc.err
      echo "probe $v $sc ok" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
      echo "bench ok" ;;
    bench=*)
      spec=${step#bench=}; name=${spec%%:*}; args=$(echo ${spec#*:} | tr '+' ' ')
      timeout -k 10 600 python bench.py $args > $O/$name.json 2> $O/$name.err
      echo "bench $name ok" ;;
    benchenv=*)
      # benchenv=NAME:VAR=VAL/VAR2=VAL2:ARGS — the full default bench line
      # (production library, every leg) with variables in the environment
      spec=${step#benchenv=}; name=${spec%%:*}; rest=${spec#*:}
      envs=$(echo ${rest%%:*} | tr '/' ' '); args=$(echo ${rest#*:} | tr '+' ' ')
      [ "$args" = "$rest" ] && args=""
      env $envs timeout -k 10 600 python bench.py $args > $O/$name.json 2> $O/$name.err
      echo "benchenv $name: $(python tools/bsum.py $O/$name.json 2>/dev/null || true)" ;;
    multi)
      timeout -k 10 600 python bench.py --gpus 2 --backend gloo $QUICK > $O/multi_gloo.json 2> $O/multi_gloo.err
      echo "multi ok" ;;
    kt)
      cd /tmp
      timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- \
        python3 $R/bench.py --no-cpu-baseline --no-direct-dispatch-leg --hard-steps 0 --latency-frames 0 > $O/kt_bench.json 2> $O/kt.err
      cd $R
      T=$(find $O/kt -name '*kernel_trace.csv' -print -quit)
      python tools/rocprof_timed_region.py "$T" $O/kt_bench.json $O/rocprof_timed_region.json > $O/rtr.log 2>&1 || true
      echo "kt ok" ;;
    ktn=*)
      # ktn=NAME: the A/B bench command under rocprofv3 --kernel-trace (does
      # the traced run land in a different pipeline state?) -> NAME.json
      name=${step#ktn=}
      cd /tmp
      timeout -s KILL 600 rocprofv3 --kernel-trace -d $O/$name -o run --output-format csv -- \
        python3 $R/bench.py --no-cpu-baseline --no-direct-dispatch-leg --latency-frames 0 --host-steps 0 $AB_ARGS > $O/$name.json 2> $O/$name.err
      cd $R
      echo "ktn $name: $(python tools/bsum.py $O/$name.json 2>/dev/null || true)" ;;
    ktv=*)
      # ktv=V: the A/B bench command under a kernel trace with variant build_V
      v=${step#ktv=}
      cd /tmp
      ODO_LIB=$(lib_of $v) timeout -s KILL 600 rocprofv3 --kernel-trace -d $O/ktv_$v -o run --output-format csv -- \
        python3 $R/bench.py --no-cpu-baseline --no-direct-dispatch-leg --latency-frames 0 --host-steps 0 --hard-steps 0 $AB_ARGS \
        > $O/ktv_$v.json 2> $O/ktv_$v.err
      cd $R
      echo "ktv $v: $(python tools/bsum.py $O/ktv_$v.json 2>/dev/null || true)" ;;
    kth)
      # kernel trace of the hard workload in the main (pipelined) leg
      cd /tmp
      timeout -s KILL 600 rocprofv3 --kernel-trace --stats -d $O/kth -o run --output-format csv -- \
        python3 $R/bench.py --no-cpu-baseline --no-direct-dispatch-leg --host-steps 0 --hard-steps 0 --latency-frames 0 --workload hard \
        --steps 10 > $O/kth_bench.json 2> $O/kth.err
      cd $R
      echo "kth ok" ;;
    serial)
      cd /tmp
      ODO_SERIAL_STREAMS=1 ODO_LIB=$TUNING timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/serial_default \
        -o run --output-format csv -- python3 $R/bench.py $QUICK --steps 10 > $O/serial_default.log 2>&1
      echo "serial default ok"
      ODO_SERIAL_STREAMS=1 ODO_LIB=$TUNING timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/serial_hard \
        -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --no-direct-dispatch-leg --host-steps 0 --latency-frames 0 \
        --steps 2 --hard-steps 0 --workload hard > $O/serial_hard.log 2>&1
      echo "serial hard ok" ;;
    vserial=*)
      # per-kernel times alone (serial streams) of a tuning-flagged variant build_V
      v=${step#vserial=}
      cd /tmp
      ODO_SERIAL_STREAMS=1 ODO_LIB=$(lib_of $v) timeout -s KILL 300 rocprofv3 --kernel-trace --stats \
        -d $O/serial_$v -o run --output-format csv -- python3 $R/bench.py $QUICK --steps 10 > $O/serial_$v.log 2>&1
      echo "vserial $v ok" ;;
    pmc=*)
      K=${step#pmc=}
      pmc_passes "$K" "$O/pmc_$(echo $K | tr -c 'A-Za-z0-9_\n' '_')" --steps 3 --warmup 1 $QUICK ;;
    vpmc=*)
      # vpmc=V:REGEX — the four PMC passes of pmc= with variant build_V (-DODO_TUNING)
      spec=${step#vpmc=}; v=${spec%%:*}; K=${spec#*:}
      PMC_LIB=$(lib_of $v) pmc_passes "$K" "$O/pmc_${v}_$(echo $K | tr -c 'A-Za-z0-9_\n' '_')" --steps 3 --warmup 1 $QUICK ;;
    pmcx=*)
      # pmcx=NAME:REGEX:CTR1,CTR2,... — one extra counter pass (tuning build,
      # serial streams) over the kernels matching REGEX, into pmcx_NAME/
      spec=${step#pmcx=}; name=${spec%%:*}; rest=${spec#*:}; K=${rest%%:*}; ctr=$(echo ${rest#*:} | tr ',' ' ')
      mkdir -p $O/pmcx_$name
      cd /tmp
      ODO_SERIAL_STREAMS=1 ODO_LIB=$TUNING timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$K" \
        -d $O/pmcx_$name/p -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $QUICK \
        > $O/pmcx_$name/p.log 2>&1
      cd $R
      echo "pmcx $name ok" ;;
    vpmcx=*)
      # vpmcx=V:NAME:REGEX:C1,C2 — pmcx with variant build_V (built with -DODO_TUNING
      # for ODO_SERIAL_STREAMS; else the pipelined bench) -> pmcx_NAME/
      spec=${step#vpmcx=}; v=${spec%%:*}; rest=${spec#*:}; name=${rest%%:*}; rest=${rest#*:}
      K=${rest%%:*}; ctr=$(echo ${rest#*:} | tr ',' ' ')
      mkdir -p $O/pmcx_$name
      cd /tmp
      ODO_SERIAL_STREAMS=1 ODO_LIB=$(lib_of $v) timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-include-regex "$K" \
        -d $O/pmcx_$name/p -o run --output-format csv -- python3 $R/bench.py --steps 3 --warmup 1 $QUICK \
        > $O/pmcx_$name/p.log 2>&1
      cd $R
      echo "vpmcx $v $name ok" ;;
    listctr)
      timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
      echo "listctr ok" ;;
    pmch=*)
      K=${step#pmch=}
      pmc_passes "$K" "$O/pmch_$(echo $K | tr -c 'A-Za-z0-9_\n' '_')" --steps 2 --warmup 1 $QUICK --workload hard ;;
    vpmch=*)
      # vpmch=V:REGEX — pmch= with variant build_V (a tuning-flagged build)
      spec=${step#vpmch=}; v=${spec%%:*}; K=${spec#*:}
      PMC_LIB=$(lib_of $v) pmc_passes "$K" "$O/pmch_${v}_$(echo $K | tr -c 'A-Za-z0-9_\n' '_')" --steps 2 --warmup 1 $QUICK --workload hard ;;
    envbench=*)
      # envbench=NAME:VAR=VAL/VAR2=VAL2:ARGS — the tuning build with knobs from the environment
      spec=${step#envbench=}; name=${spec%%:*}; rest=${spec#*:}
      envs=$(echo ${rest%%:*} | tr '/' ' '); args=$(echo ${rest#*:} | tr '+' ' ')
      [ "$args" = "$rest" ] && args=""
      env $envs ODO_LIB=$TUNING timeout -k 10 300 python bench.py --no-cpu-baseline --no-direct-dispatch-leg --latency-frames 0 --host-steps 0 \
        $args > $O/$name.json 2> $O/$name.err
      echo "envbench $name: $(python tools/bsum.py $O/$name.json 2>/dev/null || true)" ;;
    ab=*)
      spec=${step#ab=}; n=${spec%%:*}; vs=$(echo ${spec#*:} | tr ',' ' ')
      for i in $(seq 1 $n); do
        for v in $vs; do
          ODO_LIB=$(lib_of $v) timeout -k 10 300 python bench.py --no-cpu-baseline --no-direct-dispatch-leg --latency-frames 0 --host-steps 0 \
            $AB_ARGS > $O/ab_${v}_$i.json 2> $O/ab_${v}_$i.err
          echo "ab $v $i: $(python tools/bsum.py $O/ab_${v}_$i.json 2>/dev/null || true)"
        done
      done ;;
    *)
      echo "unknown step $step" >&2; exit 2 ;;
  esac
done
