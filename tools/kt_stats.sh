# rocprofv3 kernel stats of a short headline run per (name, lib, env):
#   tools/kt_stats.sh OUTDIR "name|LIB|ENV=.." ...
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-kt}; mkdir -p $O; shift
cd /tmp && export TMPDIR=/tmp
for spec in "$@"; do
  IFS='|' read -r name lib envs <<< "$spec"
  export ODO_LIB=$R/$lib
  for kv in $envs; do export "$kv"; done
  timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/$name -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-steps 0 --hard-steps 0 --latency-frames 0 > $O/$name.json 2> $O/$name.err
  for kv in $envs; do unset "${kv%%=*}"; done
  echo $name ok
done
