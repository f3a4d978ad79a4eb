# Step time of the headline leg under tuning knobs / variant builds:
#   tools/ab_knobs.sh OUTDIR "name|LIB|ENV=.. ENV2=.." ...
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-knobs}; mkdir -p $O; cd $R; shift
for spec in "$@"; do
  IFS='|' read -r name lib envs <<< "$spec"
  env ODO_LIB=$lib $envs timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --hard-steps 0 --latency-frames 0 > $O/$name.json 2> $O/$name.err
  echo $name ok
done
