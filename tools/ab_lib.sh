# A/B of library builds on the bench's headline (and hard) legs, alternated:
#   tools/ab_lib.sh OUTDIR ROUNDS LIB1 LIB2 ...   (bench args: $AB_ARGS)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-ab}; mkdir -p $O; cd $R
N=$2; shift 2
for i in $(seq 1 $N); do
  k=0
  for LIB in "$@"; do
    k=$((k+1))
    ODO_LIB=$LIB timeout -k 10 300 python bench.py --no-cpu-baseline --latency-frames 0 --host-steps 0 $AB_ARGS > $O/L${k}_$i.json 2> $O/L${k}_$i.err
    echo "L$k $i ok"
  done
done
