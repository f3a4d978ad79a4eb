# A/B of the ADAPTIVE ORB candidate band height (OA_BH 32 vs 64): bench lines
# alternated on one box.
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_oabh; mkdir -p $O
cd $R
for rep in 1 2; do
  for v in bh32 bh64; do
    ODO_LIB=adaptive-rgbd-localization-mappig_amd/build/libodo_$v.so timeout -k 10 300 python bench.py --detector adaptive-orb --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
    echo $v $rep ok
  done
done
