# A/B of the finalize staging: wave-uniform per-keypoint staging (finw) vs each
# keypoint's 16 lanes staging its own patches (fino); bench lines alternated
# on one box, then a serial kernel trace of each.
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_fins; mkdir -p $O
cd $R
for rep in 1 2; do
  for v in finw fino; do
    ODO_LIB=adaptive-rgbd-localization-mappig_amd/build/libodo_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
    echo $v $rep ok
  done
done
