# A/B of the PnP trial solves: one wave's 16-lane groups (pnpg, default) vs
# one wave per trial (pnpw); bench lines alternated on one box.
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_pnpt; mkdir -p $O
cd $R
for rep in 1 2; do
  for v in pnpg pnpw; do
    ODO_LIB=adaptive-rgbd-localization-mappig_amd/build/libodo_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
    echo $v $rep ok
  done
done
