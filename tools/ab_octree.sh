# A/B of the octree dispatch order: frames x levels (octA, level 0 first) vs levels x frames (octB)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_oct; mkdir -p $O
cd $R
for rep in 1 2; do
  for v in octA octB; do
    ODO_LIB=adaptive-rgbd-localization-mappig_amd/build/libodo_$v.so timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err
    echo $v $rep ok
  done
done
