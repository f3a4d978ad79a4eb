# Step time under CU-mask partitions of the pair / extraction streams (tuning build)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-cumask}; mkdir -p $O; cd $R
LIB=adaptive-rgbd-localization-mappig_amd/build_tuning/libodo_hip.so
F=ffffffff
run() {  # name pairmask extractmask
  ODO_LIB=$LIB ODO_PAIR_CUMASK=$2 ODO_EXTRACT_CUMASK=$3 timeout -k 10 300 python bench.py --no-cpu-baseline --host-steps 0 --hard-steps 0 --latency-frames 0 > $O/$1.json 2> $O/$1.err
  echo $1 ok
}
run base "" ""
run p64lo $F,$F,0,0,0,0,0,0 ""
run p32lo $F,0,0,0,0,0,0,0 ""
run p64s 11111111,11111111,11111111,11111111,11111111,11111111,11111111,11111111 ""
run p32s 01010101,01010101,01010101,01010101,01010101,01010101,01010101,01010101 ""
run p128s 55555555,55555555,55555555,55555555,55555555,55555555,55555555,55555555 ""
run part64 $F,$F,0,0,0,0,0,0 0,0,$F,$F,$F,$F,$F,$F
run part64s 11111111,11111111,11111111,11111111,11111111,11111111,11111111,11111111 eeeeeeee,eeeeeeee,eeeeeeee,eeeeeeee,eeeeeeee,eeeeeeee,eeeeeeee,eeeeeeee
