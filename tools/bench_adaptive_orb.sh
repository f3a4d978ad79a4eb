# ADAPTIVE with the cv::ORB inner detector: bench line (with a small CPU
# sample) and a serial-stream kernel trace, in one call.
# Usage: tools/bench_adaptive_orb.sh OUTDIR_NAME   (results under gpurun_out/OUTDIR_NAME)
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-aorb}; mkdir -p $O
cd $R
timeout -k 10 600 python bench.py --detector adaptive-orb --host-steps 0 --hard-steps 0 --cpu-frames 8 --cpu-reps 3 > $O/bench.json 2> $O/bench.err
echo bench ok
cd /tmp && export TMPDIR=/tmp
ODO_SERIAL_STREAMS=1 timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 $R/bench.py --detector adaptive-orb --steps 5 --warmup 2 --no-cpu-baseline --host-steps 0 --hard-steps 0 > $O/kt.log 2>&1
echo kt ok
