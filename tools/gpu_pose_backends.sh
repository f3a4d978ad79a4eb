# SURVEY 8(f) rank 4 back-ends: PnPRansac and GICP GPU parity tests, the
# PnPRansac bench leg and rocprofv3 kernel stats. Usage: tools/gpu_pose_backends.sh OUTDIR
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-pb}; mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gicp.py tests/test_pnpransac.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 -m pytest $R/tests/test_gicp.py -m gpu -x -q -p no:cacheprovider > $O/kt.log 2>&1
echo kt ok
