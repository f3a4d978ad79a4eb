# One build -> measure iteration on the GPU box: the named parity tests, a
# bench line (no CPU baseline), optional extra commands.
# Usage: tools/gpu_iter.sh OUTDIR "tests/a.py tests/b.py" ["extra shell command"]
set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/${1:-it}; mkdir -p $O
cd $R
if [ -n "$2" ]; then
timeout -k 10 600 python -u -m pytest $2 -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
fi
timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
echo bench ok
if [ -n "$3" ]; then
eval "$3"
echo extra ok
fi
