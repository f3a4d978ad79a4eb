set -e
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/r1; mkdir -p $O
cd $R
timeout -k 10 300 tools/ubench_peak > $O/ubench.jsonl
echo ubench ok
grep -E "mfma_scale|knn_f4_mix" $O/ubench.jsonl >> profiles/r02_ubench_peak.jsonl
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo pytest ok
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err
echo bench ok
