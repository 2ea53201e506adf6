set -o pipefail
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT; O=gpurun_out/wtb1; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py tests/test_graph_gpu.py -x -q --timeout 120 --timeout-method thread -k "transpose or weight_t or graph" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 500 python -u tools/ab_bench.py --configs "a:WT_BATCH=0" "b:WT_BATCH=1" --rounds 4 --steps 6 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -2 $O/ab.txt
