set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/tn4; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_mae_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "tn_wgrad" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/wgrad_bench.py --variants 4,0 > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
grep -v amdgpu.ids $O/bench.txt
