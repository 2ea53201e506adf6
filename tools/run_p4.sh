# stream-K GEMM: tests + A/B (24 = with stream-K where planned, 24n = plain tiled)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/sk2; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k "gemm" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u tools/gemm_nt_bench.py --variant 24,24n --kinds fwd,fwd_gelu,dgrad --iters 10 --rounds 3 > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
cat $O/bench.txt
