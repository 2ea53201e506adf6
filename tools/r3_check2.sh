#!/bin/bash
# GEMM + model GPU tests, pretrain and finetune bench, finetune rocprof.  gpurun -- bash tools/r3_check2.sh <tag>
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=$R/gpurun_out/$1; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --task finetune --steps 20 --warmup 5 > $O/bench_ft.json 2> $O/bench_ft.err || { tail -20 $O/bench_ft.err; exit 1; }
cat $O/bench_ft.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_ft -o run --output-format csv -- python $R/bench.py --task finetune --steps 10 --warmup 2 > $O/prof_ft.log 2>&1 || { tail -20 $O/prof_ft.log; exit 1; }
echo done
