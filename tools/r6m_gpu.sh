#!/bin/bash
# round 6 (s, same script as m): 8-wave dropout backward with the Q / dO fragments loaded per key tile (no spills) -- dropout GPU tests, then finetune 128-image
# step at dropout 0.1 / 0: tree vs _abbase (HEAD), alternating processes
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd $R; O=gpurun_out/r6s; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_dropout_gpu.py tests/test_kernels_gpu.py -k "drop or attn" -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
A="--task finetune --batch-per-gpu 128 --steps 30 --warmup 5"
for i in 1 2 3; do
  timeout -k 10 200 python -u _abbase/tools/bench_task.py $A --dropout 0.1 > $O/a_d$i.txt 2>&1 || { tail -20 $O/a_d$i.txt; exit 1; }
  timeout -k 10 200 python -u tools/bench_task.py $A --dropout 0.1 > $O/b_d$i.txt 2>&1 || { tail -20 $O/b_d$i.txt; exit 1; }
  timeout -k 10 200 python -u tools/bench_task.py $A > $O/b_z$i.txt 2>&1 || { tail -20 $O/b_z$i.txt; exit 1; }
done
timeout -k 10 120 python -u tools/attn_bench.py --shapes ft12 --iters 10 > $O/attn_b.txt 2>&1 && JMAE_ROOT=$R/_abbase timeout -k 10 120 python -u _abbase/tools/attn_bench.py --shapes ft12 --iters 10 > $O/attn_a.txt 2>&1 || exit 1
for f in $O/*_[dz]?.txt; do echo "$(basename $f) $(grep '^{' $f | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"; done
