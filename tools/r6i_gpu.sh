#!/bin/bash
# round 6 validation: full GPU suite (ViT-L parity summary kept), default bench + kernel trace, per-GPU shapes
set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/${1:-r6i}; mkdir -p $O
JMAE_PARITY_OUT=$O/vitl_parity.json timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/benchprof -o b -- python bench.py --steps 6 --warmup 3 > $O/benchprof.log 2>&1 || { tail -20 $O/benchprof.log; exit 1; }
python tools/trace_steps.py $(find $O/benchprof -name "*kernel_trace.csv" | head -1) --last 4 --top 40 > $O/bench_steps.txt 2>&1; head -12 $O/bench_steps.txt
for a in "vitl_b512 --batch-per-gpu 512" "vitb_b512 --model vit_base_patch16 --batch-per-gpu 512" "ft_b128 --task finetune --batch-per-gpu 128"; do
  set -- $a; n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python -c "import json;d=json.load(open('$O/$n.json'));print('$n',d['value'],'img/s',d['ms_per_step'],'ms')"
done
rm -f $(find $O/benchprof -name "*.csv" -size +20M) 2>/dev/null; true
