#!/bin/bash
# Weight-gradient side stream (JMAE_WGRAD_STREAM=1): several independent bench processes, looking for
# the intermittent collapse seen in round 1, plus a kernel trace of one run.
#   gpurun --timeout 900 -- bash tools/side_stream_check.sh <outdir> [runs]
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
N=${2:-5}
for i in $(seq 1 $N); do
  JMAE_WGRAD_STREAM=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/on_$i.json 2> $O/on_$i.err || { tail -5 $O/on_$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/on_$i.json')); print('on  run $i', d['ms_per_step'])"
done
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/off.json 2> $O/off.err || exit 1
python -c "import json; d=json.load(open('$O/off.json')); print('off run  ', d['ms_per_step'])"
cd /tmp && JMAE_WGRAD_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_on -o run --output-format csv -- python $R/bench.py --steps 4 --warmup 2 > $O/trace_on.log 2>&1 || { tail -5 $O/trace_on.log; exit 1; }
echo done
