set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
rm -rf $R/gpurun_out/prof_finetune
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_finetune -o run --output-format csv -- python $R/bench.py --task finetune --steps 10 --warmup 2 > $R/gpurun_out/prof_finetune.log 2>&1 || exit 1
cd $R
timeout -k 10 300 python bench.py --task finetune --steps 20 --warmup 5 > gpurun_out/bench_finetune.json 2> gpurun_out/bench_finetune.err || exit 1
cat gpurun_out/bench_finetune.json
