set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/final_bench.json 2> gpurun_out/final_bench.err || exit 1
cat gpurun_out/final_bench.json
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_final -o run --output-format csv -- python $R/bench.py --steps 12 --warmup 2 > $R/gpurun_out/prof_final_bench.log 2>&1
