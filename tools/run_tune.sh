set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 300 python -m jumbo_mae_tpu_amd.csrc.build > gpurun_out/build.log 2>&1 || { echo BUILD FAIL; tail -20 gpurun_out/build.log; exit 1; }
mkdir -p gpurun_out/tune
date +%s > gpurun_out/tune/t0
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 PYTORCH_TUNABLEOP_MAX_TUNING_DURATION_MS=20 PYTORCH_TUNABLEOP_FILENAME=$R/gpurun_out/tune/tunableop_results.csv timeout -k 10 900 python bench.py --steps 3 --warmup 2 > gpurun_out/tune/tune_run.json 2> gpurun_out/tune/tune_run.err; echo tune rc=$?
date +%s >> gpurun_out/tune/t0
ls -la gpurun_out/tune/; wc -l gpurun_out/tune/*.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 PYTORCH_TUNABLEOP_FILENAME=$R/gpurun_out/tune/tunableop_results0.csv timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/tune/tuned_bench.json 2> gpurun_out/tune/tuned_bench.err; echo tuned rc=$?
cat gpurun_out/tune/tuned_bench.json
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/tune/base_bench.json 2>/dev/null
cat gpurun_out/tune/base_bench.json
