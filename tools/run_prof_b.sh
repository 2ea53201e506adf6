set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
rm -rf $R/gpurun_out/prof_b
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_b -o run --output-format csv -- python $R/bench.py --model vit_base_patch16 --steps 10 --warmup 2 > $R/gpurun_out/prof_b.log 2>&1 || exit 1
echo PROF_OK
