set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for t in finetune linear; do
rm -rf $R/gpurun_out/prof_$t
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$t -o run --output-format csv -- python $R/bench.py --task $t --steps 10 --warmup 2 > $R/gpurun_out/prof_$t.log 2>&1 || exit 1
echo PROF_OK $t
done
