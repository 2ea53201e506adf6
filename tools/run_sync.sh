set -o pipefail
cd $GRAFT_REPO_ROOT
for t in finetune linear pretrain; do
timeout -k 10 300 python tools/sync_check.py --task $t > gpurun_out/sync_$t.txt 2>&1 || { tail -30 gpurun_out/sync_$t.txt; exit 1; }
head -1 gpurun_out/sync_$t.txt
done
