set -o pipefail
cd /tmp
timeout -k 10 120 rocprofv3 -L > $GRAFT_REPO_ROOT/gpurun_out/pmc_list.txt 2>&1; echo rc=$?
wc -l $GRAFT_REPO_ROOT/gpurun_out/pmc_list.txt
