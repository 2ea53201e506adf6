set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6e; mkdir -p $O
for c in 1 0; do
JMAE_GELU_CODES=$c timeout -k 10 400 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_drivers_gpu.py -k test_pretrain_driver_on_gpu > $O/drv_codes$c.log 2>&1; rc=$?
grep "driver-test\|passed\|failed" $O/drv_codes$c.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
