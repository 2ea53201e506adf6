set -o pipefail
export TMPDIR=/tmp
cd ${GRAFT_REPO_ROOT:-.}
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_kernels_gpu.py -k layernorm > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; grep -h "loss_rel" $O/pytest.log | tail -2
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
JMAE_PARITY_OUT=$O/vitl_parity.json timeout -k 10 300 python -u -m pytest -x -q -s --timeout 250 --timeout-method thread tests/test_vitl_parity_gpu.py > $O/parity.log 2>&1; tail -3 $O/parity.log
timeout -k 10 400 python -u tools/ab_bench.py --batch 2048 --configs "h:LN_FROM_H=1" "x:LN_FROM_H=0" --rounds 3 --steps 3 > $O/ab_ln.txt 2>&1 || { tail $O/ab_ln.txt; exit 1; }
tail -4 $O/ab_ln.txt
timeout -k 10 500 python -u tools/gelu_code_ab.py --task pretrain --steps 600 --out $O/gelu_ab_pretrain.json > $O/gelu_pre.txt 2>&1 || { tail $O/gelu_pre.txt; exit 1; }
tail -1 $O/gelu_pre.txt
timeout -k 10 500 python -u tools/gelu_code_ab.py --task finetune --steps 600 --out $O/gelu_ab_finetune.json > $O/gelu_ft.txt 2>&1 || { tail $O/gelu_ft.txt; exit 1; }
tail -1 $O/gelu_ft.txt
timeout -k 10 300 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
cat $O/bench.json
