# GPU: full gpu test-suite, smoke, pretrain ViT-L/ViT-B, finetune ViT-B, linear-probe ViT-L benches.
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
for t in "pretrain" "pretrain --model vit_base_patch16" "finetune" "linear"; do
  n=$(echo $t | tr ' ' '_')
  timeout -k 10 400 python bench.py --task $t --steps 20 --warmup 5 > gpurun_out/bench_$n.json 2> gpurun_out/bench_$n.err || { tail -20 gpurun_out/bench_$n.err; exit 1; }
  cat gpurun_out/bench_$n.json
done
