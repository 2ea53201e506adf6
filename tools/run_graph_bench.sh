set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
for t in "finetune" "finetune --hip-graph" "pretrain --model vit_base_patch16" "pretrain --model vit_base_patch16 --hip-graph" "pretrain" "pretrain --hip-graph"; do
  n=$(echo $t | tr ' ' '_')
  timeout -k 10 400 python bench.py --task $t --steps 20 --warmup 5 > gpurun_out/gb_$n.json 2> gpurun_out/gb_$n.err || { tail -20 gpurun_out/gb_$n.err; exit 1; }
  echo "$t: $(python -c "import json,sys; d=json.load(open('gpurun_out/gb_$n.json')); print(d['value'], d['ms_per_step'], d['config'].get('hip_graph'))")"
done
