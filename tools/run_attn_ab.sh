# A/B of two extension builds on the attention microbench: abtmp/old (PYTHONPATH) vs the tree
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd $R
for i in 1 2; do
for v in old new; do
if [ $v = old ]; then PP=$R/abtmp/old; else PP=$R; fi
JMAE_ROOT=$PP timeout -k 10 120 python tools/attn_bench.py --shapes dec,enc,ft > gpurun_out/attn_$v$i.txt 2>&1 || { cat gpurun_out/attn_$v$i.txt; exit 1; }
echo "== $v $i"; grep -v amdgpu gpurun_out/attn_$v$i.txt
done
done
