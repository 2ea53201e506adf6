set -o pipefail
cd $GRAFT_REPO_ROOT; O=gpurun_out/ftattn; mkdir -p $O
for cfg in "" "--ppw 1" "--ppw 2" "--ppw 4" "--bwd3-hd64 1" "--bwd3-hd64 1 --ppw 1" "--max-seq 128"; do
  echo "== $cfg" >> $O/out.txt
  timeout -k 10 120 python tools/attn_bench.py --shapes ft12 $cfg >> $O/out.txt 2>&1 || { echo "fail $cfg"; tail -5 $O/out.txt; exit 1; }
done
grep -v amdgpu.ids $O/out.txt
