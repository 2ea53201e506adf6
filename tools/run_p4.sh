# persistent whole-tile launch on fewer CUs (24d) vs tiled (24) vs stream-K (24s)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/sk3; mkdir -p $O
timeout -k 10 400 python -u tools/gemm_nt_bench.py --variant 24,24d,24s --only enc_wo,enc_ff2,enc_ff1,dec_wo,dec_ff2 --kinds fwd,dgrad --iters 10 --rounds 3 > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
cat $O/bench.txt
