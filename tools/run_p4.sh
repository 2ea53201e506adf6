# p4 GEMM ablations (24 = static prio; 32 = no loads; 40 = no vmcnt; 72 = no barriers; 80 = none)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/p4c; mkdir -p $O
timeout -k 10 300 python -u tools/gemm_nt_bench.py --variant 24,32,40,72,80,12 --only enc_ff1,enc_ff2,dec_ff2 --kinds fwd --iters 10 --rounds 3 > $O/bench.txt 2>&1 || { tail $O/bench.txt; exit 1; }
cat $O/bench.txt
