# step-level interleaved A/B: tools/run_ab.sh <outdir> <config>...
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; cd $R; O=gpurun_out/$1; shift; mkdir -p $O
timeout -k 10 500 python -u tools/ab_bench.py --configs "$@" --rounds 4 --steps 6 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -8 $O/ab.txt
