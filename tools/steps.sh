#!/bin/bash
# Generic GPU recipe: run named steps in order, each under its own time limit; stop at the first
# failing step (GPU fault, abort, timeout: nothing further touches the GPU in that call).
#   gpurun --timeout 900 -- bash tools/steps.sh <tag> "name:seconds:command" ["name:seconds:command" ...]
# Each step's stdout goes to gpurun_out/<tag>/<name>.out, stderr to <name>.err; the last lines of
# stdout are echoed.  A command may use $O (the output directory) and $R (the repo root).
# The special command "prof:<args>" runs `rocprofv3 --kernel-trace --stats -- python <args>` from
# /tmp into $O/<name>/ (the program is the direct child of rocprofv3, no launcher in between).
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export O R
for spec in "$@"; do
  name=${spec%%:*}; rest=${spec#*:}
  secs=${rest%%:*}; cmd=${rest#*:}
  echo "[steps] $name (${secs}s)"
  t0=$(date +%s)
  if [[ $cmd == prof:* ]]; then
    args=${cmd#prof:}
    ( cd /tmp && timeout -k 10 "$secs" rocprofv3 --kernel-trace --stats -d "$O/$name" -o run --output-format csv \
        -- python $R/$args ) > "$O/$name.out" 2> "$O/$name.err"
  else
    timeout -k 10 "$secs" bash -c "$cmd" > "$O/$name.out" 2> "$O/$name.err"
  fi
  rc=$?
  echo "[steps] $name rc=$rc $(( $(date +%s) - t0 ))s"
  tail -4 "$O/$name.out"
  if [ $rc -ne 0 ]; then
    tail -25 "$O/$name.err"
    exit $rc
  fi
done
echo "[steps] done"
