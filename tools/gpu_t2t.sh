#!/bin/bash
# GPU-box recipe: track2track leg breakdown at 1, 2, 4, 8 (16) processes.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-t2t}
mkdir -p "$OUT"
cd "$R"
for p in ${PROCS:-1 2 4 8}; do
  timeout -k 10 120 python -u tools/t2t_probe.py $p >> $OUT/probe.log 2>&1
done
