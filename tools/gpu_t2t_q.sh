#!/bin/bash
# GPU-box recipe: track2track probe under GPU_MAX_HW_QUEUES 1 / 2 / 4 and
# with the aux streams at normal priority.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-t2tq}
mkdir -p "$OUT"
cd "$R"
for q in 1 2 4; do
  for p in 8 16; do
    echo "q=$q" >> $OUT/probe.log
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python -u tools/t2t_probe.py $p >> $OUT/probe.log 2>&1
  done
done
