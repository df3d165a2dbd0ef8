#!/bin/bash
# GPU-box recipe: host-to-host chunk-size matrix with the product library
# (high-priority aux streams), wall time per 1024-track batch.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-hostmx2}"
mkdir -p "$OUT"
cd "$R"
for cfg in "256 2" "256 3" "384 3" "512 2" "512 3" "768 3"; do
    set -- $cfg
    timeout -k 10 150 python3 -u tools/host_timeline.py 4 pinned $1 $2 > "$OUT/c$1_i$2.log" 2>&1
done
