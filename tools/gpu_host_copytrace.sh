#!/bin/bash
# GPU-box recipe: the host-to-host leg's copy timeline.  One bench run (all
# device legs off but the headline) under --kernel-trace --memory-copy-trace
# --stats; tools/copy_overlap.py reports per-direction busy time, rate and
# the H2D/D2H overlap.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-r5q}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/trace" -o run \
    --output-format csv -- python3 "$R/bench.py" --steps 6 --warmup 2 --no-cpu-baseline \
    --no-verify --no-chain --no-decode --no-t2t --no-rg4 --narrow= > "$OUT/bench.log" 2>&1
cd "$R"
python3 tools/copy_overlap.py "$OUT/trace" > "$OUT/copies.txt"
