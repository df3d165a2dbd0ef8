#!/bin/bash
# GPU-box recipe: kernel trace of the config-5 chain leg alone (the
# headline leg runs 5 steps first), for tools/chain_timeline.py.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-chaintrace}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$OUT/prof" -o run --output-format csv \
    -- python3 $R/bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-verify --no-host \
    --no-t2t --no-rg4 --narrow= --no-decode > "$OUT/prof.log" 2>&1
f=$(find "$OUT/prof" -name '*kernel_trace.csv' | head -n 1)
cp "$f" "$OUT/kernel_trace.csv"
