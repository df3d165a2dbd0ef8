#!/bin/bash
# GPU-box recipe (round 4): kernel trace of the pipelined decoder probe
# (timeline: where a step's time goes between the two streams).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4l}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/trace" -o run --output-format csv \
    -- python3 $R/tools/dec_probe.py --tag trace --steps 12 > "$OUT/trace.log" 2>&1
