#!/bin/bash
# GPU-box recipe: host-to-host pipeline timeline (tools/host_timeline.py
# under a kernel + memory-copy trace), then the per-batch breakdown and the
# copy-direction overlap.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-r5s}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --memory-copy-trace -d "$OUT/trace" -o run \
    --output-format csv -- python3 "$R/tools/host_timeline.py" 5 pinned 512 3 > "$OUT/timeline.log" 2>&1
cd "$R"
python3 tools/host_breakdown.py "$OUT/trace" > "$OUT/breakdown.txt" 2>&1
python3 tools/copy_overlap.py "$OUT/trace" 16777216 > "$OUT/copies.txt" 2>&1
