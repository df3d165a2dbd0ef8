#!/bin/bash
# the headline roofline's kernel-stats pass: rocprofv3 --kernel-trace --stats
# of `bench.py --k2-profile` (every search launch one 1024-track config-2
# batch alone on the device), summary copied to profiles/<name>.
# tools/gpu_k2_profile.sh <tag> [profiles name]
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-k2prof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 $R/bench.py --k2-profile --steps 20 > "$OUT/prof.log" 2>&1
f=$(find "$OUT/prof" -name '*kernel_stats.csv' | head -n 1)
cp "$f" "$OUT/k2_alone_kernel_stats.csv"
