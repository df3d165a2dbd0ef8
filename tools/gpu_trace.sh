#!/bin/bash
# kernel timeline of a short encoder-leg bench (rocprofv3 kernel trace, no
# counters): start/end of every dispatch, for stream-overlap questions
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/tr"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/gpurun_out/tr/t" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 8 --warmup 2 --no-cpu-baseline --no-verify --no-decode --no-chain --no-host \
    > "$R/gpurun_out/tr/trace.log" 2>&1
