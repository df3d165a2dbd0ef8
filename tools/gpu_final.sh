#!/bin/bash
# GPU-box recipe for round end: the whole -m gpu suite, then a rocprofv3
# kernel-stats pass of the encoder-leg bench (the headline workload only, so
# the per-kernel averages are the bench line's launches).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/pytest_gpu.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_enc" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-decode --no-chain --no-host \
    > "$R/gpurun_out/prof_enc.log" 2>&1
