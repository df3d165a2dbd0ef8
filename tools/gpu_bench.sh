#!/bin/bash
# GPU-box recipe: smoke, bench, rocprofv3 kernel stats (run via gpurun).
#   gpurun --timeout 900 -- bash tools/gpu_bench.sh [steps]
# Every GPU step has its own time limit; the script stops at the first failure.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
STEPS=${1:-5}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" \
    > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python -u bench.py --steps "$STEPS" --warmup 2 > gpurun_out/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline \
    > "$R/gpurun_out/prof.log" 2>&1
