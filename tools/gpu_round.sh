#!/bin/bash
# GPU-box recipe for a full measurement: smoke, PMC passes -> HBM traffic,
# bench (with CPU baseline), rocprofv3 kernel-trace stats of the bench.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
ROUND=${1:-r02}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
bash tools/gpu_pmc.sh
# results land in gpurun_out/ (merged back) and in this box's profiles/ so
# the bench below already reads the fresh counters
python3 tools/pmc_traffic.py gpurun_out/pmc gpurun_out/pmc_traffic.json gpurun_out/pmc_valu.json \
    65536 "$ROUND PMC (tools/gpu_pmc.sh)" > gpurun_out/pmc_traffic.log
cp gpurun_out/pmc_traffic.json gpurun_out/pmc_valu.json profiles/
python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.json
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline \
    > "$R/gpurun_out/prof.log" 2>&1
