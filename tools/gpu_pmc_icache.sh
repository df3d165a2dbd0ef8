#!/bin/bash
# instruction-cache PMC pass over one bench step
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/pmc_ic"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_WAVES \
    -d "$OUT/ic" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-decode --no-chain --no-host > "$OUT/ic.log" 2>&1
