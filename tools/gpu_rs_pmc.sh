#!/bin/bash
# GPU-box recipe: LDS and VALU counters of the resampler (config-3 leg and
# the config-5 chain's k_rs_phase), one rocprofv3 --pmc pass.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-rspmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT \
    SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d "$OUT/sq" -o run --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 \
    --no-cpu-baseline --no-verify --no-host --no-t2t --no-rg4 --narrow= > "$OUT/sq.log" 2>&1
