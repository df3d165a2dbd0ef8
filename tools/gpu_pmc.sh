#!/bin/bash
# GPU-box recipe: PMC counter passes over one bench step (run via gpurun).
# One rocprofv3 run per pass (no pass exceeds the per-block counter limits),
# kernel-trace only alongside the counters.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-pmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify --no-host --no-chain --no-t2t --no-rg4 --narrow="
# the converter leg (k_pcm_bps) runs inside the decode legs of the same process
pass() {
    local name=$1; shift
    timeout -s KILL 90 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv \
        -- python3 $ARGS > "$OUT/$name.log" 2>&1
}
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
