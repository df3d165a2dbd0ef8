#!/bin/bash
# GPU-box recipe: PMC counter passes over one python command (run via gpurun).
#   tools/gpu_pmc_cmd.sh NAME script.py [args...]
# One rocprofv3 run per pass, each within the per-block counter limits,
# kernel-trace only alongside the counters; CSVs under gpurun_out/pmc_NAME.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
NAME=$1
shift
OUT="$R/gpurun_out/pmc_$NAME"
mkdir -p "$OUT"
SCRIPT="$R/$1"
shift
cd /tmp && export TMPDIR=/tmp
pass() {
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --pmc "$@" -d "$OUT/$name" -o run --output-format csv \
        -- python3 "$SCRIPT" "${ARGS[@]}" > "$OUT/$name.log" 2>&1
}
ARGS=("$@")
pass sq1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY
pass sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_ANY
pass grbm GRBM_GUI_ACTIVE GRBM_COUNT
