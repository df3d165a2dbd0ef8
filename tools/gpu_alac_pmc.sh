#!/bin/bash
# GPU-box recipe: instruction counters of the config-5 chain leg's kernels
# (the ALAC decode among them), one rocprofv3 --pmc pass.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-alacpmc}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM \
    SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY -d "$OUT/sq" -o run \
    --output-format csv -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    --no-verify --no-host --no-t2t --no-rg4 --narrow= --no-decode > "$OUT/sq.log" 2>&1
