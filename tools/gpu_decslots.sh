#!/bin/bash
# GPU-box recipe: decode step with 4 slots (product) vs 3 (exp build), 30 steps each
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-decslots}
mkdir -p "$OUT"
cd "$R"
A="--steps 30 --no-cpu-baseline --no-chain --no-host --no-t2t --no-rg4"
timeout -k 10 200 python -u bench.py $A > $OUT/s4.log 2>&1
ATGPU_LIB=$R/exp/libatgpu_dslot3.so timeout -k 10 200 python -u bench.py $A --dec-inflight 3 > $OUT/s3.log 2>&1
timeout -k 10 200 python -u bench.py $A > $OUT/s4b.log 2>&1
