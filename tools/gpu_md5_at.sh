#!/bin/bash
# MD5 placement experiment (encoder leg): ATG_MD5_AT = 0 after the LPC
# kernel (product), 1 at the start of the batch, 2 skipped (timing only).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/at"
cd "$R"
ARGS="--steps 30 --warmup 3 --no-cpu-baseline --no-verify --no-decode --no-chain --no-host"
for k in 1 2; do
    for a in ${AT_LIST:-0 1 2}; do
        ATG_MD5_AT=$a timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/at/at${a}_$k.log 2>&1
    done
done
