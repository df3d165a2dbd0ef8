#!/bin/bash
# MD5 split-ratio A/B on one box (encoder leg, 30 steps, alternating).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/sp"
cd "$R"
ARGS="--steps 30 --warmup 3 --no-cpu-baseline --no-verify --no-decode --no-chain --no-host"
for k in 1 2 3; do
    for pct in 50 60 70; do
        ATG_MD5_SPLIT_PCT=$pct timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/sp/p${pct}_$k.log 2>&1
    done
done
