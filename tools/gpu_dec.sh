#!/bin/bash
# Decoder MD5 priority experiment: the decode leg with the chains at raised
# (default) and normal priority, alternating.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/dec"
cd "$R"
ARGS="--steps 10 --warmup 2 --no-cpu-baseline --no-verify --no-chain --no-host"
for k in 1 2; do
    timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/dec/p1_$k.log 2>&1
    ATG_DEC_MD5_PRIO=0 timeout -k 10 300 python -u bench.py $ARGS > gpurun_out/dec/p0_$k.log 2>&1
done
