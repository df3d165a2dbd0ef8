#!/bin/bash
# MD5 placement experiment: encoder-only bench with the MD5 chains after the
# LPC kernel (default) and at the start of the batch (ATG_MD5_AT=1).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-decode --no-chain --no-host --no-cpu-baseline \
    > gpurun_out/bench_at0.log 2>&1
ATG_MD5_AT=1 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-decode --no-chain --no-host \
    --no-cpu-baseline > gpurun_out/bench_at1.log 2>&1
