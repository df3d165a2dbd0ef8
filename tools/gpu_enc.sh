#!/bin/bash
# Encoder-leg check: parity tests, then the bench at its default step count
# and at 30 steps (alternating), encoder leg only.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/enc"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_config1.py tests/test_gpu_host_pipeline.py \
    -x -q --timeout 120 --timeout-method thread > gpurun_out/enc/pytest.log 2>&1
ARGS="--no-cpu-baseline --no-decode --no-chain --no-host"
for k in 1 2; do
    timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/enc/default_$k.log 2>&1
    timeout -k 10 200 python -u bench.py $ARGS --steps 30 --warmup 3 > gpurun_out/enc/s30_$k.log 2>&1
done
