#!/bin/bash
# CU-partition experiment (encoder leg): MD5 streams on 8 CUs vs shared CUs
# (ATG_NO_CUMASK=1), alternating runs, then the encoder parity tests.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/cm"
cd "$R"
ARGS="--steps 30 --warmup 3 --no-cpu-baseline --no-verify --no-decode --no-chain --no-host"
for k in 1 2; do
    timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/cm/mask_$k.log 2>&1
    ATG_NO_CUMASK=1 timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/cm/nomask_$k.log 2>&1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_config1.py tests/test_gpu_host_pipeline.py \
    -x -q --timeout 120 --timeout-method thread > gpurun_out/cm/pytest.log 2>&1
