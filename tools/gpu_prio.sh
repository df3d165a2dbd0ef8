#!/bin/bash
# MD5 priority x in-flight depth experiment (encoder leg), then encoder tests.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/pr"
cd "$R"
ARGS="--steps 30 --warmup 3 --no-cpu-baseline --no-verify --no-decode --no-chain --no-host"
for k in 1 2; do
    timeout -k 10 200 python -u bench.py $ARGS --inflight 3 > gpurun_out/pr/p0_d3_$k.log 2>&1
    ATG_MD5_PRIO=1 timeout -k 10 200 python -u bench.py $ARGS --inflight 3 > gpurun_out/pr/p1_d3_$k.log 2>&1
    timeout -k 10 200 python -u bench.py $ARGS --inflight 2 > gpurun_out/pr/p0_d2_$k.log 2>&1
    ATG_MD5_PRIO=1 timeout -k 10 200 python -u bench.py $ARGS --inflight 2 > gpurun_out/pr/p1_d2_$k.log 2>&1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_config1.py tests/test_gpu_host_pipeline.py \
    -x -q --timeout 120 --timeout-method thread > gpurun_out/pr/pytest.log 2>&1
