#!/bin/bash
# Encoder tests + the full bench (all legs) twice.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/legs"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_config1.py tests/test_gpu_host_pipeline.py \
    tests/test_gpu_flacaudio.py tests/test_gpu_resample.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/legs/pytest.log 2>&1
for k in 1 2; do
    timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/legs/bench_$k.log 2>&1
done
