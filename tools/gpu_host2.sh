#!/bin/bash
# GPU-box recipe: host pipeline tests + the bench's host-to-host leg
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-host2}"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_pipeline.py tests/test_gpu_config1.py tests/test_gpu_flacaudio.py \
    -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-decode --no-chain --no-t2t --no-rg4 > $OUT/bench.log 2>&1
