#!/bin/bash
# GPU-box recipe: resampler tests and the bench's resample legs
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-rs}"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_resample.py tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-host --no-t2t --no-rg4 > $OUT/bench.log 2>&1
