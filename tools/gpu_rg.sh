#!/bin/bash
# GPU-box recipe: ReplayGain tests and the bench's ReplayGain legs.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-rg}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_replaygain.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-chain --no-host --no-t2t > $OUT/bench.log 2>&1
