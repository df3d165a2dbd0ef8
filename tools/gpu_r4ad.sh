#!/bin/bash
# ALAC chunked bit reader: ALAC + chain parity tests, then the chain leg
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4ad
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_alac.py tests/test_gpu_chain.py \
    -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-decode --no-host --no-t2t --no-rg4 --steps 3 --warmup 1 > $OUT/bench_chain.log 2>&1
