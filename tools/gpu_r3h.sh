#!/bin/bash
# GPU-box recipe: resampler phase tables (tests), then the bench (no CPU
# baselines / chain / t2t / rg4) with the product library and with the
# high-priority aux stream build.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3h}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_resample.py tests/test_gpu_chain.py tests/test_gpu_decode.py \
    -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
ARGS="bench.py --no-cpu-baseline --no-chain --no-t2t --no-rg4"
timeout -k 10 300 python -u $ARGS > $OUT/bench.log 2>&1
ATGPU_LIB=$R/exp/libatgpu_hiprio.so timeout -k 10 300 python -u $ARGS > $OUT/bench_hiprio.log 2>&1
