#!/bin/bash
# GPU-box recipe: decoder tests and a short bench (decode leg timings).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-dec2}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decoder_stream.py tests/test_gpu_seek.py \
    tests/test_gpu_chain.py tests/test_gpu_ext.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 200 python -u bench.py --steps 10 --no-cpu-baseline --no-chain --no-host --no-t2t --no-rg4 > $OUT/bench.log 2>&1
