#!/bin/bash
# GPU-box recipe: decoder tests + a short bench (emit gather rewrite), then
# the K2 instruction split (tools/gpu_k2split.sh).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3i}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decoder_stream.py tests/test_gpu_seek.py \
    tests/test_gpu_chain.py tests/test_gpu_async.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 10 --no-cpu-baseline --no-chain --no-t2t --no-rg4 > $OUT/bench.log 2>&1
bash tools/gpu_k2split.sh k2split
