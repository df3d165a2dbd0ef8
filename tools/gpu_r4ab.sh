#!/bin/bash
# decoder CRC chunking check: decoder parity tests, then the decoder probe
# (synchronous kernel times and the pipelined step)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4ab
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_seek.py tests/test_gpu_decoder_stream.py \
    -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 200 python -u tools/dec_probe.py --steps 20 > $OUT/dec_probe.log 2>&1
