#!/bin/bash
# GPU-box recipe (round 4): decoder tests, decoder probe twice, then the
# probe under rocprofv3 kernel stats (synchronous batches: isolated kernels).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4j}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decoder_stream.py \
    tests/test_gpu_seek.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 200 python -u tools/dec_probe.py --tag a > $OUT/dec_probe.log 2>&1
timeout -k 10 200 python -u tools/dec_probe.py --tag b >> $OUT/dec_probe.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 $R/tools/dec_probe.py --tag prof --steps 0 > "$OUT/prof.log" 2>&1
