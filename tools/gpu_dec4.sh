#!/bin/bash
# GPU-box recipe (round 4): decoder tests, then the encode + decode legs of
# the bench and their rocprof kernel stats.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-dec4}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decoder_stream.py \
    tests/test_gpu_seek.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_dec.log 2>&1
LEGS="--no-chain --no-host --no-t2t --no-rg4 --no-cpu-baseline"
timeout -k 10 300 python -u bench.py $LEGS > $OUT/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 $R/bench.py $LEGS --steps 10 > "$OUT/prof.log" 2>&1
