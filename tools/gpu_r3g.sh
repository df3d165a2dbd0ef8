#!/bin/bash
# GPU-box recipe: decoder emit rewrite (its tests + decode leg), the
# resampler / ReplayGain legs, and one PMC pass over them.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3g}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decoder_stream.py tests/test_gpu_seek.py \
    tests/test_gpu_ext.py tests/test_gpu_async.py tests/test_gpu_chain.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
ARGS="bench.py --steps 10 --no-cpu-baseline --no-chain --no-host --no-t2t --no-rg4"
timeout -k 10 300 python -u $ARGS > $OUT/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$OUT/pmc" -o run --output-format csv \
    -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-chain --no-host --no-t2t --no-rg4 \
    > "$OUT/pmc.log" 2>&1
