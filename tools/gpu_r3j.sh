#!/bin/bash
# GPU-box recipe: encoder / decoder GPU tests (side channel shift 15 on the
# fold, emit write rewrite), the bench without CPU baselines, and K2's PMC +
# kernel trace with the product library.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3j}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_decode.py tests/test_gpu_decoder_stream.py \
    tests/test_gpu_chain.py tests/test_gpu_host_pipeline.py tests/test_gpu_seek.py -x -v --timeout 200 --timeout-method thread \
    > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-chain --no-t2t --no-rg4 > $OUT/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-host --no-chain --no-decode --no-t2t --no-rg4"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
    SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
    -d "$OUT/k2/pmc" -o run --output-format csv -- python3 $ARGS > "$OUT/k2.pmc.log" 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d "$OUT/k2/kt" -o run --output-format csv -- python3 $ARGS \
    > "$OUT/k2.kt.log" 2>&1
