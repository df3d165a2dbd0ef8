#!/bin/bash
# GPU-box recipe: encoder tests and a 30-step encoder bench (+ PMC of K5)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-enc2}"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_flac_big.py tests/test_gpu_host_pipeline.py tests/test_gpu_async.py \
    -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-decode --no-chain --no-host --no-t2t --no-rg4 > $OUT/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
    SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d "$OUT/pmc" -o run --output-format csv \
    -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-host --no-chain --no-decode --no-t2t --no-rg4 \
    > "$OUT/pmc.log" 2>&1
