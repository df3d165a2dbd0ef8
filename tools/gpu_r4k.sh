#!/bin/bash
# GPU-box recipe (round 4): decoder tests, probe, isolated kernel stats and
# one SQ PMC pass over the decoder kernels (synchronous batches).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4k}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decoder_stream.py \
    tests/test_gpu_seek.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 200 python -u tools/dec_probe.py --tag a > $OUT/dec_probe.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 $R/tools/dec_probe.py --tag prof --steps 0 > "$OUT/prof.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
    -d "$OUT/pmc1" -o run --output-format csv -- python3 $R/tools/dec_probe.py --tag pmc --steps 0 > "$OUT/pmc1.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_LDS_BANK_CONFLICT \
    -d "$OUT/pmc2" -o run --output-format csv -- python3 $R/tools/dec_probe.py --tag pmc --steps 0 > "$OUT/pmc2.log" 2>&1
