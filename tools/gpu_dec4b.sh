#!/bin/bash
# GPU-box recipe (round 4): decoder tests, the decode leg at 3 slots
# (product) and with the 4- and 5-slot experiment libraries (expgpu/).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-dec4b}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decoder_stream.py \
    tests/test_gpu_seek.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest_dec.log 2>&1
LEGS="--no-chain --no-host --no-t2t --no-rg4 --no-cpu-baseline --steps 20"
timeout -k 10 300 python -u bench.py $LEGS > $OUT/bench3.log 2>&1
ATGPU_LIB=$R/expgpu/libatgpu_s4.so timeout -k 10 300 python -u bench.py $LEGS --dec-inflight 4 > $OUT/bench4.log 2>&1
ATGPU_LIB=$R/expgpu/libatgpu_s5.so timeout -k 10 300 python -u bench.py $LEGS --dec-inflight 5 > $OUT/bench5.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 $R/bench.py $LEGS --steps 10 > "$OUT/prof.log" 2>&1
cd "$R"
timeout -k 10 200 python -u tools/md5_host_probe.py > $OUT/md5_host.log 2>&1
timeout -k 10 400 python -u bench.py --no-host --no-t2t --no-rg4 --no-decode --no-cpu-baseline --steps 10 > $OUT/bench_chain.log 2>&1
# K2 MFMA prototype (tools/k2_mfma_probe.hip): parity + timing, then one PMC pass
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -mllvm -amdgpu-mfma-vgpr-form tools/k2_mfma_probe.hip \
    -o $OUT/k2_mfma_probe > $OUT/mfma_build.log 2>&1
timeout -k 10 120 $OUT/k2_mfma_probe > $OUT/mfma_probe.log 2>&1
cd /tmp
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d "$OUT/prof_mfma" -o run --output-format csv \
    -- $OUT/k2_mfma_probe > "$OUT/prof_mfma.log" 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
    -d "$OUT/pmc_mfma" -o run --output-format csv -- $OUT/k2_mfma_probe > "$OUT/pmc_mfma.log" 2>&1
