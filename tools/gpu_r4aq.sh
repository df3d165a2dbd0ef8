#!/bin/bash
# K1 register budget beside K2: product (183 VGPRs, 2 waves per SIMD) vs
# ATG_K1_WPE=3 (168 VGPRs, 26 spills) and =4 (128 VGPRs, 44 spills):
# FLAC parity on both builds, then the encoder leg, two rounds.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4aq}
mkdir -p "$OUT"
cd "$R"
for v in k1w3 k1w4; do
    ATGPU_LIB=$R/expgpu/libatgpu_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_flac.py \
        -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$v.log 2>&1
done
ARGS="--no-cpu-baseline --no-decode --no-chain --no-host --no-t2t --no-rg4 --steps 30 --warmup 3"
for k in 1 2; do
    timeout -k 10 200 python -u bench.py $ARGS > $OUT/prod_$k.log 2>&1
    for v in k1w3 k1w4; do
        ATGPU_LIB=$R/expgpu/libatgpu_$v.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/${v}_$k.log 2>&1
    done
done
