#!/bin/bash
# K2 register budget: product (4 waves per SIMD, 128 VGPRs, 8-9 scratch
# spills per job) vs expgpu/libatgpu_w3.so (3 waves per SIMD, 147 VGPRs, no
# spills): FLAC parity tests on the w3 build, then the encoder leg x2 each.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4ao}
mkdir -p "$OUT"
cd "$R"
ATGPU_LIB=$R/expgpu/libatgpu_w3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py \
    tests/test_gpu_flac_big.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_w3.log 2>&1
ARGS="--no-cpu-baseline --no-decode --no-chain --no-host --no-t2t --no-rg4 --steps 30 --warmup 3"
for k in 1 2; do
    timeout -k 10 200 python -u bench.py $ARGS > $OUT/prod_$k.log 2>&1
    ATGPU_LIB=$R/expgpu/libatgpu_w3.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/w3_$k.log 2>&1
done
