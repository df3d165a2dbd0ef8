#!/bin/bash
# ALAC decoder lanes per wave: ALAC + chain parity tests on the product
# (parse 16 / chain 1 / channel 32 lanes a wave), then the chain leg for the
# product, adec64 (64/64/64, the previous launch) and adecb (8/1/16)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4ae}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_alac.py tests/test_gpu_chain.py \
    -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
A="--no-cpu-baseline --no-decode --no-host --no-t2t --no-rg4 --steps 3 --warmup 1 --no-verify"
timeout -k 10 300 python -u bench.py $A > $OUT/prod.log 2>&1
for v in; do
    ATGPU_LIB=$R/expgpu/libatgpu_$v.so timeout -k 10 300 python -u bench.py $A > $OUT/$v.log 2>&1
done
