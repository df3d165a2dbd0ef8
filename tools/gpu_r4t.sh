#!/bin/bash
# K2 post-processing A/B (encoder leg): k2ashr (n = acc >> shv, then the
# sign fold) vs the product (sign fold, then a logical shift), then the
# encoder parity tests (incl. the back-to-back frames uploads) on the product.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4t
mkdir -p "$OUT"
cd "$R"
ARGS="--no-cpu-baseline --no-decode --no-chain --no-host --no-t2t --no-rg4 --steps 30 --warmup 3"
timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_config1.py \
    tests/test_gpu_host_pipeline.py tests/test_gpu_md5_host.py tests/test_gpu_flac_big.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
for k in 1 2; do
    ATGPU_LIB=$R/expgpu/libatgpu_k2ashr.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/k2ashr_$k.log 2>&1
    timeout -k 10 200 python -u bench.py $ARGS > $OUT/prod_$k.log 2>&1
done
