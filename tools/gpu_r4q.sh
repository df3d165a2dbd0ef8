#!/bin/bash
# K1 load-issue A/B (encoder leg): k1old (compiler-placed PCM loads) vs the
# product (all of a group's loads issued together) vs k1wpf (+ window
# prefetch) vs k1auxlf (product + K1 on the slot stream), then the encoder
# parity tests on the product.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4q
mkdir -p "$OUT"
cd "$R"
ARGS="--no-cpu-baseline --no-decode --no-chain --no-host --no-t2t --no-rg4 --steps 30 --warmup 3"
for k in 1 2; do
    ATGPU_LIB=$R/expgpu/libatgpu_k1old.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/k1old_$k.log 2>&1
    timeout -k 10 200 python -u bench.py $ARGS > $OUT/prod_$k.log 2>&1
    ATGPU_LIB=$R/expgpu/libatgpu_k1wpf.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/k1wpf_$k.log 2>&1
    ATGPU_LIB=$R/expgpu/libatgpu_k1auxlf.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/k1auxlf_$k.log 2>&1
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_config1.py \
    tests/test_gpu_host_pipeline.py tests/test_gpu_md5_host.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
