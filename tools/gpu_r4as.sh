#!/bin/bash
# K2 even orders on aligned words only (ATG_K2F_EW, product) vs v_alignbit words
# (expgpu/libatgpu_ew0.so): encoder parity tests on the product,
# then the encoder leg product/old/product/old.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4as}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_config1.py tests/test_gpu_async.py \
    tests/test_gpu_host_pipeline.py tests/test_gpu_flac_big.py tests/test_gpu_chain.py tests/test_gpu_ext.py \
    -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
ARGS="--no-cpu-baseline --no-decode --no-chain --no-host --no-t2t --no-rg4 --steps 30 --warmup 3"
for k in 1 2; do
    timeout -k 10 200 python -u bench.py $ARGS > $OUT/prod_$k.log 2>&1
    ATGPU_LIB=$R/expgpu/libatgpu_ew0.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/old_$k.log 2>&1
done
