#!/bin/bash
# Pack-stream A/B (encoder leg): product (decide/scan/pack on the main
# stream) vs packaux (on the slot stream behind MD5 part 0) vs packstr (one
# engine-wide pack stream), then the encoder parity tests on each variant.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4u
mkdir -p "$OUT"
cd "$R"
ARGS="--no-cpu-baseline --no-decode --no-chain --no-host --no-t2t --no-rg4 --steps 30 --warmup 3"
for k in 1 2; do
    timeout -k 10 200 python -u bench.py $ARGS > $OUT/prod_$k.log 2>&1
    ATGPU_LIB=$R/expgpu/libatgpu_packaux.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/packaux_$k.log 2>&1
    ATGPU_LIB=$R/expgpu/libatgpu_packstr.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/packstr_$k.log 2>&1
done
for v in packaux packstr; do
ATGPU_LIB=$R/expgpu/libatgpu_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_config1.py \
    tests/test_gpu_host_pipeline.py tests/test_gpu_md5_host.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_$v.log 2>&1
done
