#!/bin/bash
# K1-on-the-slot-stream A/B (encoder leg): product vs k1aux (K1 of the next
# batches as soon as enqueued) vs k1aux2 (K1 after the previous batch's
# search, beside its pack), then the encoder parity tests on k1aux2.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4p2
mkdir -p "$OUT"
cd "$R"
ARGS="--no-cpu-baseline --no-decode --no-chain --no-host --no-t2t --no-rg4 --steps 30 --warmup 3"
for k in 1 2; do
    timeout -k 10 200 python -u bench.py $ARGS > $OUT/prod_$k.log 2>&1
    ATGPU_LIB=$R/expgpu/libatgpu_k1aux.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/k1aux_$k.log 2>&1
    ATGPU_LIB=$R/expgpu/libatgpu_k1aux2.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/k1aux2_$k.log 2>&1
done
ATGPU_LIB=$R/expgpu/libatgpu_k1aux2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_config1.py \
    tests/test_gpu_host_pipeline.py tests/test_gpu_md5_host.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_k1aux2.log 2>&1
