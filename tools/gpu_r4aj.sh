#!/bin/bash
# K3-K5 of pipelined device batches on an engine-wide pack stream
# (ATG_PACK_STREAM, product) vs on the main stream (expgpu/libatgpu_nopack.so):
# the GPU suite on the product, then the encoder leg product/nopack x2.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4aj}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
ARGS="--no-cpu-baseline --no-decode --no-chain --no-host --no-t2t --no-rg4 --steps 30 --warmup 3"
for k in 1 2; do
    timeout -k 10 200 python -u bench.py $ARGS > $OUT/prod_$k.log 2>&1
    ATGPU_LIB=$R/expgpu/libatgpu_nopack.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/nopack_$k.log 2>&1
done
