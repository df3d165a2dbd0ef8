#!/bin/bash
# GPU-box recipe: decoder timing experiments (exp/libatgpu_dec*.so: 3 no
# CRC-16 in the parser, 4 emit without writes, 5 emit without row loads)
# beside the product library, one short bench each (decode leg timings).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-decx}
mkdir -p "$OUT"
cd "$R"
ARGS="bench.py --steps 10 --no-cpu-baseline --no-verify --no-chain --no-host --no-t2t --no-rg4"
timeout -k 10 200 python -u $ARGS > $OUT/base.log 2>&1
for e in 3 4 5; do
    ATGPU_LIB=$R/exp/libatgpu_dec$e.so timeout -k 10 200 python -u $ARGS > $OUT/dec$e.log 2>&1 || true
done
