#!/bin/bash
# K5 split, continued (timing only): product vs ATG_EXP 10 (no residual
# arithmetic in the REG path) vs 11 (one PCM load per subframe run)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4z
mkdir -p "$OUT"
cd "$R"
ARGS="--no-cpu-baseline --no-decode --no-chain --no-host --no-t2t --no-rg4 --steps 20 --warmup 3 --no-verify"
timeout -k 10 200 python -u bench.py $ARGS > $OUT/prod.log 2>&1
for e in 10; do
    ATGPU_LIB=$R/expgpu/libatgpu_k5e$e.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/k5e$e.log 2>&1
done
