#!/bin/bash
# GPU-box recipe: encoder-only bench (30 steps) with the product library and
# the experiment builds named on the command line (exp/libatgpu_<name>.so)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/encab"
mkdir -p "$OUT"
cd "$R"
A="--no-cpu-baseline --no-verify --no-decode --no-chain --no-host --no-t2t --no-rg4"
timeout -k 10 200 python -u bench.py $A > $OUT/base.log 2>&1
for n in "$@"; do
    ATGPU_LIB=$R/exp/libatgpu_$n.so timeout -k 10 200 python -u bench.py $A > $OUT/$n.log 2>&1 || true
done
