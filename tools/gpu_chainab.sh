#!/bin/bash
# GPU-box recipe: the config-5 chain leg with the product library and the
# experiment builds named on the command line
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/chainab"
mkdir -p "$OUT"
cd "$R"
A="--steps 4 --no-cpu-baseline --no-verify --no-decode --no-host --no-t2t --no-rg4"
timeout -k 10 300 python -u bench.py $A > $OUT/base.log 2>&1
for n in "$@"; do
    ATGPU_LIB=$R/exp/libatgpu_$n.so timeout -k 10 300 python -u bench.py $A > $OUT/$n.log 2>&1 || true
done
