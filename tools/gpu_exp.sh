#!/bin/bash
# GPU-box recipe: time experiment builds (exp/libatgpu_e*.so, not byte-exact)
# next to the product library; encoder leg only.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/exp"
cd "$R"
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --no-verify --no-decode --no-chain --no-host"
timeout -k 10 120 python -u bench.py $ARGS > gpurun_out/exp/base.log 2>&1
for lib in exp/libatgpu_*.so; do
    n=$(basename $lib .so)
    ATGPU_LIB=$R/$lib timeout -k 10 120 python -u bench.py $ARGS > gpurun_out/exp/$n.log 2>&1 || echo "$n failed" >> gpurun_out/exp/failed.txt
done
