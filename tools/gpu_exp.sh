#!/bin/bash
# GPU-box recipe: time experiment builds (exp/libatgpu_e*.so, not byte-exact)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/exp"
cd "$R"
for lib in exp/libatgpu_e*.so; do
    n=$(basename $lib .so)
    ATGPU_LIB=$R/$lib timeout -k 10 120 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-verify \
        > gpurun_out/exp/$n.log 2>&1
done
