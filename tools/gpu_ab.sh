#!/bin/bash
# A/B of the product library against exp/libatgpu_<name>.so on the encoder
# leg, alternating runs (bench noise between runs is a few percent).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/ab"
cd "$R"
ARGS="--steps ${AB_STEPS:-30} --warmup 3 --no-cpu-baseline --no-verify --no-decode --no-chain --no-host"
for k in 1 2; do
    timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/ab/new_$k.log 2>&1
    for lib in exp/libatgpu_*.so; do
        n=$(basename $lib .so)
        ATGPU_LIB=$R/$lib timeout -k 10 200 python -u bench.py $ARGS > gpurun_out/ab/${n}_$k.log 2>&1
    done
done
