#!/bin/bash
# A/B of two libatgpu builds on the decode leg (ATGPU_LIB selects the build)
set -e -o pipefail
OUT=gpurun_out/${1:-r5k}
mkdir -p $OUT
for rep in 1 2; do
for d in ${DEPTHS:-6 8}; do
  timeout -k 10 300 python -u bench.py --steps 30 --no-host --no-t2t --no-rg4 --no-chain --no-cpu-baseline --no-verify --narrow "" --dec-inflight $d > $OUT/A_d${d}_$rep.log 2>&1
  ATGPU_LIB=$PWD/expgpu/libatgpu.so timeout -k 10 300 python -u bench.py --steps 30 --no-host --no-t2t --no-rg4 --no-chain --no-cpu-baseline --no-verify --narrow "" --dec-inflight $d > $OUT/B_d${d}_$rep.log 2>&1
done
done
