#!/bin/bash
# GPU-box recipe: headline encode A/B -- product library vs exp/libatgpu_<name>.so,
# alternating, device-resident legs only
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-encab2}"
name=${2:-eager}
mkdir -p "$OUT"
cd "$R"
for lib in "" "$R/exp/libatgpu_$name.so" "" "$R/exp/libatgpu_$name.so"; do
  tag=${lib:+$name}; tag=${tag:-prod}
  timeout -k 10 200 env ${lib:+ATGPU_LIB=$lib} python -u bench.py --steps 20 --no-cpu-baseline --no-host --no-t2t --no-rg4 --no-chain --no-decode >> $OUT/bench_$tag.log 2>&1
done
