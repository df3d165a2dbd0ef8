#!/bin/bash
# GPU-box recipe: resampler A/B -- the product library and exp/libatgpu_<name>.so
# (parity tests + the bench's resample/chain legs under each)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-rsab}"
name=${2:-rspxd}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 env ATGPU_LIB=$R/exp/libatgpu_$name.so python -u -m pytest tests/test_gpu_resample.py tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_$name.log 2>&1
for lib in "" "$R/exp/libatgpu_$name.so" "" "$R/exp/libatgpu_$name.so"; do
  tag=${lib:+$name}; tag=${tag:-prod}
  timeout -k 10 300 env ${lib:+ATGPU_LIB=$lib} python -u bench.py --steps 10 --no-cpu-baseline --no-host --no-t2t --no-rg4 >> $OUT/bench_$tag.log 2>&1
done
