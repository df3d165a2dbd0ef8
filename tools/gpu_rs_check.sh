#!/bin/bash
# GPU-box recipe: resampler change check.  The resampler, chain and drop-in
# GPU suites, then two bench runs with the config-3 resample leg and the
# config-5 chain.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-rs}"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_resample.py tests/test_gpu_chain.py tests/test_gpu_dropin.py > "$OUT/pytest.log" 2>&1
for k in 1 2; do
    timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host \
        --no-t2t --no-rg4 --narrow= > "$OUT/chain$k.log" 2>&1
done
