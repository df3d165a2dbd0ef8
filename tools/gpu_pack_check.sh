#!/bin/bash
# GPU-box recipe: frame pack change check.  The FLAC encoder suites (every
# channel count and width, byte-identical to the port), the chain suite,
# then two bench runs with the config-5 chain (its FLAC-8 is 6-channel
# 24-bit, the multi-wave pack's case) and the headline.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-pack}"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_flac.py tests/test_gpu_flac_big.py tests/test_gpu_k2_packed.py \
    tests/test_gpu_chain.py > "$OUT/pytest.log" 2>&1
for k in 1 2; do
    timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host \
        --no-t2t --no-rg4 --narrow= > "$OUT/chain$k.log" 2>&1
done
