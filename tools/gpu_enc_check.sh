#!/bin/bash
# GPU-box recipe: encoder change check.  The FLAC encoder GPU suites, then
# two encoder-only bench runs (30 steps), then (RQ=1) the host-leg copy
# timeline (tools/gpu_host_copytrace.sh).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-r5r}"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_flac.py tests/test_gpu_flac_big.py tests/test_gpu_async.py tests/test_gpu_ext.py \
    tests/test_gpu_config1.py tests/test_gpu_host_pipeline.py > "$OUT/pytest.log" 2>&1
for k in 1 2; do
    timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-host \
        --no-chain --no-decode --no-t2t --no-rg4 --narrow= > "$OUT/bench$k.log" 2>&1
done
if [ "${RQ:-0}" = 1 ]; then
    bash tools/gpu_host_copytrace.sh "${1:-r5r}_q"
fi
