#!/bin/bash
# GPU-box recipe for encoder-search work: FLAC encoder parity tests, smoke,
# an encoder-only bench line (all tracks verified against the port), and a
# rocprofv3 kernel-stats pass of the same bench.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_flac_big.py \
    tests/test_gpu_config1.py tests/test_gpu_flacaudio.py -x -v --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_k2.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-decode --no-chain --no-host \
    > gpurun_out/bench_k2.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_k2" -o run --output-format csv \
    -- python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --no-decode --no-chain --no-host \
    > "$R/gpurun_out/prof_k2.log" 2>&1
