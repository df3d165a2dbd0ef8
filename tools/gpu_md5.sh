#!/bin/bash
# GPU-box recipe for MD5 work: the single-chain microbench, the encoder and
# decoder parity tests (STREAMINFO MD5 set / verified), smoke, and an
# encoder-only bench line.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 120 tools/bin/md5_rate 1024 16384 > gpurun_out/md5_rate.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_decode.py \
    tests/test_gpu_config1.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_md5.log 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 --no-decode --no-chain --no-host \
    > gpurun_out/bench_md5.log 2>&1
