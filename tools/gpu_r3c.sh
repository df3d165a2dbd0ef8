#!/bin/bash
# Round-3 GPU recipe: the 24-bit / multichannel encoder path (hi/lo search,
# packer, int32 MD5 wave pairs): parity tests, then the chain leg.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3c}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_chain.py tests/test_gpu_async.py \
    tests/test_gpu_flac_big.py tests/test_gpu_host_pipeline.py -x -v --timeout 200 --timeout-method thread \
    > $OUT/pytest.log 2>&1
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-decode --no-host --no-cpu-baseline \
    > $OUT/bench.log 2>&1
