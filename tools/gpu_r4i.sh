#!/bin/bash
# GPU-box recipe (round 4): decoder + host-MD5 tests, decoder probe, the
# chain leg (host MD5 for config 5).
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4i}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decoder_stream.py \
    tests/test_gpu_seek.py tests/test_gpu_md5_host.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 200 python -u tools/dec_probe.py --tag ring2 > $OUT/dec_probe.log 2>&1
timeout -k 10 400 python -u bench.py --no-host --no-t2t --no-rg4 --no-decode --no-cpu-baseline --steps 10 > $OUT/bench_chain.log 2>&1
