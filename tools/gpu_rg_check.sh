#!/bin/bash
# ReplayGain: parity tests, then the bench with the RG legs (config 2 title, config 4 album)
set -e -o pipefail
OUT=gpurun_out/${1:-r5m}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_replaygain.py tests/test_gpu_dropin.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 20 --no-host --no-t2t --no-chain --no-cpu-baseline --no-verify --narrow "" > $OUT/bench.log 2>&1
