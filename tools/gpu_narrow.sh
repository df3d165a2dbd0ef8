#!/bin/bash
# round 5: narrow-batch leg (strong-scaling rank shapes on one GPU) at several
# in-flight depths, with the async/service parity tests first
set -e -o pipefail
OUT=gpurun_out/${1:-r5b}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_async.py tests/test_gpu_service.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 400 python -u bench.py --steps 30 --no-host --no-decode --no-t2t --no-rg4 --no-chain --no-cpu-baseline --no-verify --narrow ${NARROW:-1024,512,256,128} --narrow-depths ${DEPTHS:-3,4,6,8} > $OUT/bench.log 2>&1
