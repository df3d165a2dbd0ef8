#!/bin/bash
# round 5: decode leg at several in-flight depths (rolled decoder MD5), after
# the decoder parity tests
set -e -o pipefail
OUT=gpurun_out/${1:-r5j}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
for d in ${DEPTHS:-3 4 5 6 8}; do
  timeout -k 10 300 python -u bench.py --steps 30 --no-host --no-t2t --no-rg4 --no-chain --no-cpu-baseline --no-verify --narrow "" --dec-inflight $d > $OUT/bench_d$d.log 2>&1
done
