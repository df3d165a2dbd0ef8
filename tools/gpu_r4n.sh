#!/bin/bash
# GPU-box recipe (round 4): decoder tests, then the probe at 3 slots
# (product) and the 4/5-slot exp builds, then isolated kernel stats.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4n}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest tests/test_gpu_decode.py tests/test_gpu_decoder_stream.py \
    tests/test_gpu_seek.py -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 200 python -u tools/dec_probe.py --tag s3 --inflight 3 > $OUT/dec_probe.log 2>&1
for n in 4 5; do
  ATGPU_LIB=$R/expgpu/libatgpu_ds$n.so timeout -k 10 200 python -u tools/dec_probe.py --tag s$n --inflight $n >> $OUT/dec_probe.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 $R/tools/dec_probe.py --tag prof --steps 0 > "$OUT/prof.log" 2>&1
