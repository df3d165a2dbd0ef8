#!/bin/bash
# GPU-box recipe (round 4): decoder slots A/B -- the product (3 slots) and
# exp builds with 4, 5, 6 slots, each probed with that many batches in flight.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4m}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 200 python -u tools/dec_probe.py --tag s3 --inflight 3 > $OUT/dec_probe.log 2>&1
for n in 4 5 6; do
  ATGPU_LIB=$R/expgpu/libatgpu_ds$n.so timeout -k 10 200 python -u tools/dec_probe.py --tag s$n --inflight $n >> $OUT/dec_probe.log 2>&1
done
