#!/bin/bash
# GPU-box recipe: config-5 chain step against the FLAC batches in flight
# (and ALAC decoders per thread): tools/gpu_chain_depth.sh <tag> "<depths>" "<decoders>"
set -e -o pipefail
OUT=gpurun_out/${1:-chaindepth}
mkdir -p $OUT
for d in ${2:-3 4 5 6}; do
  for n in ${3:-3}; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-verify \
        --no-host --no-t2t --no-rg4 --narrow= --no-decode --chain-inflight $d \
        --chain-decoders $n > $OUT/chain_d${d}_n$n.log 2>&1
  done
done
