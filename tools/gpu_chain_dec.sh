#!/bin/bash
# GPU-box recipe: the config-5 chain leg with 2 / 3 ALAC decoders, 4 / 6
# FLAC batches in flight (host MD5), two runs each.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-chaindec}"
mkdir -p "$OUT"
cd "$R"
for k in 1 2; do
  for cfg in "2 4" "3 4" "3 6"; do
    set -- $cfg
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-verify \
        --no-host --no-t2t --no-rg4 --narrow= --no-decode --chain-decoders $1 \
        --chain-inflight $2 > "$OUT/chain_d$1_f$2_$k.log" 2>&1
  done
done
