#!/bin/bash
# GPU-box recipe: the config-5 chain leg over ALAC decoder counts and FLAC
# batches in flight (host MD5), two runs each.
# tools/gpu_chain_dec.sh <tag> ["dec depth" ...]
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-chaindec}"
shift || true
CFGS=("$@")
[ ${#CFGS[@]} -eq 0 ] && CFGS=("2 4" "3 4" "3 6")
mkdir -p "$OUT"
cd "$R"
for k in 1 2; do
  for cfg in "${CFGS[@]}"; do
    set -- $cfg
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-verify \
        --no-host --no-t2t --no-rg4 --narrow= --no-decode --chain-decoders $1 \
        --chain-inflight $2 > "$OUT/chain_d$1_f$2_$k.log" 2>&1
  done
done
