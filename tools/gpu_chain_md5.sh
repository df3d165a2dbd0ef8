#!/bin/bash
# GPU-box recipe: the config-5 chain leg with the FLAC MD5 on host threads
# (the engine's automatic choice for its 8.6 MB tracks) against rolled GPU
# chains, two runs each, alternating.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-chainmd5}"
mkdir -p "$OUT"
cd "$R"
for k in 1 2; do
  for m in auto gpu; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-verify \
        --no-host --no-t2t --no-rg4 --narrow= --no-decode --chain-md5 $m > "$OUT/chain_${m}_$k.log" 2>&1
  done
done
