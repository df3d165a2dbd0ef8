#!/bin/bash
# GPU-box recipe: config-5 chain with 1, 2 and 3 ALAC decode threads (the
# headline leg runs 10 steps first; other legs off), chain suite first.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-chainthr}"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_chain.py > "$OUT/pytest.log" 2>&1
for t in ${2:-2 1 2 3}; do
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host \
        --no-t2t --no-rg4 --narrow= --no-decode --chain-decode-threads $t >> "$OUT/chain.log" 2>&1
done
