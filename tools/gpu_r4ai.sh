#!/bin/bash
# Round-4 product run final tree (biased K2 seed, K5 VOP3 seeds): GPU suite,
# smoke, default bench, kernel stats, then the PMC passes (tools/gpu_pmc.sh)
# that profiles/pmc_traffic.json and pmc_valu.json are refreshed from.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
N=${1:-r4ai}
OUT=$R/gpurun_out/$N
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 $R/bench.py --no-cpu-baseline > "$OUT/prof.log" 2>&1
cd "$R"
bash tools/gpu_pmc.sh pmc_$N
