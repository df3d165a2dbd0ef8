#!/bin/bash
# the round-end check on one GPU: GPU suite, smoke, default bench, kernel stats
# (rocprofv3 --kernel-trace --stats) of the same bench.  tools/gpu_full.sh <tag>
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-full}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1
if [ -z "$NO_PROF" ]; then
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 $R/bench.py --no-cpu-baseline > "$OUT/prof.log" 2>&1
fi
