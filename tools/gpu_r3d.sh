#!/bin/bash
# Round-3 GPU recipe: the whole -m gpu suite, the default bench (all legs),
# then a rocprofv3 kernel + memory-copy timeline of the pinned host pipeline.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3d}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest.log 2>&1
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1
timeout -k 10 120 python -u tools/host_timeline.py 3 pageable > $OUT/pageable.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof" -o run \
    --output-format csv -- python3 "$R/tools/host_timeline.py" 3 pinned > "$OUT/prof.log" 2>&1
