#!/bin/bash
# Round-3 GPU-box recipe: the whole -m gpu suite, then the default bench
# (all legs, every track verified).  Each GPU step has its own time limit.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r3}
mkdir -p "$R/gpurun_out/$TAG"
cd "$R"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > gpurun_out/$TAG/pytest_gpu.log 2>&1
timeout -k 10 600 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/$TAG/bench.log 2>&1
