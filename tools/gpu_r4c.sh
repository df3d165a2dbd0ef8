#!/bin/bash
# GPU-box recipe (round 4): process-per-track cold start probe, then the GPU suite.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4c}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 120 python -u tools/t2t_cold.py 1 8 > $OUT/cold_j1.json 2> $OUT/cold_j1.err
timeout -k 10 180 python -u tools/t2t_cold.py 8 48 > $OUT/cold_j8.json 2> $OUT/cold_j8.err
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
