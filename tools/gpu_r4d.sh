#!/bin/bash
# GPU-box recipe (round 4): track2track true-shape probe (fork per file, as
# ExecProgressQueue) with the encoder service vs an engine per process, then
# the GPU suite.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4d}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 120 python -u tools/t2t_cold.py 8 48 --fork --own-engine > $OUT/cold_fork_own_j8.json 2> $OUT/cold_fork_own_j8.err
timeout -k 10 120 python -u tools/t2t_cold.py 8 48 --fork > $OUT/cold_fork_svc_j8.json 2> $OUT/cold_fork_svc_j8.err
timeout -k 10 120 python -u tools/t2t_cold.py 8 128 --fork > $OUT/cold_fork_svc_j8_128.json 2> $OUT/cold_fork_svc_j8_128.err
timeout -k 10 120 python -u tools/t2t_cold.py 1 8 --fork > $OUT/cold_fork_svc_j1.json 2> $OUT/cold_fork_svc_j1.err
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
