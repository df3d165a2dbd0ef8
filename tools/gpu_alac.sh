#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_alac.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_alac.log 2>&1
echo "rc=$?" >> gpurun_out/pytest_alac.log
