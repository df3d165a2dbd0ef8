#!/bin/bash
# kernel trace of the narrow-batch leg alone (rolled MD5 at one depth)
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r5e}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 1 --no-host --no-decode --no-t2t --no-rg4 --no-chain --no-cpu-baseline --no-verify --narrow ${NARROW:-128} --narrow-depths ${DEPTHS:-8} > $OUT/bench.log 2>&1
