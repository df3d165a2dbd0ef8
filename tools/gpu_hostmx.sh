#!/bin/bash
# GPU-box recipe: host-to-host pipeline matrix (chunk size x jobs in flight x
# aux stream priority x HW queue count), wall time per batch, no profiler.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-hostmx}"
mkdir -p "$OUT"
cd "$R"
P="$R/python-audio-tools_amd/audiotools/libatgpu.so"
H="$R/exp/libatgpu_hiprio.so"
for cfg in "$P 256 2 4" "$P 1024 2 4" "$P 1024 3 4" "$P 512 3 4" "$H 256 2 4" "$H 1024 3 4" "$P 256 3 8" "$P 1024 3 8" "$H 256 3 8"; do
    set -- $cfg
    ATGPU_LIB=$1 GPU_MAX_HW_QUEUES=$4 timeout -k 10 150 python3 -u tools/host_timeline.py 3 pinned $2 $3 \
        > "$OUT/$(basename $1 .so)_c$2_i$3_q$4.log" 2>&1
done
