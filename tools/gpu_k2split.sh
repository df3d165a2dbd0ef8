#!/bin/bash
# GPU-box recipe: K2 instruction split.  For the product library and every
# exp/libatgpu_k2e*.so (tools/build_exp.sh, ATG_K2F_EXP=1..6) one encoder-only
# bench step under a PMC pass (issue counters, LDS bank conflicts) and one
# under --kernel-trace --stats (time).  tools/k2split.py tabulates.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-k2split}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-host --no-chain --no-decode --no-t2t --no-rg4"
run() {
    local name=$1 lib=$2
    ATGPU_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
        SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        -d "$OUT/$name/pmc" -o run --output-format csv -- python3 $ARGS > "$OUT/$name.pmc.log" 2>&1
    ATGPU_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --stats \
        -d "$OUT/$name/kt" -o run --output-format csv -- python3 $ARGS > "$OUT/$name.kt.log" 2>&1
}
run base "$R/python-audio-tools_amd/audiotools/libatgpu.so"
for lib in "$R"/exp/libatgpu_k2e*.so; do
    n=$(basename "$lib" .so)
    # experiment builds may fail the engine's consistency checks after K2
    # has run (EXP 2/3 leave bit counts wrong); their K2 counters still count
    run "${n#libatgpu_}" "$lib" || true
done
cd "$R"
timeout -k 10 120 python -u tools/queue_probe.py > "$OUT/queue_probe.log" 2>&1
