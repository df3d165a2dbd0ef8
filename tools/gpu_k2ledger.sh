#!/bin/bash
# GPU-box recipe: K2 instruction ledger (DESIGN 4a'').  For the product
# library and every expgpu/libatgpu_k2l_*.so (ledger builds: truncated after
# each phase, one tap pair per residual, fold-only; tools/build_exp.sh, then
# copied to expgpu/) one encoder-only bench step under a PMC pass and one
# under --kernel-trace --stats; then the event counts of the counting build.
# tools/k2split.py tabulates the PMC/time part.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT="$R/gpurun_out/${1:-k2ledger}"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS="$R/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-host --no-chain --no-decode --no-t2t --no-rg4 --narrow="
run() {
    local name=$1 lib=$2
    ATGPU_LIB=$lib timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS \
        SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
        -d "$OUT/$name/pmc" -o run --output-format csv -- python3 $ARGS > "$OUT/$name.pmc.log" 2>&1
    ATGPU_LIB=$lib timeout -s KILL 150 rocprofv3 --kernel-trace --stats \
        -d "$OUT/$name/kt" -o run --output-format csv -- python3 $ARGS > "$OUT/$name.kt.log" 2>&1
}
run base "$R/python-audio-tools_amd/audiotools/libatgpu.so"
for lib in "$R"/expgpu/libatgpu_k2l_*.so; do
    n=$(basename "$lib" .so)
    [ "$n" = libatgpu_k2l_cnt ] && continue
    run "${n#libatgpu_}" "$lib"
done
cd "$R"
ATGPU_LIB="$R/expgpu/libatgpu_k2l_cnt.so" timeout -k 10 150 python3 -u tools/k2_counts.py \
    > "$OUT/counts.json" 2> "$OUT/counts.log"
python3 tools/k2split.py "$OUT" > "$OUT/k2split.json"
