#!/bin/bash
# Round-4 checkpoint after the ALAC reader commits, plus the K2 biased
# post-processing A/B (expgpu/libatgpu_bias.so, -DATG_K2F_BIAS=1):
# product GPU suite + smoke + default bench + kernel stats, then the FLAC
# parity tests on the bias build and the encoder leg product/bias/product/bias.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r4af}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1
ATGPU_LIB=$R/expgpu/libatgpu_bias.so timeout -k 10 400 python -u -m pytest tests/test_gpu_flac.py \
    tests/test_gpu_flac_big.py tests/test_gpu_chain.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest_bias.log 2>&1
ARGS="--no-cpu-baseline --no-decode --no-chain --no-host --no-t2t --no-rg4 --steps 30 --warmup 3"
for k in 1 2; do
    timeout -k 10 200 python -u bench.py $ARGS > $OUT/prod_$k.log 2>&1
    ATGPU_LIB=$R/expgpu/libatgpu_bias.so timeout -k 10 200 python -u bench.py $ARGS > $OUT/bias_$k.log 2>&1
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv \
    -- python3 $R/bench.py --no-cpu-baseline > "$OUT/prof.log" 2>&1
