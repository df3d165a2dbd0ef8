#!/bin/bash
# Round-3 GPU recipe: streaming encoder, C extensions, host pipeline; bench
# host legs; rocprofv3 timeline of the pinned host pipeline.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3b}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_ext.py tests/test_gpu_flac.py tests/test_gpu_host_pipeline.py \
    tests/test_gpu_async.py tests/test_gpu_config1.py tests/test_gpu_flacaudio.py -x -v --timeout 200 \
    --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-decode --no-chain --no-cpu-baseline \
    > $OUT/bench.log 2>&1
timeout -k 10 120 python -u tools/host_timeline.py 3 pageable > $OUT/pageable.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof" -o run \
    --output-format csv -- python3 "$R/tools/host_timeline.py" 3 pinned > "$OUT/prof.log" 2>&1
