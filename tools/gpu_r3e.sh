#!/bin/bash
# Round-3 GPU recipe: fused decoder emit kernel, async host jobs: their GPU
# tests, the stream/queue probe, host-pipeline timelines (product library
# and the normal-priority aux stream build), then the default bench.
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r3e}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 600 python -u -m pytest tests/test_gpu_flac.py tests/test_gpu_resample.py tests/test_gpu_alac.py tests/test_gpu_replaygain.py tests/test_gpu_decoder_stream.py tests/test_gpu_decode.py tests/test_gpu_seek.py tests/test_gpu_host_pipeline.py \
    tests/test_gpu_ext.py tests/test_gpu_async.py tests/test_gpu_config1.py tests/test_gpu_flacaudio.py \
    -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
timeout -k 10 120 python -u tools/queue_probe.py > $OUT/queue_probe.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d "$OUT/prof" -o run \
    --output-format csv -- python3 "$R/tools/host_timeline.py" 3 pinned > "$OUT/prof.log" 2>&1
ATGPU_LIB=$R/exp/libatgpu_loprio.so timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats \
    -d "$OUT/prof_loprio" -o run --output-format csv -- python3 "$R/tools/host_timeline.py" 3 pinned \
    > "$OUT/prof_loprio.log" 2>&1
cd "$R"
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1
