#!/bin/bash
# GPU-box recipe: A/B of the encoder on config-5-shaped batches
# (tools/pack_probe.py: synchronous kernel times, image digest) between the
# product library and abl/libatgpu_old.so, then the wide-sample parity
# suites.  Build the baseline in this container before the call, e.g. from
# the previous commit's objects:
#   hipcc --offload-arch=gfx950 -shared -fPIC -o abl/libatgpu_old.so \
#       python-audio-tools_amd/csrc/obj/*.o   (before rebuilding the product)
set -e -o pipefail
OUT=gpurun_out/${1:-packab}
mkdir -p $OUT
for cfg in "--channels 6 --bits 24" "--channels 2 --bits 24" "--channels 8 --bits 16"; do
  timeout -k 10 240 python -u tools/pack_probe.py $cfg >> $OUT/probe.jsonl 2>>$OUT/err.log
  ATGPU_LIB=abl/libatgpu_old.so timeout -k 10 240 python -u tools/pack_probe.py $cfg >> $OUT/probe.jsonl 2>>$OUT/err.log
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_hl_range.py tests/test_gpu_flac.py tests/test_gpu_flac_big.py > $OUT/pytest.log 2>&1
