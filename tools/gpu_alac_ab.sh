#!/bin/bash
# GPU-box recipe: ALAC A/B between the product library and abl/libatgpu_{A,B}.so
# (variants: a modified alac_decode.hip compiled here and linked with the
# product's other objects, python-audio-tools_amd/csrc/obj/*.o), suites
# then chain runs.
set -e -o pipefail
OUT=gpurun_out/r6bu
mkdir -p $OUT
ATGPU_LIB=abl/libatgpu_A.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_alac.py tests/test_gpu_chain.py > $OUT/pytest_A.log 2>&1
ATGPU_LIB=abl/libatgpu_B.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_alac.py tests/test_gpu_chain.py > $OUT/pytest_B.log 2>&1
for v in P A B P A B; do
  if [ $v = P ]; then unset ATGPU_LIB; else export ATGPU_LIB=abl/libatgpu_$v.so; fi
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-verify --no-host --no-t2t --no-rg4 --narrow= --no-decode > $OUT/chain_$v.log 2>&1
  grep '^{' $OUT/chain_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['chain']; k=c['kernel_ms']; print('$v', c['ms_per_step'], k['alac_adec_parse'], k['alac_adec_interleave'], k['alac_adec_total'])" >> $OUT/summary.txt
done
