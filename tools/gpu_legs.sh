# bench legs (no CPU baseline, no verify, no chain/t2t/rg4/narrow), one run per
# library variant: tools/gpu_legs.sh [variant ...] (expgpu/libatgpu_<v>.so;
# "base" = the product library)
set -e
mkdir -p gpurun_out/legs
B="python -u bench.py --no-cpu-baseline --no-verify --no-chain --no-t2t --no-rg4 --narrow="
for v in "$@"; do
  if [ "$v" = base ]; then L=; else L=$PWD/expgpu/libatgpu_$v.so; fi
  ATGPU_LIB=${L:-$PWD/python-audio-tools_amd/audiotools/libatgpu.so} timeout -k 10 300 $B > gpurun_out/legs/$v.log 2>&1
  python3 -c "import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{\"metric\"'): d=json.loads(l); dd=d['decode']; print(sys.argv[1], d['value'], dd['ms_per_step'], dd['kernel_ms'], d['host_to_host']['value'])" gpurun_out/legs/$v.log
done
