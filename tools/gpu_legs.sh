# headline + decode legs (no CPU baseline, no verify, no host/chain/t2t/rg4/
# narrow), one run per library variant: tools/gpu_legs.sh [variant ...]
# (expgpu/libatgpu_<v>.so; "base" = the product library)
set -e
mkdir -p gpurun_out/legs
B="python -u bench.py --no-cpu-baseline --no-verify --no-chain --no-t2t --no-rg4 --narrow= --no-host"
for v in "$@"; do
  if [ "$v" = base ]; then L=$PWD/python-audio-tools_amd/audiotools/libatgpu.so; else L=$PWD/expgpu/libatgpu_$v.so; fi
  ATGPU_LIB=$L timeout -k 10 300 $B > gpurun_out/legs/$v.log 2>&1
  python3 -c "import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{\"metric\"'): d=json.loads(l); dd=d['decode']; print(sys.argv[1], d['value'], d['ms_per_step'], dd['ms_per_step'])" gpurun_out/legs/$v.log
done
