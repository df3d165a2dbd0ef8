# the BPS converter leg alone (bench decode-family legs; convert_leg runs
# with them), one run per library variant: tools/gpu_convert.sh [variant ...]
set -e
mkdir -p gpurun_out/conv
B="python -u bench.py --no-cpu-baseline --no-verify --no-chain --no-t2t --no-rg4 --narrow= --no-host --steps 30"
for v in "$@"; do
  if [ "$v" = base ]; then L=$PWD/python-audio-tools_amd/audiotools/libatgpu.so; else L=$PWD/expgpu/libatgpu_$v.so; fi
  ATGPU_LIB=$L timeout -k 10 300 $B > gpurun_out/conv/$v.log 2>&1
  python3 -c "import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{\"metric\"'): d=json.loads(l); c=d['convert']; print(sys.argv[1], c['ms_per_step'], c['roofline']['achieved'], c['verified_dither_invariant'])" gpurun_out/conv/$v.log
done
