# ReplayGain title + config-4 legs per library variant (tools/gpu_rg_legs.sh v ...)
set -e
mkdir -p gpurun_out/rgl
for v in "$@"; do
  if [ "$v" = base ]; then L=$PWD/python-audio-tools_amd/audiotools/libatgpu.so; else L=$PWD/expgpu/libatgpu_$v.so; fi
  ATGPU_LIB=$L timeout -k 10 400 python -u bench.py --no-chain --no-t2t \
    --narrow= --no-host > gpurun_out/rgl/$v.log 2>&1
  python3 -c "import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{\"metric\"'):
        d=json.loads(l); r=d['replaygain']; r4=d['replaygain_config4']
        print(sys.argv[1], r['ms_per_step'], r['fallback_tracks_last_step'], r.get('verified_vs_oracle'), r.get('verified_tracks'), r4['ms_per_step'], r4['fallback_tracks_last_step'], r4['verified_tracks'], r4.get('verified_vs_oracle'))" gpurun_out/rgl/$v.log
done
