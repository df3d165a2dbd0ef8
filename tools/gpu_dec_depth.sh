set -e
mkdir -p gpurun_out/decd
B="python -u bench.py --no-cpu-baseline --no-verify --no-chain --no-t2t --no-rg4 --narrow= --no-host"
for d in ${DEPTHS:-8 10 12 16 8 12}; do
  timeout -k 10 300 $B --dec-inflight $d > gpurun_out/decd/d$d.log 2>&1
  python3 -c "import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{\"metric\"'): d=json.loads(l); dd=d['decode']; print(sys.argv[1], dd['ms_per_step'], dd['kernel_ms']['dec_parse'], dd['kernel_ms']['dec_subframe'], dd['verified_tracks'])" gpurun_out/decd/d$d.log
done
