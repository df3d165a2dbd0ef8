set -e
mkdir -p gpurun_out/legs
B="python -u bench.py --no-cpu-baseline --no-verify --no-chain --no-t2t --no-rg4 --narrow="
for r in a b; do
timeout -k 10 300 $B > gpurun_out/legs/$r.log 2>&1 && python3 -c "import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{\"metric\"'): d=json.loads(l); print(sys.argv[1], d['value'], d['decode']['ms_per_step'], d['host_to_host']['value'], d['host_to_host']['sync_per_batch']['value'], d['resample']['ms_per_step'], d['replaygain']['ms_per_step'])" gpurun_out/legs/$r.log
done
