# headline step time against the number of timed steps (the pipeline's
# drain -- the last batches' MD5 chains -- is inside the clock)
set -e
mkdir -p gpurun_out/steps
for k in ${STEPS:-15 30 60 120}; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-verify --no-chain --no-t2t --no-rg4 \
    --narrow= --no-host --no-decode --steps $k > gpurun_out/steps/k$k.log 2>&1
  python3 -c "import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{\"metric\"'): d=json.loads(l); print(sys.argv[1], d['steps'], d['value'], d['ms_per_step'])" gpurun_out/steps/k$k.log
done
