# headline step against batches in flight (encoder legs only)
set -e
mkdir -p gpurun_out/infl
for r in a b; do for d in ${DEPTHS:-10 12 14 16}; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-verify --no-chain --no-t2t --no-rg4 \
    --narrow= --no-host --no-decode --inflight $d > gpurun_out/infl/d$d$r.log 2>&1
  python3 -c "import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{\"metric\"'): d=json.loads(l); print(sys.argv[1], d['value'], d['ms_per_step'])" gpurun_out/infl/d$d$r.log
done; done
