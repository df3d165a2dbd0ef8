# decode leg with the frame-end hypothesis off / on / self-check
set -e
mkdir -p gpurun_out/dspec
B="python -u bench.py --no-cpu-baseline --no-verify --no-chain --no-t2t --no-rg4 --narrow= --no-host"
for r in a b; do for m in 0 1 2; do
  timeout -k 10 300 $B --dec-hypothesis $m > gpurun_out/dspec/m$m$r.log 2>&1
  python3 -c "import json,sys
for l in open(sys.argv[1]):
    if l.startswith('{\"metric\"'): d=json.loads(l); dd=d['decode']; print(sys.argv[1], d['ms_per_step'], dd['ms_per_step'], dd['verified_tracks'], dd['frame_hypothesis']['batches_redone'], dd['kernel_ms'])" gpurun_out/dspec/m$m$r.log
done; done
