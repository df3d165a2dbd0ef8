set -e -o pipefail
mkdir -p gpurun_out/r6z
for d in 4 6 8; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-verify --no-host --no-t2t --no-rg4 --narrow= --no-decode --chain-inflight $d > gpurun_out/r6z/chain_d$d.log 2>&1
done
