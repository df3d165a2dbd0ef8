set -e -o pipefail
mkdir -p gpurun_out/r6az
for cfg in "--channels 6 --bits 24" "--channels 2 --bits 24" "--channels 8 --bits 16"; do
  timeout -k 10 240 python -u tools/pack_probe.py $cfg >> gpurun_out/r6az/probe.jsonl 2>>gpurun_out/r6az/err.log
  ATGPU_LIB=abl/libatgpu_old.so timeout -k 10 240 python -u tools/pack_probe.py $cfg >> gpurun_out/r6az/probe.jsonl 2>>gpurun_out/r6az/err.log
done
