"""print the narrow-batch leg of a bench JSON line (tools/gpu_narrow.sh)"""
import json
import sys

line = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(line)
print("headline", d["value"], d["ms_per_step"])
for n, per in d["narrow_batches"]["tracks_per_batch"].items():
    for k, v in per.items():
        km = {a: b for a, b in v["kernel_ms"].items() if b > 0.3}
        print(n, k, v["value"], v["ms_per_step"], "bad", v["mismatches"], km)
