"""decode leg of bench JSON lines: tools/dec_summary.py log..."""
import json
import sys

for fn in sys.argv[1:]:
    line = [x for x in open(fn) if x.startswith("{")][-1]
    d = json.loads(line)["decode"]
    print(fn, d["value"], d["ms_per_step"], d["verified_tracks"],
          {k: v for k, v in d["kernel_ms"].items()})
