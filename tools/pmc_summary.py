#!/usr/bin/env python3
"""Per-kernel PMC summary from tools/gpu_pmc.sh output (gpurun_out/pmc).

Counter values are summed over the dispatches of each kernel and divided by
the number of dispatches (per-launch figures).  FETCH_SIZE is doubled
(gfx950 reports half the bytes of wide streaming reads, MI355X_MICROARCH.md
'HBM'); FETCH_SIZE / WRITE_SIZE are in KiB."""
import collections
import csv
import glob
import json
import re
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
for f in glob.glob(root + "/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        m = re.search(r"\b(k_[A-Za-z0-9_]+(?:<[^>(]*>)?)", r["Kernel_Name"])
        if not m:
            continue
        short = m.group(1)
        agg[short][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[short][r["Counter_Name"]] += 1
out = {}
for k, d in agg.items():
    per = {c: v / cnt[k][c] for c, v in d.items()}
    if "FETCH_SIZE" in per:
        per["HBM_read_bytes"] = per["FETCH_SIZE"] * 1024 * 2
    if "WRITE_SIZE" in per:
        per["HBM_write_bytes"] = per["WRITE_SIZE"] * 1024
    if "SQ_WAVES" in per and per["SQ_WAVES"]:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM"):
            if c in per:
                per[c + "_per_wave"] = per[c] / per["SQ_WAVES"]
    out[k] = per
json.dump(out, sys.stdout, indent=1, sort_keys=True)
print()
