#!/usr/bin/env python3
"""Tabulate tools/gpu_k2split.sh output: per build, k_frame_search_ms<short>'s
per-launch PMC counts and its average duration (kernel-trace stats)."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/k2split"
KERNEL = "k_frame_search_ms<short>"
out = {}
for d in sorted(glob.glob(root + "/*/")):
    name = os.path.basename(d.rstrip("/"))
    agg, cnt = collections.defaultdict(float), collections.defaultdict(int)
    for f in glob.glob(d + "pmc/**/run_counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Kernel_Name"]:
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[r["Counter_Name"]] += 1
    per = {c: v / cnt[c] for c, v in agg.items()}
    ms = None
    for f in glob.glob(d + "kt/**/run_kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if KERNEL in r["Name"]:
                ms = float(r["AverageNs"]) / 1e6
    per["avg_ms"] = ms
    out[name] = per
json.dump(out, sys.stdout, indent=1, sort_keys=True)
print()
