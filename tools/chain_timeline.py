#!/usr/bin/env python3
"""Config-5 chain leg timeline from a rocprofv3 kernel trace
(tools/gpu_chain_trace.sh): per step (one ALAC parse launch to the next),
when each stage's kernels ran and how much of the step the device was busy.

usage: chain_timeline.py gpurun_out/<tag>/kernel_trace.csv [steps]"""
import csv
import re
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    m = re.search(r"\b(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:30]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
rows.sort()
parse = [s for s, e, n in rows if n == "k_adec_parse"]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
marks = parse[-(steps + 1):]
groups = {"alac": ("k_adec",), "resample": ("k_rs",), "md5": ("k_track_md5",),
          "flac": ("k_lpc", "k_frame", "k_track_scan", "k_stream", "k_subframe")}


def group(n):
    for g, pre in groups.items():
        if n.startswith(pre):
            return g
    return "other"


print("step  period_ms  busy_ms  " + "  ".join("%s_ms" % g for g in groups))
for a, b in zip(marks, marks[1:]):
    iv = [(max(s, a), min(e, b), group(n)) for s, e, n in rows if e > a and s < b]
    per = {g: 0.0 for g in groups}
    for s, e, g in iv:
        if g in per:
            per[g] += (e - s) / 1e6
    # union of busy intervals
    busy, cur_s, cur_e = 0.0, None, None
    for s, e, _ in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += (cur_e - cur_s) / 1e6
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += (cur_e - cur_s) / 1e6
    print("%4d  %9.2f  %7.2f  " % (len(per), (b - a) / 1e6, busy) +
          "  ".join("%8.2f" % per[g] for g in groups))
# one step in detail: the kernels of the last full step, relative start/end
a, b = marks[-2], marks[-1]
print("\nlast step, kernels (ms from the parse launch):")
for s, e, n in rows:
    if e > a and s < b and (e - s) > 200000:
        print("  %8.2f  %8.2f  %-28s %7.2f" % ((s - a) / 1e6, (e - a) / 1e6, n, (e - s) / 1e6))
