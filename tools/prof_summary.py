#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace --stats run into a small text table.

usage: prof_summary.py <run_results.db | kernel_stats.csv> [out.txt]
Keeps the libatgpu kernels (k_*) and the runtime copies, drops torch's
synthetic-data kernels.  Durations are microseconds per dispatch."""
import csv
import re
import sqlite3
import sys


def rows_from_db(path):
    c = sqlite3.connect(path)
    for name, calls, total, avg, pct in c.execute(
            "select name, total_calls, total_duration, average, percentage from top_kernels"):
        yield name, int(calls), float(total), float(avg), float(pct)


def rows_from_csv(path):
    with open(path) as f:
        for r in csv.DictReader(f):
            # rocprofv3 csv stats: durations in ns
            yield (r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]) / 1e3,
                   float(r["AverageNs"]) / 1e3, float(r["Percentage"]))


def main():
    src = sys.argv[1]
    rows = list(rows_from_db(src) if src.endswith(".db") else rows_from_csv(src))
    keep = [r for r in rows if re.search(r"\bk_[a-z]", r[0]) or "__amd_rocclr" in r[0]]
    lines = ["%-44s %6s %12s %12s" % ("kernel", "calls", "total_us", "avg_us")]
    for name, calls, total, avg, _ in keep:
        m = re.search(r"\b(k_[A-Za-z0-9_]+(?:<[^>(]*>)?)", name)
        short = m.group(1) if m else name.replace("void ", "").split("(")[0]
        lines.append("%-44s %6d %12.1f %12.1f" % (short[:44], calls, total, avg))
    text = "\n".join(lines) + "\n"
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(text)
    sys.stdout.write(text)


if __name__ == "__main__":
    main()
