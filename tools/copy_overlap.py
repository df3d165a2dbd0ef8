#!/usr/bin/env python3
"""Copy-engine timeline of a rocprofv3 --memory-copy-trace run: per
direction the busy time, the bytes and rate, and how long host->device and
device->host copies ran at the same time (full duplex).

    python tools/copy_overlap.py <dir with *memory_copy_trace.csv> [min_bytes]
"""
import csv
import glob
import sys


def merge(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def inter(x, y):
    i = j = 0
    tot = 0
    while i < len(x) and j < len(y):
        a, b = max(x[i][0], y[j][0]), min(x[i][1], y[j][1])
        if b > a:
            tot += b - a
        if x[i][1] < y[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    root = sys.argv[1]
    min_bytes = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
    rows = []
    for f in glob.glob(root + "/**/*memory_copy_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    if not rows:
        raise SystemExit("no memory_copy_trace.csv under " + root)
    by = {}
    for r in rows:
        size = int(r.get("Size") or r.get("Bytes") or 0)
        if size < min_bytes:
            continue
        d = r.get("Direction") or r.get("Operation") or r.get("Kind")
        by.setdefault(d, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), size))
    span = [min(a for v in by.values() for a, _, _ in v), max(b for v in by.values() for _, b, _ in v)]
    print("window %.1f ms, copies >= %d bytes" % ((span[1] - span[0]) / 1e6, min_bytes))
    merged = {}
    for d, v in sorted(by.items()):
        m = merge([(a, b) for a, b, _ in v])
        merged[d] = m
        busy = sum(b - a for a, b in m)
        nb = sum(s for _, _, s in v)
        lat = sum(b - a for a, b, _ in v)
        print("%-24s n=%4d  bytes %.3f GB  busy %.1f ms  %.1f GB/s over busy time, "
              "%.1f GB/s per copy" % (d, len(v), nb / 1e9, busy / 1e6, nb / busy, nb / lat))
    ks = sorted(merged)
    for i in range(len(ks)):
        for j in range(i + 1, len(ks)):
            print("overlap %s / %s: %.1f ms" % (ks[i], ks[j], inter(merged[ks[i]], merged[ks[j]]) / 1e6))


if __name__ == "__main__":
    main()
