#!/usr/bin/env python3
"""Breakdown of a host_timeline.py trace (rocprofv3 --kernel-trace
--memory-copy-trace, csv): per batch window, busy time of H2D copies, D2H
copies and each kernel (interval unions), and the time nothing ran.
    python3 tools/host_breakdown.py gpurun_out/r3f/prof [n_last_windows]
Windows are cut at each k_lpc_analyze launch of a 256-track chunk run."""
import csv
import glob
import sys


def load(root):
    ev = []
    for f in glob.glob(root + "/**/run_kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            n = r["Kernel_Name"]
            short = n.split("(")[0].split("<")[0].replace("void ", "").strip()
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short, int(r["Stream_Id"])))
    for f in glob.glob(root + "/**/run_memory_copy_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            d = "H2D" if "HOST_TO_DEVICE" in r["Direction"] else "D2H" if "DEVICE_TO_HOST" in r["Direction"] else "D2D"
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), d, int(r["Stream_Id"])))
    ev.sort()
    return ev


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


def main():
    root = sys.argv[1]
    ev = load(root)
    lpc = [s for s, e, n, st in ev if n == "k_lpc_analyze"]
    t_end = max(e for s, e, n, st in ev)
    # whole-trace tail: from the first LPC of the last `last` windows
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    t0 = lpc[-last] if len(lpc) >= last else lpc[0]
    sel = [(max(s, t0), e, n, st) for s, e, n, st in ev if e > t0]
    span = t_end - t0
    print("window %.2f ms from LPC launch %d of %d" % (span / 1e6, len(lpc) - last, len(lpc)))
    names = sorted(set(n for _, _, n, _ in sel))
    rows = []
    for n in names:
        iv = [(s, e) for s, e, m, _ in sel if m == n]
        rows.append((union(iv) / 1e6, sum(e - s for s, e in iv) / 1e6, len(iv), n))
    for u, tot, cnt, n in sorted(rows, reverse=True):
        print("  %-28s busy %8.2f ms  sum %8.2f ms  n %5d" % (n, u, tot, cnt))
    allk = [(s, e) for s, e, n, _ in sel if n not in ("H2D", "D2H", "D2D")]
    print("  any kernel busy %.2f ms; any copy busy %.2f ms; anything %.2f ms; idle %.2f ms"
          % (union(allk) / 1e6, union([(s, e) for s, e, n, _ in sel if n in ("H2D", "D2H")]) / 1e6,
             union([(s, e) for s, e, _, _ in sel]) / 1e6, (span - union([(s, e) for s, e, _, _ in sel])) / 1e6))
    h2d = [(s, e) for s, e, n, _ in sel if n == "H2D"]
    big = [(s, e) for s, e in h2d if e - s > 1e6]
    if big:
        print("  large H2D: n %d, mean %.2f ms" % (len(big), sum(e - s for s, e in big) / len(big) / 1e6))
    d2h = [(s, e) for s, e, n, _ in sel if n == "D2H" and e - s > 1e6]
    if d2h:
        print("  large D2H: n %d, mean %.2f ms" % (len(d2h), sum(e - s for s, e in d2h) / len(d2h) / 1e6))


if __name__ == "__main__":
    main()
