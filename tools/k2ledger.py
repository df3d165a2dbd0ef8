#!/usr/bin/env python3
"""K2 (k_frame_search_ms<short>) instruction ledger, DESIGN 4a''.

Inputs: tools/gpu_k2ledger.sh output (k2split.json: per-launch PMC counts of
the product and of the ledger builds; counts.json: the counting build's
dynamic events).  Phase rows are differences of cumulative truncation
builds (ATG_K2F_TRUNC 1..4), so they sum to the product's totals; the
pass-1 and pass-2 sub-rows are dynamic job counts x the static instruction
mix of the residual blocks in the product ISA (hipcc -S of
flac_search16.hip, blocks with the v_dot2 chains / the pass-2 shifts):

  packed residual block, D tap pairs:   64 D v_dot2 + 64 shift + 64 sad
                                        + 32 window perms + 12 warm-up
                                        selects + ~5       = 177 + 64 D
  side channel on packed L - R words:   208 + 64 D (pk_sub16 per word)
  side channel on (L, R) words:         ~216 + 64 TAPS, TAPS = min(2D, 13)
  pass 2 block (surviving jobs):        ~280 VALU (64 x (sub, 2 ashr, xor,
                                        add3/2) + the wave sum)
  partition search (select_fast32):     ~196 VALU + ~139 SALU

    python tools/k2ledger.py gpurun_out/r5p
"""
import json
import sys


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/k2ledger"
    k = json.load(open(root + "/k2split.json"))
    c = json.load(open(root + "/counts.json"))
    g = lambda b, ctr: k[b][ctr] / 1e9
    V, S, L = "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"
    b = {"t1": "k2l_t1", "t2": "k2l_t2", "t3": "k2l_t3", "t4": "k2l_t4", "base": "base",
         "t3e6": "k2l_t3e6"}
    jobs = c["fixed_jobs"] + c["lpc_jobs"]
    per_order = [c["jobs_order_%d" % o] for o in range(13)]
    f_lr = c["side_lr_jobs"] / jobs
    f_sp = c["side_packed_jobs"] / jobs
    f_pk = 1.0 - f_lr - f_sp
    D = [o // 2 + 1 for o in range(13)]
    D[0] = 2  # FIXED: orders 0..4, taken as 2 tap pairs on average
    taps = [min(2 * d, 13) for d in D]
    dot2 = sum(n * 64 * (f_pk * d + f_sp * d + f_lr * t) for n, d, t in zip(per_order, D, taps))
    post = jobs * 64 * 2
    block = sum(n * (f_pk * (177 + 64 * d) + f_sp * (208 + 64 * d) + f_lr * (216 + 64 * t))
                for n, d, t in zip(per_order, D, taps))
    surv = c["fast32_searches"] + c["wide_searches"]
    rows = [
        ("staging (PCM -> packed LDS images, extrema)", g(b["t1"], V), g(b["t1"], S),
         k[b["t1"]][L] / 1e6, k[b["t1"]]["avg_ms"]),
        ("phase 1: CONSTANT, wasted bits, FIXED order sums, LPC order range",
         g(b["t2"], V) - g(b["t1"], V), g(b["t2"], S) - g(b["t1"], S),
         (k[b["t2"]][L] - k[b["t1"]][L]) / 1e6, k[b["t2"]]["avg_ms"] - k[b["t1"]]["avg_ms"]),
        ("phase 2, pass 1 of all %d jobs" % jobs, g(b["t3"], V) - g(b["t2"], V),
         g(b["t3"], S) - g(b["t2"], S), (k[b["t3"]][L] - k[b["t2"]][L]) / 1e6,
         k[b["t3"]]["avg_ms"] - k[b["t2"]]["avg_ms"]),
        ("  - v_dot2 (one per tap pair and sample)", dot2 / 1e9, None, None, None),
        ("  - post-processing (shift + v_sad per sample)", post / 1e9, None, None, None),
        ("  - window words, warm-up selects, block rest", (block - dot2 - post) / 1e9,
         jobs * 37 / 1e9, None, None),
        ("  - job dispatch and setup (the rest of the row)",
         g(b["t3"], V) - g(b["t2"], V) - block / 1e9,
         g(b["t3"], S) - g(b["t2"], S) - jobs * 37 / 1e9, None, None),
        ("phase 2, pruning + partition search + pass 2 (%d of %d jobs survive)" % (surv, jobs),
         g(b["t4"], V) - g(b["t3"], V), g(b["t4"], S) - g(b["t3"], S),
         (k[b["t4"]][L] - k[b["t3"]][L]) / 1e6, k[b["t4"]]["avg_ms"] - k[b["t3"]]["avg_ms"]),
        ("  - pass 2 (exact bits)", surv * 280 / 1e9, None, None, None),
        ("  - partition search", surv * 196 / 1e9, surv * 139 / 1e9, None, None),
        ("  - pruning bound and the rest", g(b["t4"], V) - g(b["t3"], V) - surv * 476 / 1e9,
         g(b["t4"], S) - g(b["t3"], S) - surv * 139 / 1e9, None, None),
        ("phase 3: the choice, descriptors", g(b["base"], V) - g(b["t4"], V),
         g(b["base"], S) - g(b["t4"], S), (k[b["base"]][L] - k[b["t4"]][L]) / 1e6,
         k[b["base"]]["avg_ms"] - k[b["t4"]]["avg_ms"]),
        ("total (product)", g(b["base"], V), g(b["base"], S), k[b["base"]][L] / 1e6,
         k[b["base"]]["avg_ms"]),
    ]
    print("| phase | VALU (G) | SALU (G) | LDS instr (M) | ms |")
    print("|---|---|---|---|---|")
    for name, v, s, l, ms in rows:
        f = lambda x, p: "" if x is None else ("%." + str(p) + "f") % x
        print("| %s | %s | %s | %s | %s |" % (name, f(v, 3), f(s, 3), f(l, 1), f(ms, 2)))
    extra = g(b["t3"], V) - g(b["t3e6"], V)
    model = sum(n * 64 * (f_pk * (d - 1) + f_sp * (d - 1) + f_lr * (t - 2))
                for n, d, t in zip(per_order, D, taps)) / 1e9
    print()
    print("check: tap pairs beyond the first, measured (t3 - t3e6) %.3f G VALU, "
          "model %.3f G" % (extra, model))


if __name__ == "__main__":
    main()
