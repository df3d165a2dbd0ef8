#!/usr/bin/env python3
"""Search for a ReplayGain window whose value sits within 1e-9 of a bin edge
(tests/test_gpu_replaygain.py: the flagged-and-rerun case).

The gain filter (Yule then Butterworth, replaygain.c:566-610) is linear, so
one closed window's sum of squares is an exact quadratic form in any few
input samples: S(x + sum a_i e_i) = S0 + g.a + a'Ha.  The form is fitted
from oracle evaluations (oracle_port.rg_window_vals), searched over a grid of
integer offsets for the value closest to an edge, and the winner re-checked
with the oracle.  Prints the offsets for the test's construction.

    python tools/rg_near_edge.py
"""
import itertools
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import oracle_port as op  # noqa: E402

RATE, WSZ, W = 44100, 2205, 5


def base():
    rng = np.random.default_rng(5)
    n = WSZ * 12
    t = np.arange(n)
    amp = 1041.25
    x = np.stack([amp * np.sin(2 * np.pi * 440 * t / RATE) + rng.normal(0, amp / 4, n),
                  amp * np.sin(2 * np.pi * 660 * t / RATE) + rng.normal(0, amp / 4, n)],
                 1).round().astype(np.int32).reshape(-1)
    e = (W + 1) * WSZ - 1
    x[2 * e] += -107
    x[2 * (e - 1)] += -255
    return x, e


def window_sum(x, pos, a):
    y = x.copy()
    for p, d in zip(pos, a):
        y[p] += d
    v = op.rg_window_vals(y, 2, 16, RATE)[W]
    return 2.0 * WSZ * 10.0 ** (v / 1000.0), v


def main():
    x, e = base()
    pos = [2 * e, 2 * e + 1, 2 * (e - 1), 2 * (e - 1) + 1, 2 * (e - 2), 2 * (e - 2) + 1]
    k = len(pos)
    h = 64
    s0, v0 = window_sum(x, pos, [0] * k)
    g = np.zeros(k)
    H = np.zeros((k, k))
    for i in range(k):
        a = [0] * k
        a[i] = h
        sp, _ = window_sum(x, pos, a)
        a[i] = -h
        sm, _ = window_sum(x, pos, a)
        g[i] = (sp - sm) / (2 * h)
        H[i, i] = (sp + sm - 2 * s0) / (2 * h * h)
    for i, j in itertools.combinations(range(k), 2):
        a = [0] * k
        a[i] = a[j] = h
        sij, _ = window_sum(x, pos, a)
        H[i, j] = H[j, i] = (sij - s0 - h * (g[i] + g[j]) - h * h * (H[i, i] + H[j, j])) / (2 * h * h)
    print("v0 = %.12f" % v0)
    R = 40
    r = np.arange(-R, R + 1, dtype=np.float64)
    A = np.stack(np.meshgrid(r, r, r, indexing="ij"), -1).reshape(-1, 3)
    quad = np.einsum("ni,ij,nj->n", A, H[:3, :3], A)
    best = []
    # the first three offsets on a grid, the other three swept outside
    for b in itertools.product(range(-R, R + 1, 3), repeat=3):
        bb = np.array(b, dtype=np.float64)
        c0 = s0 + g[3:] @ bb + bb @ H[3:, 3:] @ bb
        S = c0 + A @ (g[:3] + 2 * H[:3, 3:] @ bb) + quad
        v = 1000.0 * np.log10(S / (2.0 * WSZ) + 1e-37)
        d = np.minimum(v - np.floor(v), np.ceil(v) - v)
        i = int(np.argmin(d))
        best.append((d[i], list(A[i].astype(int)) + list(b), v[i]))
        best.sort(key=lambda q: q[0])
        best = best[:8]
        if best[0][0] < 2e-11:
            break
    for d, a, v in best:
        _, vo = window_sum(x, pos, a)
        do = min(vo - np.floor(vo), np.ceil(vo) - vo)
        print("offsets %s  model %.3e  oracle v %.12f  dist %.3e" % (a, d, vo, do))
    print("positions (interleaved sample indices, relative to e=%d): %s" % (e, pos))


if __name__ == "__main__":
    main()
