"""Debug aid: re-create test_gpu_flac.test_presets_vs_oracle's inputs for
one (preset, channels, bps) case, encode them on the GPU and with the CPU
oracle, and print for every track that differs the first differing frame
(sizes and the first subframe's header byte on both sides).  One JSON line
per track.

    python tools/hl_debug.py [--preset 8] [--channels 2] [--bps 24]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "python-audio-tools_amd"))

import numpy as np  # noqa: E402

import oracle_port  # noqa: E402
import signals  # noqa: E402
from test_gpu_flac import gpu_encode_tracks  # noqa: E402


def frames_of(img, lst):
    _, region = oracle_port.split_flac(img)
    base = len(img) - len(region)
    out = []
    for i, (off, _n) in enumerate(lst):
        end = lst[i + 1][0] if i + 1 < len(lst) else len(img) - base
        out.append(img[base + off:base + end])
    return out


class Bits(object):
    def __init__(self, b, pos=0):
        self.b, self.p = b, pos

    def get(self, n):
        v = 0
        for _ in range(n):
            v = (v << 1) | ((self.b[self.p >> 3] >> (7 - (self.p & 7))) & 1)
            self.p += 1
        return v

    def sget(self, n):
        v = self.get(n)
        return v - (1 << n) if n and v >> (n - 1) else v

    def unary(self):
        n = 0
        while self.get(1) == 0:
            n += 1
        return n


def subframe_heads(fr, bps, nsub, hdr_len):
    """type, order, wasted, shift, coefs, method, porder, rice params of the
    first subframe (residuals are not walked)"""
    r = Bits(fr, 8 * hdr_len)
    r.get(1)
    t = r.get(6)
    w = r.unary() + 1 if r.get(1) else 0
    d = {"type": t, "wasted": w}
    sb = bps - w + (1 if assign_side(fr) else 0)
    if t >= 32 or 8 <= t < 16:
        order = t - 31 if t >= 32 else t - 8
        d["order"] = order
        d["warm"] = [r.sget(sb) for _ in range(order)]
        if t >= 32:
            prec = r.get(4) + 1
            d["shift"] = r.sget(5)
            d["coefs"] = [r.sget(prec) for _ in range(order)]
        m = r.get(2)
        po = r.get(4)
        d["method"], d["porder"] = m, po
        d["rice0"] = r.get(5 if m else 4)
    return d


def assign_side(fr):
    return False


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--preset", default="8")
    ap.add_argument("--channels", type=int, default=2)
    ap.add_argument("--bps", type=int, default=24)
    a = ap.parse_args()
    import torch
    torch.cuda.init()
    from audiotools import _atgpu
    eng = _atgpu.engine()
    opts = dict(oracle_port.PRESETS[a.preset])
    B = opts["block_size"]
    rng = np.random.default_rng(int(a.preset) * 1000 + a.channels * 100 + a.bps)
    pcms, kinds = [], []
    for kind in ["tone", "sine", "noise", "silence", "chirp", "wasted"]:
        if kind == "wasted" and a.bps == 8:
            continue
        n = int(rng.integers(1, 3 * B)) if kind != "tone" else 3 * B + 17
        pcms.append(signals.make(kind, n, a.channels, a.bps, seed=int(rng.integers(1 << 30))))
        kinds.append(kind)
    got = gpu_encode_tracks(eng, pcms, a.channels, a.bps, 44100, opts)
    for kind, p, (img, lst) in zip(kinds, pcms, got):
        want, wlst = oracle_port.encode(p, a.channels, a.bps, 44100, **opts)
        rec = {"kind": kind, "same": img == want, "gpu_bytes": len(img), "ref_bytes": len(want)}
        if img != want:
            g, w = frames_of(img, lst), frames_of(want, wlst)
            for i, (x, y) in enumerate(zip(g, w)):
                if x != y:
                    rec.update(frame=i, gpu_frame=len(x), ref_frame=len(y),
                               gpu_head=x[:12].hex(), ref_head=y[:12].hex(),
                               first_diff=next(k for k in range(min(len(x), len(y)))
                                               if x[k] != y[k]))
                    hl = 6 if i < 128 else 7
                    try:
                        rec["gpu_sub0"] = subframe_heads(x, a.bps, a.channels, hl)
                        rec["ref_sub0"] = subframe_heads(y, a.bps, a.channels, hl)
                    except Exception as e:  # noqa: BLE001
                        rec["parse_error"] = repr(e)
                    break
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
