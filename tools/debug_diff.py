#!/usr/bin/env python3
"""GPU debugging aid: encode a few cases with libatgpu and the oracle and
report where the first differing byte falls (frame index, offset, bytes)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "python-audio-tools_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import oracle_port  # noqa: E402
import signals  # noqa: E402
from audiotools import _atgpu  # noqa: E402


def run(eng, kind, n, ch, bps, preset="8", seed=1):
    opts = dict(oracle_port.PRESETS[preset])
    pcm = signals.make(kind, n, ch, bps, seed=seed)
    want, wl = oracle_port.encode(pcm, ch, bps, 44100, **opts)
    arr = pcm.astype(np.int16 if bps <= 16 else np.int32)
    out, res, offs, fp = eng.encode(_atgpu.make_options(**opts), arr, [(0, n)], ch, bps, 44100)
    got = out[res[0].out_offset:res[0].out_offset + res[0].bytes].tobytes()
    if got == want:
        print("OK   %s n=%d ch=%d bps=%d" % (kind, n, ch, bps))
        return
    i = next((k for k in range(min(len(got), len(want))) if got[k] != want[k]),
             min(len(got), len(want)))
    hdr = len(want) - sum(b for _, b in [(0, 0)]) if False else None
    starts = [o + (len(want) - sum(1 for _ in [])) * 0 for o, _ in wl]
    first = len(want) - (wl[-1][0] + 0) if wl else 0
    print("DIFF %s n=%d ch=%d bps=%d: len got %d want %d, first diff at %d"
          % (kind, n, ch, bps, len(got), len(want), i))
    # frame boundaries from the oracle's offsets (relative to first frame)
    base = len(want) - (sum(1 for _ in []) * 0)
    blocks, frames = oracle_port.split_flac(want)
    fstart = len(want) - len(frames)
    rel = i - fstart
    fidx = max([k for k, (o, _) in enumerate(wl) if o <= rel] or [0])
    fo = wl[fidx][0]
    fend = wl[fidx + 1][0] if fidx + 1 < len(wl) else len(frames)
    print("  frame %d (bytes %d..%d), offset in frame %d (frame len %d)"
          % (fidx, fo, fend, rel - fo, fend - fo))
    a = max(0, i - 4)
    print("  got  ", got[a:i + 12].hex())
    print("  want ", want[a:i + 12].hex())
    gf = [(int(offs[k]), int(fp[k])) for k in range(res[0].n_frames)]
    print("  gpu frame list head", gf[:4], "oracle", wl[:4])


def main():
    eng = _atgpu.Engine(0)
    for kind, n in (("tone", 3 * 4096 + 17), ("sine", 5000), ("noise", 4096),
                    ("silence", 300), ("chirp", 9000), ("wasted", 4096)):
        for ch, bps in ((2, 16), (1, 16)):
            try:
                run(eng, kind, n, ch, bps)
            except _atgpu.ATGError as e:
                print("ERR  %s ch=%d bps=%d: %s" % (kind, ch, bps, e))


if __name__ == "__main__":
    main()
