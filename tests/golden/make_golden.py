#!/usr/bin/env python3
"""Generate tests/golden/flac_vectors.json with the REFERENCE encoder.

Runs oracle/_ref/flacenc (the reference's own src/encoders/flac.c built in
its -DSTANDALONE mode by `make -C oracle ref`, in this container only) on
seeded inputs from tests/signals.py and records the sha256 of every .flac
it writes.  The CPU tests then pin the clean-room oracle (oracle/flac_port.c)
to these hashes on any machine, without the reference.

The standalone encoder takes -c -r -b -B -l -P -R -m -M -e and fixes the
padding at 4096 (reference src/encoders/flac.c:1637-1803); it reads LE
signed interleaved PCM from stdin.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_port  # noqa: E402
import signals  # noqa: E402

OUT = os.path.join(HERE, "flac_vectors.json")

KINDS = ["tone", "sine", "noise", "silence", "chirp", "wasted", "fsd"]
FORMATS = [(1, 8), (1, 16), (2, 16), (2, 24), (6, 16), (6, 24), (6, 8)]


def cases():
    """(name, kind, frames, channels, bps, preset, seed) — deterministic"""
    out = []
    for preset in sorted(oracle_port.PRESETS):
        B = oracle_port.PRESETS[preset]["block_size"]
        for ch, bps in FORMATS:
            for ki, kind in enumerate(KINDS):
                if kind == "wasted" and bps == 8:
                    continue
                n = {"tone": 2 * B + 17, "sine": B + 1, "noise": B // 2 + 3,
                     "silence": 300, "chirp": 3 * B - 1, "wasted": B + 100,
                     "fsd": 2 * B}[kind]
                seed = 1000 * int(preset) + 10 * ch + bps + ki
                out.append(("p%s_c%d_b%d_%s" % (preset, ch, bps, kind), kind, n, ch, bps,
                            preset, seed))
    return out


def make_pcm(kind, n, ch, bps, seed):
    if kind == "fsd":
        pats = signals.PATTERNS
        mono = signals.fsd(pats[seed % len(pats)], n, bps)
        return np.repeat(mono[:, None], ch, 1).reshape(-1).astype(np.int32)
    return signals.make(kind, n, ch, bps, seed=seed)


def ref_encode(pcm, ch, bps, preset):
    o = oracle_port.PRESETS[preset]
    args = [oracle_port.REF_FLACENC, "-c", str(ch), "-r", "44100", "-b", str(bps),
            "-B", str(o["block_size"]), "-l", str(o["max_lpc_order"]),
            "-P", str(o.get("min_residual_partition_order", 0)),
            "-R", str(o["max_residual_partition_order"])]
    if o.get("mid_side"):
        args.append("-m")
    if o.get("adaptive_mid_side"):
        args.append("-M")
    if o.get("exhaustive_model_search"):
        args.append("-e")
    dt = {8: "<i1", 16: "<i2", 24: None}[bps]
    if dt:
        raw = pcm.astype(dt).tobytes()
    else:
        b = pcm.astype("<i4").view(np.uint8).reshape(-1, 4)[:, :3]
        raw = b.tobytes()
    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, "o.flac")
        subprocess.run(args + [fn], input=raw, stdout=subprocess.DEVNULL, check=True)
        return open(fn, "rb").read()


def main():
    if not os.path.exists(oracle_port.REF_FLACENC):
        sys.exit("oracle/_ref/flacenc missing: run `make -C oracle ref` where "
                 "/root/reference exists")
    vec = []
    bad = 0
    for name, kind, n, ch, bps, preset, seed in cases():
        pcm = make_pcm(kind, n, ch, bps, seed)
        ref = ref_encode(pcm, ch, bps, preset)
        port, _ = oracle_port.encode(pcm, ch, bps, 44100, **oracle_port.PRESETS[preset])
        if port != ref:
            bad += 1
            print("port != reference:", name)
        vec.append({"name": name, "kind": kind, "n": n, "frames": len(pcm) // ch,
                    "channels": ch, "bps": bps,
                    "preset": preset, "seed": seed, "bytes": len(ref),
                    "sha256": hashlib.sha256(ref).hexdigest()})
    json.dump({"generator": "tests/golden/make_golden.py",
               "reference": "src/encoders/flac.c standalone (oracle/_ref/flacenc)",
               "vectors": vec}, open(OUT, "w"), indent=1)
    print("%d vectors, %d port mismatches -> %s" % (len(vec), bad, OUT))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
