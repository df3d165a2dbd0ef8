#!/usr/bin/env python3
"""Generate tests/golden/flac_vectors_big.json with the REFERENCE encoder:
block sizes above 4096 (up to FLAC's 65535) and residual partition orders
up to 15, outside the presets that make_golden.py covers.  The reference
accepts both (src/encoders/flac.c:1326-1505 loops the partition order while
the block divides; test/test_formats.py:3798-3844 encodes 32768- and
65535-sample blocks).

Same mechanics as make_golden.py: oracle/_ref/flacenc (the reference's own
src/encoders/flac.c, -DSTANDALONE) encodes seeded tests/signals.py inputs and
the sha256 of every .flac is recorded; the CPU tests then pin the clean-room
oracle to these hashes without the reference.
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

OUT = os.path.join(HERE, "flac_vectors_big.json")

BLOCKS = [4608, 6000, 8192, 16384, 32768, 65535]
PORDERS = [0, 6, 8, 12, 15]
FORMATS = [(2, 16), (1, 8), (2, 24), (1, 16), (6, 16)]
KINDS = ["tone", "noise", "chirp", "wasted", "silence", "sine"]


def options(block, porder, k):
    o = dict(block_size=block, max_lpc_order=(12, 8, 32, 0)[k % 4],
             min_residual_partition_order=0, max_residual_partition_order=porder,
             mid_side=k % 3 != 2, adaptive_mid_side=k % 3 == 1,
             exhaustive_model_search=k % 2 == 0)
    return o


def cases():
    out = []
    k = 0
    for rep in range(3):
        for block in BLOCKS:
            for porder in PORDERS:
                ch, bps = FORMATS[k % len(FORMATS)]
                kind = KINDS[k % len(KINDS)]
                if kind == "wasted" and bps == 8:
                    kind = "tone"
                if ch == 6 and block > 16384:
                    ch = 2
                n = {0: 2 * block + 17, 1: block, 2: block // 2 + 5}[k % 3]
                out.append(dict(name="r%d_b%d_p%d_c%d_b%d_%s" % (rep, block, porder, ch, bps, kind),
                                kind=kind, n=n, channels=ch, bps=bps, seed=7000 + k,
                                opts=options(block, porder, k)))
                k += 1
    return out


def ref_encode(pcm, ch, bps, o):
    args = [oracle_port.REF_FLACENC, "-c", str(ch), "-r", "44100", "-b", str(bps),
            "-B", str(o["block_size"]), "-l", str(o["max_lpc_order"]),
            "-P", str(o["min_residual_partition_order"]),
            "-R", str(o["max_residual_partition_order"])]
    if o["mid_side"]:
        args.append("-m")
    if o["adaptive_mid_side"]:
        args.append("-M")
    if o["exhaustive_model_search"]:
        args.append("-e")
    dt = {8: "<i1", 16: "<i2", 24: None}[bps]
    if dt:
        raw = pcm.astype(dt).tobytes()
    else:
        raw = pcm.astype("<i4").view(np.uint8).reshape(-1, 4)[:, :3].tobytes()
    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, "o.flac")
        subprocess.run(args + [fn], input=raw, stdout=subprocess.DEVNULL, check=True)
        return open(fn, "rb").read()


def main():
    if not os.path.exists(oracle_port.REF_FLACENC):
        sys.exit("oracle/_ref/flacenc missing: run `make -C oracle ref` where "
                 "/root/reference exists")
    vec, bad = [], 0
    for c in cases():
        pcm = signals.make(c["kind"], c["n"], c["channels"], c["bps"], seed=c["seed"])
        ref = ref_encode(pcm, c["channels"], c["bps"], c["opts"])
        port, _ = oracle_port.encode(pcm, c["channels"], c["bps"], 44100, **c["opts"])
        if port != ref:
            bad += 1
            print("port != reference:", c["name"])
        c.update(frames=len(pcm) // c["channels"], bytes=len(ref),
                 sha256=hashlib.sha256(ref).hexdigest())
        vec.append(c)
    json.dump({"generator": "tests/golden/make_golden_big.py",
               "reference": "src/encoders/flac.c standalone (oracle/_ref/flacenc)",
               "vectors": vec}, open(OUT, "w"), indent=1)
    print("%d vectors, %d port mismatches -> %s" % (len(vec), bad, OUT))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
