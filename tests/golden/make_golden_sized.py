#!/usr/bin/env python3
"""Generate tests/golden/flac_vectors_sized.json with the REFERENCE encoder.

Explicit frame sizes: the reference cuts one FLAC frame per pcmreader.read()
(src/encoders/flac.c:244-274), so a reader that returns short (or long) reads
gives frames whose header carries block-size code 0x6/0x7 plus an explicit
size (flac.c:412-518), while STREAMINFO's min/max block size stay the
block_size option (flac.c:193-194).  The standalone build never takes that
path (fread fills every block), so oracle/_ref/flacenc_sized drives the
reference's encoders_encode_flac with a read() wrapper
(oracle/ref_sized_reads.c, `make -C oracle ref`, this container only).

Each vector records the seeded input (tests/signals.py), the read sizes and
the sha256 of the reference's .flac; tests/test_oracle.py pins the port
(oracle/flac_port.c flacport_encode_sizes) to them, and the GPU tests compare
the GPU with the port on the same reads.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
import oracle_port  # noqa: E402
import signals  # noqa: E402

OUT = os.path.join(HERE, "flac_vectors_sized.json")

FORMATS = [(1, 8), (1, 16), (2, 16), (2, 24), (6, 16), (6, 24)]
# read-size patterns (then block_size per read): short reads mid-stream, reads
# longer than the block, 1-frame and tiny reads (fewer samples than the LPC
# order / FIXED warm-up), sizes on the standard block-size codes, and an empty
# read that ends the stream early
PATTERNS = [
    [4096, 1000, 4096, 808],
    [1, 2, 3, 4, 5, 13, 4096, 17],
    [7000, 9000],
    [192, 576, 1152, 2304, 4608, 256, 512, 1024, 2048, 8192],
    [300, 0, 5],
    [4095, 4097, 33, 65535],
]


def cases():
    out = []
    for preset in ("8", "5", "2", "0"):
        B = oracle_port.PRESETS[preset]["block_size"]
        for ch, bps in FORMATS:
            for pi, pat in enumerate(PATTERNS):
                kind = ["tone", "noise", "chirp", "sine", "tone", "wasted"][pi]
                if kind == "wasted" and bps == 8:
                    kind = "tone"
                n = sum(pat) + B // 3 + 7
                if pi == 5:
                    n = 4095 + 4097 + 33 + 20000  # ends inside the 65535 read
                seed = 7000 + 1000 * int(preset) + 10 * ch + bps + pi
                out.append(("s%s_c%d_b%d_p%d" % (preset, ch, bps, pi), kind, n, ch, bps,
                            preset, seed, pat))
    return out


def main():
    if not os.path.exists(oracle_port.REF_FLACENC_SIZED):
        sys.exit("oracle/_ref/flacenc_sized missing: run `make -C oracle ref` where "
                 "/root/reference exists")
    vec, bad = [], 0
    for name, kind, n, ch, bps, preset, seed, pat in cases():
        pcm = signals.make(kind, n, ch, bps, seed=seed)
        opts = oracle_port.PRESETS[preset]
        ref = oracle_port.ref_encode_sized(pcm, ch, bps, 44100, pat, **opts)
        port, lst = oracle_port.encode(pcm, ch, bps, 44100, frame_sizes=pat, **opts)
        if port != ref:
            bad += 1
            print("port != reference:", name)
        cut = oracle_port.cut_frames(n, opts["block_size"], pat)
        assert [m for _, m in lst] == cut
        vec.append({"name": name, "kind": kind, "n": n, "channels": ch, "bps": bps,
                    "preset": preset, "seed": seed, "read_sizes": pat,
                    "frame_lengths": cut, "bytes": len(ref),
                    "sha256": hashlib.sha256(ref).hexdigest()})
    json.dump({"generator": "tests/golden/make_golden_sized.py",
               "reference": "src/encoders/flac.c encoders_encode_flac driven by "
                            "oracle/ref_sized_reads.c (oracle/_ref/flacenc_sized)",
               "vectors": vec}, open(OUT, "w"), indent=1)
    print("%d vectors, %d port mismatches -> %s" % (len(vec), bad, OUT))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
