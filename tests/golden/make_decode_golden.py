#!/usr/bin/env python3
"""Generate tests/golden/flac_decode_vectors.json with the REFERENCE decoder.

Runs oracle/_ref/flacdec (the reference's own src/decoders/flac.c built in
its -DSTANDALONE -DEXECUTABLE mode by `make -C oracle ref`, in this container
only) on
  * the reference's own FLAC fixtures (test/*.flac, copied as data into
    tests/golden/fixtures/), and
  * seeded corruptions of them: byte XORs anywhere in the frame region and
    truncations,
and records what it reports: the error line it prints (mapped to the
decoder status codes of oracle/flac_port.h), how many PCM bytes it wrote
before stopping, and their MD5.  The standalone decoder writes each frame's
PCM (little-endian, signed) only after the frame's CRC-16 checks
(reference src/decoders/flac.c:1400-1470), exactly the frames
FlacDecoder.read() would have returned before raising.

The clean-room oracle is checked against every case here as it is
generated; the CPU tests re-check it and the GPU tests check the HIP decoder
against these records, without the reference.
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

FIX = os.path.join(HERE, "fixtures")
OUT = os.path.join(HERE, "flac_decode_vectors.json")
REF_FLACDEC = os.path.join(oracle_port.ORACLE_DIR, "_ref", "flacdec")

MSG_TO_CODE = {("*** Error: " + m): c for c, m in oracle_port.FD_MESSAGES.items()
               if c not in (15, 16)}
MSG_TO_CODE["*** I/O Error reading frame"] = 15
MSG_TO_CODE["*** MD5 mismatch at end of stream"] = 16
MSG_TO_CODE["*** Error reading streaminfo"] = 100


def ref_decode(data):
    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, "x.flac")
        with open(fn, "wb") as f:
            f.write(data)
        p = subprocess.run([REF_FLACDEC, fn], capture_output=True, timeout=120)
    err = p.stderr.decode().strip()
    # (an invalid bits-per-sample header leaves a try frame on the reader's
    # stack, so the reference also prints a "leftover etry" warning)
    lines = [ln for ln in err.splitlines() if ln in MSG_TO_CODE]
    code = 0 if p.returncode == 0 else MSG_TO_CODE[lines[0]]
    return code, p.stdout


def oracle_decode(data):
    """-> (code, pcm bytes) with the same meaning as ref_decode"""
    rc, info, _, si = oracle_port.read_metadata(data)
    if rc:
        return 100, b""
    r = oracle_port.decode_frames(data, si)
    code = r["code"]
    pcm = oracle_port.pcm_bytes(r["pcm"], info["bits_per_sample"])
    if code == 0 and info["md5"] != bytes(16):
        if hashlib.md5(pcm).digest() != info["md5"]:
            code = 16
    return code, pcm


def mutations(name, data, rng):
    rc, info, _, si = oracle_port.read_metadata(data)
    start = si.frames_offset
    n = len(data)
    out = []
    for k in range(12):
        pos = int(rng.integers(start, n))
        x = int(rng.integers(1, 256))
        out.append(("%s_xor%d" % (name, k), [[pos, x]], None))
    # flips right at frame starts (header fields, subframe headers)
    r = oracle_port.decode_frames(data, si)
    offs = [o for o, _ in r["offsets"]]
    for k in range(8):
        o = start + offs[int(rng.integers(0, len(offs)))]
        pos = o + int(rng.integers(0, 12))
        x = 1 << int(rng.integers(0, 8))
        out.append(("%s_hdr%d" % (name, k), [[pos, x]], None))
    for k in range(4):
        cut = int(rng.integers(start, n))
        out.append(("%s_cut%d" % (name, k), [], cut))
    return out


# STREAMINFO edits (body at byte 8): md5, total samples (+-), max block
# size, sample rate, channel count, bits per sample
META_EDITS = [("md5", 8 + 18, 0x01), ("total_lo", 8 + 17, 0x01),
              ("total_hi", 8 + 14, 0x01), ("total_dn", 8 + 16, 0x10),
              ("maxbs", 8 + 2, None), ("rate", 8 + 10, 0x10),
              ("chan", 8 + 12, 0x02), ("bps", 8 + 13, 0x10)]


def meta_mutations(name, data):
    if data[4] & 0x7F != 0:
        return []
    # x None: clear the byte (max block size -> its low byte)
    return [("%s_meta_%s" % (name, tag), [[pos, data[pos] if x is None else x]], None)
            for tag, pos, x in META_EDITS]


def apply(data, xors, cut):
    b = bytearray(data)
    for pos, x in xors:
        b[pos] ^= x
    if cut is not None:
        b = b[:cut]
    return bytes(b)


def main():
    rng = np.random.default_rng(0xF1AC)
    cases = []
    bad = 0
    for fn in sorted(os.listdir(FIX)):
        if not fn.endswith(".flac"):
            continue
        data = open(os.path.join(FIX, fn), "rb").read()
        name = fn[:-5]
        todo = [(name, [], None)]
        todo += meta_mutations(name, data)
        if len(data) < 200000:
            todo += mutations(name, data, rng)
        for cname, xors, cut in todo:
            d = apply(data, xors, cut)
            code, pcm = ref_decode(d)
            ocode, opcm = oracle_decode(d)
            if (code, pcm) != (ocode, opcm):
                bad += 1
                print("ORACLE MISMATCH", cname, code, ocode, len(pcm), len(opcm))
            cases.append(dict(name=cname, file=fn, xor=xors, cut=cut, code=code,
                              pcm_bytes=len(pcm), pcm_md5=hashlib.md5(pcm).hexdigest()))
    with open(OUT, "w") as f:
        json.dump(dict(generator="tests/golden/make_decode_golden.py",
                       reference="oracle/_ref/flacdec (src/decoders/flac.c)",
                       cases=cases), f, indent=0)
    codes = {}
    for c in cases:
        codes[c["code"]] = codes.get(c["code"], 0) + 1
    print("%d cases, %d oracle mismatches, codes %s" % (len(cases), bad, codes))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
