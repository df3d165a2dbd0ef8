#!/usr/bin/env python3
"""Generate tests/golden/id3_vectors.json with the REFERENCE decoder.

The reference's test/flac-id3.flac and flac-id3-2.flac (copied as data into
tests/golden/fixtures/) carry ID3v2 comments in front of "fLaC" (and
flac-id3.flac a 128-byte ID3v1 "TAG" block behind the last frame).
FlacAudio steps over the prefix before it hands the stream to FlacDecoder
(reference audiotools/flac.py:2433-2435, 1680-1684).  For each file this
script

  * finds the prefix length with a restatement of skip_id3v2_comment
    (reference audiotools/id3.py:264-310; audiotools.id3 is checked
    against it),
  * runs oracle/_ref/flacdec (the reference's src/decoders/flac.c built by
    `make -C oracle ref`, this container only) on the bytes from "fLaC" on,
  * records the prefix length, the PCM frame count and the MD5 of the PCM
    bytes it wrote (signed little-endian: what
    transfer_framelist_data(to_pcm(), md5.update) hashes).

flac-id3.flac's PCM MD5 is also a known answer of the reference's own
tracklint test (test/test_utils.py:3383-3406: 9a0ab096c517a627b0ab5a0b959e5f36);
the script asserts it.
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "python-audio-tools_amd"))
FIX = os.path.join(HERE, "fixtures")
OUT = os.path.join(HERE, "id3_vectors.json")
REF_FLACDEC = os.path.join(ROOT, "oracle", "_ref", "flacdec")
FILES = ("flac-id3.flac", "flac-id3-2.flac")
KAT = {"flac-id3.flac": "9a0ab096c517a627b0ab5a0b959e5f36"}


def id3v2_prefix(data):
    """bytes of nested ID3v2 comments at the start (id3.py:264-310)"""
    pos = 0
    while data[pos:pos + 3] == b"ID3" and len(data) >= pos + 10 and data[pos + 3] in (2, 3, 4):
        raw = data[pos + 6:pos + 10]
        if any(b & 0x80 for b in raw):
            break
        size = (raw[0] << 21) | (raw[1] << 14) | (raw[2] << 7) | raw[3]
        pos += 10 + size
    return pos


def main():
    import io
    from audiotools.id3 import skip_id3v2_comment
    out = {}
    for name in FILES:
        data = open(os.path.join(FIX, name), "rb").read()
        skip = id3v2_prefix(data)
        assert skip_id3v2_comment(io.BytesIO(data)) == skip, name
        assert data[skip:skip + 4] == b"fLaC", name
        with tempfile.TemporaryDirectory() as d:
            fn = os.path.join(d, "x.flac")
            with open(fn, "wb") as f:
                f.write(data[skip:])
            p = subprocess.run([REF_FLACDEC, fn], capture_output=True, timeout=60)
        assert p.returncode == 0, (name, p.stderr)
        # STREAMINFO: channels and bits per sample for the frame count
        si = data[skip + 8:skip + 8 + 34]
        channels = ((si[12] >> 1) & 0x7) + 1
        bps = (((si[12] & 1) << 4) | (si[13] >> 4)) + 1
        frames = len(p.stdout) // (channels * ((bps + 7) // 8))
        md5 = hashlib.md5(p.stdout).hexdigest()
        if name in KAT:
            assert md5 == KAT[name], (name, md5)
        out[name] = {"id3v2_bytes": skip, "id3v1_tag": data[-128:-125] == b"TAG",
                     "channels": channels, "bits_per_sample": bps,
                     "pcm_frames": frames, "pcm_md5": md5}
        print(name, out[name])
    with open(OUT, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
