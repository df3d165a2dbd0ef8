"""ALAC parity cases shared by the CPU oracle tests and the GPU tests: the
vectors of tests/golden/alac_vectors.json (recorded with the reference ALAC
encoder/decoder by tests/golden/make_alac_golden.py) and the inputs they
are defined on."""
import json
import os

import signals

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "alac_vectors.json")
FIX = os.path.join(HERE, "golden", "fixtures")
CREATE_DATE, VERSION = 0x7A11C0DE, "2.22alpha1"


def load():
    with open(GOLDEN) as f:
        return json.load(f)


def enc_pcm(v):
    return signals.make(v["kind"], v["n"], v["channels"], v["bps"], seed=v["seed"])


def dec_image(stream, mdat, frame_sizes):
    """the clean m4a image of a decoder stream around `mdat`"""
    from audiotools import m4a
    return m4a.m4a_file(stream["channels"], stream["bps"], 44100, 4096, stream["n"], mdat,
                        frame_sizes, create_date=CREATE_DATE, version=VERSION)


def mutate(img, case):
    b = bytearray(img)
    for pos, v in case["xor"]:
        b[pos] ^= v
    if case["cut"] is not None:
        b = b[:case["cut"]]
    return bytes(b)
