"""Decoder parity cases shared by the CPU oracle tests and the GPU tests:
the reference's FLAC fixtures and the seeded corruptions recorded in
tests/golden/flac_decode_vectors.json (generated with the reference decoder
by tests/golden/make_decode_golden.py)."""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden", "flac_decode_vectors.json")
FIX = os.path.join(HERE, "golden", "fixtures")


def load_cases():
    with open(GOLDEN) as f:
        return json.load(f)["cases"]


_files = {}


def case_bytes(case):
    fn = case["file"]
    if fn not in _files:
        with open(os.path.join(FIX, fn), "rb") as f:
            _files[fn] = f.read()
    b = bytearray(_files[fn])
    for pos, x in case["xor"]:
        b[pos] ^= x
    if case["cut"] is not None:
        b = b[:case["cut"]]
    return bytes(b)
