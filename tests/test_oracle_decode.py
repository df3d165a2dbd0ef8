"""CPU oracle decoder (oracle/flac_port.c) pinned to the reference decoder's
behaviour on its own fixtures and on 600+ seeded corruptions
(tests/golden/flac_decode_vectors.json): same status, same PCM bytes."""
import hashlib

import numpy as np
import pytest

import decode_cases
import oracle_port
import signals

CASES = decode_cases.load_cases()


def oracle_result(data):
    rc, info, _, si = oracle_port.read_metadata(data)
    if rc:
        return 100, b""
    r = oracle_port.decode_frames(data, si)
    code = r["code"]
    pcm = oracle_port.pcm_bytes(r["pcm"], info["bits_per_sample"])
    if code == 0 and info["md5"] != bytes(16) and hashlib.md5(pcm).digest() != info["md5"]:
        code = oracle_port.FD_MD5
    return code, pcm


def test_golden_covers_error_kinds():
    codes = {c["code"] for c in CASES}
    for want in (0, 2, 6, 7, 8, 9, 10, 13, 14, 15, 16):
        assert want in codes


@pytest.mark.parametrize("chunk", range(8))
def test_oracle_decoder_matches_reference_records(chunk):
    for case in CASES[chunk::8]:
        code, pcm = oracle_result(decode_cases.case_bytes(case))
        assert code == case["code"], case["name"]
        assert len(pcm) == case["pcm_bytes"], case["name"]
        assert hashlib.md5(pcm).hexdigest() == case["pcm_md5"], case["name"]


def test_oracle_offsets_round_trip():
    pcm = signals.make("tone", 4096 * 3 + 100, 2, 16, seed=5)
    data, offsets = oracle_port.encode(pcm, 2, 16, 44100, **oracle_port.PRESETS["8"])
    r = oracle_port.decode_frames(data)
    assert r["code"] == 0
    assert np.array_equal(r["pcm"], pcm)
    assert r["offsets"] == offsets
