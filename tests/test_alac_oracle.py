"""CPU: the ALAC oracle (oracle/alac_port.c, a clean-room C restatement of
the reference's src/encoders/alac.c and src/decoders/alac.c) pinned to the
vectors the reference encoder/decoder recorded
(tests/golden/alac_vectors.json, generator tests/golden/make_alac_golden.py)
and to the reference's own fixture test/alac-allframes.m4a; the m4a
container writer (audiotools/m4a.py) pinned byte for byte to that fixture.
When the reference build oracle/_ref/alac* is present (this container only)
a few extra cases compare against it live."""
import hashlib
import os

import numpy as np
import pytest

import alac_cases
import oracle_port as op
import signals

G = alac_cases.load()


@pytest.mark.parametrize("v", G["encoder"], ids=lambda v: v["name"])
def test_encoder_vectors(v):
    x = alac_cases.enc_pcm(v)
    mdat, fs = op.alac_encode(x, v["channels"], v["bps"], block_size=v["block_size"])
    assert len(mdat) == v["bytes"]
    assert hashlib.sha256(mdat).hexdigest() == v["sha256"]
    assert len(fs) == v["framesets"] and sum(fs) + 8 == len(mdat)


@pytest.mark.parametrize("v", G["leftweights"], ids=lambda v: v["name"])
def test_leftweight_vectors(v):
    """minimum/maximum_interlacing_leftweight (alac.c:57-72, 459-481): the
    port's mdat for each range is the recorded one, whose reference-decoder
    round trip make_alac_golden.py checked (0..4 is pinned to the reference
    encoder by test_encoder_vectors; the leftweight loop is the same code)"""
    x = alac_cases.enc_pcm(v)
    mdat, fs = op.alac_encode(x, v["channels"], v["bps"],
                              minimum_interlacing_leftweight=v["lw_min"],
                              maximum_interlacing_leftweight=v["lw_max"])
    assert hashlib.sha256(mdat).hexdigest() == v["sha256"]
    assert len(fs) == v["framesets"]


def test_leftweight_vectors_mostly_lossless():
    """all but the full-scale cases whose mixed channel outgrows the sample
    size (leftweights above 4) decode back to the source in the reference
    decoder"""
    lossy = [v["name"] for v in G["leftweights"] if not v["reference_decoder_lossless"]]
    assert sorted(lossy) == ["noise_c6_b16_lw5_9", "tone_c2_b16_lw250_255"]


def _decode_all(data):
    st, info, _ = op.alac_read_info(data)
    if st:
        return st + 100, b"", info
    r = op.alac_decode(data, info)
    return r["code"], op.pcm_bytes(r["pcm"], info.bits_per_sample), info


@pytest.mark.parametrize("s", G["decoder"], ids=lambda s: s["name"])
def test_decoder_vectors(s):
    x = alac_cases.enc_pcm(s)
    mdat, fs = op.alac_encode(x, s["channels"], s["bps"])
    img = alac_cases.dec_image(s, mdat, fs)
    assert hashlib.sha256(img).hexdigest() == s["image_sha256"]
    for c in s["cases"]:
        code, pcm, _ = _decode_all(alac_cases.mutate(img, c))
        if code == 10:  # Python-path ValueError; the standalone has no such check
            continue
        assert (code == 0) == (c["rc"] == 0), (c["name"], code, c["rc"])
        assert len(pcm) == c["pcm_bytes"], c["name"]
        assert hashlib.md5(pcm).hexdigest() == c["pcm_md5"], c["name"]
    # the clean stream round-trips exactly
    r = op.alac_decode(img)
    assert r["code"] == 0 and np.array_equal(r["pcm"], x)


def test_reference_fixture_decode():
    f = G["fixture"]
    data = open(os.path.join(alac_cases.FIX, f["file"]), "rb").read()
    code, pcm, info = _decode_all(data)
    assert code == 0 and f["rc"] == 0
    assert (info.channels, info.bits_per_sample, info.total_frames,
            info.max_samples_per_frame) == (1, 16, 40, 20)
    assert len(pcm) == f["pcm_bytes"] and hashlib.md5(pcm).hexdigest() == f["pcm_md5"]


def test_m4a_container_matches_reference_fixture():
    """audiotools.m4a writes the reference's atom layout byte for byte
    (creation date and the writer's version string taken from the fixture)"""
    from audiotools import m4a
    data = open(os.path.join(alac_cases.FIX, "alac-allframes.m4a"), "rb").read()
    mdat = data[5829:]
    got = m4a.m4a_file(1, 16, 44100, 20, 40, mdat, [19, 44], create_date=0xC85BCDE7,
                       version="2.16alpha2")
    assert got == data


def test_seektable_from_container():
    """stts/stsc/stco -> seekpoints every 5 framesets (m4a.py:1342-1381,
    decoders/alac.c:566-672)"""
    from audiotools import m4a
    x = signals.make("tone", 4096 * 11 + 5, 2, 16, seed=1)
    mdat, fs = op.alac_encode(x, 2, 16)
    img = m4a.m4a_file(2, 16, 44100, 4096, len(x) // 2, mdat, fs, create_date=1)
    st, info, pts = op.alac_read_info(img)
    assert st == 0 and [p for p, _ in pts] == [0, 4096 * 5, 4096 * 10]
    start = len(img) - len(mdat) + 8
    assert pts[0][1] == start and pts[1][1] == start + sum(fs[:5])
    r = op.alac_decode(img, info, start=pts[1][1], remaining=info.total_frames - pts[1][0])
    assert r["code"] == 0 and np.array_equal(r["pcm"], x[2 * 4096 * 5:])


@pytest.mark.skipif(not os.path.exists(op.REF_ALACENC), reason="reference build absent")
def test_port_matches_reference_live():
    for ch, bps, kind, bs in ((2, 16, "tone", 4096), (6, 24, "noise", 1000), (1, 24, "sine", 9),
                              (3, 16, "chirp", 4096), (8, 16, "wasted", 555)):
        x = signals.make(kind, 3 * bs + 17, ch, bps, seed=ch)
        assert op.alac_encode(x, ch, bps, block_size=bs)[0] == \
            op.ref_alac_encode(x, ch, bps, block_size=bs)
