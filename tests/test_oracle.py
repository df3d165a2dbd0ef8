"""CPU: the oracle (oracle/flac_port.c, a clean-room C restatement of the
reference FLAC encoder/decoder) pinned to the reference's own fixtures and to
golden vectors produced by the reference encoder (tests/golden/make_golden.py).

Nothing here needs a GPU.  When the reference build oracle/_ref/flacenc is
present (this container only), a few extra cases compare against it live.
"""
import hashlib
import json
import os
import struct
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_port
import signals

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
VECTORS = json.load(open(os.path.join(GOLDEN, "flac_vectors.json")))["vectors"]


def make_pcm(v):
    if v["kind"] == "fsd":
        pats = signals.PATTERNS
        mono = signals.fsd(pats[v["seed"] % len(pats)], v["n"], v["bps"])
        return np.repeat(mono[:, None], v["channels"], 1).reshape(-1).astype(np.int32)
    return signals.make(v["kind"], v["n"], v["channels"], v["bps"], seed=v["seed"])


@pytest.mark.parametrize("preset", sorted(oracle_port.PRESETS))
def test_golden_vectors(preset):
    """reference-encoder sha256 for presets 0..8 x {1,2,6} ch x {8,16,24} bit"""
    cases = [v for v in VECTORS if v["preset"] == preset]
    assert cases
    for v in cases:
        pcm = make_pcm(v)
        assert len(pcm) // v["channels"] == v["frames"]
        data, _ = oracle_port.encode(pcm, v["channels"], v["bps"], 44100,
                                     **oracle_port.PRESETS[preset])
        assert len(data) == v["bytes"], v["name"]
        assert hashlib.sha256(data).hexdigest() == v["sha256"], v["name"]


def test_golden_vectors_big_blocks():
    """reference-encoder sha256 for block sizes 4608..65535 and partition
    orders up to 15 (tests/golden/make_golden_big.py)"""
    vecs = json.load(open(os.path.join(GOLDEN, "flac_vectors_big.json")))["vectors"]
    assert len(vecs) == 90
    for v in vecs:
        pcm = signals.make(v["kind"], v["n"], v["channels"], v["bps"], seed=v["seed"])
        data, _ = oracle_port.encode(pcm, v["channels"], v["bps"], 44100, **v["opts"])
        assert len(data) == v["bytes"], v["name"]
        assert hashlib.sha256(data).hexdigest() == v["sha256"], v["name"]


SIZED = json.load(open(os.path.join(GOLDEN, "flac_vectors_sized.json")))["vectors"]


@pytest.mark.parametrize("preset", ["8", "5", "2", "0"])
def test_golden_vectors_sized_reads(preset):
    """reference-encoder sha256 for streams cut by short/long reads
    (explicit frame sizes, flac.c:244-274, 412-518;
    tests/golden/make_golden_sized.py)"""
    cases = [v for v in SIZED if v["preset"] == preset]
    assert len(cases) == 36
    for v in cases:
        pcm = signals.make(v["kind"], v["n"], v["channels"], v["bps"], seed=v["seed"])
        data, lst = oracle_port.encode(pcm, v["channels"], v["bps"], 44100,
                                       frame_sizes=v["read_sizes"],
                                       **oracle_port.PRESETS[preset])
        assert [n for _, n in lst] == v["frame_lengths"], v["name"]
        assert oracle_port.cut_frames(v["n"], oracle_port.PRESETS[preset]["block_size"],
                                      v["read_sizes"]) == v["frame_lengths"]
        assert len(data) == v["bytes"], v["name"]
        assert hashlib.sha256(data).hexdigest() == v["sha256"], v["name"]
        if max(v["frame_lengths"]) <= oracle_port.PRESETS[preset]["block_size"]:
            # (a longer frame exceeds STREAMINFO's maximum block size, which
            # the reference writes as the option: its decoder rejects it)
            dec, _, _, _ = oracle_port.decode(data)
            assert np.array_equal(dec, pcm[:len(dec)])


def test_golden_vectors_round_trip():
    for v in VECTORS[::7]:
        pcm = make_pcm(v)
        data, _ = oracle_port.encode(pcm, v["channels"], v["bps"], 44100,
                                     **oracle_port.PRESETS[v["preset"]])
        dec, ch, bps, rate = oracle_port.decode(data)
        assert (ch, bps, rate) == (v["channels"], v["bps"], 44100)
        assert np.array_equal(dec, pcm)


def test_tone_flac_kat():
    """reference fixture test/tone.flac: its frames and STREAMINFO are
    reproduced bit-for-bit by re-encoding its PCM at FLAC-8"""
    data = open(os.path.join(GOLDEN, "tone.flac"), "rb").read()
    pcm, ch, bps, rate = oracle_port.decode(data)
    assert (ch, bps, rate) == (2, 16, 44100)
    assert len(pcm) // ch == 441000
    assert oracle_port.pcm_md5(pcm, ch, bps).hex() == "31b714792d4d6d693a226a364eacb7b6"
    blocks, frames = oracle_port.split_flac(data)
    enc, offs = oracle_port.encode(pcm, ch, bps, rate, **oracle_port.PRESETS["8"])
    eblocks, eframes = oracle_port.split_flac(enc)
    assert len(eframes) == 436221 and len(offs) == 108
    assert hashlib.sha256(eframes).hexdigest() == (
        "d65c6c5624754a5963982b104446020db3214f4213b1eb97c90c92733b1e649a")
    assert eframes == frames
    assert eblocks[0][1].hex() == ("100010000009d90011980ac442f00006baa831b714792d4d6d693a"
                                   "226a364eacb7b6")
    assert eblocks[0][1] == blocks[0][1]


def read_wav(path):
    d = open(path, "rb").read()
    assert d[:4] == b"RIFF" and d[8:12] == b"WAVE"
    i, fmt, pcm = 12, None, None
    while i < len(d):
        cid, n = d[i:i + 4], struct.unpack("<I", d[i + 4:i + 8])[0]
        if cid == b"fmt ":
            fmt = struct.unpack("<HHIIHH", d[i + 8:i + 24])
        elif cid == b"data":
            pcm = d[i + 8:i + 8 + n]
        i += 8 + n + (n & 1)
    _, ch, rate, _, _, bps = fmt
    return np.frombuffer(pcm, dtype="<i2").astype(np.int32), ch, rate, bps


def test_wav_2ch_config1():
    """BASELINE config 1: test/wav-2ch.wav -> FLAC-8"""
    pcm, ch, rate, bps = read_wav(os.path.join(GOLDEN, "wav-2ch.wav"))
    assert (ch, rate, bps, len(pcm) // ch) == (2, 44100, 16, 20)
    data, offs = oracle_port.encode(pcm, ch, bps, rate, **oracle_port.PRESETS["8"])
    assert len(data) == 4204
    assert hashlib.sha256(data).hexdigest() == (
        "bf481da91f617d3ae3b4d6d2cb1f28d6f13146d2c62f90ff0f097099e8d9beb6")
    _, frames = oracle_port.split_flac(data)
    assert hashlib.sha256(frames).hexdigest() == (
        "a561eba098e65ef2f77c4ee434547051edede0b5191c061da8ce482cabfccf34")


def test_short_and_fsd_streams_round_trip():
    opts = dict(block_size=1152, max_lpc_order=16, min_residual_partition_order=0,
                max_residual_partition_order=3, mid_side=True, adaptive_mid_side=True,
                exhaustive_model_search=True)
    for samples, ch, bps in signals.SHORT_STREAMS:
        a = np.array(samples, np.int32)
        data, _ = oracle_port.encode(a, ch, bps, 44100, **opts)
        assert np.array_equal(oracle_port.decode(data)[0], a)


def test_decoder_rejects_corruption():
    pcm = signals.make("tone", 5000, 2, 16, seed=3)
    data = bytearray(oracle_port.encode(pcm, 2, 16, 44100, **oracle_port.PRESETS["8"])[0])
    data[-10] ^= 0x40
    with pytest.raises(ValueError):
        oracle_port.decode(bytes(data))


@pytest.mark.skipif(not os.path.exists(oracle_port.REF_FLACENC),
                    reason="reference build oracle/_ref absent (GPU box)")
def test_port_matches_reference_live():
    import sys
    sys.path.insert(0, GOLDEN)
    import make_golden
    rng = np.random.default_rng(7)
    for k in range(12):
        preset = str(k % 9)
        ch, bps = [(1, 16), (2, 16), (2, 24), (6, 16), (1, 8)][k % 5]
        kind = ["tone", "noise", "chirp", "sine"][k % 4]
        n = int(rng.integers(1, 3 * 4096))
        pcm = signals.make(kind, n, ch, bps, seed=k)
        ref = make_golden.ref_encode(pcm, ch, bps, preset)
        port, _ = oracle_port.encode(pcm, ch, bps, 44100, **oracle_port.PRESETS[preset])
        assert port == ref, (preset, ch, bps, kind, n)


@pytest.mark.skipif(not os.path.exists(oracle_port.REF_FLACENC_SIZED),
                    reason="reference build oracle/_ref absent (GPU box)")
def test_port_matches_reference_sized_reads_live():
    """random read sizes through the reference's encoders_encode_flac
    (oracle/ref_sized_reads.c) against the port's flacport_encode_sizes"""
    rng = np.random.default_rng(11)
    for k in range(10):
        preset = str(k % 9)
        ch, bps = [(1, 16), (2, 16), (2, 24), (6, 24), (1, 8)][k % 5]
        sizes = [int(x) for x in rng.integers(1, 9000, int(rng.integers(1, 6)))]
        n = int(rng.integers(1, 20000))
        pcm = signals.make(["tone", "noise", "chirp"][k % 3], n, ch, bps, seed=k)
        opts = oracle_port.PRESETS[preset]
        ref = oracle_port.ref_encode_sized(pcm, ch, bps, 44100, sizes, **opts)
        port, _ = oracle_port.encode(pcm, ch, bps, 44100, frame_sizes=sizes, **opts)
        assert port == ref, (preset, ch, bps, sizes, n)
