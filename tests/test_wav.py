"""CPU: audiotools.wav.WaveReader (reference audiotools/wav.py:288-553)
against the raw RIFF parse of the reference's fixture and synthetic files:
chunk walk, WAVE_FORMAT_PCM / EXTENSIBLE fmt chunks, odd chunk padding,
8-bit unsigned samples, truncation and error cases."""
import os
import struct

import numpy as np
import pytest

from test_oracle import read_wav

HERE = os.path.dirname(os.path.abspath(__file__))
WAV = os.path.join(HERE, "golden", "wav-2ch.wav")


def _riff(chunks):
    body = b"WAVE" + b"".join(cid + struct.pack("<I", len(d)) + d + (b"\0" if len(d) % 2 else b"")
                             for cid, d in chunks)
    return b"RIFF" + struct.pack("<I", len(body)) + body


def _fmt(ch, rate, bps, ext_mask=None):
    ba = ch * bps // 8
    if ext_mask is None:
        return struct.pack("<HHIIHH", 1, ch, rate, rate * ba, ba, bps)
    return struct.pack("<HHIIHHHHI", 0xFFFE, ch, rate, rate * ba, ba, bps, 22, bps,
                       ext_mask) + (b"\x01\x00\x00\x00\x00\x00\x10\x00"
                                    b"\x80\x00\x00\xaa\x00\x38\x9b\x71")


def test_reference_fixture():
    from audiotools import wav
    pcm, ch, rate, bps = read_wav(WAV)
    r = wav.WaveReader(WAV)
    assert (r.channels, r.sample_rate, r.bits_per_sample, r.channel_mask) == (2, 44100, 16, 3)
    assert r.total_pcm_frames == 20
    got = []
    while True:
        fl = r.read(7)
        if not fl.frames:
            break
        assert fl.frames <= 7
        got.append(fl.samples)
    assert np.array_equal(np.concatenate(got), pcm)
    assert r.seek(5) == 5 and np.array_equal(r.read(100).samples, pcm[10:])
    assert r.seek(10 ** 6) == 20
    with pytest.raises(ValueError):
        r.seek(-1)
    r.close()


@pytest.mark.parametrize("ch,bps,mask", [(1, 8, None), (2, 24, None), (6, 16, 0x3F),
                                         (2, 16, 0x3), (5, 16, None)])
def test_synthetic(tmp_path, ch, bps, mask):
    from audiotools import wav
    rng = np.random.default_rng(ch * 100 + bps)
    n = 101
    if bps == 8:
        raw = rng.integers(0, 256, n * ch).astype(np.uint8).tobytes()
        want = np.frombuffer(raw, np.uint8).astype(np.int32) - 128
    else:
        want = rng.integers(-(1 << (bps - 1)), 1 << (bps - 1), n * ch).astype(np.int32)
        w = bps // 8
        raw = want.astype("<i4").view(np.uint8).reshape(-1, 4)[:, :w].tobytes()
    fn = tmp_path / "x.wav"
    fn.write_bytes(_riff([(b"LIST", b"abc"), (b"fmt ", _fmt(ch, 48000, bps, mask)),
                          (b"data", raw)]))
    r = wav.WaveReader(str(fn))
    assert r.channels == ch and r.bits_per_sample == bps and r.sample_rate == 48000
    assert r.channel_mask == (mask if mask is not None else
                              {1: 0x4, 2: 0x3, 5: 0x37}[ch])
    assert np.array_equal(r.read(10 ** 6).samples, want)
    assert r.read(10).frames == 0


def test_errors(tmp_path):
    from audiotools import wav
    fn = tmp_path / "bad.wav"
    fn.write_bytes(b"RIFX" + b"\0" * 40)
    with pytest.raises(ValueError):
        wav.WaveReader(str(fn))
    fn.write_bytes(_riff([(b"data", b"\0\0"), (b"fmt ", _fmt(1, 44100, 16))]))
    with pytest.raises(ValueError):
        wav.WaveReader(str(fn))
    fn.write_bytes(_riff([(b"fmt ", _fmt(1, 44100, 16))]))
    with pytest.raises(ValueError):
        wav.WaveReader(str(fn))
    fmt = bytearray(_fmt(2, 44100, 16, 3))
    fmt[-1] ^= 1
    fn.write_bytes(_riff([(b"fmt ", bytes(fmt)), (b"data", b"\0" * 8)]))
    with pytest.raises(ValueError):
        wav.WaveReader(str(fn))
    # a data chunk that claims more than the file holds: IOError at read time
    good = _riff([(b"fmt ", _fmt(1, 44100, 16)), (b"data", b"\1\0" * 50)])
    fn.write_bytes(good[:-20])
    r = wav.WaveReader(str(fn))
    with pytest.raises(IOError):
        r.read(50)
