"""GPU: FlacDecoder.seek and offsets() semantics (reference
src/decoders/flac.c:287-356 seek, :365-443 offsets).

* test_seek_like_reference restates the reference's own AudioFile.test_seek
  (test/test_formats.py:760-834) on a FLAC file the GPU encoder wrote through
  FlacAudio.from_pcm: negative seeks raise, seek(0) rewinds to identical
  PCM, random seeks land on a seekpoint <= the request and then read exactly
  the source window, huge seeks work, closed streams raise;
* the reference's flac-seektable.flac fixture (seekpoints at odd byte
  offsets) is checked point by point against the CPU oracle decoder started
  at the same byte with the same remaining-samples count;
* offsets() walks from the current position, never checks CRC-16 (the
  oracle with check_crc=0 is the reference's walk), and returns [] once the
  stream has been read.
"""
import hashlib
import random

import numpy as np
import pytest

import decode_cases
import oracle_port
import signals

pytestmark = pytest.mark.gpu


def _read_all(dec):
    out = []
    while True:
        fl = dec.read(4096)
        if not len(fl):
            break
        out.append(fl.samples)
    return np.concatenate(out) if out else np.zeros(0, np.int32)


def test_seek_like_reference(tmp_path):
    import audiotools
    from audiotools import flac
    total = 44100 * 60 * 3
    fn = str(tmp_path / "seek.flac")
    # a deterministic non-silent signal (the reference uses silence; a
    # varying one also proves the window is the right one)
    pcm = signals.make("tone", total, 2, 16, seed=11)
    track = flac.FlacAudio.from_pcm(fn, audiotools.FrameListReader(pcm, 44100, 2, 16, 0x3),
                                    "8", total_pcm_frames=total)
    r = track.to_pcm()
    first = hashlib.md5(_read_all(r).tobytes()).digest()
    with pytest.raises(ValueError):
        r.seek(-1)
    assert r.seek(0) == 0
    assert hashlib.md5(_read_all(r).tobytes()).digest() == first
    rng = random.Random(7)
    for _ in range(10):
        position = rng.randrange(0, total)
        actual = r.seek(position)
        assert actual <= position
        assert actual % 4096 == 0
        got = _read_all(r)
        assert np.array_equal(got, pcm[actual * 2:])
    for value in (2 ** 31, 2 ** 34, 2 ** 38):
        assert r.seek(value) <= value
    r.close()
    with pytest.raises(ValueError):
        r.seek(0)


def test_seektable_fixture_points_vs_oracle(tmp_path):
    from audiotools import decoders
    data = open(decode_cases.FIX + "/flac-seektable.flac", "rb").read()
    rc, info, pts, si = oracle_port.read_metadata(data)
    assert rc == 0 and len(pts) == 6
    fn = tmp_path / "st.flac"
    fn.write_bytes(data)
    for target in (0, 1, 438272, 500000, 2203648, 2645999, 10 ** 9):
        dec = decoders.FlacDecoder(str(fn))
        got_sample = dec.seek(target)
        sample, byte = 0, 0
        for s, b, _ in pts:
            if s <= target:
                sample, byte = s, b
            else:
                break
        assert got_sample == sample
        want = oracle_port.decode_frames(data, start=si.frames_offset + byte,
                                         remaining=si.total_samples - sample)
        frames, err = [], None
        try:
            while True:
                fl = dec.read(4096)
                if not len(fl):
                    break
                frames.append(fl.samples)
        except (ValueError, IOError) as e:
            err = e
        got = np.concatenate(frames) if frames else np.zeros(0, np.int32)
        assert np.array_equal(got, np.asarray(want["pcm"], np.int32)), target
        # MD5 is validated only after a seek to sample 0 (flac.c:345-352)
        if want["code"] == 0:
            assert err is None, (target, err)
        else:
            assert err is not None and decoders._atgpu.FD_MESSAGES[want["code"]] in str(err)


def test_seek_requires_file_object():
    from audiotools import decoders
    data = open(decode_cases.FIX + "/tone2.flac", "rb").read()
    dec = decoders.FlacDecoder(data)
    with pytest.raises(TypeError):
        dec.seek(0)


def test_offsets_from_current_position(tmp_path):
    from audiotools import decoders
    data = open(decode_cases.FIX + "/tone2.flac", "rb").read()
    want = [tuple(x) for x in oracle_port.decode_frames(data)["offsets"]]
    fn = tmp_path / "t.flac"
    fn.write_bytes(data)
    assert decoders.FlacDecoder(str(fn)).offsets() == want
    dec = decoders.FlacDecoder(str(fn))
    dec.read(4096)
    dec.read(4096)
    got = dec.offsets()
    base = want[2][0]
    assert got == [(o - base, b) for o, b in want[2:]]
    # the walk finished the stream: read() now returns an empty FrameList
    assert len(dec.read(4096)) == 0
    dec2 = decoders.FlacDecoder(str(fn))
    _read_all(dec2)
    assert dec2.offsets() == []


def test_offsets_ignore_frame_crc():
    """a frame whose CRC-16 is bad still has a length: offsets() lists every
    frame (the reference never checks the CRC there) while read() raises"""
    from audiotools import decoders
    bad = [c for c in decode_cases.load_cases() if c["code"] == 14]
    assert bad
    for case in bad[:8]:
        data = decode_cases.case_bytes(case)
        walk = oracle_port.decode_frames(data, check_crc=False)
        dec = decoders.FlacDecoder(data)
        if walk["code"] in (0, 16):
            assert dec.offsets() == [tuple(x) for x in walk["offsets"]], case["name"]
        else:
            with pytest.raises((ValueError, IOError)):
                dec.offsets()
        dec = decoders.FlacDecoder(data)
        n = 0
        with pytest.raises(ValueError) as e:
            while True:
                fl = dec.read(4096)
                if not len(fl):
                    break
                n += fl.frames
        assert "invalid checksum in frame" in str(e.value)
        bb = (dec.bits_per_sample + 7) // 8
        assert n * dec.channels * bb == case["pcm_bytes"], case["name"]
