"""GPU: the compiled CPython extensions over the C ABI, byte for byte.

audiotools._encoders_c.encode_flac is the reference's encoder entry point
(src/encoders/flac.c:44-121, registered src/encoders.h:65-93) compiled
against libatgpu: BASELINE config 1 (test/wav-2ch.wav through WaveReader ->
BufferedPCMReader) must reproduce the reference encoder's file
(sha256 bf481da9...), and longer / multichannel / irregularly read streams
(several 256-frame GPU segments) the oracle's bytes.
audiotools._decoders_c.FlacDecoder is the reference's decoder type
(src/decoders/flac.c:28-443) over the GPU decoder: same frames, statuses,
offsets and seeks as the Python FlacDecoder and the oracle."""
import hashlib
import os

import numpy as np
import pytest

import oracle_port
import signals

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
WAV = os.path.join(HERE, "golden", "wav-2ch.wav")
FIX = os.path.join(HERE, "golden", "fixtures")


def test_config1_through_the_extension(tmp_path):
    import audiotools
    from audiotools import _encoders_c, wav
    fn = str(tmp_path / "wav-2ch.flac")
    offsets = _encoders_c.encode_flac(fn, audiotools.BufferedPCMReader(wav.WaveReader(WAV)),
                                      **oracle_port.PRESETS["8"])
    data = open(fn, "rb").read()
    assert hashlib.sha256(data).hexdigest() == (
        "bf481da91f617d3ae3b4d6d2cb1f28d6f13146d2c62f90ff0f097099e8d9beb6")
    _, frames = oracle_port.split_flac(data)
    assert hashlib.sha256(frames).hexdigest() == (
        "a561eba098e65ef2f77c4ee434547051edede0b5191c061da8ce482cabfccf34")
    assert offsets == [(0, 20)]


class _Reads(object):
    def __init__(self, x, rate, ch, bps, sizes=()):
        import audiotools
        self._r = audiotools.FrameListReader(x, rate, ch, bps)
        self.sample_rate, self.channels, self.bits_per_sample, self.channel_mask = rate, ch, bps, 0
        self.sizes = list(sizes)
        self.closed = False

    def read(self, n):
        return self._r.read(self.sizes.pop(0) if self.sizes else n)

    def close(self):
        self.closed = True


@pytest.mark.parametrize("kind,n,ch,bps,preset", [
    ("tone", 30000, 2, 16, "8"),
    ("tone", 4096 * 300 + 11, 2, 16, "8"),      # two GPU segments
    ("tone", 4096 * 4 + 3, 6, 24, "8"),
    ("noise", 5000, 1, 8, "5"),
    ("chirp", 70000, 2, 16, "0"),
])
def test_encode_flac_extension_vs_oracle(tmp_path, kind, n, ch, bps, preset):
    from audiotools import _encoders_c
    x = signals.make(kind, n, ch, bps, seed=n)
    opts = oracle_port.PRESETS[preset]
    r = _Reads(x, 44100, ch, bps)
    fn = str(tmp_path / "x.flac")
    lst = _encoders_c.encode_flac(fn, r, **opts)
    want, wl = oracle_port.encode(x, ch, bps, 44100, **opts)
    assert r.closed
    assert open(fn, "rb").read() == want
    assert lst == wl


def test_encode_flac_extension_irregular_reads(tmp_path):
    """every read() is one frame, across the segment boundary too; the
    Python streaming encoder and the extension agree byte for byte"""
    from audiotools import _encoders_c, encoders
    sizes = [4096] * 255 + [1000, 7] + [4096] * 3 + [4095, 1]
    n = sum(sizes) + 500
    x = signals.make("tone", n, 2, 16, seed=4)
    a, b = str(tmp_path / "c.flac"), str(tmp_path / "p.flac")
    la = _encoders_c.encode_flac(a, _Reads(x, 44100, 2, 16, sizes), **oracle_port.PRESETS["8"])
    lb = encoders.encode_flac(b, _Reads(x, 44100, 2, 16, sizes), **oracle_port.PRESETS["8"])
    assert la == lb and [m for _, m in la][:len(sizes)] == sizes
    data = open(a, "rb").read()
    assert data == open(b, "rb").read()
    want, wl = oracle_port.encode(x, 2, 16, 44100, frame_sizes=sizes,
                                  **oracle_port.PRESETS["8"])
    assert data == want and la == wl
    dec, _, _, _ = oracle_port.decode(data)
    assert np.array_equal(dec, x)


def _frames(d):
    out = []
    while True:
        fl = d.read(4096)
        if not len(fl):
            return out
        out.append(np.asarray(fl.samples).copy())


def _outcome(d):
    """(frames read, the exception type and message that ended the stream)"""
    out = []
    try:
        while True:
            fl = d.read(4096)
            if not len(fl):
                return out, None
            out.append(np.asarray(fl.samples).copy())
    except (ValueError, IOError) as e:
        return out, (type(e), str(e))


def test_flac_decoder_extension_tone():
    from audiotools import _decoders_c, decoders
    fn = os.path.join(HERE, "golden", "tone.flac")
    c, p = _decoders_c.FlacDecoder(fn), decoders.FlacDecoder(fn)
    fc, fp = _frames(c), _frames(p)
    assert len(fc) == len(fp) == 108
    assert all(np.array_equal(a, b) for a, b in zip(fc, fp))
    pcm, _, _, _ = oracle_port.decode(open(fn, "rb").read())
    assert np.array_equal(np.concatenate(fc), pcm)
    assert len(c.read(4096)) == 0                  # stays finished
    c.close()
    with pytest.raises(ValueError):
        c.read(4096)
    o1 = _decoders_c.FlacDecoder(fn).offsets()
    o2 = decoders.FlacDecoder(fn).offsets()
    assert o1 == o2 and len(o1) == 108


def test_flac_decoder_extension_seek_and_errors(tmp_path):
    from audiotools import _decoders_c, decoders
    fn = os.path.join(FIX, "flac-seektable.flac")
    # the fixture's first seekpoint is (sample 0, byte 1): a seek lands one
    # byte into the first frame and read() fails there, in both decoders
    for target in (0, 1, 44100, 438272, 44100 * 30 + 5, 10 ** 9):
        c, p = _decoders_c.FlacDecoder(fn), decoders.FlacDecoder(fn)
        assert c.seek(target) == p.seek(target)
        (fc, ec), (fp, ep) = _outcome(c), _outcome(p)
        assert ec == ep
        assert len(fc) == len(fp) and all(np.array_equal(a, b) for a, b in zip(fc, fp))
    # a flipped byte inside a frame: the same error at the same frame
    data = bytearray(open(os.path.join(HERE, "golden", "tone.flac"), "rb").read())
    data[len(data) // 2] ^= 0x10
    bad = tmp_path / "bad.flac"
    bad.write_bytes(bytes(data))
    errs = []
    for d in (_decoders_c.FlacDecoder(str(bad)), decoders.FlacDecoder(str(bad))):
        n = 0
        try:
            while len(d.read(4096)):
                n += 1
            errs.append((n, None))
        except (ValueError, IOError) as e:
            errs.append((n, (type(e), str(e))))
    assert errs[0] == errs[1] and errs[0][1] is not None
