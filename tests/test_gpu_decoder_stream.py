"""GPU: FlacDecoder (the C extension, csrc/ext/decoders_c.c) decodes in
bounded segments (8 MiB of compressed data per GPU call by default) -- windows that end inside a
frame resume at that frame (the decode's walk_end), errors are raised at the
frame where the reference's read() raises them (src/decoders/flac.c:174-285)
and the STREAMINFO MD5 is chained over the segments on the host
(flac.c:479-493).  With a window a few frames long every read crosses
segment boundaries; frames, errors and offsets() must equal the
one-segment decode and the CPU oracle."""
import numpy as np
import pytest

import decode_cases
import oracle_port
import signals

pytestmark = pytest.mark.gpu


def _frames(dec):
    out, err = [], None
    try:
        while True:
            fl = dec.read(4096)
            if not len(fl):
                break
            out.append(np.array(fl.samples))
    except (ValueError, IOError) as e:
        err = (type(e).__name__, str(e))
    return out, err


class _Segments(object):
    """decoders with a settable segment size (the extension's test hook)"""

    def __init__(self):
        from audiotools import _decoders_c, decoders
        self.FlacDecoder = decoders.FlacDecoder
        self._c = _decoders_c

    @property
    def SEGMENT_BYTES(self):
        old = self._c._set_segment_bytes(1)
        self._c._set_segment_bytes(old)
        return old

    @SEGMENT_BYTES.setter
    def SEGMENT_BYTES(self, n):
        self._c._set_segment_bytes(n)


@pytest.fixture
def small_segments():
    d = _Segments()
    old = d.SEGMENT_BYTES
    yield d
    d.SEGMENT_BYTES = old


@pytest.mark.parametrize("seg", [1 << 10, 5000, 1 << 16])
def test_segmented_read_matches_whole(small_segments, seg):
    decoders = small_segments
    from audiotools import _atgpu
    eng = _atgpu.engine()
    x = signals.make("chirp", 4096 * 9 + 123, 2, 16, seed=7)
    opts = dict(oracle_port.PRESETS["8"])
    img, _ = oracle_port.encode(x, 2, 16, 44100, **opts)
    decoders.SEGMENT_BYTES = 1 << 30
    whole, err0 = _frames(decoders.FlacDecoder(img))
    decoders.SEGMENT_BYTES = seg
    got, err = _frames(decoders.FlacDecoder(img))
    assert err0 is None and err is None
    assert len(got) == len(whole) == 10
    assert all(np.array_equal(a, b) for a, b in zip(got, whole))
    assert np.array_equal(np.concatenate(got), x)
    del eng


def test_segmented_md5_mismatch_raises_at_end(small_segments):
    decoders = small_segments
    x = signals.make("tone", 4096 * 5, 1, 16, seed=3)
    img = bytearray(oracle_port.encode(x, 1, 16, 44100, **oracle_port.PRESETS["5"])[0])
    img[26] ^= 1  # STREAMINFO MD5
    decoders.SEGMENT_BYTES = 2000
    got, err = _frames(decoders.FlacDecoder(bytes(img)))
    assert len(got) == 5 and err is not None and err[0] == "ValueError"


@pytest.mark.parametrize("c", [c for c in decode_cases.load_cases()
                               if c["file"] in ("flac-allframes.flac", "flac-seektable.flac")
                               and (c["cut"] is not None or c["xor"])][:24],
                         ids=lambda c: c["name"])
def test_segmented_errors_like_whole(small_segments, c):
    """corrupted / truncated reference fixtures: the same frames, then the
    same exception, with 300-byte windows as with one window"""
    decoders = small_segments
    data = decode_cases.case_bytes(c)
    decoders.SEGMENT_BYTES = 1 << 30
    try:
        whole, err0 = _frames(decoders.FlacDecoder(data))
    except (ValueError, IOError):
        return  # metadata errors: no frames either way
    decoders.SEGMENT_BYTES = 300
    got, err = _frames(decoders.FlacDecoder(data))
    assert len(got) == len(whole), c["name"]
    assert all(np.array_equal(a, b) for a, b in zip(got, whole)), c["name"]
    assert err == err0, c["name"]


def test_segmented_offsets(small_segments):
    decoders = small_segments
    x = signals.make("noise", 4096 * 6 + 5, 2, 16, seed=11)
    img, woffs = oracle_port.encode(x, 2, 16, 44100, **oracle_port.PRESETS["8"])
    decoders.SEGMENT_BYTES = 3000
    d = decoders.FlacDecoder(img)
    d.read(4096)
    d.read(4096)
    offs = d.offsets()
    base = woffs[2][0]
    assert [o for o, _ in offs] == [o - base for o, _ in woffs[2:]]
    assert not len(d.read(4096))
