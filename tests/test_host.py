"""CPU: the Python host layer that mirrors the reference interface on the
encode path — pcm.FrameList, the PCMReader family, and encode_flac's
reader-draining / validation logic (reference src/encoders/flac.c:44-121,
244-274; src/pcmconv.c:244-248) — up to the point where the GPU is called."""
import io

import numpy as np
import pytest

import audiotools
from audiotools import encoders, pcm


def test_framelist_bytes_round_trip():
    for bps in (8, 16, 24):
        rng = np.random.default_rng(bps)
        vals = rng.integers(-(1 << (bps - 1)), 1 << (bps - 1), 60)
        fl = pcm.from_list(vals.tolist(), 2, bps)
        for be in (False, True):
            for signed in (True, False):
                b = fl.to_bytes(be, signed)
                assert len(b) == 60 * bps // 8
                assert pcm.FrameList(b, 2, bps, be, signed) == fl


def test_framelist_le_signed_layout():
    fl = pcm.from_list([1, -1, 256, -32768], 2, 16)
    assert fl.to_bytes(False, True) == bytes([1, 0, 0xFF, 0xFF, 0, 1, 0, 0x80])
    assert fl.frames == 2 and fl.channels == 2
    assert list(fl.frame(1)) == [256, -32768]
    assert list(fl.channel(1)) == [-1, -32768]


def test_framelist_errors():
    with pytest.raises(ValueError):
        pcm.FrameList(b"\x00\x00\x00", 1, 16)
    with pytest.raises(ValueError):
        pcm.from_list([1, 2, 3], 2, 16)
    with pytest.raises(ValueError):
        pcm.from_list([40000], 1, 16)
    with pytest.raises(TypeError):
        pcm.from_list([1, 2], 2, 16) + [1, 2]
    with pytest.raises(ValueError):
        pcm.from_list([1, 2], 2, 16) + pcm.from_list([1, 2], 1, 16)


def test_split_and_channels():
    fl = pcm.from_list(list(range(20)), 2, 16)
    head, tail = fl.split(3)
    assert head.frames == 3 and tail.frames == 7
    assert head + tail == fl
    assert pcm.from_channels([fl.channel(0), fl.channel(1)]) == fl
    assert pcm.from_frames([fl.frame(i) for i in range(fl.frames)]) == fl


def test_buffered_reader_exact_counts():
    raw = pcm.from_list(list(range(-500, 500)), 2, 16).to_bytes(False, True)
    r = audiotools.BufferedPCMReader(
        audiotools.PCMReader(io.BytesIO(raw), 44100, 2, 3, 16))
    sizes = []
    while True:
        fl = r.read(128)
        if fl.frames == 0:
            break
        sizes.append(fl.frames)
    assert sizes == [128, 128, 128, 116]
    r.close()
    with pytest.raises(ValueError):
        r.read(1)


def test_collect_mirrors_reference_frame_loop():
    samples = np.arange(2 * 10000, dtype=np.int32) % 1000
    r = audiotools.BufferedPCMReader(audiotools.FrameListReader(samples, 44100, 2, 16))
    got, sizes = encoders._collect(r, 4096)
    assert sizes == [4096, 4096, 1808]
    assert np.array_equal(got, samples)
    assert encoders._frame_sizes_or_none(sizes, 4096) is None
    # an unbuffered reader that returns short reads: frames are cut there
    r = audiotools.FrameListReader(samples, 44100, 2, 16)
    got, sizes = encoders._collect(_ShortReads(r, [4096, 1000, 4096]), 4096)
    assert sizes == [4096, 1000, 4096, 808]
    assert list(encoders._frame_sizes_or_none(sizes, 4096)) == sizes


class _ShortReads(object):
    def __init__(self, r, pattern):
        self.r, self.pattern, self.i = r, pattern, 0
        self.sample_rate, self.channels = r.sample_rate, r.channels
        self.bits_per_sample, self.channel_mask = r.bits_per_sample, r.channel_mask

    def read(self, n):
        k = self.pattern[self.i] if self.i < len(self.pattern) else n
        self.i += 1
        return self.r.read(min(n, k))

    def close(self):
        pass


class _NotFrameList(object):
    sample_rate, channels, bits_per_sample, channel_mask = 44100, 2, 16, 3

    def read(self, n):
        return [0, 0]

    def close(self):
        pass


def test_encode_flac_rejects_non_framelist(tmp_path):
    """read() must return pcm.FrameList (reference pcmconv.c:244-248)"""
    with pytest.raises(TypeError):
        encoders.encode_flac(str(tmp_path / "x.flac"), _NotFrameList(), 4096, 12, 0, 6)


def test_encode_flac_reader_errors_propagate(tmp_path):
    r = audiotools.PCMReaderError(u"boom", 44100, 2, 3, 16)
    with pytest.raises(ValueError):
        encoders.encode_flac(str(tmp_path / "x.flac"), r, 4096, 12, 0, 6)


def test_encode_flac_unwritable_path():
    """fopen failure -> IOError/OSError with errno and filename (flac.c:114-116)"""
    r = audiotools.FrameListReader(np.zeros(20, np.int32), 44100, 2, 16)
    with pytest.raises(OSError) as e:
        encoders.encode_flac("/nonexistent-dir/x.flac", r, 4096, 12, 0, 6)
    assert e.value.filename == "/nonexistent-dir/x.flac"


def test_batch_requires_matching_formats(tmp_path):
    a = audiotools.FrameListReader(np.zeros(20, np.int32), 44100, 2, 16)
    b = audiotools.FrameListReader(np.zeros(20, np.int32), 48000, 2, 16)
    with pytest.raises(ValueError):
        encoders.encode_flac_batch([str(tmp_path / "a"), str(tmp_path / "b")], [a, b],
                                   4096, 12, 0, 6)


class _SegmentEngine(object):
    """stands in for the GPU engine: records the segments encode_flac hands
    over and returns one 10-byte frame per PCM frame list"""

    def __init__(self):
        self.calls = []

    def encode_frames(self, opts, pcm_, channels, bps, rate, first, sizes):
        self.calls.append((pcm_.copy(), first, list(sizes)))
        return np.zeros(10 * len(sizes), np.uint8), np.full(len(sizes), 10, np.uint32)


@pytest.mark.parametrize("bps", [8, 16, 24])
def test_encode_flac_streaming_segments_and_md5(tmp_path, monkeypatch, bps):
    """the streaming path (flac.c:244-274): SEGMENT_FRAMES frames per engine
    call, numbered on, in order; STREAMINFO's MD5 is the MD5 of the whole
    stream's little-endian sample bytes (hashed per segment on a thread)"""
    import hashlib
    from audiotools import _atgpu
    eng = _SegmentEngine()
    monkeypatch.setattr(_atgpu, "engine", lambda: eng)
    rng = np.random.default_rng(bps)
    n = 2 * (2 * encoders.SEGMENT_FRAMES * 256 + 1000)  # two full segments + a tail
    lim = 1 << (bps - 1)
    samples = rng.integers(-lim, lim, n).astype(np.int32)
    r = audiotools.BufferedPCMReader(audiotools.FrameListReader(samples, 44100, 2, bps))
    out = tmp_path / "s.flac"
    offs = encoders.encode_flac(str(out), r, 256, 8, 0, 5)
    nfr = (n // 2 + 255) // 256
    assert len(offs) == nfr
    assert [c[1] for c in eng.calls] == [0, encoders.SEGMENT_FRAMES, 2 * encoders.SEGMENT_FRAMES]
    got = np.concatenate([c[0].astype(np.int32) for c in eng.calls])
    assert np.array_equal(got, samples)
    data = out.read_bytes()
    assert data[:4] == b"fLaC"
    md5 = hashlib.md5(pcm.FrameList._wrap(samples, 2, bps).to_bytes(False, True)).digest()
    assert data[26:42] == md5
    # frame byte offsets follow the stream header, 10 bytes apart
    assert [o[0] for o in offs[:3]] == [0, 10, 20]
