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


def test_encode_flac_is_the_compiled_extension():
    """the drop-in entry point is the C-API function, as the reference's
    module function is its C extension (src/encoders.h:65-67)"""
    from audiotools import _encoders_c
    assert encoders.encode_flac is _encoders_c.encode_flac
    assert _encoders_c._set_segment_frames(256) == 256
    with pytest.raises(ValueError):
        _encoders_c._set_segment_frames(0)


def test_channel_mask_and_helpers():
    """ChannelMask / most_numerous / resampled_frame_count
    (reference audiotools/__init__.py:1862-2060, 5012-5031, 2805-2820)"""
    assert len(audiotools.ChannelMask(0x3F)) == 6
    assert audiotools.ChannelMask(0x33).channels() == [0x1, 0x2, 0x10, 0x20]
    assert audiotools.ChannelMask.from_channels(1) == 0x4
    with pytest.raises(ValueError):
        audiotools.ChannelMask.from_channels(3)
    assert audiotools.most_numerous([]) is None
    assert audiotools.most_numerous([44100]) == 44100
    assert audiotools.most_numerous([1, 2, 3], all_differ="x") == "x"
    assert audiotools.most_numerous([48000, 44100, 44100]) == 44100
    assert audiotools.resampled_frame_count(441000, 44100, 48000) == 480000
    assert audiotools.resampled_frame_count(10, 44100, 44100) == 10
    assert audiotools.resampled_frame_count(1, 48000, 44100) == 0
    assert audiotools.resampled_frame_count(123457, 44100, 8000) == 123457 * 8000 // 44100


@pytest.mark.parametrize("src,dst,chain", [
    ((44100, 2, 0x3, 24), (48000, 2, 0x3, 16), ["BPSConverter", "Resampler"]),
    ((44100, 6, 0x3F, 16), (44100, 1, 0x4, 16), ["Averager", "Downmixer"]),
    ((44100, 2, 0x3, 16), (44100, 1, 0, 16), ["Averager"]),
    ((48000, 6, 0x3F, 24), (44100, 2, 0x3, 16), ["BPSConverter", "Resampler", "Downmixer"]),
    ((44100, 6, 0x3F, 16), (44100, 4, 0x33, 16), ["RemaskedPCMReader"]),
    ((44100, 1, 0x4, 16), (44100, 2, 0x3, 8), ["BPSConverter", "ReorderedPCMReader"]),
    ((44100, 2, 0x3, 16), (44100, 2, 0x3, 16), []),
])
def test_pcmconverter_composition(src, dst, chain):
    """PCMConverter's stage order (reference audiotools/__init__.py:
    2761-2802): channels, then Resampler, then BPSConverter (outermost)"""
    base = audiotools.FrameListReader(np.zeros(10 * src[1], np.int32), src[0], src[1], src[3],
                                      channel_mask=src[2])
    r = audiotools.PCMConverter(base, *dst)
    names = []
    while r is not base:
        names.append(type(r).__name__)
        r = r.pcmreader
    assert names == chain


def test_pcmconverter_rejects():
    base = audiotools.FrameListReader(np.zeros(4, np.int32), 44100, 2, 16, channel_mask=0x3)
    for args in [(0, 2, 0x3, 16), (44100, 0, 0x3, 16), (44100, 2, 0x3, 12),
                 (44100, 2, 0x7, 16)]:
        with pytest.raises(ValueError):
            audiotools.PCMConverter(base, *args)


def test_remasked_reader_maps_speakers():
    """RemaskedPCMReader forwards matching speakers and fills the rest
    with silence (reference audiotools/__init__.py:2249-2262)"""
    x = np.arange(30, dtype=np.int32)  # 5 frames x 6 channels (0x3F)
    r = audiotools.RemaskedPCMReader(
        audiotools.FrameListReader(x, 44100, 6, 16, channel_mask=0x3F), 4, 0x1 | 0x2 | 0x100 | 0x10)
    fl = r.read(10)
    got = np.asarray(fl.samples).reshape(-1, 4)
    src = x.reshape(-1, 6)
    assert np.array_equal(got[:, 0], src[:, 0]) and np.array_equal(got[:, 1], src[:, 1])
    assert np.array_equal(got[:, 2], src[:, 4])      # back_left 0x10 -> 5th input channel
    assert not got[:, 3].any()                       # back_center 0x100: absent, silent
