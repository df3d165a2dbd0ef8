"""CPU: the track2track / trackverify callers' host logic.

Restates the reference's own tests where they exist:
  * WaveAudio.verify / init on truncated and malformed files
    (test/test_formats.py:5355-5497), on the reference's wav-8bit, wav-1ch,
    wav-2ch and wav-6ch fixtures, plus wav-misordered (data before fmt);
  * FloatFrameList (test/test_core.py:1834-1966);
  * the ID3v2 prefix skip on flac-id3.flac / flac-id3-2.flac, against the
    lengths tests/golden/make_id3_golden.py recorded with the reference
    decoder.
Host work only (RIFF parsing, byte writers, FloatFrameList); nothing here
launches a kernel -- the FLAC legs of convert / verify are in
tests/test_gpu_callers.py.
"""
import io
import json
import os

import pytest

import audiotools
from audiotools import pcm
from audiotools.id3 import skip_id3v2_comment
from audiotools.wav import RIFF_Chunk, WaveAudio

HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "golden", "fixtures")
WAVS = {"wav-8bit.wav": os.path.join(FIX, "wav-8bit.wav"),
        "wav-1ch.wav": os.path.join(FIX, "wav-1ch.wav"),
        "wav-2ch.wav": os.path.join(HERE, "golden", "wav-2ch.wav"),
        "wav-6ch.wav": os.path.join(FIX, "wav-6ch.wav")}

FMT = RIFF_Chunk(b"fmt ", 16, b"\x01\x00\x01\x00D\xac\x00\x00\x88X\x01\x00\x02\x00\x10\x00")
DATA = RIFF_Chunk(b"data", 26, b"\x00\x00\x01\x00\x02\x00\x03\x00\x02\x00\x01\x00\x00\x00"
                                b"\xff\xff\xfe\xff\xfd\xff\xfe\xff\xff\xff\x00\x00")


@pytest.mark.parametrize("name", sorted(WAVS))
def test_wave_fixture_verifies(name):
    w = WaveAudio(WAVS[name])
    assert w.verify() is True
    assert w.lossless()
    want = {"wav-8bit.wav": (1, 8, 0x4), "wav-1ch.wav": (1, 16, 0x4),
            "wav-2ch.wav": (2, 16, 0x3), "wav-6ch.wav": (6, 16, 0x3F)}[name]
    assert (w.channels(), w.bits_per_sample(), int(w.channel_mask())) == want
    assert w.sample_rate() == 44100


@pytest.mark.parametrize("name", sorted(WAVS))
def test_wave_truncated_underfoot_fails_verify(name, tmp_path):
    """test_formats.py:5358-5378: the file shrinks after WaveAudio opened it"""
    data = open(WAVS[name], "rb").read()
    fn = str(tmp_path / "t.wav")
    open(fn, "wb").write(data)
    wave = WaveAudio(fn)
    for i in range(len(data)):
        with open(fn, "wb") as f:
            f.write(data[:i])
        with pytest.raises(audiotools.InvalidFile):
            wave.verify()


@pytest.mark.parametrize("fmt_size,name", [(0x24, "wav-8bit.wav"), (0x24, "wav-1ch.wav"),
                                           (0x24, "wav-2ch.wav"), (0x3C, "wav-6ch.wav")])
def test_wave_truncated_fmt_fails_init(fmt_size, name, tmp_path):
    """test_formats.py:5400-5423"""
    data = open(WAVS[name], "rb").read()
    fn = str(tmp_path / "t.wav")
    for i in range(fmt_size + 8):
        open(fn, "wb").write(data[:i])
        with pytest.raises(audiotools.InvalidFile):
            WaveAudio(fn)


def test_wave_malformed_chunks_fail_verify(tmp_path):
    """test_formats.py:5425-5497: non-ASCII chunk id, multiple fmt, multiple
    data, data before fmt, no fmt"""
    fn = str(tmp_path / "t.wav")
    chunks = list(WaveAudio(WAVS["wav-2ch.wav"]).chunks()) + [RIFF_Chunk(b"fooz", 10, b"\0" * 10)]
    WaveAudio.wave_from_chunks(fn, iter(chunks))
    assert WaveAudio(fn).verify()
    raw = bytearray(open(fn, "rb").read())
    raw[-15] = 0
    open(fn, "wb").write(bytes(raw))
    with pytest.raises(audiotools.InvalidFile):
        WaveAudio(fn).verify()
    for chunks in ([FMT, FMT, DATA], [FMT, DATA, FMT], [FMT, DATA, DATA], [DATA, FMT], [DATA]):
        WaveAudio.wave_from_chunks(fn, chunks)
        with pytest.raises(audiotools.InvalidFile):
            WaveAudio(fn).verify()
    WaveAudio.wave_from_chunks(fn, [FMT, DATA])
    assert WaveAudio(fn).verify()


def test_wave_misordered_fixture():
    """the reference's wav-misordered.wav (data chunk before fmt): WaveAudio
    opens it, but WaveReader refuses it and verify() reports it"""
    fn = os.path.join(FIX, "wav-misordered.wav")
    w = WaveAudio(fn)
    assert (w.channels(), w.bits_per_sample(), w.total_frames()) == (1, 16, 25)
    with pytest.raises(ValueError, match="data chunk found before fmt"):
        w.to_pcm()
    with pytest.raises(audiotools.InvalidFile, match="data chunk found before fmt"):
        w.verify()


@pytest.mark.parametrize("name", sorted(WAVS))
def test_wave_convert_to_wave_is_identity(name, tmp_path):
    """AudioFile.convert -> WaveAudio.from_pcm reproduces the fixture byte
    for byte (every fixture has an even frame count), with progress"""
    src = WaveAudio(WAVS[name])
    seen = []
    out = src.convert(str(tmp_path / "o.wav"), WaveAudio,
                      progress=lambda cur, tot: seen.append((cur, tot)))
    assert open(out.filename, "rb").read() == open(WAVS[name], "rb").read()
    assert seen and seen[-1] == (src.total_frames(), src.total_frames())
    assert out == src
    assert audiotools.pcm_frame_cmp(src.to_pcm(), out.to_pcm()) is None


def test_wave_from_pcm_frame_count_mismatch(tmp_path):
    src = WaveAudio(WAVS["wav-2ch.wav"])
    fn = str(tmp_path / "o.wav")
    with pytest.raises(audiotools.EncodingError):
        WaveAudio.from_pcm(fn, src.to_pcm(), total_pcm_frames=src.total_frames() + 1)
    assert not os.path.exists(fn)


def test_wave_from_pcm_odd_frames_pad_and_header(tmp_path):
    """wav.py:705-725: odd FRAME counts get a pad byte, and without a
    total the header is rewritten with the counted frames"""
    fl = pcm.from_list(list(range(6)), 2, 16)
    r = audiotools.FrameListReader(fl, 44100, 2, 16, 0x3)
    fn = str(tmp_path / "o.wav")
    w = WaveAudio.from_pcm(fn, r)
    data = open(fn, "rb").read()
    assert len(data) == 44 + 12 + 1
    assert w.total_frames() == 3
    assert data[4:8] == (36 + 12).to_bytes(4, "little")


def test_pcm_frame_cmp_reports_first_mismatch():
    a = pcm.from_list(list(range(20)), 2, 16)
    b = pcm.from_list(list(range(14)) + [0] + list(range(15, 20)), 2, 16)
    mk = lambda fl: audiotools.FrameListReader(fl, 44100, 2, 16, 0x3)  # noqa: E731
    assert audiotools.pcm_frame_cmp(mk(a), mk(a)) is None
    assert audiotools.pcm_frame_cmp(mk(a), mk(b)) == 7
    # a shorter stream whose frames all match: the reference's for/else
    # returns the last compared index (n - 1), not n (__init__.py:2471-2475)
    assert audiotools.pcm_frame_cmp(mk(a), mk(a.split(6)[0])) == 5
    assert audiotools.pcm_cmp(mk(a), mk(a)) and not audiotools.pcm_cmp(mk(a), mk(b))


def test_id3v2_skip_matches_recorded_prefixes():
    vec = json.load(open(os.path.join(HERE, "golden", "id3_vectors.json")))
    for name, v in vec.items():
        data = open(os.path.join(FIX, name), "rb").read()
        f = io.BytesIO(data)
        assert skip_id3v2_comment(f) == v["id3v2_bytes"]
        assert f.tell() == v["id3v2_bytes"]
        assert f.read(4) == b"fLaC"
    f = io.BytesIO(b"fLaC....")
    assert skip_id3v2_comment(f) == 0 and f.tell() == 0
    # an invalid sync-safe size: no skip, position restored
    f = io.BytesIO(b"ID3\x03\x00\x00\x00\x00\x80\x00fLaC")
    assert skip_id3v2_comment(f) == 0 and f.tell() == 0


def test_float_framelist_basics():
    """test_core.py:1856-1966"""
    with pytest.raises(ValueError):
        pcm.FloatFrameList([1.0, 2.0, 3.0], 2)
    with pytest.raises(TypeError):
        pcm.FloatFrameList(0, 1)
    with pytest.raises(TypeError):
        pcm.FloatFrameList([1.0, 2.0, "a"], 1)
    for bad in ([0.0] * 5, [0.0] * 3):
        with pytest.raises(ValueError):
            pcm.FloatFrameList(bad, 2)
    for ch in (0, -1):
        with pytest.raises(ValueError):
            pcm.FloatFrameList([0.0] * 4, ch)
    f = pcm.FloatFrameList([float(i) for i in range(8)], 2)
    assert (len(f), f.channels, f.frames) == (8, 2, 4)
    with pytest.raises(IndexError):
        f[9]
    for i in range(4):
        assert list(f.frame(i)) == [2.0 * i, 2.0 * i + 1]
    for bad in (4, -1):
        with pytest.raises(IndexError):
            f.frame(bad)
    assert list(f.channel(0)) == [0.0, 2.0, 4.0, 6.0]
    assert list(f.channel(1)) == [1.0, 3.0, 5.0, 7.0]
    for bad in (2, -1):
        with pytest.raises(IndexError):
            f.channel(bad)
    assert list(f) == list(pcm.from_float_frames([f.frame(i) for i in range(4)]))
    assert list(f) == list(pcm.from_float_channels([f.channel(0), f.channel(1)]))
    with pytest.raises(IndexError):
        f.split(-1)
    f1, f2 = f.split(2)
    assert (list(f1), list(f2)) == ([0.0, 1.0, 2.0, 3.0], [4.0, 5.0, 6.0, 7.0])
    f1, f2 = f.split(0)
    assert (list(f1), list(f2)) == ([], list(f))
    f1, f2 = f.split(20)
    assert (list(f1), list(f2)) == (list(f), [])
    for i in range(f.frames):
        f1, f2 = f.split(i)
        assert len(f1) == i * f.channels and list(f1 + f2) == list(f)
    with pytest.raises(TypeError):
        pcm.FloatFrameList([float(i) for i in range(10)], 2) + [1, 2, 3]
    lst = [float(i - 128) / (1 << 7) for i in range(0, 1 << 8)]
    for bps in (8, 16, 24):
        assert lst == list(pcm.FloatFrameList(lst, 1).to_int(bps).to_float())
    for bps in (8, 16, 24):
        lst = list(range(0, 1 << bps, 4))
        assert ([i - (1 << (bps - 1)) for i in lst] ==
                list(pcm.from_list(lst, 1, bps, False).to_float().to_int(bps)))
        lst = list(range(-(1 << (bps - 1)), (1 << (bps - 1)) - 1, 4))
        assert lst == list(pcm.from_list(lst, 1, bps, True).to_float().to_int(bps))


def test_float_to_int_clamps_like_the_c_cast():
    """(int)(x * 2^(bps-1)) then MIN/MAX (src/pcm.c:1221-1224): values past
    int32 and NaN become INT_MIN (x86 cvttsd2si) and clamp to the minimum"""
    f = pcm.FloatFrameList([1.5, -1.5, 0.999999, -0.3, float("nan"), 1e30, -1e30], 1)
    assert list(f.to_int(16)) == [32767, -32768, 32767, -9830, -32768, -32768, -32768]


def test_frame_count_at_least_one():
    """FrameList.frame_count (src/pcm.c:618-631)"""
    fl = pcm.from_list([0, 0], 2, 16)
    assert fl.frame_count(0) == 1 and fl.frame_count(3) == 1 and fl.frame_count(9) == 2


def test_flac_audio_reads_streaminfo_past_id3():
    """FlacAudio.__init__ steps over the ID3v2 prefix before STREAMINFO
    (flac.py:2420-2470); metadata parsing is host code in libatgpu"""
    vec = json.load(open(os.path.join(HERE, "golden", "id3_vectors.json")))
    for name, v in vec.items():
        f = audiotools.FlacAudio(os.path.join(FIX, name))
        assert (f.channels(), f.bits_per_sample(), f.total_frames()) == (
            v["channels"], v["bits_per_sample"], v["pcm_frames"])
        assert f.lossless() and int(f.channel_mask()) == 0x3


def test_flac_audio_channel_mask_rules():
    """flac.py:1284-1341: the comment's mask when its speaker count fits,
    ChannelMask(0) when it does not, FLAC's default without one"""
    from audiotools.flac import _FLAC_MASKS, _set_comment
    body = (4).to_bytes(4, "little") + b"test" + (0).to_bytes(4, "little")
    body = _set_comment(body, u"WAVEFORMATEXTENSIBLE_CHANNEL_MASK", u"0x0607")
    from audiotools.flac import _comment_values
    assert _comment_values(body, u"waveformatextensible_channel_mask") == ["0x0607"]
    assert _FLAC_MASKS[6] == 0x3F and _FLAC_MASKS[8] == 0x63F and _FLAC_MASKS[7] == 0x70F
    assert len(audiotools.ChannelMask(_FLAC_MASKS[7])) == 7
