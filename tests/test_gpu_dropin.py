"""GPU: the drop-in callers track2track reaches (reference
audiotools/__init__.py:2729-2912) over the GPU classes.

* PCMConverter(24-bit 44.1 kHz stereo, 48000, 2, 0x3, 16) -> FlacAudio.from_pcm:
  the resampler's output equals the oracle's (MEDIUM table; parity
  unpinned), every dithered sample keeps the invariant
  out ^ (x >> 8) in {0, 1} (BPSConverter, pcmconverter.c:667-747), and the
  FLAC frames + STREAMINFO equal the port's encode of the converted PCM.
* calculate_replay_gain over tracks at mixed rates: title gains/peaks and
  the album gain equal the oracle's over the same resampled PCM and reads.
* the reference's own converter / ReplayGain tests restated
  (test/test_core.py:838-941, 4336-4424): conversion attributes and
  duration over SHORT_PCM_COMBINATIONS, close semantics, valid rates,
  a gain-applied file measuring quieter.
"""
import numpy as np
import pytest

import oracle_port
import signals

pytestmark = pytest.mark.gpu


class _Track(object):
    """an AudioFile stand-in over in-memory PCM (sample_rate(), channels(),
    total_frames(), to_pcm())"""

    def __init__(self, samples, rate, channels, bps, mask=0):
        self.samples, self.rate, self.ch, self.bps, self.mask = samples, rate, channels, bps, mask

    def sample_rate(self):
        return self.rate

    def channels(self):
        return self.ch

    def total_frames(self):
        return len(self.samples) // self.ch

    def to_pcm(self):
        import audiotools
        return audiotools.FrameListReader(self.samples, self.rate, self.ch, self.bps,
                                          channel_mask=self.mask)


class _Recorder(object):
    """a PCMReader passing reads through and keeping them"""

    def __init__(self, r):
        self.r = r
        self.sample_rate, self.channels = r.sample_rate, r.channels
        self.channel_mask, self.bits_per_sample = r.channel_mask, r.bits_per_sample
        self.parts = []

    def read(self, n):
        fl = self.r.read(n)
        self.parts.append(np.array(fl.samples))
        return fl

    def close(self):
        self.r.close()


def test_pcmconverter_chain_to_flac(tmp_path):
    import audiotools
    from audiotools.flac import FlacAudio
    x = signals.make("tone", 44100 * 2 + 333, 2, 24, seed=21)
    src = audiotools.FrameListReader(x, 44100, 2, 24, channel_mask=0x3)
    conv = audiotools.PCMConverter(src, 48000, 2, 0x3, 16)
    # the reference's composition: Resampler, then BPSConverter
    assert type(conv).__name__ == "BPSConverter"
    assert type(conv.pcmreader).__name__ == "Resampler"
    rec = _Recorder(conv)
    fn = str(tmp_path / "c.flac")
    FlacAudio.from_pcm(fn, rec, compression="8")
    out = np.concatenate(rec.parts)
    # the resampler stage against the oracle (4096-frame reads of the source)
    rs = oracle_port.resample(x, 2, 24, 48000 / 44100)
    assert len(out) == len(rs)
    # dither invariant: each output is (x >> 8) with its low bit possibly flipped
    assert np.all(((out ^ (rs >> 8)) & ~1) == 0)
    assert 0.3 < np.mean((out ^ (rs >> 8)) & 1) < 0.7      # bits do flip
    # the FLAC frames and STREAMINFO equal the port's encode of that PCM
    data = open(fn, "rb").read()
    want, _ = oracle_port.encode(out, 2, 16, 48000, **oracle_port.PRESETS["8"])
    blocks, frames = oracle_port.split_flac(data)
    wblocks, wframes = oracle_port.split_flac(want)
    assert frames == wframes
    assert blocks[0][1] == wblocks[0][1]
    dec, ch, bps, rate = oracle_port.decode(data)
    assert (ch, bps, rate) == (2, 16, 48000) and np.array_equal(dec, out)


def test_pcmconverter_downmix_average_chain():
    """5.1 -> mono: Averager(Downmixer(r)) in the reference's order, each
    stage equal to the oracle's converters over 4096-frame reads"""
    import audiotools
    x = signals.make("noise", 10000, 6, 16, seed=5)
    conv = audiotools.PCMConverter(audiotools.FrameListReader(x, 44100, 6, 16,
                                                              channel_mask=0x3F),
                                   44100, 1, 0x4, 16)
    assert type(conv).__name__ == "Averager"
    assert type(conv.pcmreader).__name__ == "Downmixer"
    parts = []
    while True:
        fl = conv.read(4096)
        if not len(fl):
            break
        parts.append(np.array(fl.samples))
    got = np.concatenate(parts)
    dm = oracle_port.convert(oracle_port.CONV_DOWNMIX, x, 6, 16, mask=0x3F)
    want = oracle_port.convert(oracle_port.CONV_AVERAGE, dm, 2, 16)
    assert np.array_equal(got, want)


def test_calculate_replay_gain_mixed_rates():
    """3 tracks, two at 44.1 kHz and one at 48 kHz: the target is 44100 (the
    most numerous), the 48 kHz track is resampled by PCMConverter, and every
    title histogram / gain / peak and the album gain equal the oracle's"""
    import audiotools
    tracks = [_Track(signals.make("tone", 44100 * 3 + 7, 2, 16, seed=1), 44100, 2, 16, 0x3),
              _Track(signals.make("chirp", 48000 * 2 + 100, 2, 16, seed=2), 48000, 2, 16, 0x3),
              _Track(signals.make("sine", 44100 * 2, 1, 16, seed=3), 44100, 1, 16, 0x4)]
    got = list(audiotools.calculate_replay_gain(tracks))
    assert [g[0] for g in got] == tracks
    hists = []
    for (tr, gain, peak, ag, ap), t in zip(got, tracks):
        pcm, reads = t.samples, None
        if t.rate != 44100:
            pcm, sizes = oracle_port.resample(t.samples, t.ch, t.bps, 44100 / t.rate,
                                              return_sizes=True)
            reads = sizes[:sizes.index(0)] if 0 in sizes else sizes  # title_gain stops at 0
        A, wpeak = oracle_port.rg_title(pcm, t.ch, t.bps, 44100, chunks=reads)
        hists.append(A)
        assert gain == oracle_port.rg_gain(A)
        assert peak == wpeak
    album = oracle_port.rg_gain(np.sum(hists, axis=0).astype(np.uint32))
    assert all(g[3] == album for g in got)
    assert all(g[4] == max(g2[2] for g2 in got) for g in got)


def test_calculate_replay_gain_progress_and_empty():
    import audiotools
    assert list(audiotools.calculate_replay_gain([])) == []
    seen = []
    t = _Track(signals.make("tone", 44100, 2, 16, seed=4), 44100, 2, 16, 0x3)
    list(audiotools.calculate_replay_gain([t], progress=lambda c, n: seen.append((c, n))))
    assert seen and seen[-1] == (44100, 44100)


# --- the reference's tests (test/test_core.py), restated --------------------
def _blank(length, rate, channels, bps, mask):
    """BLANK_PCM_Reader (test/test.py:53-90): `length` seconds of 1s"""
    import audiotools

    class Blank(object):
        def __init__(self):
            self.sample_rate, self.channels, self.bits_per_sample = rate, channels, bps
            self.channel_mask = mask
            self.left = length * rate
            self.closed = False

        def read(self, n):
            if self.closed:
                raise ValueError("unable to read closed stream")
            k = min(max(n, 1), self.left)
            self.left -= k
            return audiotools.pcm.FrameList._wrap(np.ones(k * channels, np.int32), channels,
                                                  bps)

        def close(self):
            self.closed = True

    return Blank()


SHORT_PCM_COMBINATIONS = [(11025, 1, 0x4, 8), (22050, 1, 0x4, 8), (22050, 1, 0x4, 16),
                          (32000, 2, 0x3, 16), (44100, 1, 0x4, 16), (44100, 2, 0x3, 16),
                          (48000, 1, 0x4, 16), (48000, 2, 0x3, 16), (48000, 6, 0x3F, 16),
                          (192000, 2, 0x3, 24), (96000, 6, 0x3F, 24)]


def _drain(r):
    n = 0
    while True:
        fl = r.read(4096)
        if not len(fl):
            return n
        assert fl.channels == r.channels and fl.bits_per_sample == r.bits_per_sample
        n += fl.frames


@pytest.mark.parametrize("i", range(len(SHORT_PCM_COMBINATIONS)))
def test_conversions_short_combinations(i):
    """test_core.py:847-889: every pair (in, out) of SHORT_PCM_COMBINATIONS
    -> the output's rate, channels, bps and mask are the target's and its
    duration is 5 s (here: exactly the resampled frame count, and the
    resampler's count equals the oracle's)"""
    import audiotools
    a = SHORT_PCM_COMBINATIONS[i]
    for b in SHORT_PCM_COMBINATIONS[i + 1:]:
        r = audiotools.PCMConverter(_blank(5, a[0], a[1], a[3], a[2]), sample_rate=b[0],
                                    channels=b[1], channel_mask=b[2], bits_per_sample=b[3])
        assert (r.sample_rate, r.channels, int(r.channel_mask), r.bits_per_sample) == \
            (b[0], b[1], b[2], b[3])
        n = _drain(r)
        if a[0] == b[0]:
            assert n == 5 * a[0]
        else:
            # the resampler runs after the channel stage, on b's channel
            # count (its buffers, and so its last chunks, depend on it)
            want = len(oracle_port.resample(np.ones(5 * a[0] * b[1], np.int32), b[1], 16,
                                             b[0] / a[0])) // b[1]
            assert n == want, (a, b)
            assert abs(n - audiotools.resampled_frame_count(5 * a[0], a[0], b[0])) <= 64
        assert round(n / b[0]) == 5
        r.close()


def test_converter_pcm_close_semantics():
    """test_core.py:891-941: read to the end, 10 more empty reads, then
    close: reads raise ValueError and the wrapped reader is closed"""
    import audiotools
    for rate_in in (44100, 96000):
        for ch_in, mask_in in ((1, 0x4), (2, 0x3), (4, 0x33)):
            for bps_in in (16, 24):
                for rate_out, (ch_out, mask_out), bps_out in [
                        (44100, (1, 0x4), 16), (96000, (2, 0x3), 24), (44100, (4, 0x33), 24),
                        (96000, (1, 0x4), 16)]:
                    main = _blank(1, rate_in, ch_in, bps_in, mask_in)
                    r = audiotools.PCMConverter(pcmreader=main, sample_rate=rate_out,
                                                channels=ch_out, channel_mask=mask_out,
                                                bits_per_sample=bps_out)
                    _drain(r)
                    for _ in range(10):
                        assert len(r.read(4096)) == 0
                    r.close()
                    with pytest.raises(ValueError):
                        r.read(4096)
                    with pytest.raises(ValueError):
                        main.read(4096)


def test_replaygain_valid_rates():
    """test_core.py:4336-4351: Simple_Sine(2 s, rate, 0x4, 16, (30000,
    rate/100)) at every supported rate: gain < -4.0, peak > 0.90"""
    import audiotools
    from audiotools import replaygain
    for rate in [8000, 11025, 12000, 16000, 18900, 22050, 24000, 32000, 37800, 44100, 48000,
                 56000, 64000, 88200, 96000, 112000, 128000, 144000, 176400, 192000]:
        x = signals.simple_sine(rate * 2, 30000, rate // 100)
        gain, peak = replaygain.ReplayGain(rate).title_gain(
            audiotools.FrameListReader(x, rate, 1, 16, channel_mask=0x4))
        assert gain < -4.0 and peak > 0.90, rate
        A, wpeak = oracle_port.rg_title(x, 1, 16, rate)
        assert gain == oracle_port.rg_gain(A) and peak == wpeak


def test_replaygain_reader_quieter():
    """test_core.py:4390-4424: the gain-applied stream measures quieter
    (its title gain is higher) than the original"""
    import audiotools
    from audiotools import replaygain
    x = signals.sine_stereo(44100, 44100, 441.0, 0.50, 4410.0, 0.49, 1.0, 16)
    gain, peak = replaygain.ReplayGain(44100).title_gain(
        audiotools.FrameListReader(x, 44100, 2, 16, channel_mask=0x3))
    r = replaygain.ReplayGainReader(audiotools.FrameListReader(x, 44100, 2, 16,
                                                               channel_mask=0x3), gain, peak)
    parts = []
    while True:
        fl = r.read(4096)
        if not len(fl):
            break
        parts.append(np.array(fl.samples))
    gain2, _ = replaygain.ReplayGain(44100).title_gain(
        audiotools.FrameListReader(np.concatenate(parts), 44100, 2, 16, channel_mask=0x3))
    assert gain2 > gain
