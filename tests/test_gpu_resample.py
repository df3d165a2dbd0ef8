"""GPU: the batch sinc resampler (resample.hip) against the CPU restatement
oracle/resample_port.c, bit for bit.  Parity is
unpinned to reference output (BEST table absent, see
test_resample_oracle.py); the tolerance versus the restatement is zero."""
import numpy as np
import pytest

import oracle_port

pytestmark = pytest.mark.gpu


def _batch(specs, ch, bps, seed):
    """specs: [(frames, in_rate, out_rate)] -> (pcm, tracks)"""
    rng = np.random.default_rng(seed)
    parts, tracks, off = [], [], 0
    amp = 1 << (bps - 1)
    for (n, a, b) in specs:
        t = np.arange(n)[:, None]
        tone = (0.6 * amp * np.sin(2 * np.pi * (220 + 50 * np.arange(ch)) * t / a)).astype(np.int64)
        noise = rng.integers(-amp // 8, amp // 8, (n, ch))
        x = np.clip(tone + noise, -amp, amp - 1).astype(np.int32).reshape(-1)
        parts.append(x)
        tracks.append((off, n, a, b))
        off += n
    pcm = np.concatenate(parts) if parts else np.zeros(0, np.int32)
    return pcm, tracks


def _check(pcm, tracks, ch, bps):
    from audiotools import _atgpu
    out, offs, cnt = _atgpu.resample_host(pcm, tracks, ch, bps)
    for i, (off, n, a, b) in enumerate(tracks):
        want = oracle_port.resample(pcm[off * ch:(off + n) * ch], ch, bps, b / a)
        assert int(cnt[i]) * ch == len(want), (i, a, b, n)
        got = out[int(offs[i]) * ch:(int(offs[i]) + int(cnt[i])) * ch]
        if not np.array_equal(got, want):
            bad = np.flatnonzero(got != want)
            raise AssertionError("track %d (%d->%d, %d frames): %d samples differ, first %d "
                                 "got %d want %d" % (i, a, b, n, len(bad), bad[0],
                                                     got[bad[0]], want[bad[0]]))


@pytest.mark.parametrize("ch", [1, 2, 3, 4, 5, 6, 7, 8])
def test_mixed_rates_all_channel_counts(ch):
    specs = [(5000, 44100, 48000), (3001, 48000, 44100), (4000, 192000, 48000),
             (2500, 22050, 48000), (1234, 44100, 96000), (6000, 96000, 44100),
             (0, 44100, 48000), (1, 44100, 48000), (147, 44100, 48000), (700, 8000, 48000)]
    pcm, tracks = _batch(specs, ch, 16, ch)
    _check(pcm, tracks, ch, 16)


@pytest.mark.parametrize("bps", [8, 16, 24])
def test_bits_per_sample(bps):
    pcm, tracks = _batch([(20000, 44100, 48000), (9000, 48000, 32000)], 2, bps, bps)
    _check(pcm, tracks, 2, bps)


def test_config3_shape_subset():
    """BASELINE config 3 (44.1k -> 48k stereo 24-bit) on 32 one-second
    tracks, every sample against the restatement"""
    pcm, tracks = _batch([(44100 + 37 * i, 44100, 48000) for i in range(32)], 2, 24, 3)
    _check(pcm, tracks, 2, 24)


def test_config5_shape_subset():
    """BASELINE config 5's resample (192k/24-bit 5.1 -> 48k), 4 tracks"""
    pcm, tracks = _batch([(192000 // 2 + 11 * i, 192000, 48000) for i in range(4)], 6, 24, 5)
    _check(pcm, tracks, 6, 24)


def test_full_scale_clipping():
    """full-scale square waves overshoot (Gibbs): the float -> int export
    clamps like fb_export_frames"""
    n = 8000
    x = np.where((np.arange(n) // 50) % 2 == 0, 32767, -32768).astype(np.int32)
    _check(np.repeat(x, 2), [(0, n, 44100, 48000)], 2, 16)


def test_resampler_reader_chunks(tmp_path):
    """pcmconverter.Resampler: the reference's read() chunking and samples
    over a reader returning 4096-frame and irregular reads"""
    import audiotools
    from audiotools import pcmconverter
    pcm, _ = _batch([(30001, 44100, 48000)], 2, 16, 9)
    for block in (4096, 1152, 4608):
        reads = [block] * (30001 // block) + ([30001 % block] if 30001 % block else [])
        want, sizes = oracle_port.resample(pcm, 2, 16, 48000 / 44100.0, reads=reads,
                                           return_sizes=True)
        r = pcmconverter.Resampler(
            audiotools.FrameListReader(pcm, 44100, 2, 16, 0x3) if block == 4096 else
            _FixedReads(pcm, reads), 48000)
        assert (r.sample_rate, r.channels, r.bits_per_sample) == (48000, 2, 16)
        got, got_sizes = [], []
        while True:
            fl = r.read(4096)
            got_sizes.append(fl.frames)
            if fl.frames == 0:
                break
            got.append(np.asarray(fl.samples))
        assert got_sizes == sizes
        assert np.array_equal(np.concatenate(got), want)


class _FixedReads(object):
    def __init__(self, pcm, reads):
        self.sample_rate, self.channels, self.bits_per_sample, self.channel_mask = \
            44100, 2, 16, 0x3
        self._pcm, self._reads, self._pos = pcm, list(reads), 0

    def read(self, n):
        from audiotools import pcm as P
        k = self._reads.pop(0) if self._reads else 0
        a = self._pos * 2
        self._pos += k
        return P.FrameList._wrap(self._pcm[a:a + 2 * k].copy(), 2, 16)

    def close(self):
        pass


def test_resampler_errors():
    import audiotools
    from audiotools import pcmconverter
    src = audiotools.FrameListReader(np.zeros(20, np.int32), 44100, 2, 16)
    with pytest.raises(ValueError):
        pcmconverter.Resampler(src, 0)
    r = pcmconverter.Resampler(src, 44100 * 300)
    with pytest.raises(ValueError):
        r.read(4096)
