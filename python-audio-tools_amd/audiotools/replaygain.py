"""audiotools.replaygain — ReplayGain analysis on the MI355X.

`ReplayGain` keeps the Python contract of the reference's C type
(src/replaygain.c, replaygain.h): ReplayGain(sample_rate) raises ValueError
for an unsupported rate; title_gain(pcmreader) -> (gain, peak) for one
track (0.0 gain when no 50 ms window completed); album_gain() -> (gain,
peak) over every title analysed so far, ValueError "Not enough samples to
perform calculation" when none.  Each title is analysed by replaygain.hip
(lane per track); `batch_gains` analyses many tracks/albums in one launch.
No CPU path.
"""

import math
import os

import numpy as np

from . import _atgpu
from . import pcm

RATES = (48000, 44100, 32000, 24000, 22050, 16000, 12000, 11025, 8000, 18900,
         37800, 56000, 64000, 88200, 96000, 112000, 128000, 144000, 176400, 192000)


class ReplayGain(object):
    def __init__(self, sample_rate):
        if sample_rate not in RATES:
            raise ValueError("unsupported sample rate")
        self.sample_rate = sample_rate
        self._titles = []   # (samples, channels, bps) of every title so far

    def title_gain(self, pcmreader):
        if pcmreader.sample_rate != self.sample_rate:
            raise ValueError("pcmreader's sample rate doesn't match")
        parts = []
        while True:
            fl = pcmreader.read(4096)
            if not isinstance(fl, pcm.FrameList):
                raise TypeError("pcmreader.read() must return a FrameList")
            if not fl.frames:
                break
            if fl.channels not in (1, 2):
                raise ValueError("FrameList must contain only 1 or 2 channels")
            parts.append(fl.samples)
        bps, ch = pcmreader.bits_per_sample, pcmreader.channels
        if bps not in (8, 16, 24):
            raise ValueError("unsupported bits per sample")
        samples = np.concatenate(parts) if parts else np.zeros(0, np.int32)
        self._titles.append((samples, ch, bps))
        (res,), _, _ = self._run([(samples, ch, bps)], album=False)
        return (res.title_gain, res.title_peak)

    def _run(self, titles, album):
        # the reference analyses mono as a duplicated stereo pair
        # (replaygain.c:228-229), so mono titles are widened and every title
        # of the album goes in one 2-channel batch
        bufs, tracks, off = [], [], 0
        for s, ch, bps in titles:
            st = np.repeat(s, 2) if ch == 1 else s
            frames = len(st) // 2
            tracks.append(_atgpu.RgTrack(off, frames, 2, bps, self.sample_rate, 0))
            bufs.append(st)
            off += frames
        buf = np.concatenate(bufs) if bufs else np.zeros(0, np.int32)
        return _atgpu.replaygain_host(buf, tracks, 1 if album else 0)

    def album_gain(self):
        if not self._titles:
            raise ValueError("Not enough samples to perform calculation")
        res, peaks, gains = self._run(self._titles, album=True)
        if not gains or math.isnan(gains[0]):
            raise ValueError("Not enough samples to perform calculation")
        return (gains[0], peaks[0])


def batch_gains(pcm_i32, tracks, n_albums):
    """title gains/peaks of a batch (int32 PCM in host memory, list of
    RgTrack grouped by album) and album gains/peaks.
    -> ([(title_gain, title_peak)], [(album_gain, album_peak)])"""
    res, peaks, gains = _atgpu.replaygain_host(pcm_i32, tracks, n_albums)
    return ([(r.title_gain, r.title_peak) for r in res], list(zip(gains, peaks)))


class ReplayGainReader(object):
    """reference replaygain.ReplayGainReader(pcmreader, replaygain, peak)
    (src/replaygain.c:820-925): a PCMReader applying the gain with
    lround, clamping and one XOR dither bit per sample (os.urandom, or
    `dither=` callable n -> bytes for reproducible output)"""

    def __init__(self, pcmreader, replaygain, peak, dither=None):
        self.pcmreader = pcmreader
        self.sample_rate = pcmreader.sample_rate
        self.channels = pcmreader.channels
        self.channel_mask = pcmreader.channel_mask
        self.bits_per_sample = pcmreader.bits_per_sample
        self.multiplier = _atgpu.load_library().atg_replaygain_multiplier(
            float(replaygain), float(peak))
        self._rand = dither if dither is not None else os.urandom
        self._bits = b""
        self._bitpos = 0

    def read(self, pcm_frames):
        if pcm_frames <= 0:
            raise ValueError("pcm_frames must be positive")
        fl = self.pcmreader.read(pcm_frames)
        if not isinstance(fl, pcm.FrameList):
            raise TypeError("pcmreader.read() must return a FrameList")
        if not fl.frames:
            return fl
        n = len(fl)
        have = len(self._bits) * 8 - self._bitpos
        if have < n:
            self._bits = self._bits[self._bitpos // 8:] + self._rand(
                max((n - have + 7) // 8, 4096))
            self._bitpos %= 8
        out = _atgpu.apply_gain(fl.samples, self.channels, self.bits_per_sample,
                                self.multiplier, fl.frames, self._bits, self._bitpos)
        self._bitpos += n
        return pcm.FrameList._wrap(out, self.channels, self.bits_per_sample)

    def close(self):
        self.pcmreader.close()
