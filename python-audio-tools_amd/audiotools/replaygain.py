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
    """ReplayGain(sample_rate) (replaygain.c:115-182).  Like the reference,
    the object keeps only the album state between titles -- the summed
    12000-bin window histogram B and the album peak -- never the samples."""

    def __init__(self, sample_rate):
        if sample_rate not in RATES:
            raise ValueError("unsupported sample rate")
        self.sample_rate = sample_rate
        self._album_hist = np.zeros(12000, dtype=np.uint64)
        self._album_peak = 0.0

    def title_gain(self, pcmreader):
        """(title gain, title peak) of one reader; its histogram is added
        to the album's (get_title_gain, replaygain.c:776-800)"""
        if pcmreader.sample_rate != self.sample_rate:
            raise ValueError("pcmreader's sample rate doesn't match")
        parts, sizes = [], []
        while True:
            fl = pcmreader.read(4096)
            if not isinstance(fl, pcm.FrameList):
                raise TypeError("pcmreader.read() must return a FrameList")
            if not fl.frames:
                break
            if fl.channels not in (1, 2):
                raise ValueError("FrameList must contain only 1 or 2 channels")
            parts.append(fl.samples)
            sizes.append(fl.frames)
        bps, ch = pcmreader.bits_per_sample, pcmreader.channels
        if parts and bps not in (8, 16, 24):
            raise ValueError("unsupported bits per sample")
        if not parts:
            return (0.0, 0.0)  # nothing read: no window, peak 0.0
        samples = np.concatenate(parts)
        frames = len(samples) // ch
        track = _atgpu.RgTrack(0, frames, ch, bps, self.sample_rate, 0)
        # each read() result is one analyze_samples call: its size decides
        # the fp64 summation grouping (replaygain.c:210-305)
        if any(n != 4096 for n in sizes[:-1]) or sizes[-1] > 4096:
            track.set_chunks(sizes)
        (res,), peaks, _, hist = _atgpu.replaygain_host(samples, [track], 1,
                                                        return_hist=True)
        self._album_hist += hist[0]
        self._album_peak = max(self._album_peak, peaks[0])
        return (res.title_gain, res.title_peak)

    def album_gain(self):
        """(album gain, album peak) over every title so far
        (get_album_gain, replaygain.c:803-807; ValueError when empty)"""
        if not self._album_hist.any():
            raise ValueError("Not enough samples to perform calculation")
        (gain,) = _atgpu.replaygain_hist_gain_host(
            (self._album_hist & 0xFFFFFFFF).astype(np.uint32))
        if math.isnan(gain):
            raise ValueError("Not enough samples to perform calculation")
        return (gain, self._album_peak)


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
