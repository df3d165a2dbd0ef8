"""audiotools.pcmconverter — the integer PCM converters on the MI355X.

Same names and reader contract as the reference's C types
(src/pcmconverter.c, used by audiotools/__init__.py:2729-2802 when
track2track changes bits per sample or channel count):

  BPSConverter(pcmreader, bits_per_sample)   BPSConverter_read :667-747
  Downmixer(pcmreader)   -> 2 channels       Downmixer_read    :220-342
  Averager(pcmreader)    -> 1 channel        Averager_read     :64-97
  Resampler(pcmreader, sample_rate)          Resampler_read    :439-495

Each read() pulls 4096 PCM frames from the wrapped reader, as the reference
does, and converts them with pcm_convert.hip (atg_pcm_convert_host).  Dither
bits come from os.urandom like the reference's (src/dither.c), consumed
MSB first, one per sample, channel by channel within each read; pass
`dither=` (a callable n -> bytes) to make a conversion reproducible.
No CPU path: a missing library raises ImportError.

Resampler drains the wrapped reader on its first read() (recording what each
read(4096) returned), resamples the whole track in one GPU batch
(resample.hip, atg_resample_host) and then hands out the frames in the
chunks the reference's src_process loop would have produced
(atg_resample_read_sizes).
"""

import os

import numpy as np

from . import _atgpu
from . import pcm


class _Converter(object):
    kind = None

    def __init__(self, pcmreader):
        self.pcmreader = pcmreader
        self.sample_rate = pcmreader.sample_rate
        self._closed = False

    def close(self):
        """closes the wrapped reader; later reads raise ValueError"""
        self._closed = True
        self.pcmreader.close()

    def _input(self):
        if self._closed:
            raise ValueError("cannot read closed stream")
        fl = self.pcmreader.read(4096)
        if not isinstance(fl, pcm.FrameList):
            raise TypeError("pcmreader.read() must return a FrameList")
        return fl


class BPSConverter(_Converter):
    kind = _atgpu.CONV_BPS

    def __init__(self, pcmreader, bits_per_sample, dither=None):
        _Converter.__init__(self, pcmreader)
        self.channels = pcmreader.channels
        self.channel_mask = pcmreader.channel_mask
        self.bits_per_sample = bits_per_sample
        self._rand = dither if dither is not None else os.urandom
        self._bits = b""
        self._bitpos = 0

    def _dither_bits(self, n):
        """bytes holding the next n dither bits at offset self._bitpos"""
        have = len(self._bits) * 8 - self._bitpos
        if have < n:
            need = (n - have + 7) // 8
            self._bits = self._bits[self._bitpos // 8:] + self._rand(max(need, 4096))
            self._bitpos %= 8
        start = self._bitpos
        self._bitpos += n
        return self._bits, start

    def read(self, pcm_frames):
        fl = self._input()
        ib, ob = self.pcmreader.bits_per_sample, self.bits_per_sample
        if ib == ob or fl.frames == 0:
            return pcm.FrameList._wrap(fl.samples, self.channels, ob)
        kw = {}
        if ob < ib:
            bits, bit0 = self._dither_bits(len(fl))
            kw = dict(dither=bits, dither_bit0=bit0)
        out = _atgpu.pcm_convert(self.kind, fl.samples, self.channels, ib, ob, **kw)
        return pcm.FrameList._wrap(out, self.channels, ob)


class Downmixer(_Converter):
    kind = _atgpu.CONV_DOWNMIX

    def __init__(self, pcmreader):
        _Converter.__init__(self, pcmreader)
        self.channels = 2
        self.channel_mask = 0x3
        self.bits_per_sample = pcmreader.bits_per_sample

    def read(self, pcm_frames):
        fl = self._input()
        if fl.frames == 0:
            return pcm.empty_framelist(2, self.bits_per_sample)
        out = _atgpu.pcm_convert(self.kind, fl.samples, self.pcmreader.channels,
                                 self.bits_per_sample,
                                 channel_mask=self.pcmreader.channel_mask)
        return pcm.FrameList._wrap(out, 2, self.bits_per_sample)


class Averager(_Converter):
    kind = _atgpu.CONV_AVERAGE

    def __init__(self, pcmreader):
        _Converter.__init__(self, pcmreader)
        self.channels = 1
        self.channel_mask = 0x4
        self.bits_per_sample = pcmreader.bits_per_sample

    def read(self, pcm_frames):
        fl = self._input()
        if fl.frames == 0:
            return pcm.empty_framelist(1, self.bits_per_sample)
        out = _atgpu.pcm_convert(self.kind, fl.samples, self.pcmreader.channels,
                                 self.bits_per_sample)
        return pcm.FrameList._wrap(out, 1, self.bits_per_sample)


class Resampler(object):
    """reference pcmconverter.Resampler (src/pcmconverter.c:370-495):
    libsamplerate sinc interpolation to `sample_rate`, bits per sample and
    channels unchanged; read() returns what one src_process round yields
    and an empty FrameList at the end"""

    def __init__(self, pcmreader, sample_rate):
        sample_rate = int(sample_rate)
        if sample_rate <= 0:
            raise ValueError("new sample rate must be positive")
        self.pcmreader = pcmreader
        self.sample_rate = sample_rate
        self.channels = pcmreader.channels
        self.channel_mask = pcmreader.channel_mask
        self.bits_per_sample = pcmreader.bits_per_sample
        self._chunks = None
        self._closed = False

    def _run(self):
        ratio = float(self.sample_rate) / float(self.pcmreader.sample_rate)
        if ratio > 256 or ratio < 1.0 / 256:
            raise ValueError("SRC ratio outside [1/256, 256] range.")
        parts, reads = [], []
        while True:
            fl = self.pcmreader.read(4096)
            if not isinstance(fl, pcm.FrameList):
                raise TypeError("pcmreader.read() must return a FrameList")
            if fl.frames == 0:
                break
            parts.append(fl.samples)
            reads.append(fl.frames)
        data = np.concatenate(parts) if parts else np.zeros(0, dtype=np.int32)
        frames = len(data) // self.channels
        out, _, counts = _atgpu.resample_host(
            data, [(0, frames, self.pcmreader.sample_rate, self.sample_rate, reads)],
            self.channels, self.bits_per_sample)
        sizes = _atgpu.resample_read_sizes(frames, self.channels,
                                           self.pcmreader.sample_rate, self.sample_rate, reads)
        if sum(sizes) != int(counts[0]):
            raise RuntimeError("resampler frame count disagrees with its read sizes")
        self._out = out
        self._chunks = sizes
        self._next = 0
        self._pos = 0

    def read(self, pcm_frames):
        if self._closed:
            raise ValueError("cannot read closed stream")
        if self._chunks is None:
            self._run()
        if self._next >= len(self._chunks):
            return pcm.empty_framelist(self.channels, self.bits_per_sample)
        n = self._chunks[self._next]
        self._next += 1
        a = self._pos * self.channels
        self._pos += n
        return pcm.FrameList._wrap(self._out[a:a + n * self.channels].copy(), self.channels,
                                   self.bits_per_sample)

    def close(self):
        self._closed = True
        self.pcmreader.close()
