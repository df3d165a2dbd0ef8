"""audiotools — Python 3 host side of the MI355X FLAC encode hot path.

This package mirrors the slice of python-audio-tools 2.22alpha1's public
API that sits on the PCM -> FLAC encode path, so callers of the reference
find the same names with the same meaning:

  audiotools.pcm.FrameList ...... reference src/pcm.c (C type)
  audiotools.PCMReader .......... reference audiotools/__init__.py:2063-2131
  audiotools.BufferedPCMReader .. reference audiotools/__init__.py:2561-2606
  audiotools.encoders.encode_flac reference src/encoders/flac.c:44-307

The encoding itself runs in libatgpu.so (HIP kernels for gfx950) through
the C ABI declared in include/atgpu.h.  There is no CPU encoding path: if
the library or a GPU is missing, encode_flac raises.
"""

from . import pcm

VERSION = "2.22alpha1"
BUFFER_SIZE = 0x100000
FRAMELIST_SIZE = 0x100000 // 4   # reference audiotools/__init__.py:93-94


class EncodingError(IOError):
    """raised if an audio file cannot be created correctly
    (reference audiotools/__init__.py:1282-1300)"""

    def __init__(self, error_message):
        IOError.__init__(self, error_message)
        self.error_message = error_message

    def __reduce__(self):
        return (EncodingError, (self.error_message,))

    def __str__(self):
        return str(self.error_message)


class PCMReader(object):
    """wraps a file object of raw PCM bytes and yields pcm.FrameLists
    (reference audiotools/__init__.py:2063-2131)"""

    def __init__(self, file, sample_rate, channels, channel_mask,
                 bits_per_sample, process=None, signed=True,
                 big_endian=False):
        self.file = file
        self.sample_rate = sample_rate
        self.channels = channels
        self.channel_mask = channel_mask
        self.bits_per_sample = bits_per_sample
        self.process = process
        self.signed = signed
        self.big_endian = big_endian
        self.bytes_per_frame = self.channels * (self.bits_per_sample // 8)

    def read(self, pcm_frames):
        framelist = pcm.FrameList(
            self.file.read(max(pcm_frames, 1) * self.bytes_per_frame),
            self.channels, self.bits_per_sample, self.big_endian, self.signed)
        if framelist.frames > 0:
            return framelist
        elif self.process is not None:
            if self.process.wait() == 0:
                return framelist
            raise ValueError(u"subprocess exited with error")
        return framelist

    def close(self):
        self.file.close()


class PCMReaderError(object):
    """a PCMReader whose read() raises ValueError
    (reference audiotools/__init__.py:2133-2160)"""

    def __init__(self, error_message, sample_rate, channels, channel_mask,
                 bits_per_sample):
        self.sample_rate = sample_rate
        self.channels = channels
        self.channel_mask = channel_mask
        self.bits_per_sample = bits_per_sample
        self.error_message = error_message

    def read(self, pcm_frames):
        raise ValueError(self.error_message)

    def close(self):
        pass


class BufferedPCMReader(object):
    """a PCMReader which reads exact counts of PCM frames
    (reference audiotools/__init__.py:2561-2606)"""

    def __init__(self, pcmreader):
        self.pcmreader = pcmreader
        self.sample_rate = pcmreader.sample_rate
        self.channels = pcmreader.channels
        self.channel_mask = pcmreader.channel_mask
        self.bits_per_sample = pcmreader.bits_per_sample
        self.buffer = pcm.empty_framelist(self.channels, self.bits_per_sample)

    def close(self):
        self.pcmreader.close()
        self.read = self.read_closed

    def read(self, pcm_frames):
        while self.buffer.frames < pcm_frames:
            frame = self.pcmreader.read(FRAMELIST_SIZE)
            if len(frame):
                self.buffer += frame
            else:
                break
        (output, self.buffer) = self.buffer.split(pcm_frames)
        return output

    def read_closed(self, pcm_frames):
        raise ValueError()


class FrameListReader(object):
    """PCMReader over an in-memory FrameList (or interleaved int array),
    handing out at most `pcm_frames` frames per read()"""

    def __init__(self, samples, sample_rate, channels, bits_per_sample,
                 channel_mask=0):
        if isinstance(samples, pcm.FrameList):
            self._fl = samples
        else:
            import numpy as np
            self._fl = pcm.FrameList._wrap(np.asarray(samples, dtype=np.int32),
                                           channels, bits_per_sample)
        self.sample_rate = sample_rate
        self.channels = channels
        self.channel_mask = channel_mask
        self.bits_per_sample = bits_per_sample

    def read(self, pcm_frames):
        (head, self._fl) = self._fl.split(max(pcm_frames, 1))
        return head

    def close(self):
        pass
