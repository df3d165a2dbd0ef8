"""audiotools — Python 3 host side of the MI355X FLAC encode hot path.

This package mirrors the slice of python-audio-tools 2.22alpha1's public
API that sits on the PCM -> FLAC encode path, so callers of the reference
find the same names with the same meaning:

  audiotools.pcm.FrameList ...... reference src/pcm.c (C type)
  audiotools.PCMReader .......... reference audiotools/__init__.py:2063-2131
  audiotools.BufferedPCMReader .. reference audiotools/__init__.py:2561-2606
  audiotools.encoders.encode_flac reference src/encoders/flac.c:44-307
  audiotools.PCMConverter ....... reference audiotools/__init__.py:2729-2802
  audiotools.resampled_frame_count reference audiotools/__init__.py:2805-2820
  audiotools.calculate_replay_gain reference audiotools/__init__.py:2845-2912
  audiotools.AudioFile.convert .. reference audiotools/__init__.py:3760-3774
  audiotools.AudioFile.verify ... reference audiotools/__init__.py:3939-3970
  audiotools.FlacAudio / WaveAudio / ALACAudio (flac.py, wav.py, m4a.py)

track2track's per-file step is `AudioFile.convert(target, FlacAudio, "8")`
and trackverify's is `AudioFile.verify()`; both run through these classes,
so under the drop-in they reach the GPU encoder and decoders.

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


class InvalidFile(Exception):
    """raised if a file is invalid in some way
    (reference audiotools/__init__.py:1276-1279)"""


class DecodingError(IOError):
    """raised if a decoder exits with an error
    (reference audiotools/__init__.py:1342-1350)"""

    def __init__(self, error_message):
        IOError.__init__(self, error_message)
        self.error_message = error_message


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


class ChannelMask(object):
    """the speaker bits of a channel mask (reference
    audiotools/__init__.py:1862-2030): len() counts the defined speakers,
    channels() lists their bits in RIFF WAVE order (least significant
    first), as the reference's speaker-name list is ordered"""

    SPEAKER_BITS = 18  # front_left 0x1 ... top_back_right 0x20000

    def __init__(self, mask):
        self.mask = int(mask) & ((1 << self.SPEAKER_BITS) - 1)

    def __int__(self):
        return self.mask

    def __len__(self):
        return bin(self.mask).count("1")

    def __eq__(self, other):
        return int(self) == int(other)

    def __ne__(self, other):
        return int(self) != int(other)

    def __hash__(self):
        return hash(self.mask)

    def channels(self):
        return [1 << b for b in range(self.SPEAKER_BITS) if self.mask >> b & 1]

    @classmethod
    def from_channels(cls, channel_count):
        """0x4 for mono, 0x3 for stereo; ValueError otherwise"""
        if channel_count == 2:
            return cls(0x3)
        if channel_count == 1:
            return cls(0x4)
        raise ValueError("ambiguous channel assignment")


class PCMReaderProgress(object):
    """a PCMReader reporting progress(current, total) after every read
    (reference audiotools/__init__.py:2167-2191)"""

    def __init__(self, pcmreader, total_frames, progress, current_frames=0):
        self._read = pcmreader.read
        self._close = pcmreader.close
        self.sample_rate = pcmreader.sample_rate
        self.channels = pcmreader.channels
        self.channel_mask = pcmreader.channel_mask
        self.bits_per_sample = pcmreader.bits_per_sample
        self.current_frames = current_frames
        self.total_frames = total_frames
        self.progress = progress

    def read(self, pcm_frames):
        frame = self._read(pcm_frames)
        self.current_frames += frame.frames
        self.progress(self.current_frames, self.total_frames)
        return frame

    def close(self):
        self._close()


def to_pcm_progress(audiofile, progress):
    """audiofile.to_pcm(), wrapped in a PCMReaderProgress when a progress
    callback is given (reference audiotools/__init__.py:2158-2164)"""
    if progress is None:
        return audiofile.to_pcm()
    return PCMReaderProgress(audiofile.to_pcm(), audiofile.total_frames(), progress)


class CounterPCMReader(object):
    """a PCMReader counting the frames read through it
    (reference audiotools/__init__.py:2608-2631)"""

    def __init__(self, pcmreader):
        self.sample_rate = pcmreader.sample_rate
        self.channels = pcmreader.channels
        self.channel_mask = pcmreader.channel_mask
        self.bits_per_sample = pcmreader.bits_per_sample
        self.__pcmreader = pcmreader
        self.frames_written = 0

    def bytes_written(self):
        return self.frames_written * self.channels * (self.bits_per_sample // 8)

    def read(self, pcm_frames):
        frame = self.__pcmreader.read(pcm_frames)
        self.frames_written += frame.frames
        return frame

    def close(self):
        self.__pcmreader.close()


def transfer_data(from_function, to_function):
    """BUFFER_SIZE strings from from_function to to_function until an empty
    one; an IOError ends the transfer quietly
    (reference audiotools/__init__.py:2301-2314)"""
    try:
        s = from_function(BUFFER_SIZE)
        while len(s) > 0:
            to_function(s)
            s = from_function(BUFFER_SIZE)
    except IOError:
        pass


def transfer_framelist_data(pcmreader, to_function, signed=True, big_endian=False):
    """FrameLists from pcmreader as bytes to to_function until an empty one
    (reference audiotools/__init__.py:2317-2328)"""
    f = pcmreader.read(FRAMELIST_SIZE)
    while len(f) > 0:
        to_function(f.to_bytes(big_endian, signed))
        f = pcmreader.read(FRAMELIST_SIZE)


def pcm_cmp(pcmreader1, pcmreader2):
    """True if the two readers' PCM data are equal
    (reference audiotools/__init__.py:2384-2409)"""
    if (pcmreader1.sample_rate != pcmreader2.sample_rate or
            pcmreader1.channels != pcmreader2.channels or
            pcmreader1.bits_per_sample != pcmreader2.bits_per_sample):
        return False
    reader1 = BufferedPCMReader(pcmreader1)
    reader2 = BufferedPCMReader(pcmreader2)
    s1 = reader1.read(FRAMELIST_SIZE)
    s2 = reader2.read(FRAMELIST_SIZE)
    while len(s1) > 0 and len(s2) > 0:
        if s1 != s2:
            return False
        s1 = reader1.read(FRAMELIST_SIZE)
        s2 = reader2.read(FRAMELIST_SIZE)
    return True


def pcm_frame_cmp(pcmreader1, pcmreader2):
    """the PCM frame number of the first mismatch, None if the streams
    match (reference audiotools/__init__.py:2445-2481); may raise IOError
    or ValueError from the readers"""
    if (pcmreader1.sample_rate != pcmreader2.sample_rate or
            pcmreader1.channels != pcmreader2.channels or
            pcmreader1.bits_per_sample != pcmreader2.bits_per_sample):
        return 0
    if (int(pcmreader1.channel_mask) != 0 and int(pcmreader2.channel_mask) != 0 and
            int(pcmreader1.channel_mask) != int(pcmreader2.channel_mask)):
        return 0
    frame_number = 0
    reader1 = BufferedPCMReader(pcmreader1)
    reader2 = BufferedPCMReader(pcmreader2)
    framelist1 = reader1.read(FRAMELIST_SIZE)
    framelist2 = reader2.read(FRAMELIST_SIZE)
    while len(framelist1) > 0 and len(framelist2) > 0:
        if framelist1 != framelist2:
            n = min(framelist1.frames, framelist2.frames)
            for i in range(n):
                if framelist1.frame(i) != framelist2.frame(i):
                    return frame_number + i
            return frame_number + max(n - 1, 0)
        frame_number += framelist1.frames
        framelist1 = reader1.read(FRAMELIST_SIZE)
        framelist2 = reader2.read(FRAMELIST_SIZE)
    if len(framelist1) == 0 and len(framelist2) == 0:
        return None
    return frame_number


class AudioFile(object):
    """the format-independent part of the reference's AudioFile
    (audiotools/__init__.py:3595-3990) the transcode callers use:
    convert() is track2track's per-file step, verify() trackverify's."""

    SUFFIX = ""
    NAME = ""

    def __init__(self, filename):
        self.filename = filename

    def lossless(self):
        return False

    def convert(self, target_path, target_class, compression=None, progress=None):
        """encode a new target_class file from this one
        (reference audiotools/__init__.py:3760-3774); EncodingError on a
        problem"""
        return target_class.from_pcm(
            target_path, to_pcm_progress(self, progress), compression,
            total_pcm_frames=(self.total_frames() if self.lossless() else None))

    @classmethod
    def __unlink__(cls, filename):
        import os
        try:
            os.unlink(filename)
        except OSError:
            pass

    def __eq__(self, audiofile):
        """equal PCM data (reference audiotools/__init__.py:3926-3934)"""
        if hasattr(audiofile, "to_pcm") and callable(audiofile.to_pcm):
            try:
                return pcm_frame_cmp(self.to_pcm(), audiofile.to_pcm()) is None
            except (ValueError, IOError):
                return False
        return False

    def __ne__(self, audiofile):
        return not self.__eq__(audiofile)

    __hash__ = object.__hash__

    def verify(self, progress=None):
        """decode the whole file; True if it is sound, InvalidFile with the
        decoder's message otherwise (reference
        audiotools/__init__.py:3939-3970)"""
        try:
            total_frames = self.total_frames()
            decoder = self.to_pcm()
            pcm_frame_count = 0
            framelist = decoder.read(FRAMELIST_SIZE)
            while len(framelist) > 0:
                pcm_frame_count += framelist.frames
                if progress is not None:
                    progress(pcm_frame_count, total_frames)
                framelist = decoder.read(FRAMELIST_SIZE)
        except (IOError, ValueError) as err:
            raise InvalidFile(str(err))
        try:
            decoder.close()
        except DecodingError as err:
            raise InvalidFile(err.error_message)
        if self.lossless():
            if pcm_frame_count == total_frames:
                return True
            raise InvalidFile("incorrect PCM frame count")
        return True


def _check_mask(channel_mask, channels):
    if channel_mask != 0 and len(ChannelMask(channel_mask)) != channels:
        raise ValueError("channel count and channel mask mismatch")


class ReorderedPCMReader(object):
    """a PCMReader whose output channels are the listed input channels
    (reference audiotools/__init__.py:2194-2236)"""

    def __init__(self, pcmreader, channel_order, channel_mask=None):
        self.pcmreader = pcmreader
        self.sample_rate = pcmreader.sample_rate
        self.channels = len(channel_order)
        self.channel_mask = pcmreader.channel_mask if channel_mask is None else channel_mask
        _check_mask(self.channel_mask, self.channels)
        self.bits_per_sample = pcmreader.bits_per_sample
        self.channel_order = list(channel_order)

    def read(self, pcm_frames):
        fl = self.pcmreader.read(pcm_frames)
        return pcm.from_channels([fl.channel(c) for c in self.channel_order])

    def close(self):
        self.pcmreader.close()


class RemaskedPCMReader(object):
    """a PCMReader with another channel count and mask: matching speakers
    forwarded, missing ones silent (reference
    audiotools/__init__.py:2239-2298)"""

    def __init__(self, pcmreader, channel_count, channel_mask):
        self.pcmreader = pcmreader
        self.sample_rate = pcmreader.sample_rate
        self.channels = channel_count
        self.channel_mask = channel_mask
        self.bits_per_sample = pcmreader.bits_per_sample
        if pcmreader.channel_mask != 0 and channel_mask != 0:
            mask = ChannelMask(channel_mask)
            if len(mask) != channel_count:
                raise ValueError("channel count and channel mask mismatch")
            have = ChannelMask(pcmreader.channel_mask).channels()
            self._map = [have.index(c) if c in have else None for c in mask.channels()]
        elif channel_count <= pcmreader.channels:
            self._map = list(range(channel_count))
        else:
            # the reference's list here is range(channel_count) + [None] *
            # (channel_count - pcmreader.channels): longer than
            # channel_count, and channel() of an input it lacks raises --
            # kept as written
            self._map = (list(range(channel_count)) +
                         [None] * (channel_count - pcmreader.channels))

    def read(self, pcm_frames):
        fl = self.pcmreader.read(pcm_frames)
        blank = pcm.from_list([0] * fl.frames, 1, self.pcmreader.bits_per_sample, True)
        return pcm.from_channels([fl.channel(c) if c is not None else blank
                                  for c in self._map])

    def close(self):
        self.pcmreader.close()


def PCMConverter(pcmreader, sample_rate, channels, channel_mask, bits_per_sample):
    """a PCMReader wrapper converting sample rate, channel count / mask and
    bits per sample (reference audiotools/__init__.py:2729-2802), composed
    in the reference's order: channels first (Downmixer / Averager /
    RemaskedPCMReader / ReorderedPCMReader), then Resampler, then
    BPSConverter -- the order decides what each stage reads, and so the
    resampler's chunking and the dither bits' order.  The converters run on
    the GPU (audiotools.pcmconverter).  ValueError for an unsupported
    target."""
    if sample_rate <= 0:
        raise ValueError("invalid sample rate")
    if channels <= 0:
        raise ValueError("invalid channel count")
    if bits_per_sample not in (8, 16, 24):
        raise ValueError("invalid bits-per-sample")
    _check_mask(channel_mask, channels)
    from . import pcmconverter
    if pcmreader.channels > channels:
        if channels == 1 and channel_mask in (0, 0x4):
            if pcmreader.channels > 2:
                pcmreader = pcmconverter.Averager(pcmconverter.Downmixer(pcmreader))
            else:
                pcmreader = pcmconverter.Averager(pcmreader)
        elif channels == 2 and channel_mask in (0, 0x3):
            pcmreader = pcmconverter.Downmixer(pcmreader)
        else:
            pcmreader = RemaskedPCMReader(pcmreader, channels, channel_mask)
    elif pcmreader.channels < channels:
        # duplicate the first channel (mono -> stereo)
        pcmreader = ReorderedPCMReader(
            pcmreader, list(range(pcmreader.channels)) + [0] * (channels - pcmreader.channels),
            channel_mask)
    if pcmreader.sample_rate != sample_rate:
        pcmreader = pcmconverter.Resampler(pcmreader, sample_rate)
    if pcmreader.bits_per_sample != bits_per_sample:
        pcmreader = pcmconverter.BPSConverter(pcmreader, bits_per_sample)
    return pcmreader


def resampled_frame_count(initial_frame_count, initial_sample_rate, new_sample_rate):
    """the PCM frame count after resampling, rounded down
    (reference audiotools/__init__.py:2805-2820)"""
    if initial_sample_rate == new_sample_rate:
        return initial_frame_count
    return (int(initial_frame_count) * int(new_sample_rate)) // int(initial_sample_rate)


def most_numerous(item_list, empty_list=None, all_differ=None):
    """the item occurring most often (reference
    audiotools/__init__.py:5012-5031); empty_list for an empty list,
    all_differ when every item differs.  Ties: the reference takes the last
    of a stable sort over Py2 dict order; here the item seen first wins."""
    if len(item_list) == 0:
        return empty_list
    counts = {}
    for item in item_list:
        counts[item] = counts.get(item, 0) + 1
    best = max(counts.values())
    if best == 1 and len(item_list) > 1:
        return all_differ
    return next(i for i in item_list if counts[i] == best)


REPLAY_GAIN_RATES = [8000, 11025, 12000, 16000, 18900, 22050, 24000, 32000, 37800, 44100,
                     48000, 56000, 64000, 88200, 96000, 112000, 128000, 144000, 176400,
                     192000]


def applicable_replay_gain(tracks):
    """True when the tracks share one supported sample rate and 1 or 2
    channels (reference audiotools/__init__.py:2823-2842)"""
    rates = set(t.sample_rate() for t in tracks)
    if len(rates) > 1 or list(rates)[0] not in REPLAY_GAIN_RATES:
        return False
    chans = set(t.channels() for t in tracks)
    return not (len(chans) > 1 or list(chans)[0] not in (1, 2))


def calculate_replay_gain(tracks, progress=None):
    """yields (track, track_gain, track_peak, album_gain, album_peak) for
    every AudioFile of `tracks` (reference audiotools/__init__.py:2845-2912):
    the album's most numerous sample rate rounded up to a supported
    ReplayGain rate is the target, each track converted to it (channels
    above 2 downmixed) by PCMConverter and read as the reference's
    ReplayGain.title_gain reads it; then the whole album is analysed in one
    GPU batch per device (replaygain.album_scan: titles sharded over the
    node's GPUs, the shards' window histograms summed and peaks max'd), the
    album gain from the summed histogram.  Gains and peaks are those of the
    title-by-title reference computation.  ValueError if a problem occurs."""
    if len(tracks) == 0:
        return
    from bisect import bisect
    from . import replaygain
    rates = REPLAY_GAIN_RATES
    target_rate = ([rates[0]] + rates)[bisect(rates, most_numerous(
        [t.sample_rate() for t in tracks]))]
    track_frames = [resampled_frame_count(t.total_frames(), t.sample_rate(), target_rate)
                    for t in tracks]
    current, total = 0, sum(track_frames)
    if target_rate not in replaygain.RATES:
        raise ValueError("unsupported sample rate")
    titles = []
    for track, frames in zip(tracks, track_frames):
        reader = track.to_pcm()
        if reader.channels > 2:
            out_ch, out_mask = 2, 0x3
        else:
            out_ch, out_mask = reader.channels, reader.channel_mask
        if (reader.channels != out_ch or reader.channel_mask != out_mask or
                reader.sample_rate != target_rate):
            reader = PCMConverter(reader, target_rate, out_ch, out_mask,
                                  reader.bits_per_sample)
        if progress is not None:
            reader = PCMReaderProgress(reader, total, progress, current_frames=current)
            current += frames
        titles.append(replaygain._read_title(reader, target_rate))
    gains, hist, peak = replaygain.album_scan(titles, target_rate)
    album_gain, album_peak = replaygain.album_gain_of(hist, peak)
    for track, (gain, tpeak) in zip(tracks, gains):
        yield (track, gain, tpeak, album_gain, album_peak)


# the format classes (their modules import the names above)
from .flac import FlacAudio, InvalidFLAC  # noqa: E402,F401
from .wav import WaveAudio, InvalidWave  # noqa: E402,F401
from .m4a import ALACAudio, InvalidALAC  # noqa: E402,F401
