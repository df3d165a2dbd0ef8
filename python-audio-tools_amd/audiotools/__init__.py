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
    above 2 downmixed) by PCMConverter, its title gain and peak measured by
    one ReplayGain object (replaygain.hip), the album gain from the summed
    window histogram.  ValueError if a problem occurs."""
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
    rg = replaygain.ReplayGain(target_rate)
    gains = []
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
            gain, peak = rg.title_gain(PCMReaderProgress(reader, total, progress,
                                                         current_frames=current))
            current += frames
        else:
            gain, peak = rg.title_gain(reader)
        gains.append((track, gain, peak))
    album_gain, album_peak = rg.album_gain()
    for track, gain, peak in gains:
        yield (track, gain, peak, album_gain, album_peak)
