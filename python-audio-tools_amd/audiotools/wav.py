"""audiotools.wav — RIFF WAVE input for the encode path (BASELINE config 1).

Only the reading side the encoder needs: `WaveReader` (reference
audiotools/wav.py:421-553) walks the RIFF chunks to "fmt " and "data" and
hands out pcm.FrameLists; `parse_fmt` (:288-354) decodes the "fmt " chunk
(WAVE_FORMAT_PCM with the SMPTE/ITU-R default masks, or
WAVE_FORMAT_EXTENSIBLE with the PCM sub-format GUID); `WaveAudio.to_pcm`
(:652-655) returns a WaveReader.  Config 1 is
`encode_flac(out, BufferedPCMReader(WaveReader("wav-2ch.wav")), **FLAC8)`.

Host byte work: the samples are converted by pcm.FrameList and the encode
itself runs in libatgpu on the GPU.
"""

import struct

from . import pcm as _pcm

PRINTABLE_ASCII = frozenset(range(0x20, 0x7E + 1))

# WAVE_FORMAT_EXTENSIBLE KSDATAFORMAT_SUBTYPE_PCM GUID (wav.py:343-345)
_PCM_SUBFORMAT = (b"\x01\x00\x00\x00\x00\x00\x10\x00"
                  b"\x80\x00\x00\xaa\x00\x38\x9b\x71")

# channel masks assumed for plain WAVE_FORMAT_PCM files (wav.py:304-335):
# 1 = front center, 2 = FL FR, 3 = FL FR FC, 4 = FL FR BL BR,
# 5 = FL FR FC BL BR, 6 = FL FR FC LFE BL BR
_DEFAULT_MASKS = {1: 0x4, 2: 0x3, 3: 0x7, 4: 0x33, 5: 0x37, 6: 0x3F}


def parse_fmt(chunk):
    """bytes of a "fmt " chunk -> (channels, sample_rate, bits_per_sample,
    channel_mask); ValueError on an unsupported or invalid chunk,
    IOError when the chunk is truncated (BitstreamReader EOF)"""
    if len(chunk) < 16:
        raise IOError("I/O error reading fmt chunk")
    (compression, channels, sample_rate, _bytes_per_second, _block_align,
     bits_per_sample) = struct.unpack("<HHIIHH", chunk[:16])
    if compression == 1:
        return channels, sample_rate, bits_per_sample, _DEFAULT_MASKS.get(channels, 0)
    if compression == 0xFFFE:
        if len(chunk) < 40:
            raise IOError("I/O error reading fmt chunk")
        _cb_size, _valid_bits, channel_mask = struct.unpack("<HHI", chunk[16:24])
        if chunk[24:40] != _PCM_SUBFORMAT:
            raise ValueError("invalid WAVE sub-format")
        return channels, sample_rate, bits_per_sample, channel_mask
    raise ValueError("unsupported WAVE compression")


class WaveReader(object):
    """PCMReader over a wave file's "data" chunk
    (reference audiotools/wav.py:421-553)"""

    def __init__(self, wave_filename):
        self.file = open(wave_filename, "rb")
        try:
            self._open()
        except Exception:
            self.file.close()
            raise

    def _open(self):
        head = self.file.read(12)
        if len(head) < 12:
            raise ValueError("invalid WAVE file")
        riff, total_size, wave = struct.unpack("<4sI4s", head)
        if riff != b"RIFF":
            raise ValueError("not a RIFF WAVE file")
        if wave != b"WAVE":
            raise ValueError("invalid WAVE file")
        total_size -= 4
        fmt_read = False
        # walk the chunks until "data" (wav.py:451-502)
        while total_size > 0:
            hdr = self.file.read(8)
            if len(hdr) < 8:
                raise ValueError("invalid WAVE file")
            chunk_id, chunk_size = struct.unpack("<4sI", hdr)
            if not frozenset(chunk_id).issubset(PRINTABLE_ASCII):
                raise ValueError("invalid RIFF WAVE chunk ID")
            total_size -= 8
            if chunk_id == b"fmt ":
                (self.channels, self.sample_rate, self.bits_per_sample,
                 self.channel_mask) = parse_fmt(self.file.read(chunk_size))
                self.bytes_per_pcm_frame = (self.bits_per_sample // 8) * self.channels
                fmt_read = True
            elif chunk_id == b"data":
                if not fmt_read:
                    raise ValueError("data chunk found before fmt")
                self.total_pcm_frames = chunk_size // self.bytes_per_pcm_frame
                self.remaining_pcm_frames = self.total_pcm_frames
                self.data_chunk_offset = self.file.tell()
                return
            else:
                self.file.read(chunk_size)
            if chunk_size % 2:
                if len(self.file.read(1)) < 1:
                    raise ValueError("invalid RIFF WAVE chunk")
                total_size -= chunk_size + 1
            else:
                total_size -= chunk_size
        raise ValueError("data chunk not found")

    def read(self, pcm_frames):
        """a FrameList of min(max(pcm_frames, 1), remaining) frames
        (wav.py:504-527); IOError if the data chunk ends early"""
        requested = min(max(pcm_frames, 1), self.remaining_pcm_frames)
        nbytes = self.bytes_per_pcm_frame * requested
        data = self.file.read(nbytes)
        if len(data) < nbytes:
            raise IOError("data chunk ends prematurely")
        self.remaining_pcm_frames -= requested
        # 8-bit WAVE samples are unsigned, wider ones signed (wav.py:523-527)
        return _pcm.FrameList(data, self.channels, self.bits_per_sample, False,
                              self.bits_per_sample != 8)

    def seek(self, pcm_frame_offset):
        """position at a PCM frame; returns the frames actually skipped
        (wav.py:529-548)"""
        if pcm_frame_offset < 0:
            raise ValueError("cannot seek to negative value")
        pcm_frame_offset = min(pcm_frame_offset, self.total_pcm_frames)
        self.file.seek(self.data_chunk_offset +
                       pcm_frame_offset * self.bytes_per_pcm_frame, 0)
        self.remaining_pcm_frames = self.total_pcm_frames - pcm_frame_offset
        return pcm_frame_offset

    def close(self):
        self.file.close()


class WaveAudio(object):
    """the slice of the reference's WaveAudio (wav.py:580-655) the
    transcode path uses: stream attributes and to_pcm()"""

    SUFFIX = "wav"
    NAME = SUFFIX

    def __init__(self, filename):
        self.filename = filename
        r = WaveReader(filename)
        try:
            self.__channels = r.channels
            self.__sample_rate = r.sample_rate
            self.__bits_per_sample = r.bits_per_sample
            self.__channel_mask = r.channel_mask
            self.__total_frames = r.total_pcm_frames
        finally:
            r.close()

    def channels(self):
        return self.__channels

    def sample_rate(self):
        return self.__sample_rate

    def bits_per_sample(self):
        return self.__bits_per_sample

    def channel_mask(self):
        return self.__channel_mask

    def total_frames(self):
        return self.__total_frames

    def lossless(self):
        return True

    def to_pcm(self):
        return WaveReader(self.filename)
