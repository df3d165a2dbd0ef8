"""audiotools.wav — RIFF WAVE on either side of the transcode path.

`WaveReader` (reference audiotools/wav.py:421-553) walks the RIFF chunks to
"fmt " and "data" and hands out pcm.FrameLists; `parse_fmt` (:288-354)
decodes the "fmt " chunk (WAVE_FORMAT_PCM with the SMPTE/ITU-R default
masks, or WAVE_FORMAT_EXTENSIBLE with the PCM sub-format GUID).  Config 1
is `encode_flac(out, BufferedPCMReader(WaveReader("wav-2ch.wav")), **FLAC8)`.

`WaveAudio` (:580-1128) carries what track2track / trackverify call on a
wave file: `to_pcm`, `convert` (AudioFile's), `verify` (header, data chunk
and footer checks, :1077-1128), `from_pcm` (a FLAC -> WAV conversion's
writer, :659-729), `chunks` / `wave_header_footer` / `wave_from_chunks`
and the header validators they use (:146-286, :357-418, :839-1003).

Host byte work: the samples are converted by pcm.FrameList; encoding and
decoding run in libatgpu on the GPU.
"""

import io
import struct

from . import pcm as _pcm
from . import AudioFile, ChannelMask, EncodingError, InvalidFile

ERR_WAV_NOT_WAVE = u"not a RIFF WAVE file"
ERR_WAV_INVALID_WAVE = u"invalid RIFF WAVE file"
ERR_WAV_NO_DATA_CHUNK = u"data chunk not found"
ERR_WAV_INVALID_CHUNK = u"invalid RIFF WAVE chunk ID"
ERR_WAV_MULTIPLE_FMT = u"multiple fmt chunks found"
ERR_WAV_PREMATURE_DATA = u"data chunk found before fmt"
ERR_WAV_MULTIPLE_DATA = u"multiple data chunks found"
ERR_WAV_NO_FMT_CHUNK = u"fmt chunk not found"
ERR_WAV_HEADER_EXTRA_DATA = u"%d bytes found after data chunk header"
ERR_WAV_HEADER_IOERROR = u"I/O error reading header data"
ERR_WAV_FOOTER_IOERROR = u"I/O error reading footer data"
ERR_WAV_TRUNCATED_DATA_CHUNK = u"premature end of data chunk"
ERR_WAV_INVALID_SIZE = u"total wave file size mismatch"
ERR_TOTAL_PCM_FRAMES_MISMATCH = u"total_pcm_frames mismatch"

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


class InvalidWave(InvalidFile):
    """reference audiotools/wav.py:574-577"""


def _printable(chunk_id):
    return frozenset(chunk_id).issubset(PRINTABLE_ASCII)


class RIFF_Chunk(object):
    """a raw RIFF chunk: id, declared size, data (reference wav.py:30-83)"""

    def __init__(self, chunk_id, chunk_size, chunk_data):
        self.id = chunk_id
        self.__size = chunk_size
        self.__data = chunk_data

    def __repr__(self):
        return "RIFF_Chunk(%r)" % (self.id,)

    def size(self):
        return self.__size

    def total_size(self):
        return 8 + self.__size + (self.__size % 2)

    def data(self):
        return io.BytesIO(self.__data)

    def verify(self):
        return self.__size == len(self.__data)

    def write(self, f):
        f.write(self.id)
        f.write(struct.pack("<I", self.__size))
        f.write(self.__data)
        if self.__size % 2:
            f.write(b"\0")
        return self.total_size()


class _Reader(object):
    """little-endian field reader over bytes; IOError past the end (the
    BitstreamReader behaviour the validators rely on)"""

    def __init__(self, data):
        self.data, self.pos = data, 0

    def take(self, n):
        if self.pos + n > len(self.data):
            raise IOError("I/O error")
        b = self.data[self.pos:self.pos + n]
        self.pos += n
        return b

    def chunk_header(self):
        return struct.unpack("<4sI", self.take(8))


def validate_header(header):
    """header bytes as wave_header_footer returns them -> (total size, data
    size); ValueError if invalid (reference wav.py:153-236)"""
    header_size = len(header)
    r = _Reader(header)
    try:
        riff, remaining_size, wave = struct.unpack("<4sI4s", r.take(12))
        if riff != b"RIFF":
            raise ValueError(ERR_WAV_NOT_WAVE)
        if wave != b"WAVE":
            raise ValueError(ERR_WAV_INVALID_WAVE)
        total_size = remaining_size + 8
        header_size -= 12
        fmt_found = False
        while header_size > 0:
            chunk_id, chunk_size = r.chunk_header()
            if not _printable(chunk_id):
                raise ValueError(ERR_WAV_INVALID_CHUNK)
            header_size -= 8
            if chunk_id == b"fmt ":
                if fmt_found:
                    raise ValueError(ERR_WAV_MULTIPLE_FMT)
                fmt_found = True
                r.take(chunk_size + chunk_size % 2)
                header_size -= chunk_size + chunk_size % 2
            elif chunk_id == b"data":
                if not fmt_found:
                    raise ValueError(ERR_WAV_PREMATURE_DATA)
                if header_size > 0:
                    raise ValueError(ERR_WAV_HEADER_EXTRA_DATA % header_size)
                return (total_size, chunk_size)
            else:
                r.take(chunk_size + chunk_size % 2)
                header_size -= chunk_size + chunk_size % 2
        raise ValueError(ERR_WAV_NO_DATA_CHUNK)
    except IOError:
        raise ValueError(ERR_WAV_HEADER_IOERROR)


def validate_footer(footer, data_bytes_written):
    """True if the footer after the data chunk is valid; ValueError
    otherwise (reference wav.py:239-285)"""
    total_size = len(footer)
    r = _Reader(footer)
    try:
        if data_bytes_written % 2:
            r.take(1)
            total_size -= 1
        while total_size > 0:
            chunk_id, chunk_size = r.chunk_header()
            if not _printable(chunk_id):
                raise ValueError(ERR_WAV_INVALID_CHUNK)
            total_size -= 8
            if chunk_id == b"fmt ":
                raise ValueError(ERR_WAV_MULTIPLE_FMT)
            if chunk_id == b"data":
                raise ValueError(ERR_WAV_MULTIPLE_DATA)
            r.take(chunk_size + chunk_size % 2)
            total_size -= chunk_size + chunk_size % 2
        return True
    except IOError:
        raise ValueError(ERR_WAV_FOOTER_IOERROR)


def wave_header(sample_rate, channels, channel_mask, bits_per_sample, total_pcm_frames):
    """everything before a RIFF WAVE's PCM data (reference wav.py:357-418):
    a plain fmt chunk for <= 2 channels of <= 16 bits, else
    WAVE_FORMAT_EXTENSIBLE; ValueError if the file would reach 4 GiB"""
    bytes_ps = bits_per_sample // 8
    avg_bytes_per_second = sample_rate * channels * bytes_ps
    block_align = channels * bytes_ps
    if channels <= 2 and bits_per_sample <= 16:
        fmt = struct.pack("<HHIIHH", 1, channels, sample_rate, avg_bytes_per_second,
                          block_align, bits_per_sample)
    else:
        if int(channel_mask) == 0:
            channel_mask = _DEFAULT_MASKS.get(channels, 0)
        fmt = (struct.pack("<HHIIHH", 0xFFFE, channels, sample_rate, avg_bytes_per_second,
                           block_align, bits_per_sample) +
               struct.pack("<HHI", 22, bits_per_sample, int(channel_mask)) + _PCM_SUBFORMAT)
    data_size = bytes_ps * channels * total_pcm_frames
    total_size = 4 + 8 + len(fmt) + 8 + data_size + (data_size % 2)
    if total_size >= (1 << 32):
        raise ValueError("total size too large for wave file")
    return (struct.pack("<4sI4s", b"RIFF", total_size, b"WAVE") +
            struct.pack("<4sI", b"fmt ", len(fmt)) + fmt +
            struct.pack("<4sI", b"data", data_size))


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
            if not _printable(chunk_id):
                raise ValueError(ERR_WAV_INVALID_CHUNK)
            total_size -= 8
            if chunk_id == b"fmt ":
                (self.channels, self.sample_rate, self.bits_per_sample,
                 self.channel_mask) = parse_fmt(self.file.read(chunk_size))
                self.bytes_per_pcm_frame = (self.bits_per_sample // 8) * self.channels
                fmt_read = True
            elif chunk_id == b"data":
                if not fmt_read:
                    raise ValueError(ERR_WAV_PREMATURE_DATA)
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
            raise IOError(ERR_WAV_TRUNCATED_DATA_CHUNK)
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


class WaveAudio(AudioFile):
    """a RIFF WAVE file (reference audiotools/wav.py:580-1128)"""

    SUFFIX = "wav"
    NAME = SUFFIX
    PRINTABLE_ASCII = PRINTABLE_ASCII

    def __init__(self, filename):
        """the stream attributes from the first "fmt " chunk and the size of
        the first "data" chunk, in whatever order they come; a truncated
        "fmt " chunk is passed over, an invalid one raises InvalidWave
        (wav.py:589-629)"""
        AudioFile.__init__(self, filename)
        self.__channels = 0
        self.__sample_rate = 0
        self.__bits_per_sample = 0
        self.__data_size = 0
        self.__channel_mask = 0
        fmt_read = data_read = False
        try:
            for chunk in self.chunks():
                if chunk.id == b"fmt ":
                    try:
                        (self.__channels, self.__sample_rate, self.__bits_per_sample,
                         self.__channel_mask) = parse_fmt(chunk.data().read())
                        fmt_read = True
                        if fmt_read and data_read:
                            break
                    except IOError:
                        continue
                    except ValueError as err:
                        raise InvalidWave(str(err))
                elif chunk.id == b"data":
                    self.__data_size = chunk.size()
                    data_read = True
                    if fmt_read and data_read:
                        break
        except IOError:
            raise InvalidWave("I/O error reading wave")

    def channels(self):
        return self.__channels

    def sample_rate(self):
        return self.__sample_rate

    def bits_per_sample(self):
        return self.__bits_per_sample

    def channel_mask(self):
        return ChannelMask(self.__channel_mask)

    def total_frames(self):
        return self.__data_size // (self.__bits_per_sample // 8) // self.__channels

    def lossless(self):
        return True

    def has_foreign_wave_chunks(self):
        return set([b"fmt ", b"data"]) != set(c.id for c in self.chunks())

    def to_pcm(self):
        return WaveReader(self.filename)

    def chunks(self):
        """RIFF_Chunk for every chunk, data read as far as the file goes
        (wav.py:839-893; the reference defers chunks of 1 MiB or more to a
        file-backed chunk, here they are read the same way); InvalidWave on
        a broken header or chunk id"""
        with open(self.filename, "rb") as wave_file:
            head = wave_file.read(12)
            if len(head) < 12:
                raise InvalidWave(ERR_WAV_INVALID_WAVE)
            riff, total_size, wave = struct.unpack("<4sI4s", head)
            if riff != b"RIFF":
                raise InvalidWave(ERR_WAV_NOT_WAVE)
            if wave != b"WAVE":
                raise InvalidWave(ERR_WAV_INVALID_WAVE)
            total_size -= 4
            while total_size > 0:
                hdr = wave_file.read(8)
                if len(hdr) < 8:
                    raise InvalidWave(ERR_WAV_INVALID_WAVE)
                chunk_id, chunk_size = struct.unpack("<4sI", hdr)
                if not _printable(chunk_id):
                    raise InvalidWave(ERR_WAV_INVALID_CHUNK)
                total_size -= 8
                yield RIFF_Chunk(chunk_id, chunk_size, wave_file.read(chunk_size))
                if chunk_size % 2:
                    if len(wave_file.read(1)) < 1:
                        raise InvalidWave(ERR_WAV_INVALID_CHUNK)
                    total_size -= chunk_size + 1
                else:
                    total_size -= chunk_size

    @classmethod
    def wave_from_chunks(cls, filename, chunk_iter):
        """a RIFF WAVE file from RIFF_Chunk-like objects (wav.py:895-918)"""
        with open(filename, "wb") as wave_file:
            total_size = 4
            wave_file.write(struct.pack("<4sI4s", b"RIFF", total_size, b"WAVE"))
            for chunk in chunk_iter:
                total_size += chunk.write(wave_file)
            wave_file.seek(0, 0)
            wave_file.write(struct.pack("<4sI4s", b"RIFF", total_size, b"WAVE"))

    def wave_header_footer(self):
        """(everything before the data chunk's PCM, everything after it)
        (wav.py:920-1003); ValueError on a broken file, IOError if it ends
        inside a chunk"""
        with open(self.filename, "rb") as f:
            r = _Reader(f.read())
        head, tail = [], []
        cur = head
        fmt_found = False
        riff, size, wave = struct.unpack("<4sI4s", r.take(12))
        if riff != b"RIFF":
            raise ValueError(ERR_WAV_NOT_WAVE)
        if wave != b"WAVE":
            raise ValueError(ERR_WAV_INVALID_WAVE)
        cur.append(struct.pack("<4sI4s", riff, size, wave))
        total_size = size - 4
        while total_size > 0:
            chunk_id, chunk_size = r.chunk_header()
            if not _printable(chunk_id):
                raise ValueError(ERR_WAV_INVALID_CHUNK)
            cur.append(struct.pack("<4sI", chunk_id, chunk_size))
            total_size -= 8
            if chunk_id != b"data":
                if chunk_id == b"fmt ":
                    if fmt_found:
                        raise ValueError(ERR_WAV_MULTIPLE_FMT)
                    fmt_found = True
                cur.append(r.take(chunk_size + chunk_size % 2))
                total_size -= chunk_size + chunk_size % 2
            else:
                r.take(chunk_size)
                cur = tail
                if chunk_size % 2:
                    cur.append(r.take(1))
                    total_size -= chunk_size + 1
                else:
                    total_size -= chunk_size
        if not fmt_found:
            # the reference returns (not raises) this error, whose unpacking
            # in verify() then fails with a ValueError: same outcome
            raise ValueError(ERR_WAV_NO_FMT_CHUNK)
        return (b"".join(head), b"".join(tail))

    def verify(self, progress=None):
        """True if header, data chunk and footer are consistent; InvalidWave
        otherwise (wav.py:1077-1128)"""
        from . import CounterPCMReader, to_pcm_progress, transfer_framelist_data
        try:
            (header, footer) = self.wave_header_footer()
        except (IOError, ValueError) as err:
            raise InvalidWave(str(err))
        try:
            (total_size, data_size) = validate_header(header)
        except ValueError as err:
            raise InvalidWave(str(err))
        counter = CounterPCMReader(to_pcm_progress(self, progress))
        try:
            transfer_framelist_data(counter, lambda f: f)
        except IOError:
            raise InvalidWave(ERR_WAV_TRUNCATED_DATA_CHUNK)
        data_bytes_written = counter.bytes_written()
        if data_size != data_bytes_written:
            raise InvalidWave(ERR_WAV_TRUNCATED_DATA_CHUNK)
        try:
            validate_footer(footer, data_bytes_written)
        except ValueError:
            raise InvalidWave(ERR_WAV_INVALID_SIZE)
        if len(header) + data_size + len(footer) != total_size:
            raise InvalidWave(ERR_WAV_INVALID_SIZE)
        return True

    @classmethod
    def from_pcm(cls, filename, pcmreader, compression=None, total_pcm_frames=None):
        """write pcmreader's data as a RIFF WAVE file (wav.py:659-729), the
        writer of a FLAC/ALAC -> WAV conversion.  As the reference does, a
        pad byte follows the data when the FRAME count is odd, and the
        header is rewritten with the counted frames when no total was given"""
        from . import CounterPCMReader, transfer_framelist_data
        try:
            header = wave_header(pcmreader.sample_rate, pcmreader.channels,
                                 pcmreader.channel_mask, pcmreader.bits_per_sample,
                                 total_pcm_frames if total_pcm_frames is not None else 0)
        except ValueError as err:
            raise EncodingError(str(err))
        try:
            f = open(filename, "wb")
        except IOError as err:
            raise EncodingError(str(err))
        try:
            counter = CounterPCMReader(pcmreader)
            f.write(header)
            try:
                transfer_framelist_data(counter, f.write, pcmreader.bits_per_sample > 8,
                                        False)
            except (IOError, ValueError) as err:
                f.close()
                cls.__unlink__(filename)
                raise EncodingError(str(err))
            except Exception:
                f.close()
                cls.__unlink__(filename)
                raise
            if counter.frames_written % 2:
                f.write(b"\0")
            if total_pcm_frames is not None:
                if counter.frames_written != total_pcm_frames:
                    f.close()
                    cls.__unlink__(filename)
                    raise EncodingError(ERR_TOTAL_PCM_FRAMES_MISMATCH)
            else:
                f.seek(0, 0)
                f.write(wave_header(pcmreader.sample_rate, pcmreader.channels,
                                    pcmreader.channel_mask, pcmreader.bits_per_sample,
                                    counter.frames_written))
        finally:
            if not f.closed:
                f.close()
        return WaveAudio(filename)
