"""audiotools.flac — FlacAudio.from_pcm on the MI355X encoder.

Mirrors the slice of the reference's FlacAudio (audiotools/flac.py) that
turns encoder output into the finished file:

  FlacAudio.from_pcm(filename, pcmreader, compression, total_pcm_frames,
                     encoding_function)           flac.py:1696-1845
    - compression presets "0".."8"                 flac.py:1719-1764
    - channel-mask validation                      flac.py:1772-1797
    - PADDING sized for the expected SEEKTABLE     flac.py:1799-1805
    - encode (audiotools.encoders.encode_flac, the GPU path)
    - SEEKTABLE from the encoder's frame offsets, one point per 10 s
      (FlacAudio.seektable, flac.py:1847-1876)
    - WAVEFORMATEXTENSIBLE_CHANNEL_MASK comment for >2 channels or >16 bits
    - metadata rewritten in place, PADDING shrunk by the growth
      (FlacMetaData.add_block ordering flac.py:53-75, update_metadata
      :1369-1427)
  FlacAudio(filename).to_pcm() -> audiotools.decoders.FlacDecoder (GPU),
    positioned past any ID3v2 prefix; PCMReaderError if the decoder cannot
    open the stream                                flac.py:1674-1693
  FlacAudio.convert / verify (AudioFile's, flac.py:2360-2398 and
    __init__.py:3939-3970) -- the track2track / trackverify steps
  FlacAudio.channel_mask()                         flac.py:1284-1341

The rewrite is byte-level host work; encoding and decoding run in libatgpu.
"""

import struct
from bisect import bisect_right

from . import AudioFile, BufferedPCMReader, ChannelMask, EncodingError, InvalidFile
from . import _atgpu
from .id3 import skip_id3v2_comment

# FLAC metadata block ids
STREAMINFO, PADDING, APPLICATION, SEEKTABLE, VORBIS_COMMENT, CUESHEET, PICTURE = \
    0, 1, 2, 3, 4, 5, 6
PREFERRED_ORDER = [STREAMINFO, SEEKTABLE, CUESHEET, VORBIS_COMMENT, PICTURE, APPLICATION,
                   PADDING]

COMPRESSION_PRESETS = {
    "0": dict(block_size=1152, max_lpc_order=0, min_residual_partition_order=0,
              max_residual_partition_order=3),
    "1": dict(block_size=1152, max_lpc_order=0, adaptive_mid_side=True,
              min_residual_partition_order=0, max_residual_partition_order=3),
    "2": dict(block_size=1152, max_lpc_order=0, exhaustive_model_search=True,
              min_residual_partition_order=0, max_residual_partition_order=3),
    "3": dict(block_size=4096, max_lpc_order=6, min_residual_partition_order=0,
              max_residual_partition_order=4),
    "4": dict(block_size=4096, max_lpc_order=8, adaptive_mid_side=True,
              min_residual_partition_order=0, max_residual_partition_order=4),
    "5": dict(block_size=4096, max_lpc_order=8, mid_side=True,
              min_residual_partition_order=0, max_residual_partition_order=5),
    "6": dict(block_size=4096, max_lpc_order=8, mid_side=True,
              min_residual_partition_order=0, max_residual_partition_order=6),
    "7": dict(block_size=4096, max_lpc_order=8, mid_side=True,
              exhaustive_model_search=True, min_residual_partition_order=0,
              max_residual_partition_order=6),
    "8": dict(block_size=4096, max_lpc_order=12, mid_side=True,
              exhaustive_model_search=True, min_residual_partition_order=0,
              max_residual_partition_order=6),
}
DEFAULT_COMPRESSION = "8"

_DEFAULT_MASKS = {1: 0x0004, 2: 0x0003, 3: 0x0007, 4: 0x0033, 5: 0x0037, 6: 0x003F}
_VALID_MASKS = (0x0001, 0x0004, 0x0003, 0x0007, 0x0033, 0x0603, 0x0037, 0x0607,
                0x003F, 0x060F)


class InvalidFLAC(InvalidFile):
    """reference audiotools/flac.py:32-33"""


# FLAC's channel assignments for 3..8 channels without a
# WAVEFORMATEXTENSIBLE_CHANNEL_MASK comment (flac.py:1312-1341)
_FLAC_MASKS = {3: 0x007, 4: 0x033, 5: 0x037, 6: 0x03F, 7: 0x70F, 8: 0x63F}


class UnsupportedChannelCount(EncodingError):
    def __init__(self, filename, count):
        EncodingError.__init__(self, "unsupported channel count %d for %s"
                               % (count, filename))


class UnsupportedChannelMask(EncodingError):
    def __init__(self, filename, mask):
        EncodingError.__init__(self, "unsupported channel mask 0x%X for %s"
                               % (mask, filename))


def _blocks(data):
    """-> ([(type, body)], offset of the first frame)"""
    if data[:4] != b"fLaC":
        raise ValueError("not a FLAC file")
    pos, out = 4, []
    while True:
        h = data[pos]
        length = int.from_bytes(data[pos + 1:pos + 4], "big")
        out.append((h & 0x7F, bytes(data[pos + 4:pos + 4 + length])))
        pos += 4 + length
        if h & 0x80:
            return out, pos


def _comment_values(body, key):
    """the values of KEY=value entries of a VORBIS_COMMENT body (keys
    compared case-insensitively, as VorbisComment's lookup does)"""
    vl = int.from_bytes(body[:4], "little")
    n = int.from_bytes(body[4 + vl:8 + vl], "little")
    pos, prefix, out = 8 + vl, (key + "=").upper().encode("ascii"), []
    for _ in range(n):
        ll = int.from_bytes(body[pos:pos + 4], "little")
        line = body[pos + 4:pos + 4 + ll]
        if line[:len(prefix)].upper() == prefix:
            out.append(line[len(prefix):].decode("utf-8", "replace"))
        pos += 4 + ll
    return out


def _build(blocks):
    out = [b"fLaC"]
    for i, (t, body) in enumerate(blocks):
        last = 0x80 if i == len(blocks) - 1 else 0
        out.append(bytes([last | t]) + len(body).to_bytes(3, "big") + body)
    return b"".join(out)


def _add_block(blocks, block):
    """FlacMetaData.add_block: before the first block later in PREFERRED_ORDER"""
    stop = set(PREFERRED_ORDER[PREFERRED_ORDER.index(block[0]) + 1:])
    for i, (t, _) in enumerate(blocks):
        if t in stop:
            blocks.insert(i, block)
            return
    blocks.append(block)


def seektable_points(offsets, total_frames, seekpoint_interval):
    """FlacAudio.seektable (flac.py:1847-1876): for every interval start, the
    FLAC frame containing it -> (first sample, byte offset, pcm frames)"""
    sample_offsets, frames, total = [], {}, 0
    for byte_offset, pcm_frames in offsets:
        frames[total] = (byte_offset, pcm_frames)
        sample_offsets.append(total)
        total += pcm_frames
    points = []
    for pcm_frame in range(0, total_frames, seekpoint_interval):
        s = sample_offsets[bisect_right(sample_offsets, pcm_frame) - 1]
        points.append((s, frames[s][0], frames[s][1]))
    return points


def _seektable_body(points):
    return b"".join(struct.pack(">QQH", s, o, n) for s, o, n in points)


def _set_comment(body, key, value):
    """VorbisComment[key] = [value] on a VORBIS_COMMENT body (little-endian
    lengths): existing KEY= entries replaced in place, else appended"""
    vl = int.from_bytes(body[:4], "little")
    vendor = body[4:4 + vl]
    n = int.from_bytes(body[4 + vl:8 + vl], "little")
    pos, lines = 8 + vl, []
    for _ in range(n):
        ll = int.from_bytes(body[pos:pos + 4], "little")
        lines.append(body[pos + 4:pos + 4 + ll])
        pos += 4 + ll
    entry = ("%s=%s" % (key, value)).encode("utf-8")
    prefix = (key + "=").upper().encode("ascii")
    hit = [i for i, l in enumerate(lines) if l[:len(prefix)].upper() == prefix]
    if hit:
        lines[hit[0]] = entry
        for i in reversed(hit[1:]):
            del lines[i]
    else:
        lines.append(entry)
    out = [len(vendor).to_bytes(4, "little"), vendor, len(lines).to_bytes(4, "little")]
    for l in lines:
        out += [len(l).to_bytes(4, "little"), l]
    return b"".join(out)


class FlacAudio(AudioFile):
    NAME = "flac"
    SUFFIX = "flac"
    DEFAULT_COMPRESSION = DEFAULT_COMPRESSION
    COMPRESSION_MODES = tuple(map(str, range(0, 9)))

    def __init__(self, filename):
        """read STREAMINFO past any ID3v2 prefix (__read_streaminfo__,
        flac.py:2420-2470); InvalidFLAC if the file cannot be read"""
        AudioFile.__init__(self, filename)
        try:
            with open(filename, "rb") as f:
                f.seek(0, 2)
                size = f.tell()
                self.__stream_suffix = 0
                if size >= 128:
                    f.seek(-128, 2)
                    if f.read(3) == b"TAG":
                        self.__stream_suffix = 128
                f.seek(0, 0)
                self.__stream_offset = skip_id3v2_comment(f)
                data = f.read()
        except IOError as err:
            raise InvalidFLAC(str(err))
        rc, si, _ = _atgpu.read_metadata(data)
        if rc:
            raise InvalidFLAC("Invalid FLAC file" if rc == 1 else "EOF while reading metadata")
        self._si = si
        self._comments = []
        try:
            blocks, _ = _blocks(data)
            for t, body in blocks:
                if t == VORBIS_COMMENT:
                    self._comments.append(body)
        except (ValueError, IndexError):
            pass

    def lossless(self):
        return True

    def channel_mask(self):
        """ChannelMask of the track's layout (flac.py:1284-1341): stereo and
        mono fixed, else the WAVEFORMATEXTENSIBLE_CHANNEL_MASK comment when
        its speaker count matches, else FLAC's default for the count"""
        if self.channels() <= 2:
            return ChannelMask.from_channels(self.channels())
        try:
            if not self._comments:
                raise ValueError()
            mask = ChannelMask(int(_comment_values(
                self._comments[0], u"WAVEFORMATEXTENSIBLE_CHANNEL_MASK")[0], 16))
            return mask if len(mask) == self.channels() else ChannelMask(0)
        except (IndexError, KeyError, ValueError):
            return ChannelMask(_FLAC_MASKS.get(self.channels(), 0))

    def sample_rate(self):
        return self._si.sample_rate

    def channels(self):
        return self._si.channels

    def bits_per_sample(self):
        return self._si.bits_per_sample

    def total_frames(self):
        return self._si.total_samples

    def to_pcm(self):
        """FlacDecoder over the stream from the "fLaC" marker on; if it
        cannot be opened (the file changed since), a PCMReaderError
        carrying the message (flac.py:1674-1693)"""
        from .decoders import FlacDecoder
        from . import PCMReaderError
        try:
            with open(self.filename, "rb") as flac:
                if self.__stream_offset > 0:
                    flac.seek(self.__stream_offset)
                return FlacDecoder(flac)
        except (IOError, ValueError) as msg:
            return PCMReaderError(error_message=str(msg),
                                  sample_rate=self.sample_rate(),
                                  channels=self.channels(),
                                  channel_mask=int(self.channel_mask()),
                                  bits_per_sample=self.bits_per_sample())

    def convert(self, target_path, target_class, compression=None, progress=None):
        """FlacAudio.convert (flac.py:2360-2398): files with foreign RIFF /
        AIFF chunks go through the target's from_wave / from_aiff, which no
        class here has, so every conversion is from_pcm with the exact
        frame count"""
        from . import to_pcm_progress
        return target_class.from_pcm(target_path, to_pcm_progress(self, progress),
                                     compression, total_pcm_frames=self.total_frames())

    @classmethod
    def from_pcm(cls, filename, pcmreader, compression=None, total_pcm_frames=None,
                 encoding_function=None):
        from .encoders import encode_flac
        if compression is None or compression not in cls.COMPRESSION_MODES:
            compression = DEFAULT_COMPRESSION
        if pcmreader.channels > 8:
            raise UnsupportedChannelCount(filename, pcmreader.channels)
        if int(pcmreader.channel_mask) == 0:
            channel_mask = _DEFAULT_MASKS.get(pcmreader.channels, 0)
        elif int(pcmreader.channel_mask) not in _VALID_MASKS:
            raise UnsupportedChannelMask(filename, int(pcmreader.channel_mask))
        else:
            channel_mask = int(pcmreader.channel_mask)
        interval = pcmreader.sample_rate * 10
        if total_pcm_frames is not None:
            expected = total_pcm_frames // interval + (1 if total_pcm_frames % interval else 0)
            padding_size = 4096 + 4 + expected * 18
        else:
            padding_size = 4096
        try:
            offsets = (encode_flac if encoding_function is None else encoding_function)(
                filename, pcmreader=BufferedPCMReader(pcmreader), padding_size=padding_size,
                **COMPRESSION_PRESETS[compression])
            with open(filename, "rb") as f:
                data = f.read()
            blocks, frames_at = _blocks(data)
            old_len = frames_at - 4
            si_body = blocks[0][1]
            total = int.from_bytes(si_body[13:18], "big") & ((1 << 36) - 1)
            _add_block(blocks, (SEEKTABLE, _seektable_body(
                seektable_points(offsets, total, interval))))
            if (pcmreader.channels > 2 or pcmreader.bits_per_sample > 16) and channel_mask:
                for i, (t, body) in enumerate(blocks):
                    if t == VORBIS_COMMENT:
                        blocks[i] = (t, _set_comment(body, u"WAVEFORMATEXTENSIBLE_CHANNEL_MASK",
                                                     u"0x%.4X" % channel_mask))
                        break
            # update_metadata (flac.py:1389-1427): absorb the growth in PADDING
            new_len = sum(4 + len(b) for _, b in blocks)
            delta = new_len - old_len
            pads = [i for i, (t, _) in enumerate(blocks) if t == PADDING]
            if pads and delta <= sum(len(blocks[i][1]) for i in pads):
                for i in pads:
                    plen = len(blocks[i][1])
                    if delta > 0:
                        take = min(delta, plen)
                        blocks[i] = (PADDING, b"\0" * (plen - take))
                        delta -= take
                    elif delta < 0:
                        blocks[i] = (PADDING, b"\0" * (plen - delta))
                        delta = 0
                    else:
                        break
                out = _build(blocks) + data[frames_at:]
            else:
                # padding too small: the metadata grows and the frames move
                out = _build(blocks) + data[frames_at:]
            with open(filename, "wb") as f:
                f.write(out)
            return cls(filename)
        except (IOError, ValueError) as err:
            _unlink(filename)
            raise EncodingError(str(err))
        except Exception:
            _unlink(filename)
            raise


def _unlink(filename):
    import os
    try:
        os.unlink(filename)
    except OSError:
        pass
