"""audiotools.m4a — ALAC in an M4A container on the MI355X engine.

Mirrors the slice of the reference's audiotools/m4a.py that the transcode
path uses:

  ALACAudio.from_pcm(filename, pcmreader, compression=None,
                     total_pcm_frames=None, block_size=4096,
                     encoding_function=None)          m4a.py:941-1124
    - bits per sample 16/24 and the channel masks it accepts (:953-972)
    - encode (audiotools.encoders.encode_alac, the GPU path) into the mdat
    - ftyp / moov (mvhd, trak/tkhd, mdia/mdhd/hdlr/minf(smhd, dinf/dref,
      stbl(stsd/alac, stts, stsc, stsz, stco))), udta/meta) / free / mdat,
      byte for byte as the reference's atom builders write them
      (m4a.py:1126-1400, m4a_atoms.py)
  ALACAudio(filename).to_pcm() -> audiotools.decoders.ALACDecoder (GPU)
  ALACAudio.convert / verify (AudioFile's, __init__.py:3760-3774,
    3939-3970): the config-5 chain's source side under track2track /
    trackverify; InvalidALAC for a file the decoder cannot open

The container is host byte work; the ALAC bitstreams are encoded and
decoded by libatgpu (alac_encode.hip / alac_decode.hip).
"""

import struct
import time

from . import AudioFile, BufferedPCMReader, ChannelMask, EncodingError, InvalidFile, VERSION

INITIAL_HISTORY = 10      # m4a.py:759-762
HISTORY_MULTIPLIER = 40
MAXIMUM_K = 14
BLOCK_SIZE = 4096
ALAC_FRAMES_PER_CHUNK = 5  # m4a.py:1348, 1366
APPLE_EPOCH = 2082844800

VALID_MASKS = (0x0001, 0x0004, 0x0003, 0x0007, 0x0107, 0x0037, 0x003F, 0x013F, 0x00FF,
               0x0000)
_MATRIX = (0x10000, 0, 0, 0, 0x10000, 0, 0, 0, 0x40000000)


class InvalidALAC(InvalidFile):
    """reference audiotools/m4a.py:745-746"""


class UnsupportedBitsPerSample(EncodingError):
    def __init__(self, filename, bits_per_sample):
        EncodingError.__init__(self, "unsupported bits per sample %d for %s"
                               % (bits_per_sample, filename))


class UnsupportedChannelMask(EncodingError):
    def __init__(self, filename, mask):
        EncodingError.__init__(self, "unsupported channel mask 0x%X for %s" % (mask, filename))


def atom(name, body):
    """32-bit size + 4-byte name + body (M4A_Tree_Atom / Leaf builds)"""
    return struct.pack(">I", len(body) + 8) + name + body


def ftyp_atom():
    """M4A_FTYP_Atom('M4A ', 0, ['M4A ', 'mp42', 'isom', 4 x NUL])"""
    return atom(b"ftyp", b"M4A " + struct.pack(">I", 0) + b"M4A mp42isom\0\0\0\0")


def _mvhd(rate, date, total):
    # "8u 24u" "32u 32u 32u 32u 32u 16u 10P" "9* 32u" "64U 32u 64U 32u 32u"
    return atom(b"mvhd", struct.pack(">B3xIIIIIH10x", 0, date, date, rate, total, 0x10000,
                                     0x100) +
                struct.pack(">9I", *_MATRIX) + struct.pack(">QIQII", 0, 0, 0, 0, 2))


def _tkhd(date, total):
    # "8u 20p 1u 1u 1u 1u": version 0, in preview/movie/enabled
    # "32u 32u 32u 4P 32u 8P 16u 16u 16u 2P" "9* 32u" "32u 32u"
    return atom(b"tkhd", struct.pack(">I", 0x7) +
                struct.pack(">III4xI8xHHH2x", date, date, 1, total, 0, 0, 0x100) +
                struct.pack(">9I", *_MATRIX) + struct.pack(">II", 0, 0))


def _mdhd(rate, date, total):
    lang = 0
    for c in "und":  # "1p 5u 5u 5u"
        lang = (lang << 5) | (ord(c) - 0x60)
    return atom(b"mdhd", struct.pack(">B3xIIIIHH", 0, date, date, rate, total, lang, 0))


def _hdlr(subtype, manufacturer):
    # "8u 24u 4b 4b 4b 32u 32u 8u %db %dP": empty name + 1 padding byte
    return atom(b"hdlr", struct.pack(">I4s4s4sIIB", 0, b"\0" * 4, subtype, manufacturer, 0, 0,
                                     0) + b"\0")


def _stsd(channels, bps, rate, block_size, max_frame, bitrate):
    sub = atom(b"alac", struct.pack(">4xIxBBBBBHIII", block_size, bps, HISTORY_MULTIPLIER,
                                    INITIAL_HISTORY, MAXIMUM_K, channels, 0x00FF, max_frame,
                                    bitrate, rate))
    desc = atom(b"alac", struct.pack(">6xHHH4sHHHHI", 1, 0, 0, b"\0" * 4, channels, bps, 0, 0,
                                     0xAC440000) + sub)
    return atom(b"stsd", struct.pack(">II", 0, 1) + desc)


def stts_times(total, block_size):
    """m4a.py:1330-1340: full blocks + one short block, empty ones dropped"""
    times = [(total // block_size, block_size), (1, total % block_size)]
    return [t for t in times if t[0] > 0 and t[1] > 0]


def stsc_blocks(total, block_size):
    """m4a.py:1342-1358"""
    frames = total // block_size + (1 if total % block_size else 0)
    if frames < ALAC_FRAMES_PER_CHUNK:
        return [(1, frames, 1)]
    blocks = [(1, ALAC_FRAMES_PER_CHUNK, 1)]
    if frames % ALAC_FRAMES_PER_CHUNK:
        blocks.append((1 + frames // ALAC_FRAMES_PER_CHUNK, frames % ALAC_FRAMES_PER_CHUNK, 1))
    return blocks


def stco_offsets(mdat_offset, frame_sizes):
    """m4a.py:1369-1381: one chunk of 5 framesets per offset"""
    offs = [mdat_offset + 8]
    for i in range(0, len(frame_sizes), ALAC_FRAMES_PER_CHUNK):
        offs.append(offs[-1] + sum(frame_sizes[i:i + ALAC_FRAMES_PER_CHUNK]))
    return offs[:-1]


def _meta(version):
    data = atom(b"data", struct.pack(">I4x", 1) +
                ("Python Audio Tools %s" % version).encode("utf-8"))
    ilst = atom(b"ilst", atom(b"\xa9too", data))
    return atom(b"meta", struct.pack(">I", 0) + _hdlr(b"mdir", b"appl") + ilst +
                atom(b"free", b"\0" * 1024))


def moov_atom(channels, bps, rate, date, mdat_offset, mdat_size, block_size, total,
              frame_sizes, version=VERSION):
    """__moov_atom__ (m4a.py:1136-1180) with every child atom"""
    bitrate = (mdat_size * 8 * rate) // total if total else 0
    times = stts_times(total, block_size)
    stts = atom(b"stts", struct.pack(">II", 0, len(times)) +
                b"".join(struct.pack(">II", *t) for t in times))
    blocks = stsc_blocks(total, block_size)
    stsc = atom(b"stsc", struct.pack(">II", 0, len(blocks)) +
                b"".join(struct.pack(">III", *b) for b in blocks))
    stsz = atom(b"stsz", struct.pack(">III", 0, 0, len(frame_sizes)) +
                b"".join(struct.pack(">I", s) for s in frame_sizes))
    offs = stco_offsets(mdat_offset, frame_sizes)
    stco = atom(b"stco", struct.pack(">II", 0, len(offs)) +
                b"".join(struct.pack(">I", o & 0xFFFFFFFF) for o in offs))
    stbl = atom(b"stbl", _stsd(channels, bps, rate, block_size,
                               max(frame_sizes) if frame_sizes else 0, bitrate) +
                stts + stsc + stsz + stco)
    dinf = atom(b"dinf", atom(b"dref", struct.pack(">II", 0, 1) +
                              atom(b"url ", b"\x00\x00\x00\x01")))
    minf = atom(b"minf", atom(b"smhd", b"\0" * 8) + dinf + stbl)
    mdia = atom(b"mdia", _mdhd(rate, date, total) + _hdlr(b"soun", b"\0" * 4) + minf)
    trak = atom(b"trak", _tkhd(date, total) + mdia)
    return atom(b"moov", _mvhd(rate, date, total) + trak + atom(b"udta", _meta(version)))


def free_atom(size=0x1000):
    return atom(b"free", b"\0" * size)


def m4a_file(channels, bps, rate, block_size, total, mdat, frame_sizes, create_date=None,
             version=VERSION):
    """complete file: ftyp, moov, free(4096), then the mdat atom (whose
    8-byte header is part of `mdat`); moov's stco points into it
    (m4a.py:1085-1124)"""
    date = (int(time.time()) + APPLE_EPOCH if create_date is None else create_date) & 0xFFFFFFFF
    ftyp = ftyp_atom()
    free = free_atom()
    probe = moov_atom(channels, bps, rate, date, 0, len(mdat), block_size, total, frame_sizes,
                      version)
    pre = len(ftyp) + len(probe) + len(free)
    moov = moov_atom(channels, bps, rate, date, pre, len(mdat), block_size, total,
                     frame_sizes, version)
    return ftyp + moov + free + bytes(mdat)


class ALACAudio(AudioFile):
    """the reference's ALACAudio (m4a.py:750-1124), transcode slice"""

    SUFFIX = "m4a"
    NAME = "alac"
    BINARIES = ()
    BLOCK_SIZE = BLOCK_SIZE
    INITIAL_HISTORY = INITIAL_HISTORY
    HISTORY_MULTIPLIER = HISTORY_MULTIPLIER
    MAXIMUM_K = MAXIMUM_K

    def __init__(self, filename):
        from . import decoders
        AudioFile.__init__(self, filename)
        try:
            d = decoders.ALACDecoder(filename)
        except (IOError, ValueError) as err:
            raise InvalidALAC(str(err))
        self._channels = d.channels
        self._rate = d.sample_rate
        self._bps = d.bits_per_sample
        self._mask = d.channel_mask
        self._total = d.total_frames
        d.close()

    def channels(self):
        return self._channels

    def sample_rate(self):
        return self._rate

    def bits_per_sample(self):
        return self._bps

    def channel_mask(self):
        return ChannelMask(self._mask)

    def total_frames(self):
        return self._total

    def lossless(self):
        return True

    def to_pcm(self):
        from .decoders import ALACDecoder
        return ALACDecoder(self.filename)

    @classmethod
    def from_pcm(cls, filename, pcmreader, compression=None, total_pcm_frames=None,
                 block_size=4096, encoding_function=None, create_date=None):
        """encode pcmreader to a new ALAC file (m4a.py:941-1124); the mdat is
        produced by encode_alac on the GPU, the atoms around it here"""
        import io
        from .encoders import encode_alac
        if pcmreader.bits_per_sample not in (16, 24):
            raise UnsupportedBitsPerSample(filename, pcmreader.bits_per_sample)
        if int(pcmreader.channel_mask) not in VALID_MASKS:
            raise UnsupportedChannelMask(filename, int(pcmreader.channel_mask))
        mdat = io.BytesIO()
        try:
            (frame_sizes, frames) = (encode_alac if encoding_function is None else
                                     encoding_function)(
                file=mdat, pcmreader=BufferedPCMReader(pcmreader), block_size=block_size,
                initial_history=cls.INITIAL_HISTORY,
                history_multiplier=cls.HISTORY_MULTIPLIER, maximum_k=cls.MAXIMUM_K)
        except (IOError, ValueError) as err:
            raise EncodingError(str(err))
        if total_pcm_frames is not None and frames != total_pcm_frames:
            raise EncodingError("total PCM frames mismatch")
        data = m4a_file(pcmreader.channels, pcmreader.bits_per_sample,
                        pcmreader.sample_rate, block_size, frames, mdat.getvalue(),
                        frame_sizes, create_date)
        try:
            with open(filename, "wb") as f:
                f.write(data)
        except IOError as err:
            raise EncodingError(str(err))
        return cls(filename)
