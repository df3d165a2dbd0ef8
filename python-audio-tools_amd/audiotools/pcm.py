"""audiotools.pcm — the FrameList PCM container, Python 3 / numpy edition.

Mirrors the reference's C type `pcm.FrameList` (reference src/pcm.c:37-96,
layout src/pcm.h:40-54): `frames` PCM frames of `channels` interleaved
signed integer samples of `bits_per_sample` bits.  The samples live in a
numpy int32 array in exactly the reference's interleaved order
(`samples[f * channels + c]`), so the GPU engine can take it as its
ATG_PCM_S32 container without a copy.
"""

import numpy as np

__all__ = ["FrameList", "FloatFrameList", "from_list", "from_frames",
           "from_channels", "from_float_frames", "from_float_channels",
           "empty_framelist", "empty_float_framelist"]


def _check_bps(bits_per_sample):
    if bits_per_sample not in (8, 16, 24):
        raise ValueError("bits_per_sample must be 8, 16 or 24")


class FrameList(object):
    """FrameList(string, channels, bits_per_sample, is_big_endian, is_signed)

    Builds a FrameList from raw PCM bytes (reference FrameList_init,
    src/pcm.c; byte conversion src/pcm.c:1599-1700).
    """

    __slots__ = ("_samples", "channels", "bits_per_sample")

    def __init__(self, data=b"", channels=1, bits_per_sample=16,
                 is_big_endian=False, is_signed=True):
        _check_bps(bits_per_sample)
        if channels < 1:
            raise ValueError("number of channels must be > 0")
        width = bits_per_sample // 8
        data = bytes(data)
        if len(data) % (channels * width):
            raise ValueError(
                "number of samples must be divisible by bits-per-sample "
                "and number of channels")
        self.channels = channels
        self.bits_per_sample = bits_per_sample
        # the common containers straight through numpy's own dtypes
        # (WAVE: 16-bit signed little-endian, 8-bit unsigned)
        if width == 2 and is_signed:
            self._samples = np.frombuffer(
                data, dtype=">i2" if is_big_endian else "<i2").astype(np.int32)
            return
        if width == 1:
            v = np.frombuffer(data, dtype=np.int8 if is_signed else np.uint8)
            self._samples = v.astype(np.int32) - (0 if is_signed else 128)
            return
        raw = np.frombuffer(data, dtype=np.uint8).reshape(-1, width)
        if is_big_endian:
            raw = raw[:, ::-1]
        value = np.zeros(raw.shape[0], dtype=np.int64)
        for b in range(width):
            value |= raw[:, b].astype(np.int64) << (8 * b)
        if is_signed:
            sign = np.int64(1) << (bits_per_sample - 1)
            value = (value ^ sign) - sign
        else:
            value = value - (np.int64(1) << (bits_per_sample - 1))
        self._samples = value.astype(np.int32)

    @classmethod
    def _wrap(cls, samples, channels, bits_per_sample):
        fl = cls.__new__(cls)
        fl._samples = np.ascontiguousarray(samples, dtype=np.int32)
        fl.channels = channels
        fl.bits_per_sample = bits_per_sample
        return fl

    # --- attributes -------------------------------------------------
    @property
    def frames(self):
        return len(self._samples) // self.channels

    @property
    def samples(self):
        """interleaved int32 samples (numpy array, read-only by convention)"""
        return self._samples

    def frame_count(self, bytes_count):
        """whole PCM frames in `bytes_count` bytes, at least 1
        (FrameList_frame_count, src/pcm.c:618-631)"""
        per = self.channels * (self.bits_per_sample // 8)
        bytes_count -= bytes_count % per
        return bytes_count // per if bytes_count else 1

    # --- sequence protocol ------------------------------------------
    def __len__(self):
        return len(self._samples)

    def __getitem__(self, i):
        return int(self._samples[i])

    def __iter__(self):
        return iter(int(x) for x in self._samples)

    def __eq__(self, other):
        return (isinstance(other, FrameList) and
                self.channels == other.channels and
                self.bits_per_sample == other.bits_per_sample and
                np.array_equal(self._samples, other._samples))

    def __ne__(self, other):
        return not self.__eq__(other)

    def __add__(self, other):
        if not isinstance(other, FrameList):
            raise TypeError("can only concatenate FrameList with other FrameLists")
        if (other.channels != self.channels or
                other.bits_per_sample != self.bits_per_sample):
            raise ValueError("FrameLists must have the same number of "
                             "channels and bits per sample")
        return FrameList._wrap(np.concatenate([self._samples, other._samples]),
                               self.channels, self.bits_per_sample)

    def __repr__(self):
        return "FrameList(frames=%d, channels=%d, bits_per_sample=%d)" % (
            self.frames, self.channels, self.bits_per_sample)

    # --- methods (src/pcm.c:70-96) ----------------------------------
    def frame(self, index):
        if index < 0 or index >= self.frames:
            raise IndexError("frame index out of range")
        c = self.channels
        return FrameList._wrap(self._samples[index * c:(index + 1) * c], c,
                               self.bits_per_sample)

    def channel(self, index):
        if index < 0 or index >= self.channels:
            raise IndexError("channel index out of range")
        return FrameList._wrap(self._samples[index::self.channels], 1,
                               self.bits_per_sample)

    def split(self, count):
        """split(count) -> (head, tail); head holds up to `count` frames"""
        if count < 0:
            raise ValueError("split size must be >= 0")
        cut = min(count, self.frames) * self.channels
        return (FrameList._wrap(self._samples[:cut], self.channels,
                                self.bits_per_sample),
                FrameList._wrap(self._samples[cut:], self.channels,
                                self.bits_per_sample))

    def to_bytes(self, is_big_endian, is_signed=True):
        width = self.bits_per_sample // 8
        v = self._samples.astype(np.int64)
        if not is_signed:
            v = v + (np.int64(1) << (self.bits_per_sample - 1))
        u = (v & ((np.int64(1) << (8 * width)) - 1)).astype(np.uint64)
        out = np.empty((len(u), width), dtype=np.uint8)
        for b in range(width):
            out[:, b] = (u >> np.uint64(8 * b)) & np.uint64(0xFF)
        if is_big_endian:
            out = out[:, ::-1]
        return out.tobytes()

    def to_float(self):
        """-> FloatFrameList of samples / 2^(bps-1) in fp64
        (FrameList_to_float, src/pcm.c:599-615)"""
        return FloatFrameList._wrap(
            self._samples.astype(np.float64) / float(1 << (self.bits_per_sample - 1)),
            self.channels)


def _cvttsd2si(values):
    """(int) of fp64 values with x86 cvttsd2si semantics: truncation toward
    zero, and INT_MIN for NaN and anything outside int32 (the reference's
    C cast, src/pcm.c:1222, compiled for x86-64)"""
    v = np.asarray(values, dtype=np.float64)
    out = np.full(v.shape, -(1 << 31), dtype=np.int64)
    ok = np.isfinite(v) & (v > -2147483649.0) & (v < 2147483648.0)
    out[ok] = np.trunc(v[ok]).astype(np.int64)
    return out


class FloatFrameList(object):
    """FloatFrameList(float_list, channels): `frames` PCM frames of
    `channels` interleaved fp64 samples in [-1.0, 1.0) (reference C type
    pcm.FloatFrameList, src/pcm.c:907-1380)"""

    __slots__ = ("_samples", "channels")

    def __init__(self, data, channels):
        if isinstance(data, (str, bytes)) or not hasattr(data, "__len__"):
            raise TypeError("FloatFrameList requires a sequence of floats")
        if channels < 1:
            raise ValueError("number of channels must be > 0")
        if len(data) % channels:
            raise ValueError("number of samples must be divisible by number of channels")
        try:
            self._samples = np.array([float(x) for x in data], dtype=np.float64)
        except (TypeError, ValueError):
            raise TypeError("FloatFrameList samples must be floats")
        self.channels = channels

    @classmethod
    def _wrap(cls, samples, channels):
        fl = cls.__new__(cls)
        fl._samples = np.ascontiguousarray(samples, dtype=np.float64)
        fl.channels = channels
        return fl

    @property
    def frames(self):
        return len(self._samples) // self.channels

    @property
    def samples(self):
        return self._samples

    def __len__(self):
        return len(self._samples)

    def __getitem__(self, i):
        if i < 0 or i >= len(self._samples):
            raise IndexError("index out of range")
        return float(self._samples[i])

    def __iter__(self):
        return iter(float(x) for x in self._samples)

    def __eq__(self, other):
        return (isinstance(other, FloatFrameList) and self.channels == other.channels and
                np.array_equal(self._samples, other._samples))

    def __ne__(self, other):
        return not self.__eq__(other)

    def __add__(self, other):
        if not isinstance(other, FloatFrameList):
            raise TypeError("can only concatenate FloatFrameList with other FloatFrameLists")
        if other.channels != self.channels:
            raise ValueError("both FloatFrameLists must have the same number of channels")
        return FloatFrameList._wrap(np.concatenate([self._samples, other._samples]),
                                    self.channels)

    def __mul__(self, count):
        return FloatFrameList._wrap(np.tile(self._samples, max(int(count), 0)), self.channels)

    def __repr__(self):
        return "FloatFrameList(frames=%d, channels=%d)" % (self.frames, self.channels)

    def frame(self, index):
        if index < 0 or index >= self.frames:
            raise IndexError("frame number out of range")
        c = self.channels
        return FloatFrameList._wrap(self._samples[index * c:(index + 1) * c], c)

    def channel(self, index):
        if index < 0 or index >= self.channels:
            raise IndexError("channel number out of range")
        return FloatFrameList._wrap(self._samples[index::self.channels], 1)

    def split(self, count):
        """split(frames) -> (head, tail) (FloatFrameList_split,
        src/pcm.c:1229-1288); IndexError for a negative split point"""
        if count < 0:
            raise IndexError("split point must be positive")
        cut = min(count, self.frames) * self.channels
        return (FloatFrameList._wrap(self._samples[:cut], self.channels),
                FloatFrameList._wrap(self._samples[cut:], self.channels))

    @staticmethod
    def from_frames(frames):
        return from_float_frames(frames)

    @staticmethod
    def from_channels(channels):
        return from_float_channels(channels)

    def to_int(self, bits_per_sample):
        """-> FrameList of (int)(sample * 2^(bps-1)) clamped to the bps range
        (FloatFrameList_to_int, src/pcm.c:1198-1227)"""
        adjustment = 1 << (bits_per_sample - 1)
        v = _cvttsd2si(self._samples * adjustment)
        v = np.maximum(np.minimum(v, adjustment - 1), -adjustment)
        return FrameList._wrap(v, self.channels, bits_per_sample)


def from_list(values, channels, bits_per_sample, is_signed=True):
    """from_list(list, channels, bits_per_sample, is_signed) -> FrameList"""
    _check_bps(bits_per_sample)
    arr = np.asarray(list(values), dtype=np.int64)
    if len(arr) % channels:
        raise ValueError("number of samples must be divisible by channels")
    if not is_signed:
        arr = arr - (np.int64(1) << (bits_per_sample - 1))
    lo, hi = -(1 << (bits_per_sample - 1)), (1 << (bits_per_sample - 1)) - 1
    if len(arr) and (arr.min() < lo or arr.max() > hi):
        raise ValueError("sample value out of range for bits_per_sample")
    return FrameList._wrap(arr, channels, bits_per_sample)


def from_frames(frames):
    """concatenate single-frame FrameLists"""
    frames = list(frames)
    if not frames:
        raise ValueError("at least one FrameList required")
    out = frames[0]
    for f in frames[1:]:
        out = out + f
    return out


def from_channels(channels):
    """interleave single-channel FrameLists"""
    channels = list(channels)
    if not channels:
        raise ValueError("at least one FrameList required")
    n = channels[0].frames
    bps = channels[0].bits_per_sample
    for c in channels:
        if c.channels != 1 or c.frames != n or c.bits_per_sample != bps:
            raise ValueError("all channels must be mono FrameLists of equal length")
    stacked = np.stack([c.samples for c in channels], axis=1).reshape(-1)
    return FrameList._wrap(stacked, len(channels), bps)


def empty_framelist(channels, bits_per_sample):
    return FrameList._wrap(np.zeros(0, dtype=np.int32), channels, bits_per_sample)


def empty_float_framelist(channels):
    return FloatFrameList._wrap(np.zeros(0, dtype=np.float64), channels)


def from_float_frames(frames):
    """concatenate single-frame FloatFrameLists (src/pcm.c FloatFrameList_from_frames)"""
    frames = list(frames)
    if not frames:
        raise IndexError("list index out of range")
    for f in frames:
        if not isinstance(f, FloatFrameList):
            raise TypeError("frames must be of type FloatFrameList")
        if f.channels != frames[0].channels:
            raise ValueError("all subframes must have the same number of channels")
        if f.frames != 1:
            raise ValueError("all subframes must be 1 frame long")
    return FloatFrameList._wrap(np.concatenate([f.samples for f in frames]),
                                frames[0].channels)


def from_float_channels(channels):
    """interleave single-channel FloatFrameLists (src/pcm.c
    FloatFrameList_from_channels)"""
    channels = list(channels)
    if not channels:
        raise IndexError("list index out of range")
    for c in channels:
        if not isinstance(c, FloatFrameList):
            raise TypeError("channels must be of type FloatFrameList")
        if c.frames != channels[0].frames:
            raise ValueError("all channels must have the same number of frames")
        if c.channels != 1:
            raise ValueError("all channels must be 1 channel wide")
    return FloatFrameList._wrap(np.stack([c.samples for c in channels], axis=1).reshape(-1),
                                len(channels))
