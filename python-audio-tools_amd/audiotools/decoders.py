"""audiotools.decoders — FLAC decoding on the MI355X.

`FlacDecoder` keeps the Python-visible contract of the reference's C type
audiotools.decoders.FlacDecoder (src/decoders/flac.c, methods :145-166):

  FlacDecoder(file)        file object (or filename) positioned at "fLaC";
                           ValueError / IOError from the metadata reader
                           (flacdec_read_metadata, flac.c:568-707)
  .sample_rate .bits_per_sample .channels .channel_mask
  .read(n)                 one FLAC frame per call as a pcm.FrameList; an
                           empty FrameList once the stream is done, after
                           the STREAMINFO MD5 check (flac.c:174-285, 479-493);
                           ValueError with the reference's message on a bad
                           frame, IOError "EOF reading frame" on truncation
  .seek(pcm_frame_offset)  last SEEKTABLE point at or before the offset
                           (flac.c:287-356)
  .offsets()               [(byte offset from the current position, block
                           size)] of the frames left, CRC-16 unchecked
                           (flac.c:365-443)
  .close()                 further reads raise ValueError

The stream is decoded by libatgpu (HIP kernels, flac_decode.hip) in bounded
segments as read() needs them (SEGMENT_BYTES of compressed data per GPU
call, the MD5 chained on the host); read() hands out the decoded frames in
order and raises the decode status at the frame where the reference would.
`decode_flac_batch` is the batch entry trackverify-style callers use.
`ALACDecoder` / `decode_alac_batch` do the same for ALAC in M4A
(reference src/decoders/alac.c; GPU kernels alac_decode.hip).
There is no CPU decoding path.
"""

import hashlib

import numpy as np

from . import _atgpu
from . import pcm


def _read_all(file):
    """-> (bytes, seekable): filenames and file objects can seek, raw bytes
    cannot (the reference seeks only streams from file objects,
    flac.c:298-307)"""
    if isinstance(file, str):
        with open(file, "rb") as f:
            return f.read(), True
    if isinstance(file, (bytes, bytearray, memoryview)):
        return bytes(file), False
    return file.read(), True


def _metadata_error(rc):
    if rc == 1:
        return ValueError("not a FLAC file")
    return IOError("EOF while reading metadata")


def _status_error(status):
    if status == _atgpu.FD_EOF:
        return IOError(_atgpu.FD_MESSAGES[_atgpu.FD_EOF])
    return ValueError(_atgpu.FD_MESSAGES.get(status, "Error"))


# compressed bytes per GPU decode call of a streaming FlacDecoder: bounds
# the decoded PCM held in host memory (int32 samples: about 4x this for
# 16-bit audio) whatever the stream's length
SEGMENT_BYTES = 8 << 20


def _frame_bytes(samples, bits_per_sample):
    """FrameList.to_bytes(False, True) of int32 samples: little-endian,
    saturated to the bps range (src/pcm.c:1826-1948)"""
    bb = (bits_per_sample + 7) // 8
    hi = (1 << (bits_per_sample - 1)) - 1
    a = np.clip(np.asarray(samples, dtype=np.int64), -hi - 1, hi).astype("<i4")
    return a.view(np.uint8).reshape(-1, 4)[:, :bb].tobytes()


class FlacDecoder(object):
    """reference src/decoders/flac.c FlacDecoder, decoded on the GPU in
    bounded segments: each GPU call decodes the frames of SEGMENT_BYTES of
    compressed data (a window that ends inside a frame resumes at that
    frame, whose byte position the decode reports as walk_end; an error is
    raised only when the frame that stops a walk is the first of its window,
    so it cannot be the window's cut), and the STREAMINFO MD5 runs over the
    handed-out PCM on the host, chained across segments"""

    def __init__(self, file):
        data, self._seekable = _read_all(file)
        rc, si, points = _atgpu.read_metadata(data)
        if rc:
            raise _metadata_error(rc)
        self._data = data
        self._si = si
        self._seekpoints = points
        self.sample_rate = si.sample_rate
        self.bits_per_sample = si.bits_per_sample
        self.channels = si.channels
        self.channel_mask = si.channel_mask
        self._closed = False
        # the bitstream position: byte offset from the first frame and
        # remaining_samples there; MD5 validation only from sample 0
        # (FlacDecoder_seek, flac.c:317-352)
        self._start_byte = 0
        self._remaining = si.total_samples
        self._validate = True
        self._reset()

    def _reset(self):
        self._finalized = False
        self._seg_byte = self._start_byte      # next window's first byte
        self._seg_remaining = self._remaining  # remaining_samples there
        self._seg = None                       # (pcm, frame starts, byte offsets)
        self._seg_n = 0
        self._next = 0
        self._stop = None                      # status after the current segment
        # FlacDecoder_verify_okay (flac.c:479-493): a blank MD5 always passes
        self._md5 = hashlib.md5() if self._validate and any(self._si.md5) else None

    def _body(self):
        return memoryview(self._data)[self._si.frames_offset:]

    def _decode_segment(self):
        body = self._body()
        start, rem = self._seg_byte, self._seg_remaining
        win = SEGMENT_BYTES
        while True:
            end = min(start + win, len(body))
            final = end >= len(body)
            chunk = bytes(body[start:end])
            track = _atgpu.dec_track(0, len(chunk), self._si)
            track.total_samples = rem
            track.md5[:] = bytes(16)  # the MD5 is chained on the host
            pcm_i32, res, offs, bss = _atgpu.decoder().decode(
                chunk + b"\0" * ((-len(chunk)) % 4), [track])
            r = res[0]
            if r.status == _atgpu.FD_OK or final or r.n_frames > 0 or \
                    r.status == _atgpu.FD_FRAME_CRC:
                break
            win *= 4  # the window's first frame may be longer than the window
        n, ch = r.n_frames, self.channels
        lens, rems = [], []
        for bs in bss[r.first_frame:r.first_frame + n]:
            rems.append(rem)
            lens.append(min(int(bs), rem))
            rem = (rem - int(bs)) % (1 << 64)
        self._seg_rems = rems
        # where the frame after these n sits (offsets() resumes there)
        self._after = (start + (int(offs[r.first_frame + n]) if r.walk_frames > n
                                else int(r.walk_end)), rem)
        starts = np.concatenate([[0], np.cumsum(lens, dtype=np.int64)]) if lens \
            else np.zeros(1, dtype=np.int64)
        pcm_seg = pcm_i32[r.pcm_offset * ch:(r.pcm_offset + int(starts[-1])) * ch]
        self._seg = (pcm_seg, starts, [start + int(o) for o in
                                       offs[r.first_frame:r.first_frame + n]])
        self._seg_n = n
        self._next = 0
        if r.status == _atgpu.FD_OK:
            self._stop = _atgpu.FD_OK          # remaining_samples reached 0
        elif final or n == 0 or r.status == _atgpu.FD_FRAME_CRC:
            self._stop = r.status              # a real error at frame n
        else:                                  # the window's cut: resume there
            self._stop = None
            self._seg_byte = start + int(r.walk_end)
            self._seg_remaining = rem

    def read(self, pcm_frames):
        """one FLAC frame per call (flac.c:174-285)"""
        if self._closed:
            raise ValueError("cannot read closed stream")
        if self._finalized:
            return pcm.empty_framelist(self.channels, self.bits_per_sample)
        while self._seg is None or self._next >= self._seg_n:
            if self._seg is not None and self._stop is not None:
                # every good frame handed out: the stream either reached
                # remaining_samples == 0 (MD5 verdict) or stops on an error
                if self._stop == _atgpu.FD_OK:
                    self._finalized = True
                    if self._md5 is not None and self._md5.digest() != bytes(self._si.md5):
                        raise ValueError(_atgpu.FD_MESSAGES[_atgpu.FD_MD5])
                    return pcm.empty_framelist(self.channels, self.bits_per_sample)
                raise _status_error(self._stop)
            self._decode_segment()
        pcm_seg, starts, _ = self._seg
        k = self._next
        self._next += 1
        a = int(starts[k]) * self.channels
        b = int(starts[k + 1]) * self.channels
        frame = pcm_seg[a:b].copy()
        if self._md5 is not None:
            self._md5.update(_frame_bytes(frame, self.bits_per_sample))
        return pcm.FrameList._wrap(frame, self.channels, self.bits_per_sample)

    def seek(self, pcm_frame_offset):
        """position at the last SEEKTABLE point at or before
        pcm_frame_offset (sample 0 without one) and return its sample
        number (FlacDecoder_seek, flac.c:287-356); reads then continue from
        that frame, with MD5 validation only when it is sample 0"""
        if self._closed:
            raise ValueError("cannot seek closed stream")
        if not self._seekable:
            raise TypeError("can only seek streams from file objects")
        pcm_frame_offset = int(pcm_frame_offset)
        if pcm_frame_offset < 0:
            raise ValueError("cannot seek to negative value")
        sample, byte = 0, 0
        for (sample_number, byte_offset, _samples) in self._seekpoints:
            if sample_number <= pcm_frame_offset:
                sample, byte = sample_number, byte_offset
            else:
                break
        self._start_byte = int(byte)
        self._remaining = (self._si.total_samples - sample) % (1 << 64)
        self._validate = sample == 0
        self._reset()
        return sample

    def offsets(self):
        """[(byte offset from the current position, block size)] of every
        frame from the current position to the end, CRC-16 unchecked; the
        stream is then finished (flac.c:365-443)"""
        # the current position: the next frame read() would hand out
        if self._seg is not None and self._next < self._seg_n:
            pos, rem = self._seg[2][self._next], self._seg_rems[self._next]
        elif self._seg is not None and self._stop == _atgpu.FD_OK:
            self._finalized = True
            return []  # remaining_samples already 0
        elif self._seg is not None:
            pos, rem = self._after  # the next window, or the frame that failed
        else:
            pos, rem = self._seg_byte, self._seg_remaining
        body = self._body()
        chunk = bytes(body[pos:])
        track = _atgpu.dec_track(0, len(chunk), self._si)
        track.total_samples = rem
        track.md5[:] = bytes(16)
        _, res, offs, bss = _atgpu.decoder().decode(chunk + b"\0" * ((-len(chunk)) % 4),
                                                    [track], fetch_pcm=False)
        r = res[0]
        if r.walk_status != _atgpu.FD_OK:
            raise _status_error(r.walk_status)
        self._finalized = True
        return [(int(o), int(b)) for o, b in
                zip(offs[r.first_frame:r.first_frame + r.walk_frames],
                    bss[r.first_frame:r.first_frame + r.walk_frames])]

    def close(self):
        self._closed = True


def decode_flac_batch(images):
    """decode a list of .flac images (bytes) in one GPU batch.
    -> list of (status, streaminfo, int32 interleaved PCM); status is an
    ATG_FD_* code (0 = decoded and MD5-verified)."""
    parts, tracks, infos, pos = [], [], [], 0
    for img in images:
        rc, si, _ = _atgpu.read_metadata(img)
        if rc:
            raise _metadata_error(rc)
        body = bytes(img[si.frames_offset:])
        pad = (-len(body)) % 4
        tracks.append(_atgpu.dec_track(pos, len(body), si))
        parts.append(body + b"\0" * pad)
        infos.append(si)
        pos += len(body) + pad
    pcm_i32, res, _, _ = _atgpu.decoder().decode(b"".join(parts), tracks)
    out = []
    for si, r in zip(infos, res):
        a = r.pcm_offset * si.channels
        out.append((r.status, si, pcm_i32[a:a + r.pcm_frames * si.channels]))
    return out


def pcm_md5(samples, bits_per_sample):
    """MD5 of FrameList.to_bytes(False, True) for int32 samples (test aid)"""
    a = np.asarray(samples, dtype=np.int32)
    bb = (bits_per_sample + 7) // 8
    b = a.astype("<i4").view(np.uint8).reshape(-1, 4)[:, :bb]
    return hashlib.md5(b.tobytes()).digest()


# ------------------------------------------------------------------ ALAC
ALAC_CHANNEL_MASKS = {1: 0x0004, 2: 0x0003, 3: 0x0007, 4: 0x0107, 5: 0x0037, 6: 0x003F,
                      7: 0x013F, 8: 0x00FF}  # ALACDecoder_channel_mask (alac.c:157-180)


def _alac_init_error(status):
    msg = _atgpu.AD_INIT_MESSAGES.get(status, "no error")
    if status in (_atgpu.AD_IO_ERROR, _atgpu.AD_NO_MDAT):
        return IOError(msg)
    return ValueError(msg)


def _alac_read_error(status):
    msg = _atgpu.AD_READ_MESSAGES.get(status, "no error")
    return IOError(msg) if status == _atgpu.AD_IO_ERROR else ValueError(msg)


class ALACDecoder(object):
    """reference src/decoders/alac.c ALACDecoder(filename), decoded on the
    GPU (alac_decode.hip):

      .sample_rate .bits_per_sample .channels .channel_mask
      .read(n)       one ALAC frameset per call (wave channel order); an
                     empty FrameList once remaining_frames is 0 (:183-254)
      .seek(offset)  last seektable entry at or before offset (:256-301)
      .close()
    """

    def __init__(self, filename):
        with open(filename, "rb") as f:  # IOError with errno + filename
            data = f.read()
        self.filename = filename
        st, info, points, sizes = _atgpu.alac_read_info(data)
        if st:
            raise _alac_init_error(st)
        self._data = data
        self._info = info
        self._sizes = sizes
        # an empty seektable rewinds to the mdat start (alac.c:82-87)
        self._seektable = points if points else [(0, info.mdat_offset)]
        self.sample_rate = info.sample_rate
        self.bits_per_sample = info.bits_per_sample
        self.channels = info.channels
        self.channel_mask = ALAC_CHANNEL_MASKS.get(info.channels, 0)
        self.total_frames = info.total_frames
        self._pos = info.mdat_offset
        self._remaining = info.total_frames
        self._closed = False
        self._decoded = False

    def _hint(self):
        """the stsz sizes from the current position on (a decoding hint)"""
        if not len(self._sizes):
            return None
        starts = self._info.mdat_offset + np.concatenate(
            [[0], np.cumsum(self._sizes.astype(np.int64))])
        k = int(np.searchsorted(starts, self._pos))
        if k < len(self._sizes) and starts[k] == self._pos:
            return self._sizes[k:]
        return None

    def _decode(self):
        if self._decoded:
            return
        pad = (-len(self._data)) % 4
        track = _atgpu.alac_dec_track(0, len(self._data), self._info, start=self._pos,
                                      remaining=self._remaining, frameset_bytes=self._hint())
        pcm_i32, res, ff, _ = _atgpu.alac_decoder().decode(self._data + b"\0" * pad, [track])
        r = res[0]
        self._pcm = pcm_i32[r.sample_offset:r.sample_offset + r.pcm_frames * self.channels]
        self._fs = [int(x) for x in ff[r.first_frameset:r.first_frameset + r.n_framesets]]
        self._starts = np.concatenate([[0], np.cumsum(self._fs, dtype=np.int64)])
        self._status = r.status
        self._next = 0
        self._decoded = True

    def read(self, pcm_frames):
        if self._closed:
            raise ValueError("cannot read closed stream")
        if self._remaining == 0:
            return pcm.empty_framelist(self.channels, self.bits_per_sample)
        self._decode()
        if self._next < len(self._fs):
            k = self._next
            self._next += 1
            n = self._fs[k]
            self._remaining -= min(self._remaining, n)
            a, b = int(self._starts[k]) * self.channels, int(self._starts[k + 1]) * self.channels
            return pcm.FrameList._wrap(self._pcm[a:b].copy(), self.channels,
                                       self.bits_per_sample)
        if self._status == _atgpu.AD_OK:  # remaining reached 0 with this walk
            return pcm.empty_framelist(self.channels, self.bits_per_sample)
        raise _alac_read_error(self._status)

    def seek(self, pcm_frame_offset):
        if self._closed:
            raise ValueError("cannot seek closed stream")
        pcm_frame_offset = int(pcm_frame_offset)
        if pcm_frame_offset < 0:
            raise ValueError("cannot seek to negative value")
        best = None
        for entry in self._seektable:
            if entry[0] <= pcm_frame_offset:
                best = entry
            else:
                break
        if best is None:
            raise ValueError("no offset found in seektable")
        self._remaining = (self.total_frames - best[0]) % (1 << 32)
        self._pos = best[1]
        self._decoded = False
        return best[0]

    def close(self):
        self._closed = True


def decode_alac_batch(images):
    """decode a list of M4A/ALAC images (bytes) in one GPU batch
    -> list of (status, AlacInfo, int32 interleaved PCM); status is an
    ATG_AD_* code (0 = every frame up to total_frames decoded)"""
    parts, tracks, infos, pos = [], [], [], 0
    for img in images:
        st, info, _, sizes = _atgpu.alac_read_info(img)
        if st:
            raise _alac_init_error(st)
        img = bytes(img)
        pad = (-len(img)) % 4
        tracks.append(_atgpu.alac_dec_track(pos, len(img), info, frameset_bytes=sizes))
        parts.append(img + b"\0" * pad)
        infos.append(info)
        pos += len(img) + pad
    pcm_i32, res, _, _ = _atgpu.alac_decoder().decode(b"".join(parts), tracks)
    out = []
    for info, r in zip(infos, res):
        out.append((r.status, info,
                    pcm_i32[r.sample_offset:r.sample_offset + r.pcm_frames * info.channels]))
    return out
