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
  .offsets()               [(byte offset from the first frame, block size)]
                           (flac.c:365-443)
  .close()                 further reads raise ValueError

The whole stream is decoded by libatgpu (HIP kernels, flac_decode.hip) the
first time it is needed; read() then hands out the decoded frames in order
and raises the decode status at the frame where the reference would.
`decode_flac_batch` is the batch entry trackverify-style callers use.
There is no CPU decoding path.
"""

import hashlib

import numpy as np

from . import _atgpu
from . import pcm


def _read_all(file):
    if isinstance(file, (str, bytes)) and not isinstance(file, bytes):
        with open(file, "rb") as f:
            return f.read()
    if isinstance(file, (bytes, bytearray, memoryview)):
        return bytes(file)
    return file.read()


def _metadata_error(rc):
    if rc == 1:
        return ValueError("not a FLAC file")
    return IOError("EOF while reading metadata")


class FlacDecoder(object):
    """reference src/decoders/flac.c FlacDecoder, decoded on the GPU"""

    def __init__(self, file):
        data = _read_all(file)
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
        self._decoded = False
        self._closed = False
        self._finalized = False
        self._next = 0

    def _decode(self):
        if self._decoded:
            return
        start = self._si.frames_offset
        track = _atgpu.dec_track(0, len(self._data) - start, self._si)
        pcm_i32, res, offs, bss = _atgpu.decoder().decode(self._data[start:], [track])
        r = res[0]
        n = r.pcm_frames * self.channels
        self._pcm = pcm_i32[r.pcm_offset * self.channels:r.pcm_offset * self.channels + n]
        self._offsets = offs[r.first_frame:r.first_frame + r.n_frames]
        self._block_sizes = bss[r.first_frame:r.first_frame + r.n_frames]
        # PCM frames of each decoded frame: MIN(block size, remaining)
        lens, remaining = [], self._si.total_samples
        for bs in self._block_sizes:
            lens.append(min(int(bs), remaining))
            remaining = (remaining - int(bs)) % (1 << 64)
        self._lens = lens
        self._starts = np.concatenate([[0], np.cumsum(lens, dtype=np.int64)]) \
            if lens else np.zeros(1, dtype=np.int64)
        self._status = r.status
        self._decoded = True

    def read(self, pcm_frames):
        if self._closed:
            raise ValueError("cannot read closed stream")
        if self._finalized:
            return pcm.empty_framelist(self.channels, self.bits_per_sample)
        self._decode()
        if self._next < len(self._lens):
            k = self._next
            self._next += 1
            a = int(self._starts[k]) * self.channels
            b = int(self._starts[k + 1]) * self.channels
            return pcm.FrameList._wrap(self._pcm[a:b].copy(), self.channels,
                                       self.bits_per_sample)
        # every decoded frame handed out: the stream either reached
        # remaining_samples == 0 (MD5 verdict) or stopped on an error
        if self._status in (_atgpu.FD_OK, _atgpu.FD_MD5):
            self._finalized = True
            if self._status == _atgpu.FD_MD5:
                raise ValueError(_atgpu.FD_MESSAGES[_atgpu.FD_MD5])
            return pcm.empty_framelist(self.channels, self.bits_per_sample)
        if self._status == _atgpu.FD_EOF:
            raise IOError(_atgpu.FD_MESSAGES[_atgpu.FD_EOF])
        raise ValueError(_atgpu.FD_MESSAGES.get(self._status, "Error"))

    def offsets(self):
        self._decode()
        if self._status not in (_atgpu.FD_OK, _atgpu.FD_MD5):
            if self._status == _atgpu.FD_EOF:
                raise IOError(_atgpu.FD_MESSAGES[_atgpu.FD_EOF])
            raise ValueError(_atgpu.FD_MESSAGES.get(self._status, "Error"))
        self._finalized = True
        return [(int(o), int(b)) for o, b in zip(self._offsets, self._block_sizes)]

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
