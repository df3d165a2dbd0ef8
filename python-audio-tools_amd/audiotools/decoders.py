"""audiotools.decoders — FLAC decoding on the MI355X.

`FlacDecoder` IS the compiled C-API type `audiotools._decoders_c.FlacDecoder`
(csrc/ext/decoders_c.c over libatgpu's C ABI), with the Python-visible
contract of the reference's C type audiotools.decoders.FlacDecoder
(src/decoders/flac.c, methods :145-166):

  FlacDecoder(file)        file object, filename or bytes positioned at
                           "fLaC"; ValueError / IOError from the metadata
                           reader (flacdec_read_metadata, flac.c:568-707)
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
segments as read() needs them (8 MiB of compressed data per GPU call, the
MD5 chained on the host); read() hands out the decoded frames in order and
raises the decode status at the frame where the reference would.
`decode_flac_batch` is the batch entry trackverify-style callers use.
`ALACDecoder` / `decode_alac_batch` do the same for ALAC in M4A
(reference src/decoders/alac.c; GPU kernels alac_decode.hip).
There is no CPU decoding path.
"""

import hashlib

import numpy as np

from . import _atgpu
from . import pcm
# the drop-in decoder type: the compiled C-API FlacDecoder
# (csrc/ext/decoders_c.c over libatgpu), as the reference's is its C type
from ._decoders_c import FlacDecoder  # noqa: F401


def _metadata_error(rc):
    if rc == 1:
        return ValueError("not a FLAC file")
    return IOError("EOF while reading metadata")




def decode_flac_batch(images):
    """decode a list of .flac images (bytes) in one GPU batch.
    -> list of (status, streaminfo, int32 interleaved PCM); status is an
    ATG_FD_* code (0 = decoded and MD5-verified)."""
    infos, bodies = [], []
    for img in images:
        rc, si, _ = _atgpu.read_metadata(img)
        if rc:
            raise _metadata_error(rc)
        infos.append(si)
        bodies.append(bytes(img[si.frames_offset:]))
    # the streams sharded over the node's GPUs (_atgpu.batch_devices),
    # balanced by PCM frames
    devs = _atgpu.batch_devices()
    ranges = (_atgpu.shard_ranges([si.total_samples for si in infos], len(devs))
              if len(devs) > 1 else [(0, len(infos))])

    def shard(i):
        t0, t1 = ranges[i]
        parts, tracks, pos = [], [], 0
        for si, body in zip(infos[t0:t1], bodies[t0:t1]):
            pad = (-len(body)) % 4
            tracks.append(_atgpu.dec_track(pos, len(body), si))
            parts.append(body + b"\0" * pad)
            pos += len(body) + pad
        dec = (_atgpu.decoder() if len(ranges) == 1
               else _atgpu.shard_object("decoder", i, devs[i]))
        return dec.decode(b"".join(parts), tracks)

    out = []
    for (t0, t1), (pcm_i32, res, _, _) in zip(ranges, _atgpu.run_shards(shard, len(ranges))):
        for si, r in zip(infos[t0:t1], res):
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
