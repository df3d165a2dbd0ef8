"""audiotools.replaygain — ReplayGain analysis on the MI355X.

`ReplayGain` keeps the Python contract of the reference's C type
(src/replaygain.c, replaygain.h): ReplayGain(sample_rate) raises ValueError
for an unsupported rate; title_gain(pcmreader) -> (gain, peak) for one
track (0.0 gain when no 50 ms window completed); album_gain() -> (gain,
peak) over every title analysed so far, ValueError "Not enough samples to
perform calculation" when none.  Each title is analysed by replaygain.hip
(lane per track); `batch_gains` analyses many tracks/albums in one launch.
No CPU path.
"""

import math
import os
import time

import numpy as np

from . import _atgpu
from . import _encoders_c
from . import pcm

# album_scan's last call: host seconds per phase (summed over shards)
_last_phases = {}
# bytes per upload chunk of album_scan (pinned staging, per shard)
STAGE_BYTES = 256 << 20

RATES = (48000, 44100, 32000, 24000, 22050, 16000, 12000, 11025, 8000, 18900,
         37800, 56000, 64000, 88200, 96000, 112000, 128000, 144000, 176400, 192000)


def _read_title(pcmreader, sample_rate):
    """drain one title the way ReplayGain.title_gain reads it (read(4096)
    until an empty FrameList, replaygain.c:210-305) -> (int32 samples, read
    sizes, channels, bits) or None when nothing was read; the samples are
    the reads' arrays, not concatenated (album_scan copies them once, into
    the upload staging)"""
    if pcmreader.sample_rate != sample_rate:
        raise ValueError("pcmreader's sample rate doesn't match")
    parts, sizes = [], []
    while True:
        fl = pcmreader.read(4096)
        if not isinstance(fl, pcm.FrameList):
            raise TypeError("pcmreader.read() must return a FrameList")
        if not fl.frames:
            break
        if fl.channels not in (1, 2):
            raise ValueError("FrameList must contain only 1 or 2 channels")
        parts.append(np.ascontiguousarray(fl.samples, dtype=np.int32))
        sizes.append(fl.frames)
    bps, ch = pcmreader.bits_per_sample, pcmreader.channels
    if parts and bps not in (8, 16, 24):
        raise ValueError("unsupported bits per sample")
    if not parts:
        return None
    return parts, sizes, ch, bps


def _rg_track(offset, frames, sizes, ch, bps, rate):
    t = _atgpu.RgTrack(offset, frames, ch, bps, rate, 0)
    # each read() result is one analyze_samples call: its size decides the
    # fp64 summation grouping (replaygain.c:210-305)
    if any(n != 4096 for n in sizes[:-1]) or sizes[-1] > 4096:
        t.set_chunks(sizes)
    return t


class ReplayGain(object):
    """ReplayGain(sample_rate) (replaygain.c:115-182).  Like the reference,
    the object keeps only the album state between titles -- the summed
    12000-bin window histogram B and the album peak -- never the samples."""

    def __init__(self, sample_rate):
        if sample_rate not in RATES:
            raise ValueError("unsupported sample rate")
        self.sample_rate = sample_rate
        self._album_hist = np.zeros(12000, dtype=np.uint64)
        self._album_peak = 0.0

    def title_gain(self, pcmreader):
        """(title gain, title peak) of one reader; its histogram is added
        to the album's (get_title_gain, replaygain.c:776-800)"""
        title = _read_title(pcmreader, self.sample_rate)
        if title is None:
            return (0.0, 0.0)  # nothing read: no window, peak 0.0
        parts, sizes, ch, bps = title
        samples = np.concatenate(parts)
        track = _rg_track(0, len(samples) // ch, sizes, ch, bps, self.sample_rate)
        (res,), peaks, _, hist = _atgpu.replaygain_host(samples, [track], 1,
                                                        return_hist=True)
        self._album_hist += hist[0]
        self._album_peak = max(self._album_peak, peaks[0])
        return (res.title_gain, res.title_peak)

    def add_album_state(self, hist, peak):
        """fold another analysis' album histogram and peak into this one
        (an album scanned in shards, album_scan)"""
        self._album_hist += np.asarray(hist, dtype=np.uint64)
        self._album_peak = max(self._album_peak, float(peak))

    def album_gain(self):
        """(album gain, album peak) over every title so far
        (get_album_gain, replaygain.c:803-807; ValueError when empty)"""
        return album_gain_of(self._album_hist, self._album_peak)


def album_gain_of(hist, peak):
    """(album gain, album peak) of a summed 12000-bin histogram
    (analyzeResult, replaygain.c:754-776; ValueError when empty)"""
    hist = np.asarray(hist, dtype=np.uint64)
    if not hist.any():
        raise ValueError("Not enough samples to perform calculation")
    (gain,) = _atgpu.replaygain_hist_gain_host((hist & 0xFFFFFFFF).astype(np.uint32))
    if math.isnan(gain):
        raise ValueError("Not enough samples to perform calculation")
    return (gain, float(peak))


def album_scan(titles, sample_rate):
    """ReplayGain of a whole album in one GPU call per device.

    titles: one entry per track, in album order: None (nothing read) or
    (int32 samples -- one array or the list of the reads' arrays --, read
    sizes, channels, bits_per_sample) as _read_title gives.  The non-empty titles are sharded over the node's GPUs
    (_atgpu.batch_devices, contiguous groups balanced by frames); each
    shard is one atg_replaygain_device batch whose album histogram and peak
    come back with the titles' gains; the shards' histograms are summed and
    their peaks max'd -- the album state the reference accumulates title by
    title (replaygain.c:776-807).
    -> ([(title_gain, title_peak)], album histogram uint64[12000], album peak)"""
    if sample_rate not in RATES:
        raise ValueError("unsupported sample rate")
    idx = [i for i, t in enumerate(titles) if t is not None]
    out = [(0.0, 0.0)] * len(titles)
    hist = np.zeros(12000, dtype=np.uint64)
    peak = 0.0
    if not idx:
        return out, hist, peak
    nsamp = {i: sum(len(p) for p in _parts(titles[i][0])) for i in idx}
    devs = _atgpu.batch_devices()
    frames = [nsamp[i] // titles[i][2] for i in idx]
    ranges = _atgpu.shard_ranges(frames, len(devs)) if len(devs) > 1 else [(0, len(idx))]
    _last_phases.update(fill_s=0.0, upload_wait_s=0.0, gpu_s=0.0)

    def shard(k):
        t0, t1 = ranges[k]
        eng = (_atgpu.engine() if len(ranges) == 1
               else _atgpu.shard_object("engine", k, devs[k]))
        # one device buffer; a title's pcm_offset counts frames of its own
        # channel count (sample pcm_offset * channels), so mono and stereo
        # titles sit at disjoint sample ranges
        tracks, starts, spos = [], [], 0
        for i in idx[t0:t1]:
            parts, sizes, ch, bps = titles[i]
            off = -(-spos // ch)
            tracks.append(_rg_track(off, nsamp[i] // ch, sizes, ch, bps, sample_rate))
            starts.append(off * ch)
            spos = off * ch + nsamp[i]
        d_pcm = eng.device_alloc(4 * spos)
        d_hist = eng.device_alloc(4 * 12000)
        try:
            # the titles' reads copied once, by host threads, into pinned
            # staging (two buffers), each chunk uploaded by a thread of its
            # own while the next chunk is filled
            cap = max(STAGE_BYTES, 4 * max(nsamp[i] for i in idx[t0:t1]))
            stages = [_atgpu.staging(("rg", k, b), cap).view(np.int32) for b in (0, 1)]
            titles_k = idx[t0:t1]
            chunks, j = [], 0
            while j < len(titles_k):
                m = j
                while m < len(titles_k) and starts[m] + nsamp[titles_k[m]] - starts[j] <= \
                        len(stages[0]):
                    m += 1
                chunks.append((j, m))
                j = m
            pending = [None, None]
            for c, (j, m) in enumerate(chunks):
                a = starts[j]
                b = starts[m - 1] + nsamp[titles_k[m - 1]]
                if pending[c % 2] is not None:
                    pending[c % 2].result()  # that buffer's upload is done
                view = stages[c % 2][:b - a]

                # the chunk's reads in one threaded host gather (GIL
                # released); a mono/stereo alignment gap is zeroed
                segs = []
                for q in range(j, m):
                    i = titles_k[q]
                    end = starts[q + 1] if q + 1 < m else b
                    segs.extend(_parts(titles[i][0]))
                    if end > starts[q] + nsamp[i]:
                        segs.append(np.zeros(end - starts[q] - nsamp[i], dtype=np.int32))
                tf = time.perf_counter()
                _encoders_c.gather_into(view, segs)
                _last_phases["fill_s"] += time.perf_counter() - tf
                pending[c % 2] = _atgpu.upload_pool().submit(
                    eng.copy_to_device, d_pcm + 4 * a, view)
            tw = time.perf_counter()
            for f in pending:
                if f is not None:
                    f.result()
            _last_phases["upload_wait_s"] += time.perf_counter() - tw
            tg = time.perf_counter()
            res, peaks = _atgpu.replaygain_device(d_pcm, tracks, 1, d_hist)
            h = np.empty(12000, dtype=np.uint32)
            eng.copy_to_host(h, d_hist)
            _last_phases["gpu_s"] += time.perf_counter() - tg
        finally:
            eng.device_free(d_pcm)
            eng.device_free(d_hist)
        return res, peaks[0], h

    for (t0, t1), (res, pk, h) in zip(ranges, _atgpu.run_shards(shard, len(ranges))):
        for i, r in zip(idx[t0:t1], res):
            out[i] = (r.title_gain, r.title_peak)
        hist += h.astype(np.uint64)
        peak = max(peak, pk)
    return out, hist, peak


def _parts(samples):
    """a title's samples: the list of its reads' arrays, or one array"""
    return samples if isinstance(samples, (list, tuple)) else [samples]


def album_allreduce(hist, peak, group=None):
    """an album scanned by several processes (one per GPU, torch.distributed
    initialised -- the config-4 layout): SUM of the 12000-bin
    window histograms and MAX of the peaks over the group -- exact and
    order-independent.  torch tensors on the device (the histogram as int32:
    two's-complement sums are the uint32 bits) are reduced in place over
    RCCL ("nccl" backend) and returned; numpy / float inputs go through a
    tensor on the process's device (gloo: on the host).
    -> (hist, peak)"""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return hist, peak
    if torch.is_tensor(hist):
        pk = peak if torch.is_tensor(peak) else torch.tensor(
            [float(peak)], dtype=torch.float64, device=hist.device)
        dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(pk, op=dist.ReduceOp.MAX, group=group)
        return hist, pk
    dev = (torch.device("cuda", torch.cuda.current_device())
           if dist.get_backend(group) == "nccl" else torch.device("cpu"))
    h = torch.as_tensor(np.asarray(hist, dtype=np.int64), device=dev)
    p = torch.tensor([float(peak)], dtype=torch.float64, device=dev)
    dist.all_reduce(h, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(p, op=dist.ReduceOp.MAX, group=group)
    return h.cpu().numpy().astype(np.uint64), float(p.item())


def batch_gains(pcm_i32, tracks, n_albums):
    """title gains/peaks of a batch (int32 PCM in host memory, list of
    RgTrack grouped by album) and album gains/peaks.
    -> ([(title_gain, title_peak)], [(album_gain, album_peak)])"""
    res, peaks, gains = _atgpu.replaygain_host(pcm_i32, tracks, n_albums)
    return ([(r.title_gain, r.title_peak) for r in res], list(zip(gains, peaks)))


class ReplayGainReader(object):
    """reference replaygain.ReplayGainReader(pcmreader, replaygain, peak)
    (src/replaygain.c:820-925): a PCMReader applying the gain with
    lround, clamping and one XOR dither bit per sample (os.urandom, or
    `dither=` callable n -> bytes for reproducible output)"""

    def __init__(self, pcmreader, replaygain, peak, dither=None):
        self.pcmreader = pcmreader
        self.sample_rate = pcmreader.sample_rate
        self.channels = pcmreader.channels
        self.channel_mask = pcmreader.channel_mask
        self.bits_per_sample = pcmreader.bits_per_sample
        self.multiplier = _atgpu.load_library().atg_replaygain_multiplier(
            float(replaygain), float(peak))
        self._rand = dither if dither is not None else os.urandom
        self._bits = b""
        self._bitpos = 0

    def read(self, pcm_frames):
        if pcm_frames <= 0:
            raise ValueError("pcm_frames must be positive")
        fl = self.pcmreader.read(pcm_frames)
        if not isinstance(fl, pcm.FrameList):
            raise TypeError("pcmreader.read() must return a FrameList")
        if not fl.frames:
            return fl
        n = len(fl)
        have = len(self._bits) * 8 - self._bitpos
        if have < n:
            self._bits = self._bits[self._bitpos // 8:] + self._rand(
                max((n - have + 7) // 8, 4096))
            self._bitpos %= 8
        out = _atgpu.apply_gain(fl.samples, self.channels, self.bits_per_sample,
                                self.multiplier, fl.frames, self._bits, self._bitpos)
        self._bitpos += n
        return pcm.FrameList._wrap(out, self.channels, self.bits_per_sample)

    def close(self):
        self.pcmreader.close()
