"""audiotools.encoders — FLAC / ALAC encoding on the MI355X engine.

`encode_flac` IS the compiled C-API entry point `audiotools._encoders_c.
encode_flac` (csrc/ext/encoders_c.c over libatgpu's C ABI), as the
reference's module function is its C extension (src/encoders/flac.c:44-121,
registered src/encoders.h:65-67):

    encode_flac(filename, pcmreader, block_size, max_lpc_order,
                min_residual_partition_order, max_residual_partition_order,
                mid_side=0, adaptive_mid_side=0, exhaustive_model_search=0,
                disable_verbatim_subframes=0, disable_constant_subframes=0,
                disable_fixed_subframes=0, disable_lpc_subframes=0,
                padding_size=4096) -> [(byte_offset, pcm_frames), ...]

* the output file is opened first; failure raises OSError/IOError carrying
  errno and filename (flac.c:114-116);
* PCM is pulled with pcmreader.read(block_size) until an empty FrameList,
  and every read becomes one FLAC frame, exactly as the reference frame loop
  does (flac.c:244-274) — with a BufferedPCMReader that is block_size
  frames plus a shorter final frame;
* read() must return pcm.FrameList objects (TypeError otherwise,
  pcmconv.c:244-248); exceptions raised by read() propagate;
* on success the reader is closed (flac.c:282) and the list of
  (offset of the frame from the first frame, pcm frames) is returned.

It streams: up to 256 FLAC frames per GPU call (atg_flac_encode_frames) with
the GIL released, the MD5 of each segment's PCM bytes on a host thread
beside the GPU call, STREAMINFO rewritten at the end (flac.c:276-279), on a
streaming engine (two HIP streams per process, for one process per track
under track2track).

`encode_flac_batch` is the batch form the engine is built for: many tracks
in one GPU pass (what track2track -j N achieves with N processes), MD5
chains on the GPU, the tracks sharded over the node's GPUs.

`encode_alac` / `encode_alac_batch` do the same for ALAC (reference
src/encoders/alac.c:30-189; GPU kernels alac_encode.hip).
"""

import numpy as np

from . import pcm as _pcm
from . import _atgpu
from ._encoders_c import encode_flac  # noqa: F401  (the drop-in entry point)


def pcm_le_bytes(samples, bits_per_sample):
    """little-endian signed PCM bytes of interleaved samples: what the
    reference's MD5 callback hashes (FrameList.to_bytes(False, True),
    flac.c:187-188 -> pcmconv.c:266-291)"""
    a = np.asarray(samples)
    if bits_per_sample <= 8:
        return a.astype(np.int8).tobytes()
    if bits_per_sample <= 16:
        return a.astype("<i2").tobytes()
    w = (bits_per_sample + 7) // 8
    return np.ascontiguousarray(a.astype("<i4").view(np.uint8).reshape(-1, 4)[:, :w]).tobytes()


def _collect(pcmreader, block_size):
    """drain a PCMReader the way the reference frame loop does"""
    chunks, sizes = [], []
    while True:
        fl = pcmreader.read(block_size)
        if not isinstance(fl, _pcm.FrameList):
            raise TypeError("results from pcmreader.read() must be FrameLists")
        if fl.frames == 0:
            break
        if fl.channels != pcmreader.channels:
            raise ValueError("FrameList channel count does not match pcmreader")
        chunks.append(fl.samples)
        sizes.append(fl.frames)
    samples = (np.concatenate(chunks) if chunks else np.zeros(0, dtype=np.int32))
    return samples, sizes


def _frame_sizes_or_none(sizes, block_size):
    """None when the chunks are plain block_size blocking (+ short tail)"""
    if all(s == block_size for s in sizes[:-1]) and (not sizes or sizes[-1] <= block_size):
        return None
    return np.asarray(sizes, dtype=np.uint32)


def encode_flac_batch(filenames, pcmreaders, block_size, max_lpc_order,
                      min_residual_partition_order, max_residual_partition_order,
                      mid_side=0, adaptive_mid_side=0, exhaustive_model_search=0,
                      disable_verbatim_subframes=0, disable_constant_subframes=0,
                      disable_fixed_subframes=0, disable_lpc_subframes=0,
                      padding_size=4096):
    """encode several PCMReaders (same channels / bits / rate) to several
    .flac files in one GPU batch; returns one offsets list per file"""
    filenames = list(filenames)
    pcmreaders = list(pcmreaders)
    if len(filenames) != len(pcmreaders):
        raise ValueError("filenames and pcmreaders differ in length")
    if not pcmreaders:
        return []
    r0 = pcmreaders[0]
    channels, bps, rate = r0.channels, r0.bits_per_sample, r0.sample_rate
    for r in pcmreaders:
        if (r.channels, r.bits_per_sample, r.sample_rate) != (channels, bps, rate):
            raise ValueError("all pcmreaders of a batch must share channels, "
                             "bits-per-sample and sample rate")
    files = [open(fn, "wb") for fn in filenames]
    try:
        opts = _atgpu.make_options(
            block_size, max_lpc_order, min_residual_partition_order,
            max_residual_partition_order, mid_side, adaptive_mid_side,
            exhaustive_model_search, disable_verbatim_subframes,
            disable_constant_subframes, disable_fixed_subframes,
            disable_lpc_subframes, padding_size)
        parts, tracks, start = [], [], 0
        for r in pcmreaders:
            samples, sizes = _collect(r, block_size)
            frames = len(samples) // channels
            tracks.append((start, frames, _frame_sizes_or_none(sizes, block_size)))
            parts.append(samples)
            start += frames
        pcm = np.concatenate(parts) if parts else np.zeros(0, dtype=np.int32)
        if bps <= 16:
            pcm = pcm.astype(np.int16)
        # the tracks sharded over the node's GPUs (contiguous groups balanced
        # by frames, one engine per device, _atgpu.batch_devices)
        devs = _atgpu.batch_devices()
        ranges = (_atgpu.shard_ranges([t[1] for t in tracks], len(devs))
                  if len(devs) > 1 else [(0, len(tracks))])

        def shard(i):
            t0, t1 = ranges[i]
            s0 = tracks[t0][0]
            s1 = tracks[t1 - 1][0] + tracks[t1 - 1][1]
            eng = (_atgpu.engine() if len(ranges) == 1
                   else _atgpu.shard_object("engine", i, devs[i]))
            return eng.encode(opts, pcm[s0 * channels:s1 * channels],
                              [(a - s0, n, fs) for a, n, fs in tracks[t0:t1]],
                              channels, bps, rate)

        lists = []
        for (t0, t1), (out, results, offsets, pcm_frames) in zip(
                ranges, _atgpu.run_shards(shard, len(ranges))):
            for f, res in zip(files[t0:t1], results):
                f.write(memoryview(out[res.out_offset:res.out_offset + res.bytes]))
                lo, n = res.first_frame, res.n_frames
                lists.append([(int(offsets[lo + i]), int(pcm_frames[lo + i]))
                              for i in range(n)])
        for r in pcmreaders:
            r.close()
        return lists
    finally:
        for f in files:
            f.close()


def encode_alac_batch(files, pcmreaders, block_size, initial_history, history_multiplier,
                      maximum_k, minimum_interlacing_leftweight=0,
                      maximum_interlacing_leftweight=4):
    """several PCMReaders (same channels / bits) -> one mdat atom written to
    each file object in one GPU batch; one (frame_byte_sizes,
    total_pcm_frames) tuple per file"""
    files = list(files)
    pcmreaders = list(pcmreaders)
    if len(files) != len(pcmreaders):
        raise ValueError("files and pcmreaders differ in length")
    if not pcmreaders:
        return []
    # the leftweights tried per stereo frame (alac.c:57-72, 459-481); the
    # reference writes them in 8 bits and, with min > max, emits a stale
    # frame: both refused here
    if not (0 <= minimum_interlacing_leftweight <= maximum_interlacing_leftweight <= 255):
        raise ValueError("interlacing leftweights must satisfy 0 <= minimum <= maximum <= 255")
    r0 = pcmreaders[0]
    channels, bps = r0.channels, r0.bits_per_sample
    if bps not in (16, 24):
        raise ValueError("bits per sample must be 16 or 24")
    for r in pcmreaders:
        if (r.channels, r.bits_per_sample) != (channels, bps):
            raise ValueError("all pcmreaders of a batch must share channels and "
                             "bits-per-sample")
    parts, tracks, start = [], [], 0
    for r in pcmreaders:
        samples, sizes = _collect(r, block_size)
        frames = len(samples) // channels
        tracks.append((start, frames, _frame_sizes_or_none(sizes, block_size)))
        parts.append(samples)
        start += frames
    pcm = np.concatenate(parts) if parts else np.zeros(0, dtype=np.int32)
    if bps <= 16:
        pcm = pcm.astype(np.int16)
    enc = _atgpu.alac_encoder()
    opts = enc.options(block_size, initial_history, history_multiplier, maximum_k,
                       minimum_interlacing_leftweight, maximum_interlacing_leftweight)
    out, results, fsb = enc.encode(opts, pcm, tracks, channels, bps)
    logs = []
    for f, res in zip(files, results):
        f.write(memoryview(out[res.out_offset:res.out_offset + res.bytes]))
        lo = res.first_frameset
        logs.append(([int(x) for x in fsb[lo:lo + res.n_framesets]], int(res.pcm_frames)))
    for r in pcmreaders:
        r.close()
    return logs


def encode_alac(file, pcmreader, block_size, initial_history, history_multiplier, maximum_k,
                minimum_interlacing_leftweight=0, maximum_interlacing_leftweight=4):
    """encode_alac(file, pcmreader, block_size, initial_history,
    history_multiplier, maximum_k) -> ([frameset byte sizes], total PCM frames)

    writes the mdat atom (size, "mdat", framesets) to the file object at
    its position, as the reference does (src/encoders/alac.c:30-189)"""
    if not hasattr(file, "write"):
        raise TypeError("file must by a concrete file object")
    return encode_alac_batch([file], [pcmreader], block_size, initial_history,
                             history_multiplier, maximum_k, minimum_interlacing_leftweight,
                             maximum_interlacing_leftweight)[0]
