"""ctypes wrapper of oracle/libflacport.so — the CPU restatement of the
reference FLAC encoder/decoder.  TEST INFRASTRUCTURE ONLY: used by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, never by the
product path.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "libflacport.so")
REF_FLACENC = os.path.join(ORACLE_DIR, "_ref", "flacenc")

c_u32, c_i32, c_u64 = ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64


class PortOptions(ctypes.Structure):
    _fields_ = [("block_size", c_u32), ("max_lpc_order", c_u32),
                ("min_residual_partition_order", c_u32),
                ("max_residual_partition_order", c_u32),
                ("mid_side", c_i32), ("adaptive_mid_side", c_i32),
                ("exhaustive_model_search", c_i32),
                ("disable_verbatim_subframes", c_i32),
                ("disable_constant_subframes", c_i32),
                ("disable_fixed_subframes", c_i32),
                ("disable_lpc_subframes", c_i32), ("padding_size", c_u32)]


# reference FLAC presets (audiotools/flac.py:1719-1764)
PRESETS = {
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

_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-C", ORACLE_DIR, "port"],
                                  stdout=subprocess.DEVNULL)
        lib = ctypes.CDLL(LIB)
        lib.flacport_max_stream_bytes.restype = ctypes.c_size_t
        lib.flacport_max_stream_bytes.argtypes = [c_u64, c_u32, c_u32, c_u32, c_u32]
        lib.flacport_encode.restype = ctypes.c_int
        lib.flacport_encode.argtypes = [
            ctypes.c_void_p, c_u64, c_u32, c_u32, c_u32, ctypes.POINTER(PortOptions),
            ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
            ctypes.POINTER(ctypes.c_size_t)]
        lib.flacport_decode.restype = ctypes.c_int
        lib.flacport_decode.argtypes = [
            ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(c_u32),
            ctypes.POINTER(c_u32), ctypes.POINTER(c_u32), ctypes.POINTER(c_u64),
            ctypes.c_void_p, ctypes.c_size_t]
        lib.flacport_pcm_md5.restype = None
        lib.flacport_pcm_md5.argtypes = [ctypes.c_void_p, c_u64, c_u32, c_u32,
                                         ctypes.c_void_p]
        _lib = lib
    return _lib


def options(**kw):
    d = dict(mid_side=0, adaptive_mid_side=0, exhaustive_model_search=0,
             disable_verbatim_subframes=0, disable_constant_subframes=0,
             disable_fixed_subframes=0, disable_lpc_subframes=0,
             padding_size=4096)
    d.update(kw)
    return PortOptions(d["block_size"], d["max_lpc_order"],
                       d.get("min_residual_partition_order", 0),
                       d["max_residual_partition_order"], int(bool(d["mid_side"])),
                       int(bool(d["adaptive_mid_side"])),
                       int(bool(d["exhaustive_model_search"])),
                       int(bool(d["disable_verbatim_subframes"])),
                       int(bool(d["disable_constant_subframes"])),
                       int(bool(d["disable_fixed_subframes"])),
                       int(bool(d["disable_lpc_subframes"])), int(d["padding_size"]))


def encode(pcm, channels, bps, rate, frame_sizes=None, **opts):
    """-> (flac bytes, [(offset, pcm_frames), ...]).  frame_sizes = the frame
    counts a reader's successive read() calls returned (then block_size per
    read): one frame per read, as the reference (flac.c:244-274)."""
    lib = load()
    o = options(**opts)
    a = np.ascontiguousarray(pcm, dtype=np.int32)
    frames = len(a) // channels
    sizes = None if frame_sizes is None else np.ascontiguousarray(frame_sizes, dtype=np.uint32)
    cap = lib.flacport_max_stream_bytes(frames, channels, bps, o.block_size,
                                        o.padding_size)
    nfmax = frames // max(1, o.block_size) + 2
    if sizes is not None and len(sizes):
        # per listed read: a verbatim frame of its own size plus headers
        per = 32 + channels * (12 + (sizes.astype(np.int64) * (bps + 1) + 7) // 8)
        cap += int(per.sum()) + 64
        nfmax += len(sizes)
    if opts.get("disable_verbatim_subframes"):
        # without VERBATIM a predictor may exceed the verbatim bound (24-bit
        # noise): leave room for twice that
        cap = 2 * cap + (1 << 20)
    out = np.empty(cap, dtype=np.uint8)
    olen = ctypes.c_size_t()
    offs = np.zeros(nfmax, dtype=np.uint64)
    lens = np.zeros(nfmax, dtype=np.uint32)
    nf = ctypes.c_size_t()
    if not hasattr(lib, "_sizes_ready"):
        lib.flacport_encode_sizes.restype = ctypes.c_int
        lib.flacport_encode_sizes.argtypes = [
            ctypes.c_void_p, c_u64, c_u32, c_u32, c_u32, ctypes.POINTER(PortOptions),
            ctypes.c_void_p, ctypes.c_size_t,
            ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
            ctypes.POINTER(ctypes.c_size_t)]
        lib._sizes_ready = True
    rc = lib.flacport_encode_sizes(
        a.ctypes.data_as(ctypes.c_void_p), frames, channels, bps, rate, ctypes.byref(o),
        None if sizes is None else sizes.ctypes.data_as(ctypes.c_void_p),
        0 if sizes is None else len(sizes), out.ctypes.data_as(ctypes.c_void_p),
        cap, ctypes.byref(olen), offs.ctypes.data_as(ctypes.c_void_p),
        lens.ctypes.data_as(ctypes.c_void_p), nfmax, ctypes.byref(nf))
    if rc != 0:
        raise RuntimeError("flacport_encode failed: %d" % rc)
    n = nf.value
    return out[:olen.value].tobytes(), [(int(offs[i]), int(lens[i])) for i in range(n)]


def cut_frames(frames, block_size, frame_sizes):
    """the frame lengths a stream of `frames` PCM frames is cut into when the
    reader's reads return frame_sizes, then block_size per read"""
    cut, left = [], frames
    for n in frame_sizes:
        if left <= 0 or n == 0:
            return cut
        cut.append(min(n, left))
        left -= cut[-1]
    while left > 0:
        cut.append(min(block_size, left))
        left -= cut[-1]
    return cut


REF_FLACENC_SIZED = os.path.join(ORACLE_DIR, "_ref", "flacenc_sized")


def ref_encode_sized(pcm, channels, bps, rate, frame_sizes, **opts):
    """the REFERENCE encoder (oracle/_ref/flacenc_sized: src/encoders/flac.c's
    encoders_encode_flac behind oracle/ref_sized_reads.c) with reads of the
    listed sizes -> .flac bytes (padding fixed at 4096, as the standalone
    build)"""
    import tempfile
    args = [REF_FLACENC_SIZED, "-c", str(channels), "-r", str(rate), "-b", str(bps),
            "-B", str(opts["block_size"]), "-l", str(opts["max_lpc_order"]),
            "-P", str(opts.get("min_residual_partition_order", 0)),
            "-R", str(opts["max_residual_partition_order"]),
            "-S", ",".join(str(int(x)) for x in frame_sizes)]
    for k, f in (("mid_side", "-m"), ("adaptive_mid_side", "-M"),
                 ("exhaustive_model_search", "-e")):
        if opts.get(k):
            args.append(f)
    raw = pcm_bytes(pcm, bps)
    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, "o.flac")
        subprocess.run(args + [fn], input=raw, stdout=subprocess.DEVNULL, check=True)
        return open(fn, "rb").read()


def decode(data):
    """-> (pcm int32 interleaved, channels, bps, rate); raises on CRC/MD5 error"""
    lib = load()
    ch, bps, rate, tot = c_u32(), c_u32(), c_u32(), c_u64()
    rc = lib.flacport_decode(data, len(data), ctypes.byref(ch), ctypes.byref(bps),
                             ctypes.byref(rate), ctypes.byref(tot), None, 0)
    if rc != 0:
        raise ValueError("flacport_decode header failed: %d" % rc)
    pcm = np.zeros(tot.value * ch.value, dtype=np.int32)
    rc = lib.flacport_decode(data, len(data), ctypes.byref(ch), ctypes.byref(bps),
                             ctypes.byref(rate), ctypes.byref(tot),
                             pcm.ctypes.data_as(ctypes.c_void_p), len(pcm))
    if rc != 0:
        raise ValueError("flacport_decode failed: %d" % rc)
    return pcm, ch.value, bps.value, rate.value


def pcm_md5(pcm, channels, bps):
    lib = load()
    a = np.ascontiguousarray(pcm, dtype=np.int32)
    d = np.zeros(16, dtype=np.uint8)
    lib.flacport_pcm_md5(a.ctypes.data_as(ctypes.c_void_p), len(a) // channels,
                         channels, bps, d.ctypes.data_as(ctypes.c_void_p))
    return d.tobytes()


def split_flac(data):
    """-> (list of (block_type, payload bytes), frame region bytes)"""
    assert data[:4] == b"fLaC"
    i, blocks = 4, []
    while True:
        last, btype = data[i] & 0x80, data[i] & 0x7F
        n = int.from_bytes(data[i + 1:i + 4], "big")
        blocks.append((btype, data[i + 4:i + 4 + n]))
        i += 4 + n
        if last:
            break
    return blocks, data[i:]


# ---------------------------------------------------------------- decoder
class PortStreamInfo(ctypes.Structure):
    _fields_ = [("min_block_size", c_u32), ("max_block_size", c_u32),
                ("min_frame_size", c_u32), ("max_frame_size", c_u32),
                ("sample_rate", c_u32), ("channels", c_u32),
                ("bits_per_sample", c_u32), ("channel_mask", c_u32),
                ("total_samples", c_u64), ("md5", ctypes.c_uint8 * 16),
                ("frames_offset", c_u64), ("n_seekpoints", c_u32),
                ("reserved", c_u32)]


class PortSeekPoint(ctypes.Structure):
    _fields_ = [("sample_number", c_u64), ("byte_offset", c_u64),
                ("samples", c_u32), ("reserved", c_u32)]


# decoder status codes: the reference's flac_status values
# (src/decoders/flac.h:68-81) plus the conditions FlacDecoder.read raises
FD_OK, FD_ERROR, FD_FRAME_CRC, FD_EOF, FD_MD5 = 0, 1, 14, 15, 16
FD_MESSAGES = {
    1: "Error", 2: "invalid sync code", 3: "invalid reserved bit",
    4: "invalid bits per sample", 5: "invalid sample rate",
    6: "invalid checksum in frame header",
    7: "frame sample rate does not match STREAMINFO sample rate",
    8: "frame channel count does not match STREAMINFO channel count",
    9: "frame bits-per-sample does not match STREAMINFO bits per sample",
    10: "frame block size exceeds STREAMINFO's maximum block size",
    11: "invalid residual partition coding method",
    12: "invalid FIXED subframe order", 13: "invalid subframe type",
    14: "invalid checksum in frame", 15: "EOF reading frame",
    16: "MD5 mismatch at end of stream",
}


def _dec_lib():
    lib = load()
    if not hasattr(lib, "_dec_ready"):
        lib.flacport_read_metadata.restype = ctypes.c_int
        lib.flacport_read_metadata.argtypes = [
            ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(PortStreamInfo),
            ctypes.c_void_p, ctypes.c_size_t]
        lib.flacport_decode_frames.restype = ctypes.c_int
        lib.flacport_decode_frames.argtypes = [
            ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(PortStreamInfo), c_u64,
            ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t),
            ctypes.POINTER(c_u64)]
        lib._dec_ready = True
    return lib


def read_metadata(data):
    """-> (rc, streaminfo dict, [(sample, byte_offset, samples)]);
    rc 0 ok, 1 not FLAC (ValueError), 2 EOF (IOError)"""
    lib = _dec_lib()
    si = PortStreamInfo()
    sp = (PortSeekPoint * 4096)()
    rc = lib.flacport_read_metadata(data, len(data), ctypes.byref(si),
                                    ctypes.cast(sp, ctypes.c_void_p), 4096)
    info = {f: getattr(si, f) for f, _ in PortStreamInfo._fields_ if f != "md5"}
    info["md5"] = bytes(si.md5)
    pts = [(sp[i].sample_number, sp[i].byte_offset, sp[i].samples)
           for i in range(min(si.n_seekpoints, 4096))]
    return rc, info, pts, si


def decode_frames(data, si=None, start=None, remaining=None, check_crc=True,
                  extra_frames=4):
    """Frame loop of the reference decoder over a whole file image.
    -> dict(code, pcm int32 interleaved, offsets [(byte offset from start,
    block_size)], pcm_frames)"""
    lib = _dec_lib()
    if si is None:
        rc, _, _, si = read_metadata(data)
        if rc:
            raise ValueError("metadata rc %d" % rc)
    if start is None:
        start = si.frames_offset
    if remaining is None:
        remaining = si.total_samples
    bs = max(1, si.max_block_size)
    minbs = max(1, min(si.min_block_size or 1, bs))
    want = int(min(remaining, si.total_samples)) + bs * extra_frames
    body = data[start:]
    while True:  # a wrapped remaining count decodes past the total: grow
        frame_cap = want // minbs + extra_frames + 2
        cap = want * max(1, si.channels)
        pcm = np.zeros(cap, dtype=np.int32)
        offs = np.zeros(frame_cap, dtype=np.uint64)
        bss = np.zeros(frame_cap, dtype=np.uint32)
        nf, got = ctypes.c_size_t(), c_u64()
        code = lib.flacport_decode_frames(body, len(body), ctypes.byref(si), remaining,
                                          int(check_crc), pcm.ctypes.data_as(ctypes.c_void_p),
                                          cap, offs.ctypes.data_as(ctypes.c_void_p),
                                          bss.ctypes.data_as(ctypes.c_void_p), frame_cap,
                                          ctypes.byref(nf), ctypes.byref(got))
        if code != -1:
            break
        want *= 4
    n = nf.value
    return dict(code=code, pcm=pcm[:got.value * si.channels],
                offsets=[(int(offs[i]), int(bss[i])) for i in range(n)],
                pcm_frames=got.value)


def pcm_bytes(pcm, bps):
    """FrameList.to_bytes(little_endian, signed) for 8/16/24-bit samples;
    out-of-range values saturate as the reference's int_to_char converters
    do (src/pcm.c:1826-1948)"""
    a = np.asarray(pcm, dtype=np.int32)
    lim = 1 << (bps - 1)
    a = np.clip(a, -lim, lim - 1)
    if a.size == 0:
        return b""
    if bps == 8:
        return a.astype(np.int8).tobytes()
    if bps == 16:
        return a.astype("<i2").tobytes()
    if bps == 24:
        u = a.astype("<i4").view(np.uint8).reshape(-1, 4)[:, :3]
        return u.tobytes()
    raise ValueError("unsupported bps %d" % bps)


# --- PCM converters (oracle/pcmconv_port.c; parity unpinned, see header) ---
CONV_BPS, CONV_DOWNMIX, CONV_AVERAGE = 0, 1, 2


def convert(kind, pcm, channels, in_bps, out_bps=None, mask=0, dither=b""):
    """oracle conversion of interleaved int32 PCM -> int32 array"""
    lib = load()
    a = np.ascontiguousarray(pcm, dtype=np.int32)
    frames = len(a) // channels
    P = ctypes.c_void_p
    if kind == CONV_BPS:
        out = np.empty(max(1, frames * channels), dtype=np.int32)
        d = np.frombuffer(bytes(dither) or b"\0", dtype=np.uint8)
        lib.pcmconvport_bps.argtypes = [P, P, c_u64, c_u32, c_u32, c_u32, P]
        lib.pcmconvport_bps(a.ctypes.data, out.ctypes.data, frames, channels, in_bps,
                            out_bps, d.ctypes.data)
        return out[:frames * channels]
    if kind == CONV_DOWNMIX:
        out = np.empty(max(1, frames * 2), dtype=np.int32)
        lib.pcmconvport_downmix.argtypes = [P, P, c_u64, c_u32, c_u32, c_u32]
        lib.pcmconvport_downmix(a.ctypes.data, out.ctypes.data, frames, channels, mask,
                                in_bps)
        return out[:frames * 2]
    out = np.empty(max(1, frames), dtype=np.int32)
    lib.pcmconvport_average.argtypes = [P, P, c_u64, c_u32]
    lib.pcmconvport_average(a.ctypes.data, out.ctypes.data, frames, channels)
    return out[:frames]


# --- ReplayGain (oracle/replaygain_port.c; parity unpinned, see header) ---
def rg_title(pcm, channels, bps, rate, chunks=None):
    """-> (histogram uint32[12000], title peak); chunks = the frame counts
    the reader's read(4096) calls returned (None: 4096-frame reads)"""
    lib = load()
    a = np.ascontiguousarray(pcm, dtype=np.int32)
    A = np.zeros(12000, dtype=np.uint32)
    P = ctypes.c_void_p
    lib.rgport_title_chunks.argtypes = [P, c_u64, c_u32, c_u32, c_u32, P, c_u64, P]
    lib.rgport_title_chunks.restype = ctypes.c_double
    ch = None if chunks is None else np.ascontiguousarray(chunks, dtype=np.uint32)
    peak = lib.rgport_title_chunks(a.ctypes.data, len(a) // channels, channels, bps, rate,
                                   None if ch is None else ch.ctypes.data,
                                   0 if ch is None else len(ch), A.ctypes.data)
    if peak < 0:
        raise ValueError("rgport_title_chunks rejected the track")
    return A, peak


def rg_window_vals(pcm, channels, bps, rate):
    """the value 1000 log10(mean square / 2 + 1e-37) of every closed 50 ms
    window (what the histogram bins), 4096-frame reads"""
    lib = load()
    a = np.ascontiguousarray(pcm, dtype=np.int32)
    P = ctypes.c_void_p
    lib.rgport_window_vals.argtypes = [P, c_u64, c_u32, c_u32, c_u32, P, c_u64]
    lib.rgport_window_vals.restype = ctypes.c_int64
    cap = len(a) // channels // int(np.ceil(rate * 0.05)) + 2
    vals = np.zeros(cap, dtype=np.float64)
    n = lib.rgport_window_vals(a.ctypes.data, len(a) // channels, channels, bps, rate,
                               vals.ctypes.data, cap)
    if n < 0:
        raise ValueError("rgport_window_vals rejected the track")
    return vals[:n]


def rg_gain(A):
    lib = load()
    A = np.ascontiguousarray(A, dtype=np.uint32)
    lib.rgport_gain.argtypes = [ctypes.c_void_p]
    lib.rgport_gain.restype = ctypes.c_double
    return lib.rgport_gain(A.ctypes.data)


def rg_multiplier(gain, peak):
    lib = load()
    lib.pcmconvport_rg_multiplier.argtypes = [ctypes.c_double, ctypes.c_double]
    lib.pcmconvport_rg_multiplier.restype = ctypes.c_double
    return lib.pcmconvport_rg_multiplier(gain, peak)


def rg_apply(pcm, channels, bps, multiplier, chunk_frames, dither):
    lib = load()
    a = np.ascontiguousarray(pcm, dtype=np.int32)
    out = np.empty(max(1, len(a)), dtype=np.int32)
    d = np.frombuffer(bytes(dither) or b"\0", dtype=np.uint8)
    P = ctypes.c_void_p
    lib.pcmconvport_apply_gain.argtypes = [P, P, c_u64, c_u32, c_u32, ctypes.c_double,
                                           c_u32, P]
    lib.pcmconvport_apply_gain(a.ctypes.data, out.ctypes.data, len(a) // channels, channels,
                               bps, multiplier, chunk_frames, d.ctypes.data)
    return out[:len(a)]


# --- ALAC (oracle/alac_port.c; pinned to oracle/_ref/alacenc / alacdec) ---
REF_ALACENC = os.path.join(ORACLE_DIR, "_ref", "alacenc")
REF_ALACDEC = os.path.join(ORACLE_DIR, "_ref", "alacdec")
ALAC_DEFAULTS = dict(block_size=4096, initial_history=10, history_multiplier=40, maximum_k=14,
                     minimum_interlacing_leftweight=0, maximum_interlacing_leftweight=4)


class AlacOptions(ctypes.Structure):
    _fields_ = [("block_size", c_u32), ("initial_history", c_u32),
                ("history_multiplier", c_u32), ("maximum_k", c_u32),
                ("min_leftweight", c_u32), ("max_leftweight", c_u32)]


class AlacInfo(ctypes.Structure):
    _fields_ = [("max_samples_per_frame", c_u32), ("bits_per_sample", c_u32),
                ("history_multiplier", c_u32), ("initial_history", c_u32),
                ("maximum_k", c_u32), ("channels", c_u32), ("sample_rate", c_u32),
                ("total_frames", c_u32), ("mdat_offset", c_u64), ("n_seekpoints", c_u32),
                ("reserved", c_u32)]


class AlacSeekPoint(ctypes.Structure):
    _fields_ = [("pcm_frames_offset", c_u64), ("file_offset", c_u64)]


ALAC_OK, ALAC_IO_ERROR, ALAC_INVALID_UNUSED_BITS = 0, 1, 2
ALAC_MESSAGES = {1: "I/O Errror", 2: "invalid unused bits", 3: "invalid alac atom",
                 4: "invalid mdhd atom", 5: "mdia atom not found", 6: "stsd atom not found",
                 7: "mdhd atom not found", 8: "invalid seektable entries",
                 9: "Unable to locate 'mdat' atom in stream", 10: "channel length mismatch"}


def _alac_lib():
    lib = load()
    if not hasattr(lib, "_alac_ready"):
        P = ctypes.c_void_p
        lib.alacport_encode.restype = ctypes.c_int
        lib.alacport_encode.argtypes = [P, c_u64, c_u32, c_u32, ctypes.POINTER(AlacOptions), P,
                                        ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t), P,
                                        ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        lib.alacport_max_mdat_bytes.restype = ctypes.c_size_t
        lib.alacport_max_mdat_bytes.argtypes = [c_u64, c_u32, c_u32, c_u32]
        lib.alacport_read_info.restype = ctypes.c_int
        lib.alacport_read_info.argtypes = [ctypes.c_char_p, ctypes.c_size_t,
                                           ctypes.POINTER(AlacInfo), P, ctypes.c_size_t]
        lib.alacport_decode.restype = ctypes.c_int
        lib.alacport_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t,
                                        ctypes.POINTER(AlacInfo), c_u64, c_u64, P,
                                        ctypes.c_size_t, ctypes.POINTER(c_u64), P, P,
                                        ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        lib._alac_ready = True
    return lib


def alac_encode(pcm, channels, bps, **opts):
    """-> (mdat atom bytes, [frameset byte sizes])"""
    lib = _alac_lib()
    o = dict(ALAC_DEFAULTS)
    o.update(opts)
    op = AlacOptions(o["block_size"], o["initial_history"], o["history_multiplier"],
                     o["maximum_k"], o["minimum_interlacing_leftweight"],
                     o["maximum_interlacing_leftweight"])
    a = np.ascontiguousarray(pcm, dtype=np.int32)
    frames = len(a) // channels
    cap = lib.alacport_max_mdat_bytes(frames, channels, bps, op.block_size)
    out = np.zeros(cap, dtype=np.uint8)
    olen = ctypes.c_size_t()
    nfs_cap = frames // op.block_size + 2
    fs = np.zeros(nfs_cap, dtype=np.uint32)
    nfs = ctypes.c_size_t()
    rc = lib.alacport_encode(a.ctypes.data_as(ctypes.c_void_p), frames, channels, bps,
                             ctypes.byref(op), out.ctypes.data_as(ctypes.c_void_p), cap,
                             ctypes.byref(olen), fs.ctypes.data_as(ctypes.c_void_p), nfs_cap,
                             ctypes.byref(nfs))
    if rc != 0:
        raise ValueError("alacport_encode failed: %d" % rc)
    return out[:olen.value].tobytes(), [int(x) for x in fs[:nfs.value]]


def alac_read_info(data):
    """-> (status, AlacInfo, [(pcm_frames_offset, file_offset)])"""
    lib = _alac_lib()
    info = AlacInfo()
    sp = (AlacSeekPoint * 65536)()
    rc = lib.alacport_read_info(bytes(data), len(data), ctypes.byref(info),
                                ctypes.cast(sp, ctypes.c_void_p), 65536)
    pts = [(sp[i].pcm_frames_offset, sp[i].file_offset)
           for i in range(min(info.n_seekpoints, 65536))]
    return rc, info, pts


def alac_decode(data, info=None, start=None, remaining=None):
    """the read() loop over an m4a image -> dict(code, pcm (wave order,
    interleaved int32), framesets [(pcm frames, absolute byte offset)])"""
    lib = _alac_lib()
    data = bytes(data)
    if info is None:
        rc, info, _ = alac_read_info(data)
        if rc:
            return dict(code=100 + rc, pcm=np.zeros(0, np.int32), framesets=[])
    if start is None:
        start = info.mdat_offset
    if remaining is None:
        remaining = info.total_frames
    ch = max(1, info.channels)
    cap = (int(remaining) + 2 * max(1, info.max_samples_per_frame) + 64) * ch
    while True:
        pcm = np.zeros(cap, dtype=np.int32)
        fsn = len(data) // 2 + 4
        fsf = np.zeros(fsn, dtype=np.uint32)
        fso = np.zeros(fsn, dtype=np.uint64)
        got, nfs = c_u64(), ctypes.c_size_t()
        code = lib.alacport_decode(data, len(data), ctypes.byref(info), start, remaining,
                                   pcm.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(got),
                                   fsf.ctypes.data_as(ctypes.c_void_p),
                                   fso.ctypes.data_as(ctypes.c_void_p), fsn, ctypes.byref(nfs))
        if code != -1:
            break
        cap *= 4
    n = min(nfs.value, fsn)
    return dict(code=code, pcm=pcm[:got.value * ch],
                framesets=[(int(fsf[i]), int(fso[i])) for i in range(n)])


def ref_alac_encode(pcm, channels, bps, **opts):
    """the reference encoder (oracle/_ref/alacenc) -> mdat bytes"""
    import tempfile
    o = dict(ALAC_DEFAULTS)
    o.update(opts)
    args = [REF_ALACENC, "-c", str(channels), "-b", str(bps), "-B", str(o["block_size"]),
            "-M", str(o["history_multiplier"]), "-K", str(o["maximum_k"])]
    raw = pcm_bytes(pcm, bps)
    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, "o.mdat")
        subprocess.run(args + [fn], input=raw, stdout=subprocess.DEVNULL, check=True)
        return open(fn, "rb").read()


def ref_alac_decode(m4a_bytes):
    """the reference decoder (oracle/_ref/alacdec) -> (exit code, PCM bytes,
    stderr text)"""
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        fn = os.path.join(d, "i.m4a")
        open(fn, "wb").write(m4a_bytes)
        p = subprocess.run([REF_ALACDEC, fn], capture_output=True)
        return p.returncode, p.stdout, p.stderr.decode("latin-1")


# --- Resampler (oracle/resample_port.c; parity unpinned, see its header) ---
def resample(pcm, channels, bps, ratio, reads=None, return_sizes=False):
    """Resampler(reader, rate) read to the end, libsamplerate sinc (MEDIUM
    table) over int32 interleaved PCM; reads = the wrapped reader's read()
    frame counts (None: 4096-frame reads) -> int32 interleaved output
    [, frame count of every read() including the final 0]"""
    lib = load()
    a = np.ascontiguousarray(pcm, dtype=np.int32)
    frames = len(a) // channels
    P, L = ctypes.c_void_p, ctypes.c_long
    lib.rsport_resample.argtypes = [P, L, ctypes.c_int, ctypes.c_int, ctypes.c_double, P, L,
                                    P, L, P, L, ctypes.POINTER(L)]
    lib.rsport_resample.restype = L
    cap = int(frames * ratio) + 64
    out = np.zeros(max(1, cap * channels), dtype=np.int32)
    r = None if reads is None else np.ascontiguousarray(reads, dtype=np.uint32)
    scap = (len(r) if r is not None else frames // 4096 + 1) + 64
    sizes = np.zeros(scap, dtype=np.uint32)
    ns = L()
    n = lib.rsport_resample(a.ctypes.data, frames, channels, bps, ratio,
                            None if r is None else r.ctypes.data, 0 if r is None else len(r),
                            out.ctypes.data, cap, sizes.ctypes.data, scap, ctypes.byref(ns))
    assert 0 <= n <= cap and ns.value <= scap
    if return_sizes:
        return out[:n * channels], [int(x) for x in sizes[:ns.value]]
    return out[:n * channels]


def resample_positions(n_out, ratio):
    """-> (center frames uint32, start filter indices int32) of the first
    n_out outputs (the fp64 position recurrence)"""
    lib = load()
    P = ctypes.c_void_p
    lib.rsport_positions.argtypes = [c_u64, ctypes.c_double, P, P]
    lib.rsport_positions.restype = c_u64
    c = np.zeros(max(1, n_out), dtype=np.uint32)
    s = np.zeros(max(1, n_out), dtype=np.int32)
    lib.rsport_positions(n_out, ratio, c.ctypes.data, s.ctypes.data)
    return c[:n_out], s[:n_out]
