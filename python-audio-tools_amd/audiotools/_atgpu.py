"""ctypes binding of libatgpu.so — the C ABI declared in include/atgpu.h.

The library holds the HIP kernels (gfx950) and the batch engine.  This
module only marshals arguments; it never encodes anything itself.  Missing
library => ImportError, missing GPU => ATGError(ATG_ERR_DEVICE): there is no
CPU fallback on the product path.
"""

import atexit
import ctypes
import itertools
import os
import threading
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("ATGPU_LIB", os.path.join(_HERE, "libatgpu.so"))

ATG_OK = 0
ATG_ERR_INVALID = -1
ATG_ERR_UNSUPPORTED = -2
ATG_ERR_DEVICE = -3
ATG_ERR_NOMEM = -4
ATG_ERR_CAPACITY = -5

PCM_S16 = 0
PCM_S32 = 1

# every function include/atgpu.h declares (tests check the .so exports them)
EXPORTS = (
    "atg_abi_version", "atg_last_error", "atg_engine_create", "atg_engine_create_ex",
    "atg_engine_destroy", "atg_flac_batch_bounds", "atg_flac_encode_host",
    "atg_flac_encode_host_async", "atg_flac_encode_host_wait",
    "atg_flac_encode_device", "atg_flac_encode_device_async", "atg_flac_encode_wait",
    "atg_engine_kernel_times", "atg_engine_set_host_chunk_bytes", "atg_engine_set_inflight",
    "atg_engine_inflight", "atg_pick_device", "atg_visible_devices",
    "atg_host_gather", "atg_replaygain_rb_factor",
    "atg_flac_encode_frames",
    "atg_flac_max_frames_bytes", "atg_flac_stream_header", "atg_host_alloc",
    "atg_flac_encode_frames_batch", "atg_service_connect", "atg_service_close",
    "atg_service_last_error", "atg_service_encode_frames",
    "atg_host_free", "atg_device_alloc",
    "atg_device_free", "atg_copy_to_device", "atg_copy_device", "atg_copy_to_host",
    "atg_flac_read_metadata", "atg_decoder_create", "atg_decoder_destroy",
    "atg_decoder_last_error", "atg_flac_decode_host", "atg_flac_decode_fetch",
    "atg_flac_decode_device", "atg_flac_decode_device_async", "atg_flac_decode_wait",
    "atg_decoder_kernel_times", "atg_decoder_set_inflight",
    "atg_decoder_set_frame_hypothesis", "atg_decoder_frame_hypothesis_redos",
    "atg_pcm_convert_last_error", "atg_pcm_convert_out_channels",
    "atg_pcm_convert_device", "atg_pcm_convert_host",
    "atg_replaygain_last_error", "atg_replaygain_device", "atg_replaygain_hist_gain",
    "atg_replaygain_set_warmup", "atg_replaygain_fallback_tracks",
    "atg_replaygain_bound", "atg_replaygain_rebinned_windows",
    "atg_replaygain_multiplier", "atg_pcm_apply_gain_device", "atg_pcm_apply_gain_host",
    "atg_alac_last_error", "atg_alac_encoder_create", "atg_alac_encoder_destroy",
    "atg_alac_batch_bounds", "atg_alac_encode_device", "atg_alac_encode_host",
    "atg_alac_encoder_kernel_times", "atg_alac_decoder_last_error", "atg_alac_read_info",
    "atg_alac_decoder_create", "atg_alac_decoder_destroy", "atg_alac_decode_host",
    "atg_alac_decode_fetch", "atg_alac_decode_device", "atg_alac_decoder_kernel_times",
    "atg_resample_last_error", "atg_resample_output_frames", "atg_resample_device",
    "atg_resample_host", "atg_resample_read_sizes", "atg_resample_kernel_times",
)

CONV_BPS, CONV_DOWNMIX, CONV_AVERAGE = 0, 1, 2

c_u32, c_i32, c_u64 = ctypes.c_uint32, ctypes.c_int32, ctypes.c_uint64


class FlacOptions(ctypes.Structure):
    _fields_ = [("block_size", c_u32), ("max_lpc_order", c_u32),
                ("min_residual_partition_order", c_u32),
                ("max_residual_partition_order", c_u32),
                ("mid_side", c_i32), ("adaptive_mid_side", c_i32),
                ("exhaustive_model_search", c_i32),
                ("disable_verbatim_subframes", c_i32),
                ("disable_constant_subframes", c_i32),
                ("disable_fixed_subframes", c_i32),
                ("disable_lpc_subframes", c_i32), ("padding_size", c_u32)]


class Track(ctypes.Structure):
    _fields_ = [("pcm_offset", c_u64), ("pcm_frames", c_u64),
                ("frame_sizes", ctypes.POINTER(c_u32)), ("n_frame_sizes", c_u64)]


class TrackResult(ctypes.Structure):
    _fields_ = [("out_offset", c_u64), ("bytes", c_u64),
                ("first_frame", c_u32), ("n_frames", c_u32),
                ("min_frame_bytes", c_u32), ("max_frame_bytes", c_u32),
                ("md5", ctypes.c_uint8 * 16), ("status", c_i32),
                ("reserved", c_u32)]


class StreamInfo(ctypes.Structure):
    _fields_ = [("min_block_size", c_u32), ("max_block_size", c_u32),
                ("min_frame_size", c_u32), ("max_frame_size", c_u32),
                ("sample_rate", c_u32), ("channels", c_u32),
                ("bits_per_sample", c_u32), ("channel_mask", c_u32),
                ("total_samples", c_u64), ("md5", ctypes.c_uint8 * 16),
                ("frames_offset", c_u64), ("n_seekpoints", c_u32),
                ("reserved", c_u32)]


class SeekPoint(ctypes.Structure):
    _fields_ = [("sample_number", c_u64), ("byte_offset", c_u64),
                ("samples", c_u32), ("reserved", c_u32)]


class DecTrack(ctypes.Structure):
    _fields_ = [("data_offset", c_u64), ("data_bytes", c_u64),
                ("total_samples", c_u64), ("sample_rate", c_u32),
                ("channels", c_u32), ("bits_per_sample", c_u32),
                ("max_block_size", c_u32), ("md5", ctypes.c_uint8 * 16)]


class DecResult(ctypes.Structure):
    _fields_ = [("pcm_offset", c_u64), ("pcm_frames", c_u64),
                ("first_frame", c_u32), ("n_frames", c_u32),
                ("status", c_i32), ("walk_frames", c_u32),
                ("md5", ctypes.c_uint8 * 16), ("walk_status", c_i32),
                ("reserved", c_u32), ("walk_end", c_u64)]


# decode status codes (include/atgpu.h ATG_FD_*) and the reference's
# messages for them (src/decoders/flac.c FlacDecoder_strerror, read())
FD_OK, FD_FRAME_CRC, FD_EOF, FD_MD5 = 0, 14, 15, 16
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


class RgTrack(ctypes.Structure):
    _fields_ = [("pcm_offset", c_u64), ("pcm_frames", c_u64), ("channels", c_u32),
                ("bits_per_sample", c_u32), ("sample_rate", c_u32), ("album", c_u32),
                ("chunk_frames", ctypes.POINTER(c_u32)), ("n_chunks", c_u64)]

    def set_chunks(self, chunks):
        """attach the read() chunk sizes (kept alive on the object)"""
        if chunks is None:
            self._chunks = None
            self.chunk_frames = None
            self.n_chunks = 0
        else:
            self._chunks = np.ascontiguousarray(chunks, dtype=np.uint32)
            self.chunk_frames = self._chunks.ctypes.data_as(ctypes.POINTER(c_u32))
            self.n_chunks = len(self._chunks)
        return self


class RgResult(ctypes.Structure):
    _fields_ = [("title_gain", ctypes.c_double), ("title_peak", ctypes.c_double),
                ("status", c_i32), ("reserved", c_u32)]


class AlacOptions(ctypes.Structure):
    _fields_ = [("block_size", c_u32), ("initial_history", c_u32),
                ("history_multiplier", c_u32), ("maximum_k", c_u32),
                ("minimum_interlacing_leftweight", c_u32),
                ("maximum_interlacing_leftweight", c_u32)]


class AlacTrackResult(ctypes.Structure):
    _fields_ = [("out_offset", c_u64), ("bytes", c_u64), ("pcm_frames", c_u64),
                ("first_frameset", c_u32), ("n_framesets", c_u32), ("status", c_i32),
                ("reserved", c_u32)]


class AlacInfo(ctypes.Structure):
    _fields_ = [("max_samples_per_frame", c_u32), ("bits_per_sample", c_u32),
                ("history_multiplier", c_u32), ("initial_history", c_u32),
                ("maximum_k", c_u32), ("channels", c_u32), ("sample_rate", c_u32),
                ("total_frames", c_u32), ("mdat_offset", c_u64), ("n_seekpoints", c_u32),
                ("reserved", c_u32)]


class AlacSeekPoint(ctypes.Structure):
    _fields_ = [("pcm_frames_offset", c_u64), ("file_offset", c_u64)]


class AlacDecTrack(ctypes.Structure):
    _fields_ = [("data_offset", c_u64), ("data_bytes", c_u64), ("start", c_u64),
                ("remaining", c_u64), ("max_samples_per_frame", c_u32),
                ("bits_per_sample", c_u32), ("history_multiplier", c_u32),
                ("initial_history", c_u32), ("maximum_k", c_u32), ("channels", c_u32),
                ("frameset_bytes", ctypes.POINTER(c_u32)), ("n_frameset_bytes", c_u64)]


class AlacDecResult(ctypes.Structure):
    _fields_ = [("sample_offset", c_u64), ("pcm_frames", c_u64), ("first_frameset", c_u32),
                ("n_framesets", c_u32), ("status", c_i32), ("channels", c_u32)]


class RsTrack(ctypes.Structure):
    _fields_ = [("pcm_offset", c_u64), ("pcm_frames", c_u64), ("in_rate", c_u32),
                ("out_rate", c_u32), ("reads", ctypes.POINTER(c_u32)), ("n_reads", c_u64)]


# ALAC decoder status (include/atgpu.h ATG_AD_*) -> (exception, message) as
# the reference raises them (src/decoders/alac.c alac_exception/strerror,
# ALACDecoder_read, pcmconv.c aa_int_to_FrameList)
AD_OK, AD_IO_ERROR, AD_NO_MDAT, AD_CHANNEL_MISMATCH = 0, 1, 9, 10
AD_INIT_MESSAGES = {1: "I/O Errror", 2: "invalid unused bits", 3: "invalid alac atom",
                    4: "invalid mdhd atom", 5: "mdia atom not found",
                    6: "stsd atom not found", 7: "mdhd atom not found",
                    8: "invalid seektable entries",
                    9: "Unable to locate 'mdat' atom in stream"}
AD_READ_MESSAGES = {1: "EOF during frame reading", 2: "invalid unused bits",
                    10: "channel length mismatch"}


class ATGError(RuntimeError):
    """failure reported by libatgpu (status code + message)"""

    def __init__(self, status, message):
        RuntimeError.__init__(self, "%s (atg status %d)" % (message, status))
        self.status = status
        self.message = message


_lib = None
_lib_lock = threading.Lock()


def load_library():
    """dlopen libatgpu.so (built in-tree by __graft_entry__.build())"""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError("libatgpu.so not found at %s: build it with "
                              "`make -C python-audio-tools_amd/csrc` or "
                              "__graft_entry__.build()" % LIB_PATH)
        lib = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        lib.atg_abi_version.restype = ctypes.c_int
        lib.atg_last_error.restype = ctypes.c_char_p
        lib.atg_engine_create.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
        lib.atg_engine_create.restype = ctypes.c_int
        lib.atg_engine_create_ex.argtypes = [ctypes.c_int, c_u32, ctypes.POINTER(P)]
        lib.atg_engine_create_ex.restype = ctypes.c_int
        lib.atg_engine_destroy.argtypes = [P]
        lib.atg_engine_destroy.restype = None
        lib.atg_flac_batch_bounds.argtypes = [
            ctypes.POINTER(FlacOptions), ctypes.POINTER(Track), c_u32, c_u32, c_u32,
            ctypes.POINTER(c_u64), ctypes.POINTER(c_u64)]
        lib.atg_flac_batch_bounds.restype = ctypes.c_int
        lib.atg_flac_encode_host.argtypes = [
            P, ctypes.POINTER(FlacOptions), P, ctypes.c_int, ctypes.POINTER(Track),
            c_u32, c_u32, c_u32, c_u32, P, c_u64, ctypes.POINTER(TrackResult),
            P, P]
        lib.atg_flac_encode_host.restype = ctypes.c_int
        lib.atg_flac_encode_host_async.argtypes = [
            P, ctypes.POINTER(FlacOptions), P, ctypes.c_int, ctypes.POINTER(Track),
            c_u32, c_u32, c_u32, c_u32, P, c_u64, ctypes.POINTER(TrackResult),
            P, P, ctypes.POINTER(c_u64)]
        lib.atg_flac_encode_host_async.restype = ctypes.c_int
        lib.atg_flac_encode_host_wait.argtypes = [P, c_u64]
        lib.atg_flac_encode_host_wait.restype = ctypes.c_int
        lib.atg_flac_encode_device.argtypes = [
            P, ctypes.POINTER(FlacOptions), P, ctypes.c_int, ctypes.POINTER(Track),
            c_u32, c_u32, c_u32, c_u32, P, c_u64, ctypes.POINTER(TrackResult)]
        lib.atg_flac_encode_device.restype = ctypes.c_int
        lib.atg_flac_encode_device_async.argtypes = [
            P, ctypes.POINTER(FlacOptions), P, ctypes.c_int, ctypes.POINTER(Track),
            c_u32, c_u32, c_u32, c_u32, P, c_u64, ctypes.POINTER(c_u64)]
        lib.atg_flac_encode_device_async.restype = ctypes.c_int
        lib.atg_flac_encode_wait.argtypes = [P, c_u64, ctypes.POINTER(TrackResult)]
        lib.atg_flac_encode_wait.restype = ctypes.c_int
        lib.atg_flac_encode_frames.argtypes = [
            P, ctypes.POINTER(FlacOptions), P, ctypes.c_int, c_u64, P, c_u64, c_u32, c_u32,
            c_u32, c_u64, P, c_u64, ctypes.POINTER(c_u64), P]
        lib.atg_flac_encode_frames.restype = ctypes.c_int
        lib.atg_flac_max_frames_bytes.argtypes = [ctypes.POINTER(FlacOptions), c_u64, P, c_u64,
                                                  c_u32, c_u32]
        lib.atg_flac_max_frames_bytes.restype = c_u64
        lib.atg_flac_stream_header.argtypes = [ctypes.POINTER(FlacOptions), c_u32, c_u32, c_u32,
                                               c_u64, c_u32, c_u32, P, P, c_u64]
        lib.atg_flac_stream_header.restype = c_u64
        lib.atg_host_alloc.argtypes = [c_u64, ctypes.POINTER(P)]
        lib.atg_host_alloc.restype = ctypes.c_int
        lib.atg_host_free.argtypes = [P]
        lib.atg_host_free.restype = None
        lib.atg_engine_set_host_chunk_bytes.argtypes = [P, c_u64]
        lib.atg_engine_set_host_chunk_bytes.restype = ctypes.c_int
        lib.atg_engine_set_inflight.argtypes = [P, c_u32]
        lib.atg_engine_set_inflight.restype = ctypes.c_int
        lib.atg_engine_inflight.argtypes = [P]
        lib.atg_engine_inflight.restype = c_u32
        lib.atg_pick_device.argtypes = []
        lib.atg_pick_device.restype = ctypes.c_int
        lib.atg_visible_devices.argtypes = []
        lib.atg_visible_devices.restype = ctypes.c_int
        lib.atg_engine_kernel_times.argtypes = [
            P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_float),
            ctypes.c_int]
        lib.atg_engine_kernel_times.restype = ctypes.c_int
        lib.atg_device_alloc.argtypes = [P, c_u64, ctypes.POINTER(P)]
        lib.atg_device_alloc.restype = ctypes.c_int
        lib.atg_device_free.argtypes = [P, P]
        lib.atg_device_free.restype = ctypes.c_int
        lib.atg_copy_to_device.argtypes = [P, P, P, c_u64]
        lib.atg_copy_to_device.restype = ctypes.c_int
        lib.atg_copy_device.argtypes = [P, P, P, c_u64]
        lib.atg_copy_device.restype = ctypes.c_int
        lib.atg_copy_to_host.argtypes = [P, P, P, c_u64]
        lib.atg_copy_to_host.restype = ctypes.c_int
        lib.atg_flac_read_metadata.argtypes = [
            ctypes.c_char_p, c_u64, ctypes.POINTER(StreamInfo), P, c_u32]
        lib.atg_flac_read_metadata.restype = ctypes.c_int
        lib.atg_decoder_create.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
        lib.atg_decoder_create.restype = ctypes.c_int
        lib.atg_decoder_destroy.argtypes = [P]
        lib.atg_decoder_destroy.restype = None
        lib.atg_decoder_last_error.restype = ctypes.c_char_p
        lib.atg_flac_decode_host.argtypes = [
            P, P, c_u64, ctypes.POINTER(DecTrack), c_u32, ctypes.POINTER(DecResult),
            ctypes.POINTER(c_u64), ctypes.POINTER(c_u64)]
        lib.atg_flac_decode_host.restype = ctypes.c_int
        lib.atg_flac_decode_fetch.argtypes = [P, P, c_u64, P, P, c_u64]
        lib.atg_flac_decode_fetch.restype = ctypes.c_int
        lib.atg_flac_decode_device.argtypes = [
            P, P, c_u64, ctypes.POINTER(DecTrack), c_u32, ctypes.POINTER(DecResult),
            ctypes.POINTER(P), ctypes.POINTER(c_u64)]
        lib.atg_flac_decode_device.restype = ctypes.c_int
        lib.atg_flac_decode_device_async.argtypes = [
            P, P, c_u64, ctypes.POINTER(DecTrack), c_u32, ctypes.POINTER(c_u64)]
        lib.atg_flac_decode_device_async.restype = ctypes.c_int
        lib.atg_flac_decode_wait.argtypes = [
            P, c_u64, ctypes.POINTER(DecResult), ctypes.POINTER(P), ctypes.POINTER(c_u64)]
        lib.atg_flac_decode_wait.restype = ctypes.c_int
        lib.atg_decoder_set_inflight.argtypes = [P, c_u32]
        lib.atg_decoder_set_inflight.restype = ctypes.c_int
        lib.atg_decoder_set_frame_hypothesis.argtypes = [P, ctypes.c_int]
        lib.atg_decoder_set_frame_hypothesis.restype = ctypes.c_int
        lib.atg_decoder_frame_hypothesis_redos.argtypes = [P]
        lib.atg_decoder_frame_hypothesis_redos.restype = c_u64
        lib.atg_decoder_kernel_times.argtypes = [
            P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_float),
            ctypes.c_int]
        lib.atg_decoder_kernel_times.restype = ctypes.c_int
        lib.atg_pcm_convert_last_error.restype = ctypes.c_char_p
        lib.atg_pcm_convert_out_channels.argtypes = [ctypes.c_int, c_u32]
        lib.atg_pcm_convert_out_channels.restype = c_u32
        lib.atg_pcm_convert_device.argtypes = [
            ctypes.c_int, P, P, c_u64, c_u32, c_u32, c_u32, c_u32, P, c_u64, P]
        lib.atg_pcm_convert_device.restype = ctypes.c_int
        lib.atg_pcm_convert_host.argtypes = [
            ctypes.c_int, ctypes.c_int, P, P, c_u64, c_u32, c_u32, c_u32, c_u32, P, c_u64,
            c_u64]
        lib.atg_pcm_convert_host.restype = ctypes.c_int
        lib.atg_replaygain_last_error.restype = ctypes.c_char_p
        lib.atg_replaygain_device.argtypes = [
            P, ctypes.POINTER(RgTrack), c_u32, c_u32, ctypes.POINTER(RgResult), P,
            ctypes.POINTER(ctypes.c_double), P]
        lib.atg_replaygain_device.restype = ctypes.c_int
        lib.atg_replaygain_hist_gain.argtypes = [P, c_u32, ctypes.POINTER(ctypes.c_double), P]
        lib.atg_replaygain_hist_gain.restype = ctypes.c_int
        lib.atg_replaygain_multiplier.argtypes = [ctypes.c_double, ctypes.c_double]
        lib.atg_replaygain_multiplier.restype = ctypes.c_double
        lib.atg_pcm_apply_gain_device.argtypes = [
            P, P, c_u64, c_u32, c_u32, ctypes.c_double, c_u32, P, c_u64, P]
        lib.atg_pcm_apply_gain_device.restype = ctypes.c_int
        lib.atg_pcm_apply_gain_host.argtypes = [
            ctypes.c_int, P, P, c_u64, c_u32, c_u32, ctypes.c_double, c_u32, P, c_u64, c_u64]
        lib.atg_pcm_apply_gain_host.restype = ctypes.c_int
        lib.atg_alac_last_error.restype = ctypes.c_char_p
        lib.atg_alac_encoder_create.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
        lib.atg_alac_encoder_create.restype = ctypes.c_int
        lib.atg_alac_encoder_destroy.argtypes = [P]
        lib.atg_alac_encoder_destroy.restype = None
        lib.atg_alac_batch_bounds.argtypes = [
            P, ctypes.POINTER(AlacOptions), ctypes.POINTER(Track), c_u32, c_u32, c_u32,
            ctypes.POINTER(c_u64), ctypes.POINTER(c_u64)]
        lib.atg_alac_batch_bounds.restype = ctypes.c_int
        lib.atg_alac_encode_device.argtypes = [
            P, ctypes.POINTER(AlacOptions), P, ctypes.c_int, ctypes.POINTER(Track), c_u32,
            c_u32, c_u32, P, c_u64, ctypes.POINTER(AlacTrackResult), P]
        lib.atg_alac_encode_device.restype = ctypes.c_int
        lib.atg_alac_encode_host.argtypes = [
            P, ctypes.POINTER(AlacOptions), P, ctypes.c_int, ctypes.POINTER(Track), c_u32,
            c_u32, c_u32, P, c_u64, ctypes.POINTER(AlacTrackResult), P]
        lib.atg_alac_encode_host.restype = ctypes.c_int
        lib.atg_alac_encoder_kernel_times.argtypes = [
            P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_float), ctypes.c_int]
        lib.atg_alac_encoder_kernel_times.restype = ctypes.c_int
        lib.atg_alac_decoder_last_error.restype = ctypes.c_char_p
        lib.atg_alac_read_info.argtypes = [ctypes.c_char_p, c_u64, ctypes.POINTER(AlacInfo), P,
                                           c_u32, P, c_u32, ctypes.POINTER(c_u32)]
        lib.atg_alac_read_info.restype = ctypes.c_int
        lib.atg_alac_decoder_create.argtypes = [ctypes.c_int, ctypes.POINTER(P)]
        lib.atg_alac_decoder_create.restype = ctypes.c_int
        lib.atg_alac_decoder_destroy.argtypes = [P]
        lib.atg_alac_decoder_destroy.restype = None
        lib.atg_alac_decode_host.argtypes = [
            P, P, c_u64, ctypes.POINTER(AlacDecTrack), c_u32, ctypes.POINTER(AlacDecResult),
            ctypes.POINTER(c_u64), ctypes.POINTER(c_u64)]
        lib.atg_alac_decode_host.restype = ctypes.c_int
        lib.atg_alac_decode_fetch.argtypes = [P, P, c_u64, P, P, c_u64]
        lib.atg_alac_decode_fetch.restype = ctypes.c_int
        lib.atg_alac_decode_device.argtypes = [
            P, P, c_u64, ctypes.POINTER(AlacDecTrack), c_u32, ctypes.POINTER(AlacDecResult),
            ctypes.POINTER(P), ctypes.POINTER(c_u64)]
        lib.atg_alac_decode_device.restype = ctypes.c_int
        lib.atg_alac_decoder_kernel_times.argtypes = [
            P, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_float), ctypes.c_int]
        lib.atg_alac_decoder_kernel_times.restype = ctypes.c_int
        lib.atg_resample_last_error.restype = ctypes.c_char_p
        lib.atg_resample_output_frames.argtypes = [c_u64, c_u32, c_u32, c_u32]
        lib.atg_resample_output_frames.restype = c_u64
        lib.atg_resample_device.argtypes = [
            ctypes.POINTER(RsTrack), c_u32, c_u32, c_u32, P, P, c_u64, P, P, P]
        lib.atg_resample_device.restype = ctypes.c_int
        lib.atg_resample_host.argtypes = [
            ctypes.c_int, ctypes.POINTER(RsTrack), c_u32, c_u32, c_u32, P, c_u64, P, c_u64,
            P, P]
        lib.atg_resample_host.restype = ctypes.c_int
        lib.atg_resample_read_sizes.argtypes = [c_u64, c_u32, c_u32, c_u32, P, c_u64, P, c_u64]
        lib.atg_resample_read_sizes.restype = ctypes.c_int64
        lib.atg_resample_kernel_times.argtypes = [
            ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_float), ctypes.c_int]
        lib.atg_resample_kernel_times.restype = ctypes.c_int
        _lib = lib
        return lib


def _check(lib, status):
    if status != ATG_OK:
        raise ATGError(status, lib.atg_last_error().decode("utf-8", "replace"))


def make_options(block_size, max_lpc_order, min_residual_partition_order,
                 max_residual_partition_order, mid_side=0, adaptive_mid_side=0,
                 exhaustive_model_search=0, disable_verbatim_subframes=0,
                 disable_constant_subframes=0, disable_fixed_subframes=0,
                 disable_lpc_subframes=0, padding_size=4096):
    return FlacOptions(int(block_size), int(max_lpc_order),
                       int(min_residual_partition_order),
                       int(max_residual_partition_order), int(bool(mid_side)),
                       int(bool(adaptive_mid_side)),
                       int(bool(exhaustive_model_search)),
                       int(bool(disable_verbatim_subframes)),
                       int(bool(disable_constant_subframes)),
                       int(bool(disable_fixed_subframes)),
                       int(bool(disable_lpc_subframes)), int(padding_size))


def _track_array(tracks):
    """tracks: iterable of (pcm_offset, pcm_frames[, frame_sizes])"""
    tracks = list(tracks)
    arr = (Track * max(1, len(tracks)))()
    keep = []
    for i, t in enumerate(tracks):
        arr[i].pcm_offset = int(t[0])
        arr[i].pcm_frames = int(t[1])
        sizes = t[2] if len(t) > 2 else None
        if sizes is not None:
            s = np.ascontiguousarray(sizes, dtype=np.uint32)
            keep.append(s)
            arr[i].frame_sizes = s.ctypes.data_as(ctypes.POINTER(c_u32))
            arr[i].n_frame_sizes = len(s)
        else:
            arr[i].frame_sizes = None
            arr[i].n_frame_sizes = 0
    return arr, len(tracks), keep


# Every engine / decoder / encoder handle this process opened, by opening
# order.  At interpreter exit the atexit hook below closes those still open,
# newest first, while the interpreter and the HIP runtime are both intact:
# otherwise their destroy calls run from __del__ during module teardown (or
# never), interleaved with torch's and the HIP runtime's own teardown.  Round
# 5's two exit-time crashes came from that path.
_live_handles = weakref.WeakValueDictionary()
_handle_serial = itertools.count()


def _track_handle(obj):
    _live_handles[next(_handle_serial)] = obj


def close_all():
    """close every handle still open (newest first); registered with atexit"""
    for k in sorted(_live_handles.keys(), reverse=True):
        obj = _live_handles.get(k)
        if obj is not None:
            try:
                obj.close()
            except Exception:
                pass


atexit.register(close_all)


class TrackTable(object):
    """a batch's atg_track array, built once (batches repeat in pipelines)"""

    def __init__(self, tracks):
        self.arr, self.n, self._keep = _track_array(tracks)


class HostJob:
    """a queued host-memory encode (Engine.encode_async).

    The engine DMAs into the job's pcm / out / result arrays until the job is
    waited, so the arrays are held by the Engine (not only by this object)
    until then, and a job dropped unwaited -- an exception between submit and
    wait, a discarded result -- is waited by its finalizer."""

    def __init__(self, engine, ticket, keep, n, nf):
        self.engine, self.ticket, self.n, self.nf = engine, ticket, n, nf
        engine._inflight[ticket] = keep
        self._done = None

    def wait(self):
        if self._done is None:
            keep = self.engine._inflight.get(self.ticket)
            if keep is None:
                raise ATGError(ATG_ERR_INVALID, "host job already waited or its engine closed")
            try:
                _check(self.engine.lib, self.engine.lib.atg_flac_encode_host_wait(
                    self.engine.handle, self.ticket))
            finally:
                del self.engine._inflight[self.ticket]
            _pcm, out, res, offs, fpcm, _arr, _k = keep
            self._done = (out, [res[i] for i in range(self.n)], offs[:self.nf], fpcm[:self.nf])
        return self._done

    def __del__(self):
        if self._done is None:
            try:
                if self.engine.handle and self.ticket in self.engine._inflight:
                    self.wait()
            except Exception:
                pass


ENGINE_STREAMING = 1  # atg_engine_create_ex flag (include/atgpu.h)
ENGINE_MD5_GPU = 2  # MD5 always on GPU chains
ENGINE_MD5_HOST = 4  # MD5 always on host threads


class Engine(object):
    """one libatgpu engine (streams + workspace) on one device; streaming=True
    for a process that encodes one track at a time (streams on first use,
    ATG_ENGINE_STREAMING); md5 = "auto" (the engine picks GPU chains or host
    threads per batch), "gpu" or "host" (ATG_ENGINE_MD5_GPU / _HOST)"""

    def __init__(self, device=0, streaming=False, md5="auto"):
        self.lib = load_library()
        self.device = device
        self._inflight = {}  # host-job ticket -> the arrays the engine writes
        flags = ENGINE_STREAMING if streaming else 0
        flags |= {"auto": 0, "gpu": ENGINE_MD5_GPU, "host": ENGINE_MD5_HOST}[md5]
        h = ctypes.c_void_p()
        _check(self.lib, self.lib.atg_engine_create_ex(int(device), flags, ctypes.byref(h)))
        self.handle = h
        _track_handle(self)

    def close(self):
        if self.handle:
            # atg_engine_destroy drains the device; the arrays of unwaited host
            # jobs are released only after it
            self.lib.atg_engine_destroy(self.handle)
            self.handle = None
            self._inflight.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def bounds(self, options, tracks, channels, bits_per_sample):
        arr, n, _keep = _track_array(tracks)
        nf, nb = c_u64(), c_u64()
        _check(self.lib, self.lib.atg_flac_batch_bounds(
            ctypes.byref(options), arr, n, channels, bits_per_sample,
            ctypes.byref(nf), ctypes.byref(nb)))
        return nf.value, nb.value

    def encode(self, options, pcm, tracks, channels, bits_per_sample,
               sample_rate, out=None):
        """encode a batch held in host memory.

        pcm: numpy int16 (bits <= 16) or int32 interleaved samples; out: an
        optional uint8 array of at least bounds() bytes (e.g. pinned_empty)
        the images are written to.  Page-locked pcm / out are moved by DMA
        without staging.
        Returns (out: uint8 array, results: list of TrackResult,
                 frame_offsets: uint64 array, frame_pcm: uint32 array)."""
        pcm = np.ascontiguousarray(pcm)
        if pcm.dtype == np.int16:
            fmt = PCM_S16
        elif pcm.dtype == np.int32:
            fmt = PCM_S32
        else:
            raise TypeError("pcm must be int16 or int32")
        tracks = list(tracks)
        nf, nb = self.bounds(options, tracks, channels, bits_per_sample)
        arr, n, keep = _track_array(tracks)
        if out is None:
            out = np.empty(max(1, nb), dtype=np.uint8)
        elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.nbytes < nb:
            raise ValueError("out must be a contiguous uint8 array of >= %d bytes" % nb)
        res = (TrackResult * max(1, n))()
        offs = np.zeros(max(1, nf), dtype=np.uint64)
        fpcm = np.zeros(max(1, nf), dtype=np.uint32)
        _check(self.lib, self.lib.atg_flac_encode_host(
            self.handle, ctypes.byref(options), pcm.ctypes.data_as(ctypes.c_void_p),
            fmt, arr, n, channels, bits_per_sample, sample_rate,
            out.ctypes.data_as(ctypes.c_void_p), nb, res,
            offs.ctypes.data_as(ctypes.c_void_p), fpcm.ctypes.data_as(ctypes.c_void_p)))
        return out, [res[i] for i in range(n)], offs[:nf], fpcm[:nf]

    def encode_async(self, options, pcm, tracks, channels, bits_per_sample,
                     sample_rate, out=None):
        """queue a host-memory batch (atg_flac_encode_host_async); returns a
        HostJob whose wait() gives encode()'s (out, results, frame_offsets,
        frame_pcm).  The job keeps pcm, out and the result arrays alive
        until it is waited; jobs overlap in submission order."""
        pcm = np.ascontiguousarray(pcm)
        if pcm.dtype == np.int16:
            fmt = PCM_S16
        elif pcm.dtype == np.int32:
            fmt = PCM_S32
        else:
            raise TypeError("pcm must be int16 or int32")
        tracks = list(tracks)
        nf, nb = self.bounds(options, tracks, channels, bits_per_sample)
        arr, n, keep = _track_array(tracks)
        if out is None:
            out = np.empty(max(1, nb), dtype=np.uint8)
        elif out.dtype != np.uint8 or not out.flags.c_contiguous or out.nbytes < nb:
            raise ValueError("out must be a contiguous uint8 array of >= %d bytes" % nb)
        res = (TrackResult * max(1, n))()
        offs = np.zeros(max(1, nf), dtype=np.uint64)
        fpcm = np.zeros(max(1, nf), dtype=np.uint32)
        t = c_u64()
        _check(self.lib, self.lib.atg_flac_encode_host_async(
            self.handle, ctypes.byref(options), pcm.ctypes.data_as(ctypes.c_void_p),
            fmt, arr, n, channels, bits_per_sample, sample_rate,
            out.ctypes.data_as(ctypes.c_void_p), nb, res,
            offs.ctypes.data_as(ctypes.c_void_p), fpcm.ctypes.data_as(ctypes.c_void_p),
            ctypes.byref(t)))
        return HostJob(self, t.value, (pcm, out, res, offs, fpcm, arr, keep), n, nf)

    def encode_device(self, options, d_pcm, fmt, tracks, channels,
                      bits_per_sample, sample_rate, d_out, out_cap):
        """encode a batch whose PCM is already in device memory; the .flac
        images stay in device memory at d_out.  Returns the TrackResults.
        `tracks` may be a TrackTable (prepared once, reused across calls)."""
        if isinstance(tracks, TrackTable):
            arr, n = tracks.arr, tracks.n
        else:
            arr, n, keep = _track_array(tracks)
        res = (TrackResult * max(1, n))()
        _check(self.lib, self.lib.atg_flac_encode_device(
            self.handle, ctypes.byref(options), ctypes.c_void_p(d_pcm), fmt, arr, n,
            channels, bits_per_sample, sample_rate, ctypes.c_void_p(d_out),
            out_cap, res))
        return [res[i] for i in range(n)]

    def encode_device_async(self, options, d_pcm, fmt, tracks, channels, bits_per_sample,
                            sample_rate, d_out, out_cap):
        """enqueue a device-memory batch; -> (ticket, n_tracks) for wait()"""
        if isinstance(tracks, TrackTable):
            arr, n = tracks.arr, tracks.n
        else:
            arr, n, keep = _track_array(tracks)
        t = c_u64()
        _check(self.lib, self.lib.atg_flac_encode_device_async(
            self.handle, ctypes.byref(options), ctypes.c_void_p(d_pcm), fmt, arr, n,
            channels, bits_per_sample, sample_rate, ctypes.c_void_p(d_out), out_cap,
            ctypes.byref(t)))
        return (t.value, n)

    def wait(self, ticket):
        """TrackResults of an enqueued batch (waits for it)"""
        t, n = ticket
        res = (TrackResult * max(1, n))()
        _check(self.lib, self.lib.atg_flac_encode_wait(self.handle, t, res))
        return [res[i] for i in range(n)]

    def encode_frames(self, options, pcm, channels, bits_per_sample, sample_rate,
                      first_frame_number=0, frame_sizes=None):
        """one track's PCM (host numpy int16 / int32, interleaved) as FLAC
        frames only, numbered from first_frame_number (atg_flac_encode_frames)
        -> (frame bytes: uint8 array, per-frame byte counts: uint32 array)"""
        pcm = np.ascontiguousarray(pcm)
        if pcm.dtype == np.int16:
            fmt = PCM_S16
        elif pcm.dtype == np.int32:
            fmt = PCM_S32
        else:
            raise TypeError("pcm must be int16 or int32")
        frames = len(pcm) // channels
        fs = None if frame_sizes is None else np.ascontiguousarray(frame_sizes, dtype=np.uint32)
        fs_p = fs.ctypes.data_as(ctypes.c_void_p) if fs is not None else None
        nfs = len(fs) if fs is not None else 0
        cap = self.lib.atg_flac_max_frames_bytes(ctypes.byref(options), frames, fs_p, nfs,
                                                 channels, bits_per_sample)
        if not cap:
            raise ATGError(ATG_ERR_INVALID, "invalid encoder options")
        n_fr = nfs if fs is not None else (frames + options.block_size - 1) // options.block_size
        out = np.empty(max(1, cap), dtype=np.uint8)
        fb = np.zeros(max(1, n_fr), dtype=np.uint32)
        nb = c_u64()
        _check(self.lib, self.lib.atg_flac_encode_frames(
            self.handle, ctypes.byref(options), pcm.ctypes.data_as(ctypes.c_void_p), fmt,
            frames, fs_p, nfs, channels, bits_per_sample, sample_rate, int(first_frame_number),
            out.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(nb),
            fb.ctypes.data_as(ctypes.c_void_p)))
        return out[:nb.value], fb[:n_fr]

    def set_inflight(self, n):
        """batches encode_device_async keeps in flight (3..32; 0 = automatic,
        the default: the first batch of a pipeline picks it, include/atgpu.h)"""
        _check(self.lib, self.lib.atg_engine_set_inflight(self.handle, int(n)))

    def inflight(self):
        """the current depth D: keep up to D device batches in flight (with
        the automatic depth, read it after the pipeline's first enqueue)"""
        return int(self.lib.atg_engine_inflight(self.handle))

    def set_host_chunk_bytes(self, nbytes):
        """PCM bytes per chunk of the host-memory pipeline (encode())"""
        _check(self.lib, self.lib.atg_engine_set_host_chunk_bytes(self.handle, int(nbytes)))

    def kernel_times(self):
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_float * 16)()
        k = self.lib.atg_engine_kernel_times(self.handle, names, ms, 16)
        return {names[i].decode(): float(ms[i]) for i in range(k)}

    def copy_device(self, d_dst, d_src, nbytes):
        """device-to-device copy on this engine's device"""
        _check(self.lib, self.lib.atg_copy_device(self.handle, ctypes.c_void_p(d_dst),
                                                  ctypes.c_void_p(d_src), nbytes))

    def copy_to_host(self, dst, d_src):
        """device bytes at d_src -> the numpy array dst (its full size)"""
        _check(self.lib, self.lib.atg_copy_to_host(
            self.handle, dst.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(d_src),
            dst.nbytes))
        return dst

    def copy_to_device(self, d_dst, src):
        """the numpy array src (its full size) -> device bytes at d_dst"""
        src = np.ascontiguousarray(src)
        _check(self.lib, self.lib.atg_copy_to_device(
            self.handle, ctypes.c_void_p(d_dst), src.ctypes.data_as(ctypes.c_void_p), src.nbytes))

    def device_alloc(self, nbytes):
        """device memory on this engine's device -> pointer (device_free)"""
        p = ctypes.c_void_p()
        _check(self.lib, self.lib.atg_device_alloc(self.handle, max(4, int(nbytes)),
                                                   ctypes.byref(p)))
        return p.value

    def device_free(self, d_ptr):
        _check(self.lib, self.lib.atg_device_free(self.handle, ctypes.c_void_p(d_ptr)))


def stream_header(options, channels, bits_per_sample, sample_rate, total_samples=0,
                  min_frame_bytes=0xFFFFFF, max_frame_bytes=0, md5=b"\0" * 16):
    """fLaC + STREAMINFO + VORBIS_COMMENT + PADDING (atg_flac_stream_header)"""
    lib = load_library()
    cap = 4096 + int(options.padding_size)
    out = ctypes.create_string_buffer(cap)
    m = ctypes.create_string_buffer(bytes(md5), 16)
    n = lib.atg_flac_stream_header(ctypes.byref(options), channels, bits_per_sample,
                                   sample_rate, int(total_samples), int(min_frame_bytes),
                                   int(max_frame_bytes), m, out, cap)
    if not n:
        raise ATGError(ATG_ERR_INVALID, "invalid stream header arguments")
    return out.raw[:n]


def pinned_empty(shape, dtype=np.uint8):
    """a numpy array in page-locked host memory (atg_host_alloc), freed
    when the array is collected"""
    lib = load_library()
    dtype = np.dtype(dtype)
    count = int(np.prod(shape)) if np.ndim(shape) else int(shape)
    nbytes = max(1, count * dtype.itemsize)
    p = ctypes.c_void_p()
    _check(lib, lib.atg_host_alloc(nbytes, ctypes.byref(p)))
    buf = (ctypes.c_uint8 * nbytes).from_address(p.value)
    # not freed by weakref's own atexit hook: that hook runs before
    # close_all (it registers later), and a buffer an unwaited host job still
    # DMAs into must outlive the engine; at exit the process takes it back
    weakref.finalize(buf, lib.atg_host_free, p.value).atexit = False
    return np.frombuffer(buf, dtype=dtype, count=count).reshape(shape)


_staging = {}
_staging_lock = threading.Lock()


def staging(key, nbytes):
    """a page-locked host buffer of at least nbytes, one per key, kept for
    the process's lifetime (grown on demand): uploads from it run at DMA
    rate without a pinning cost per call"""
    with _staging_lock:
        b = _staging.get(key)
        if b is None or b.nbytes < nbytes:
            b = pinned_empty(max(int(nbytes), 1 << 20), np.uint8)
            _staging[key] = b
        return b


_upool = None


def upload_pool():
    """a thread for host-to-device copies beside the host threads' fills"""
    global _upool
    with _staging_lock:
        if _upool is None:
            import concurrent.futures
            _upool = concurrent.futures.ThreadPoolExecutor(4)
        return _upool


def read_metadata(data, sp_cap=4096):
    """flacdec_read_metadata over an in-memory image (host C in libatgpu).
    -> (rc, StreamInfo, [(sample_number, byte_offset, samples)]);
    rc 0 ok, 1 not a FLAC stream, 2 EOF"""
    lib = load_library()
    si = StreamInfo()
    sp = (SeekPoint * max(1, sp_cap))()
    rc = lib.atg_flac_read_metadata(bytes(data), len(data), ctypes.byref(si),
                                    ctypes.cast(sp, ctypes.c_void_p), sp_cap)
    pts = [(sp[i].sample_number, sp[i].byte_offset, sp[i].samples)
           for i in range(min(si.n_seekpoints, sp_cap))]
    return rc, si, pts


def dec_track(offset, nbytes, si):
    """DecTrack for a stream whose first frame is at `offset` of the batch"""
    t = DecTrack()
    t.data_offset = offset
    t.data_bytes = nbytes
    t.total_samples = si.total_samples
    t.sample_rate = si.sample_rate
    t.channels = si.channels
    t.bits_per_sample = si.bits_per_sample
    t.max_block_size = si.max_block_size
    t.md5[:] = bytes(si.md5)
    return t


class Decoder(object):
    """one libatgpu FLAC decoder (HIP stream + workspace) on one device"""

    def __init__(self, device=0):
        self.lib = load_library()
        self.device = device
        h = ctypes.c_void_p()
        self._check(self.lib.atg_decoder_create(int(device), ctypes.byref(h)))
        self.handle = h
        _track_handle(self)
        self._pending = {}

    def _check(self, status):
        if status != ATG_OK:
            raise ATGError(status, self.lib.atg_decoder_last_error().decode(
                "utf-8", "replace"))

    def close(self):
        if self.handle:
            self.lib.atg_decoder_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_inflight(self, n):
        """decode batches decode_device_async keeps in flight (3..16)"""
        self._check(self.lib.atg_decoder_set_inflight(self.handle, int(n)))

    def set_frame_hypothesis(self, mode):
        """the parse's frame-end hypothesis: 0 off (every subframe walked),
        1 on (default), 2 on with every batch redone (self-check)"""
        self._check(self.lib.atg_decoder_set_frame_hypothesis(self.handle, int(mode)))

    def frame_hypothesis_redos(self):
        """batches redone with the full parse after a failed check"""
        return int(self.lib.atg_decoder_frame_hypothesis_redos(self.handle))

    def decode(self, data, tracks, fetch_pcm=True):
        """decode a batch in host memory.  data: bytes-like holding every
        stream; tracks: list of DecTrack.  -> (pcm int32 array, [DecResult],
        frame byte offsets (uint64), frame block sizes (uint32)); pcm is
        None when fetch_pcm is false (results carry the PCM MD5s)"""
        buf = np.frombuffer(bytes(data), dtype=np.uint8)
        n = len(tracks)
        arr = (DecTrack * max(1, n))(*tracks)
        res = (DecResult * max(1, n))()
        ns, nf = c_u64(), c_u64()
        self._check(self.lib.atg_flac_decode_host(
            self.handle, buf.ctypes.data_as(ctypes.c_void_p), len(buf), arr, n, res,
            ctypes.byref(ns), ctypes.byref(nf)))
        pcm = np.empty(max(1, ns.value), dtype=np.int32) if fetch_pcm else None
        offs = np.empty(max(1, nf.value), dtype=np.uint64)
        bss = np.empty(max(1, nf.value), dtype=np.uint32)
        self._check(self.lib.atg_flac_decode_fetch(
            self.handle, pcm.ctypes.data_as(ctypes.c_void_p) if fetch_pcm else None,
            ns.value, offs.ctypes.data_as(ctypes.c_void_p),
            bss.ctypes.data_as(ctypes.c_void_p), nf.value))
        return (pcm[:ns.value] if fetch_pcm else None, [res[i] for i in range(n)],
                offs[:nf.value], bss[:nf.value])

    def decode_device(self, d_data, nbytes, tracks):
        """decode a batch already in device memory -> ([DecResult],
        device pointer of the int32 PCM, interleaved samples)"""
        n = len(tracks)
        arr = (DecTrack * max(1, n))(*tracks)
        res = (DecResult * max(1, n))()
        dp = ctypes.c_void_p()
        ns = c_u64()
        self._check(self.lib.atg_flac_decode_device(
            self.handle, ctypes.c_void_p(d_data), nbytes, arr, n, res, ctypes.byref(dp),
            ctypes.byref(ns)))
        return [res[i] for i in range(n)], dp.value, ns.value

    def decode_device_async(self, d_data, nbytes, tracks):
        """enqueue a device-resident batch (three may be in flight) -> ticket;
        d_data must stay valid until decode_wait(ticket)"""
        n = len(tracks)
        arr = (DecTrack * max(1, n))(*tracks)
        ticket = c_u64()
        self._check(self.lib.atg_flac_decode_device_async(
            self.handle, ctypes.c_void_p(d_data), nbytes, arr, n, ctypes.byref(ticket)))
        self._pending[ticket.value] = n
        return ticket.value

    def decode_wait(self, ticket):
        """-> ([DecResult], device pointer of the int32 PCM, interleaved samples)"""
        n = self._pending.pop(ticket, 0)
        res = (DecResult * max(1, n))()
        dp = ctypes.c_void_p()
        ns = c_u64()
        self._check(self.lib.atg_flac_decode_wait(self.handle, ticket, res, ctypes.byref(dp),
                                                  ctypes.byref(ns)))
        return [res[i] for i in range(n)], dp.value, ns.value

    def kernel_times(self):
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_float * 16)()
        k = self.lib.atg_decoder_kernel_times(self.handle, names, ms, 16)
        return {names[i].decode(): float(ms[i]) for i in range(k)}


class AlacEncoder(object):
    """one libatgpu ALAC encoder (HIP stream + workspace) on one device"""

    def __init__(self, device=0):
        self.lib = load_library()
        self.device = device
        h = ctypes.c_void_p()
        self._check(self.lib.atg_alac_encoder_create(int(device), ctypes.byref(h)))
        self.handle = h
        _track_handle(self)

    def _check(self, status):
        if status != ATG_OK:
            raise ATGError(status, self.lib.atg_alac_last_error().decode("utf-8", "replace"))

    def close(self):
        if self.handle:
            self.lib.atg_alac_encoder_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def options(block_size=4096, initial_history=10, history_multiplier=40, maximum_k=14,
                minimum_interlacing_leftweight=0, maximum_interlacing_leftweight=4):
        return AlacOptions(int(block_size), int(initial_history), int(history_multiplier),
                           int(maximum_k), int(minimum_interlacing_leftweight),
                           int(maximum_interlacing_leftweight))

    def bounds(self, options, tracks, channels, bits_per_sample):
        arr, n, _keep = _track_array(tracks)
        nf, nb = c_u64(), c_u64()
        self._check(self.lib.atg_alac_batch_bounds(self.handle, ctypes.byref(options), arr, n,
                                                   channels, bits_per_sample, ctypes.byref(nf),
                                                   ctypes.byref(nb)))
        return nf.value, nb.value

    def encode(self, options, pcm, tracks, channels, bits_per_sample):
        """host PCM (int16 for 16-bit, int32 otherwise) -> (out bytes array,
        [AlacTrackResult], frameset byte sizes uint32 array)"""
        pcm = np.ascontiguousarray(pcm)
        fmt = PCM_S16 if pcm.dtype == np.int16 else PCM_S32
        if pcm.dtype not in (np.int16, np.int32):
            raise TypeError("pcm must be int16 or int32")
        tracks = list(tracks)
        nf, nb = self.bounds(options, tracks, channels, bits_per_sample)
        arr, n, keep = _track_array(tracks)
        out = np.empty(max(1, nb), dtype=np.uint8)
        res = (AlacTrackResult * max(1, n))()
        fsb = np.zeros(max(1, nf), dtype=np.uint32)
        self._check(self.lib.atg_alac_encode_host(
            self.handle, ctypes.byref(options), pcm.ctypes.data_as(ctypes.c_void_p), fmt, arr,
            n, channels, bits_per_sample, out.ctypes.data_as(ctypes.c_void_p), nb, res,
            fsb.ctypes.data_as(ctypes.c_void_p)))
        return out, [res[i] for i in range(n)], fsb[:nf]

    def encode_device(self, options, d_pcm, fmt, tracks, channels, bits_per_sample, d_out,
                      out_cap, frameset_bytes=None):
        if isinstance(tracks, TrackTable):
            arr, n = tracks.arr, tracks.n
        else:
            arr, n, keep = _track_array(tracks)
        res = (AlacTrackResult * max(1, n))()
        self._check(self.lib.atg_alac_encode_device(
            self.handle, ctypes.byref(options), ctypes.c_void_p(d_pcm), fmt, arr, n, channels,
            bits_per_sample, ctypes.c_void_p(d_out), out_cap, res,
            frameset_bytes.ctypes.data_as(ctypes.c_void_p) if frameset_bytes is not None
            else None))
        return [res[i] for i in range(n)]

    def kernel_times(self):
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_float * 16)()
        k = self.lib.atg_alac_encoder_kernel_times(self.handle, names, ms, 16)
        return {names[i].decode(): float(ms[i]) for i in range(k)}


def alac_read_info(data, sp_cap=65536):
    """parse_decoding_parameters + seek_mdat (host C in libatgpu)
    -> (status, AlacInfo, [(pcm_frames_offset, file_offset)], stsz sizes)"""
    lib = load_library()
    data = bytes(data)
    info = AlacInfo()
    sp = (AlacSeekPoint * max(1, sp_cap))()
    nfs = c_u32()
    lib.atg_alac_read_info(data, len(data), ctypes.byref(info), None, 0, None, 0,
                           ctypes.byref(nfs))
    sizes = np.zeros(max(1, nfs.value), dtype=np.uint32)
    st = lib.atg_alac_read_info(data, len(data), ctypes.byref(info),
                                ctypes.cast(sp, ctypes.c_void_p), sp_cap,
                                sizes.ctypes.data_as(ctypes.c_void_p), len(sizes),
                                ctypes.byref(nfs))
    pts = [(sp[i].pcm_frames_offset, sp[i].file_offset)
           for i in range(min(info.n_seekpoints, sp_cap))]
    return st, info, pts, sizes[:nfs.value]


def alac_dec_track(offset, nbytes, info, start=None, remaining=None, frameset_bytes=None):
    """AlacDecTrack for an image at `offset` of the batch buffer; keeps the
    hint array alive on the returned object"""
    t = AlacDecTrack()
    t.data_offset = offset
    t.data_bytes = nbytes
    t.start = info.mdat_offset if start is None else start
    t.remaining = info.total_frames if remaining is None else remaining
    t.max_samples_per_frame = info.max_samples_per_frame
    t.bits_per_sample = info.bits_per_sample
    t.history_multiplier = info.history_multiplier
    t.initial_history = info.initial_history
    t.maximum_k = info.maximum_k
    t.channels = info.channels
    if frameset_bytes is not None and len(frameset_bytes):
        hint = np.ascontiguousarray(frameset_bytes, dtype=np.uint32)
        t._hint = hint
        t.frameset_bytes = hint.ctypes.data_as(ctypes.POINTER(c_u32))
        t.n_frameset_bytes = len(hint)
    else:
        t._hint = None
        t.frameset_bytes = None
        t.n_frameset_bytes = 0
    return t


class AlacDecoder(object):
    """one libatgpu ALAC decoder (HIP stream + workspace) on one device"""

    def __init__(self, device=0):
        self.lib = load_library()
        self.device = device
        h = ctypes.c_void_p()
        self._check(self.lib.atg_alac_decoder_create(int(device), ctypes.byref(h)))
        self.handle = h
        _track_handle(self)

    def _check(self, status):
        if status != ATG_OK:
            raise ATGError(status, self.lib.atg_alac_decoder_last_error().decode(
                "utf-8", "replace"))

    def close(self):
        if self.handle:
            self.lib.atg_alac_decoder_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def decode(self, data, tracks):
        """decode a batch in host memory (images 4-byte aligned in data)
        -> (pcm int32, [AlacDecResult], frameset frames, frameset offsets)"""
        buf = np.frombuffer(bytes(data), dtype=np.uint8)
        n = len(tracks)
        arr = (AlacDecTrack * max(1, n))(*tracks)
        res = (AlacDecResult * max(1, n))()
        ns, nf = c_u64(), c_u64()
        self._check(self.lib.atg_alac_decode_host(
            self.handle, buf.ctypes.data_as(ctypes.c_void_p), len(buf), arr, n, res,
            ctypes.byref(ns), ctypes.byref(nf)))
        pcm = np.empty(max(1, ns.value), dtype=np.int32)
        ff = np.empty(max(1, nf.value), dtype=np.uint32)
        fo = np.empty(max(1, nf.value), dtype=np.uint64)
        self._check(self.lib.atg_alac_decode_fetch(
            self.handle, pcm.ctypes.data_as(ctypes.c_void_p), ns.value,
            ff.ctypes.data_as(ctypes.c_void_p), fo.ctypes.data_as(ctypes.c_void_p), nf.value))
        return pcm[:ns.value], [res[i] for i in range(n)], ff[:nf.value], fo[:nf.value]

    def decode_device(self, d_data, nbytes, tracks):
        n = len(tracks)
        arr = (AlacDecTrack * max(1, n))(*tracks)
        res = (AlacDecResult * max(1, n))()
        dp = ctypes.c_void_p()
        ns = c_u64()
        self._check(self.lib.atg_alac_decode_device(
            self.handle, ctypes.c_void_p(d_data), nbytes, arr, n, res, ctypes.byref(dp),
            ctypes.byref(ns)))
        return [res[i] for i in range(n)], dp.value, ns.value

    def kernel_times(self):
        names = (ctypes.c_char_p * 16)()
        ms = (ctypes.c_float * 16)()
        k = self.lib.atg_alac_decoder_kernel_times(self.handle, names, ms, 16)
        return {names[i].decode(): float(ms[i]) for i in range(k)}


_engine = None
_engine_lock = threading.Lock()
_alac_decoder = None
_decoder = None
_alac_encoder = None


def default_device():
    """ATG_DEVICE, else LOCAL_RANK, else this process's turn of a node-wide
    round robin over the visible GPUs (atg_pick_device, csrc/devices.hip):
    one process per track under track2track -j N lands on N GPUs"""
    return int(load_library().atg_pick_device())


def visible_devices():
    """GPUs this process may use (atg_visible_devices; no HIP call)"""
    return int(load_library().atg_visible_devices())


def engine():
    """process-wide engine on ATG_DEVICE / LOCAL_RANK / device 0"""
    global _engine
    with _engine_lock:
        if _engine is None:
            _engine = Engine(default_device())
        return _engine


def decoder():
    """process-wide FLAC decoder on ATG_DEVICE / LOCAL_RANK / device 0"""
    global _decoder
    with _engine_lock:
        if _decoder is None:
            _decoder = Decoder(default_device())
        return _decoder


def alac_decoder():
    """process-wide ALAC decoder on ATG_DEVICE / LOCAL_RANK / device 0"""
    global _alac_decoder
    with _engine_lock:
        if _alac_decoder is None:
            _alac_decoder = AlacDecoder(default_device())
        return _alac_decoder


def alac_encoder():
    """process-wide ALAC encoder on ATG_DEVICE / LOCAL_RANK / device 0"""
    global _alac_encoder
    with _engine_lock:
        if _alac_encoder is None:
            _alac_encoder = AlacEncoder(default_device())
        return _alac_encoder


# ---- batches sharded over the node's GPUs ---------------------
# A batch entry point (encode_flac_batch, decode_flac_batch,
# calculate_replay_gain) splits its tracks into contiguous groups, one per
# device, balanced by PCM frames, and runs every group on its device's
# engine in a thread of its own (the C calls release the GIL); results are
# merged in track order.  No collective: the groups are independent, except
# ReplayGain's album histogram / peak, reduced by the caller (replaygain.py).
_shard_objs = {}


def batch_devices():
    """devices a batch call shards over: the one ATG_DEVICE / LOCAL_RANK
    names (a process bound to a GPU), else every visible GPU.
    ATG_SHARD_DEVICES="0,0" lists them explicitly (tests: two shards on one
    GPU take the multi-device path)"""
    v = os.environ.get("ATG_SHARD_DEVICES", "")
    if v.strip():
        return [int(x) for x in v.split(",") if x.strip()]
    for var in ("ATG_DEVICE", "LOCAL_RANK"):
        if os.environ.get(var, "").strip():
            return [int(os.environ[var])]
    return list(range(visible_devices()))


def shard_ranges(weights, n):
    """contiguous [t0, t1) ranges of len(weights) tracks over at most n
    shards, each ending where the running weight first reaches its share
    of the total; empty ranges dropped"""
    weights = [max(0, int(w)) for w in weights]
    t, n = len(weights), max(1, min(n, len(weights)))
    if t == 0:
        return []
    total = float(sum(weights)) or float(t)
    w = weights if sum(weights) else [1] * t
    out, t0, run = [], 0, 0
    for k in range(1, n + 1):
        goal = total * k / n
        t1 = t0
        while t1 < t and (run + w[t1] <= goal or t1 == t0) and (t - t1) > (n - k):
            run += w[t1]
            t1 += 1
        if k == n:
            t1 = t
        if t1 > t0:
            out.append((t0, t1))
        t0 = t1
    return out


def shard_object(kind, i, device):
    """the engine / decoder of shard i on `device` (one per shard, kept for
    the process's lifetime like engine())"""
    key = (kind, i, device)
    with _engine_lock:
        obj = _shard_objs.get(key)
        if obj is None:
            obj = {"engine": Engine, "decoder": Decoder, "alac_decoder": AlacDecoder}[kind](
                device)
            _shard_objs[key] = obj
        return obj


def run_shards(fn, n):
    """fn(i) for i in range(n) on n threads (one per device); results in
    order; the first exception is raised"""
    if n == 1:
        return [fn(0)]
    out, err = [None] * n, []

    def one(i):
        try:
            out[i] = fn(i)
        except BaseException as e:  # noqa: B902 -- re-raised below
            err.append(e)

    th = [threading.Thread(target=one, args=(i,)) for i in range(n)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    if err:
        raise err[0]
    return out


def pcm_convert(kind, pcm, channels, in_bps, out_bps=None, channel_mask=0,
                dither=b"", dither_bit0=0, device=None):
    """one GPU conversion of interleaved int32 PCM held in host memory
    (atg_pcm_convert_host) -> int32 numpy array"""
    lib = load_library()
    a = np.ascontiguousarray(pcm, dtype=np.int32)
    frames = len(a) // channels
    oc = lib.atg_pcm_convert_out_channels(kind, channels)
    out = np.empty(max(1, frames * oc), dtype=np.int32)
    d = np.frombuffer(bytes(dither), dtype=np.uint8) if dither else None
    st = lib.atg_pcm_convert_host(
        default_device() if device is None else device, kind,
        a.ctypes.data_as(ctypes.c_void_p), out.ctypes.data_as(ctypes.c_void_p), frames,
        channels, channel_mask, in_bps, in_bps if out_bps is None else out_bps,
        d.ctypes.data_as(ctypes.c_void_p) if d is not None else None,
        0 if d is None else len(d), dither_bit0)
    if st != ATG_OK:
        raise ATGError(st, lib.atg_pcm_convert_last_error().decode("utf-8", "replace"))
    return out[:frames * oc]


def _rg_check(lib, st):
    if st != ATG_OK:
        raise ATGError(st, lib.atg_replaygain_last_error().decode("utf-8", "replace"))


def replaygain_device(d_pcm, tracks, n_albums=0, d_album_hist=None):
    """ReplayGain of a batch whose int32 PCM is in device memory.
    tracks: list of RgTrack.  -> ([RgResult], [album peak])"""
    lib = load_library()
    n = len(tracks)
    arr = (RgTrack * max(1, n))(*tracks)
    res = (RgResult * max(1, n))()
    peaks = (ctypes.c_double * max(1, n_albums))()
    _rg_check(lib, lib.atg_replaygain_device(
        ctypes.c_void_p(d_pcm), arr, n, n_albums, res,
        ctypes.c_void_p(d_album_hist) if d_album_hist else None, peaks, None))
    return [res[i] for i in range(n)], [peaks[i] for i in range(n_albums)]


def replaygain_hist_gain(d_hist, n):
    """analyzeResult of n device histograms -> list of gains (NaN = none)"""
    lib = load_library()
    g = (ctypes.c_double * max(1, n))()
    _rg_check(lib, lib.atg_replaygain_hist_gain(ctypes.c_void_p(d_hist), n, g, None))
    return [g[i] for i in range(n)]


def replaygain_host(pcm, tracks, n_albums=0, return_hist=False, eng=None):
    """same as replaygain_device for int32 PCM in host memory, on `eng`'s
    device (the process-wide engine's by default)
    -> (results, album_peaks, album_gains[, album histograms uint32])"""
    lib = load_library()
    eng = eng or engine()
    a = np.ascontiguousarray(pcm, dtype=np.int32)
    d_pcm, d_hist = ctypes.c_void_p(), ctypes.c_void_p()
    _check(lib, lib.atg_device_alloc(eng.handle, max(4, a.nbytes), ctypes.byref(d_pcm)))
    _check(lib, lib.atg_device_alloc(eng.handle, max(4, 48000 * n_albums),
                                     ctypes.byref(d_hist)))
    try:
        if a.nbytes:
            _check(lib, lib.atg_copy_to_device(eng.handle, d_pcm,
                                               a.ctypes.data_as(ctypes.c_void_p), a.nbytes))
        res, peaks = replaygain_device(d_pcm.value, tracks, n_albums, d_hist.value)
        gains = replaygain_hist_gain(d_hist.value, n_albums) if n_albums else []
        hist = None
        if return_hist:
            hist = np.zeros((max(1, n_albums), 12000), dtype=np.uint32)
            if n_albums:
                _check(lib, lib.atg_copy_to_host(eng.handle, hist.ctypes.data_as(ctypes.c_void_p),
                                                 d_hist, hist.nbytes))
    finally:
        lib.atg_device_free(eng.handle, d_pcm)
        lib.atg_device_free(eng.handle, d_hist)
    if return_hist:
        return res, peaks, gains, hist[:n_albums]
    return res, peaks, gains


def replaygain_hist_gain_host(hists):
    """analyzeResult of host uint32[n][12000] histograms on the GPU
    -> list of gains (NaN = not enough samples)"""
    lib = load_library()
    eng = engine()
    h = np.ascontiguousarray(np.atleast_2d(hists), dtype=np.uint32)
    n = h.shape[0]
    d = ctypes.c_void_p()
    _check(lib, lib.atg_device_alloc(eng.handle, max(4, h.nbytes), ctypes.byref(d)))
    try:
        _check(lib, lib.atg_copy_to_device(eng.handle, d, h.ctypes.data_as(ctypes.c_void_p),
                                           h.nbytes))
        return replaygain_hist_gain(d.value, n)
    finally:
        lib.atg_device_free(eng.handle, d)


def apply_gain(pcm, channels, bits_per_sample, multiplier, chunk_frames, dither,
               dither_bit0=0, device=None):
    """ReplayGainReader sample transform on the GPU (atg_pcm_apply_gain_host)"""
    lib = load_library()
    a = np.ascontiguousarray(pcm, dtype=np.int32)
    out = np.empty(max(1, len(a)), dtype=np.int32)
    d = np.frombuffer(bytes(dither) or b"\0", dtype=np.uint8)
    st = lib.atg_pcm_apply_gain_host(
        default_device() if device is None else device, a.ctypes.data_as(ctypes.c_void_p),
        out.ctypes.data_as(ctypes.c_void_p), len(a) // channels, channels, bits_per_sample,
        multiplier, chunk_frames, d.ctypes.data_as(ctypes.c_void_p), len(d), dither_bit0)
    if st != ATG_OK:
        raise ATGError(st, lib.atg_pcm_convert_last_error().decode("utf-8", "replace"))
    return out[:len(a)]


# ------------------------------------------------------------------ resampler
def _rs_check(lib, st):
    if st != ATG_OK:
        raise ATGError(st, lib.atg_resample_last_error().decode("utf-8", "replace"))


def resample_output_frames(in_frames, channels, in_rate, out_rate):
    return int(load_library().atg_resample_output_frames(in_frames, channels, in_rate, out_rate))


def resample_tracks(tracks, channels):
    """[(pcm_offset, pcm_frames, in_rate, out_rate[, reads])] -> RsTrack
    array (reads: the upstream read() frame counts, None = 4096-frame
    reads); the read arrays are kept alive on the returned object"""
    arr = (RsTrack * max(1, len(tracks)))()
    keep = []
    for i, t in enumerate(tracks):
        off, n, a, b = t[:4]
        arr[i].pcm_offset, arr[i].pcm_frames = off, n
        arr[i].in_rate, arr[i].out_rate = a, b
        reads = t[4] if len(t) > 4 else None
        if reads is not None:
            r = np.ascontiguousarray(reads, dtype=np.uint32)
            keep.append(r)
            arr[i].reads = r.ctypes.data_as(ctypes.POINTER(c_u32))
            arr[i].n_reads = len(r)
    arr._keep = keep
    return arr


def resample_device(d_in, d_out, out_cap_samples, tracks, channels, bits_per_sample,
                    stream=None):
    """resample a batch whose int32 PCM is in device memory
    -> (out frame offsets, out frame counts) numpy uint64"""
    lib = load_library()
    n = len(tracks)
    arr = resample_tracks(tracks, channels)
    offs = np.zeros(max(1, n), dtype=np.uint64)
    cnt = np.zeros(max(1, n), dtype=np.uint64)
    _rs_check(lib, lib.atg_resample_device(
        arr, n, channels, bits_per_sample, ctypes.c_void_p(d_in), ctypes.c_void_p(d_out),
        out_cap_samples, offs.ctypes.data_as(ctypes.c_void_p),
        cnt.ctypes.data_as(ctypes.c_void_p), stream))
    return offs[:n], cnt[:n]


def resample_host(pcm, tracks, channels, bits_per_sample, device=None):
    """resample int32 interleaved PCM held in host memory (atg_resample_host)
    -> (int32 output, out frame offsets, out frame counts)"""
    lib = load_library()
    a = np.ascontiguousarray(pcm, dtype=np.int32)
    n = len(tracks)
    total = 0
    for t in tracks:
        if len(t) > 4 and t[4] is not None:
            total += sum(resample_read_sizes(t[1], channels, t[2], t[3], t[4]))
        else:
            total += resample_output_frames(t[1], channels, t[2], t[3])
    out = np.empty(max(1, total * channels), dtype=np.int32)
    offs = np.zeros(max(1, n), dtype=np.uint64)
    cnt = np.zeros(max(1, n), dtype=np.uint64)
    _rs_check(lib, lib.atg_resample_host(
        default_device() if device is None else device, resample_tracks(tracks, channels), n,
        channels, bits_per_sample, a.ctypes.data_as(ctypes.c_void_p), len(a),
        out.ctypes.data_as(ctypes.c_void_p), total * channels,
        offs.ctypes.data_as(ctypes.c_void_p), cnt.ctypes.data_as(ctypes.c_void_p)))
    return out[:total * channels], offs[:n], cnt[:n]


def resample_read_sizes(in_frames, channels, in_rate, out_rate, reads):
    """frame counts of successive Resampler.read() calls (the last is 0)"""
    lib = load_library()
    r = np.ascontiguousarray(reads, dtype=np.uint32)
    cap = len(r) + 16
    while True:
        sizes = np.zeros(cap, dtype=np.uint32)
        k = lib.atg_resample_read_sizes(in_frames, channels, in_rate, out_rate,
                                        r.ctypes.data_as(ctypes.c_void_p), len(r),
                                        sizes.ctypes.data_as(ctypes.c_void_p), cap)
        if k < 0:
            raise ValueError("invalid sample rate")
        if k <= cap:
            return [int(x) for x in sizes[:k]]
        cap = int(k)


def resample_kernel_times():
    lib = load_library()
    names = (ctypes.c_char_p * 4)()
    ms = (ctypes.c_float * 4)()
    k = lib.atg_resample_kernel_times(names, ms, 4)
    return {names[i].decode(): float(ms[i]) for i in range(k)}
