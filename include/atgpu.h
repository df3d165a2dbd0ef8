/*
 * atgpu.h — C ABI of libatgpu, the MI355X (gfx950) batch FLAC encoder.
 *
 * This is the drop-in boundary for python-audio-tools' FLAC encode hot path.
 * The reference binds the encoder through its CPython-2 extension
 * `audiotools.encoders.encode_flac` (reference src/encoders/flac.c:44-121,
 * registered at src/encoders.h:65-67); that function pulls PCM from a
 * PCMReader (src/pcmconv.c:207-329), encodes frame by frame
 * (src/encoders/flac.c:240-274) and returns [(byte_offset, pcm_frames)].
 * The entry points below replace the body of that function (and of the
 * frame loop) for a whole batch of tracks at once; the Python-visible
 * `encode_flac` in python-audio-tools_amd/audiotools/encoders.py keeps the
 * reference's signature and error behaviour and calls into this ABI.
 *
 * Plain C types only.  No exceptions cross the ABI: every entry point
 * returns an atg_status; atg_last_error() describes the most recent failure
 * on the calling thread.
 */
#ifndef ATGPU_H
#define ATGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ATG_ABI_VERSION 1

typedef enum {
    ATG_OK = 0,
    ATG_ERR_INVALID = -1,     /* bad argument (maps to ValueError) */
    ATG_ERR_UNSUPPORTED = -2, /* option combination not supported on GPU */
    ATG_ERR_DEVICE = -3,      /* HIP runtime failure */
    ATG_ERR_NOMEM = -4,       /* device or host allocation failed */
    ATG_ERR_CAPACITY = -5     /* caller output buffer too small */
} atg_status;

/* Encoder options: the keyword arguments of encode_flac
   (reference src/encoders/flac.c:52-67; struct flac_encoding_options,
   src/encoders/flac.h:30-55).  Derived options (QLP precision, maximum Rice
   parameter) are computed inside, as the reference does (flac.c:164-184). */
typedef struct {
    uint32_t block_size;
    uint32_t max_lpc_order;
    uint32_t min_residual_partition_order; /* accepted; unused, as reference */
    uint32_t max_residual_partition_order;
    int32_t mid_side;
    int32_t adaptive_mid_side;
    int32_t exhaustive_model_search;
    int32_t disable_verbatim_subframes;
    int32_t disable_constant_subframes;
    int32_t disable_fixed_subframes;
    int32_t disable_lpc_subframes;
    uint32_t padding_size;
} atg_flac_options;

/* PCM sample containers the engine reads. */
typedef enum {
    ATG_PCM_S16 = 0, /* interleaved int16 (bits_per_sample <= 16) */
    ATG_PCM_S32 = 1  /* interleaved int32 (any bits_per_sample <= 24), the
                        reference FrameList layout (src/pcm.h:40-54) */
} atg_pcm_format;

/* One track of a batch: a contiguous run of interleaved PCM frames.
   By default the track is cut into block_size frames plus a shorter last
   one (what BufferedPCMReader feeds the reference encoder,
   audiotools/__init__.py:2561-2606).  When frame_sizes is non-NULL the
   track is cut exactly as listed instead (the reference encodes whatever
   each pcmreader.read(block_size) call returns as one frame,
   src/encoders/flac.c:244-274); sizes must sum to pcm_frames and each be
   1..4096. */
typedef struct {
    uint64_t pcm_offset; /* index of the track's first PCM frame */
    uint64_t pcm_frames; /* number of PCM frames (samples per channel) */
    const uint32_t *frame_sizes; /* optional explicit frame lengths */
    uint64_t n_frame_sizes;
} atg_track;

/* Per-track result.  `bytes` is the length of the complete .flac image
   (stream marker, STREAMINFO, VORBIS_COMMENT, PADDING, frames) written at
   out + out_offset.  frame_offsets[] (caller array indexed by
   first_frame .. first_frame+n_frames-1) hold each frame's byte offset from
   the first frame, as encode_flac's return list does (flac.c:249-253). */
typedef struct {
    uint64_t out_offset;
    uint64_t bytes;
    uint32_t first_frame;
    uint32_t n_frames;
    uint32_t min_frame_bytes;
    uint32_t max_frame_bytes;
    uint8_t md5[16];
    int32_t status;
    uint32_t reserved;
} atg_track_result;

typedef struct atg_engine atg_engine;

/* Library / device management */
int atg_abi_version(void);
const char *atg_last_error(void);
atg_status atg_engine_create(int device, atg_engine **out);
void atg_engine_destroy(atg_engine *eng);

/* Number of FLAC frames and worst-case output bytes of a batch, so callers
   can size outputs (the reference's recorders grow on demand; a batch
   engine needs bounds up front). */
atg_status atg_flac_batch_bounds(const atg_flac_options *opts,
                                 const atg_track *tracks, uint32_t n_tracks,
                                 uint32_t channels, uint32_t bits_per_sample,
                                 uint64_t *total_frames, uint64_t *out_bytes);

/* Encode a batch whose PCM and output live in host memory.
   pcm: interleaved samples in `format`; out: out_cap bytes; results:
   n_tracks entries; frame_offsets / frame_pcm_frames: total_frames entries
   each (may be NULL).  Each track's image starts at results[t].out_offset. */
atg_status atg_flac_encode_host(atg_engine *eng, const atg_flac_options *opts,
                                const void *pcm, atg_pcm_format format,
                                const atg_track *tracks, uint32_t n_tracks,
                                uint32_t channels, uint32_t bits_per_sample,
                                uint32_t sample_rate, uint8_t *out,
                                uint64_t out_cap, atg_track_result *results,
                                uint64_t *frame_offsets,
                                uint32_t *frame_pcm_frames);

/* Encode a batch whose PCM already lives in device memory (HBM) and leave
   the .flac images in device memory at d_out (out_cap bytes).  Results are
   copied back to host `results` (small).  Runs on the engine's streams and
   returns when the images are complete. */
atg_status atg_flac_encode_device(atg_engine *eng, const atg_flac_options *opts,
                                  const void *d_pcm, atg_pcm_format format,
                                  const atg_track *tracks, uint32_t n_tracks,
                                  uint32_t channels, uint32_t bits_per_sample,
                                  uint32_t sample_rate, void *d_out,
                                  uint64_t out_cap, atg_track_result *results);

/* Per-kernel device time of the engine's most recent encode, measured with
   HIP events recorded on the stream each kernel ran on.  names/ms arrays of
   capacity `cap`; returns the number of entries written. */
int atg_engine_kernel_times(atg_engine *eng, const char **names, float *ms, int cap);

/* Device-memory helpers so callers without a GPU framework can stage data. */
atg_status atg_device_alloc(atg_engine *eng, uint64_t bytes, void **d_ptr);
atg_status atg_device_free(atg_engine *eng, void *d_ptr);
atg_status atg_copy_to_device(atg_engine *eng, void *d_dst, const void *src,
                              uint64_t bytes);
atg_status atg_copy_to_host(atg_engine *eng, void *dst, const void *d_src,
                            uint64_t bytes);

#ifdef __cplusplus
}
#endif
#endif
