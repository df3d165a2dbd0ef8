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

#define ATG_ABI_VERSION 4

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
   1..65535 (frames above 4096 samples take the large-frame kernels). */
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
/* flags for atg_engine_create_ex */
#define ATG_ENGINE_STREAMING 1u /* streams on first use: a process that only
                                   encodes one track at a time through
                                   atg_flac_encode_frames (encode_flac, one
                                   process per track under track2track -j N)
                                   then holds two HIP streams, so many such
                                   processes fit the device's hardware queues */
/* Where a device batch's STREAMINFO MD5 is computed.  By default the engine
   picks per batch: one GPU hash chain per track (md5.hip) unless the tracks
   are few and long enough that host cores hash the PCM sooner than the
   longest serial chain ends (config 5: 64 tracks x 8.6 MB of 24-bit 5.1 PCM
   -- the PCM goes to pinned host memory and host threads hash it beside the
   next batch's GPU work).  These flags force one side (the images are the
   same bytes either way). */
#define ATG_ENGINE_MD5_GPU 2u
#define ATG_ENGINE_MD5_HOST 4u
/* atg_engine_create with flags.  Without ATG_ENGINE_STREAMING every stream
   is created at once in a fixed order (the batch APIs' queue layout). */
atg_status atg_engine_create_ex(int device, uint32_t flags, atg_engine **out);
void atg_engine_destroy(atg_engine *eng);

/* Device choice for callers that do not name one (the drop-in entry points:
   encode_flac, FlacDecoder, the process-wide engines), host code only, no
   HIP call.  atg_pick_device: ATG_DEVICE, else LOCAL_RANK, else the next
   visible device of a node-wide round robin (a flock'ed counter in
   /dev/shm, per user; ATG_RR_FILE names another file), so the reference's
   one-process-per-track conversions (audiotools/__init__.py:5263-5529)
   spread over the node's GPUs.  Decided once per process (again after a
   fork).  atg_visible_devices: the entries of HIP_VISIBLE_DEVICES /
   CUDA_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES, else the GPU nodes of the KFD
   topology (ATG_DEVICE_COUNT overrides, for tests); at least 1. */
int atg_pick_device(void);
int atg_visible_devices(void);

/* Number of FLAC frames and worst-case output bytes of a batch, so callers
   can size outputs (the reference's recorders grow on demand; a batch
   engine needs bounds up front). */
atg_status atg_flac_batch_bounds(const atg_flac_options *opts,
                                 const atg_track *tracks, uint32_t n_tracks,
                                 uint32_t channels, uint32_t bits_per_sample,
                                 uint64_t *total_frames, uint64_t *out_bytes);

/* Encode a batch whose PCM and output live in host memory.
   pcm: interleaved samples in `format`; out: out_cap bytes (>= the
   atg_flac_batch_bounds size); results: n_tracks entries; frame_offsets /
   frame_pcm_frames: total_frames entries each (may be NULL).  Each track's
   image starts at results[t].out_offset; the images are packed back to back
   (16-byte aligned) from out on.  The batch runs as a pipeline of chunks of
   consecutive tracks (atg_engine_set_host_chunk_bytes), three in flight:
   chunk c+1's upload, chunk c's encode and chunk c-1's download overlap.
   Page-locked buffers (atg_host_alloc, hipHostMalloc, hipHostRegister) are
   copied by DMA directly; pageable ones through pinned staging. */
atg_status atg_flac_encode_host(atg_engine *eng, const atg_flac_options *opts,
                                const void *pcm, atg_pcm_format format,
                                const atg_track *tracks, uint32_t n_tracks,
                                uint32_t channels, uint32_t bits_per_sample,
                                uint32_t sample_rate, uint8_t *out,
                                uint64_t out_cap, atg_track_result *results,
                                uint64_t *frame_offsets,
                                uint32_t *frame_pcm_frames);

/* Asynchronous form of atg_flac_encode_host: plans the job, queues its
   chunks on the pipeline (collecting older chunks, of this or earlier jobs,
   as stages free up) and returns a ticket; pcm, out, results and the frame
   arrays must stay valid until atg_flac_encode_host_wait(ticket).  Jobs
   share the pipeline in submission order, so job k+1's uploads overlap job
   k's last chunks: back to back, the PCIe link stays busy.  Fails with
   ATG_ERR_INVALID while an atg_flac_encode_device_async batch is unwaited
   (and that call fails while a host job is in flight). */
atg_status atg_flac_encode_host_async(atg_engine *eng, const atg_flac_options *opts,
                                      const void *pcm, atg_pcm_format format,
                                      const atg_track *tracks, uint32_t n_tracks,
                                      uint32_t channels, uint32_t bits_per_sample,
                                      uint32_t sample_rate, uint8_t *out, uint64_t out_cap,
                                      atg_track_result *results, uint64_t *frame_offsets,
                                      uint32_t *frame_pcm_frames, uint64_t *ticket);
/* Wait for host job `ticket` (and the jobs before it); its results and
   images are then complete.  A job's ticket can be waited once. */
atg_status atg_flac_encode_host_wait(atg_engine *eng, uint64_t ticket);

/* Streaming form for ONE track (the reference's frame loop,
   src/encoders/flac.c:244-274, run over bounded segments of a long track):
   encodes pcm_frames PCM frames (host memory, cut into block_size frames or
   the explicit frame_sizes, as atg_track) as FLAC frames only -- no stream
   header, no MD5 -- numbered from first_frame_number (the frame header's
   UTF-8 frame number, flac.c:1531-1566).  The frames land back to back at
   out (*out_bytes in total, frame_bytes[i] each; out_cap >=
   atg_flac_max_frames_bytes).  The caller hashes the PCM (a serial MD5
   chain per track runs faster on a host core than on one GPU lane) and
   writes the stream header with atg_flac_stream_header before the first
   segment and again, with the final STREAMINFO, at the end (the reference
   rewrites STREAMINFO once the frames are written, flac.c:276-279). */
atg_status atg_flac_encode_frames(atg_engine *eng, const atg_flac_options *opts,
                                  const void *pcm, atg_pcm_format format, uint64_t pcm_frames,
                                  const uint32_t *frame_sizes, uint64_t n_frame_sizes,
                                  uint32_t channels, uint32_t bits_per_sample,
                                  uint32_t sample_rate, uint64_t first_frame_number,
                                  uint8_t *out, uint64_t out_cap, uint64_t *out_bytes,
                                  uint32_t *frame_bytes);
/* One segment of atg_flac_encode_frames_batch: PCM frames
   [pcm_offset, pcm_offset + pcm_frames) of the batch buffer, cut as
   atg_track, numbered from first_frame_number. */
typedef struct {
    uint64_t pcm_offset;
    uint64_t pcm_frames;
    const uint32_t *frame_sizes; /* NULL: block_size frames + a short last one */
    uint64_t n_frame_sizes;
    uint64_t first_frame_number;
} atg_segment;

/* atg_flac_encode_frames for many segments (of many tracks, from many
   callers) in one GPU pass: what the encoder service (atgpu-encoderd)
   runs for the encode_flac calls of concurrent processes.  Segments share
   the options and the PCM format.  Segment k's frames land at
   out + seg_offsets[k] (seg_bytes[k] bytes; offsets 16-byte aligned, packed
   in segment order; out_cap >= the sum of atg_flac_max_frames_bytes rounded
   up to 16 each); frame_bytes (may be NULL) receives every frame's size in
   segment order.  The engine's results of earlier batches are gone. */
atg_status atg_flac_encode_frames_batch(atg_engine *eng, const atg_flac_options *opts,
                                        const void *pcm, atg_pcm_format format,
                                        const atg_segment *segs, uint32_t n_segs,
                                        uint32_t channels, uint32_t bits_per_sample,
                                        uint32_t sample_rate, uint8_t *out, uint64_t out_cap,
                                        uint64_t *seg_offsets, uint64_t *seg_bytes,
                                        uint32_t *frame_bytes);
/* worst-case bytes of atg_flac_encode_frames' output (0: invalid options) */
uint64_t atg_flac_max_frames_bytes(const atg_flac_options *opts, uint64_t pcm_frames,
                                   const uint32_t *frame_sizes, uint64_t n_frame_sizes,
                                   uint32_t channels, uint32_t bits_per_sample);
/* fLaC + STREAMINFO (fields clamped as flacenc_write_streaminfo,
   flac.c:376-409) + VORBIS_COMMENT (vendor string) + PADDING of
   opts->padding_size bytes (flac.c:208-238), host-side; returns the header
   size, or 0 when cap is too small or an argument is invalid. */
uint64_t atg_flac_stream_header(const atg_flac_options *opts, uint32_t channels,
                                uint32_t bits_per_sample, uint32_t sample_rate,
                                uint64_t total_samples, uint32_t min_frame_bytes,
                                uint32_t max_frame_bytes, const uint8_t *md5, uint8_t *out,
                                uint64_t cap);

/* ------------------------------------------------------------------ */
/* Encoder service.  track2track converts every track in a fresh process */
/* (reference audiotools/__init__.py:5494-5521), and a process that      */
/* brings up its own HIP context, engine and code objects pays ~0.3-0.5 s */
/* for it.  atgpu-encoderd (beside libatgpu.so) owns one engine per GPU  */
/* and encodes the segments of every client process, batching concurrent */
/* clients' segments that share options and format into one GPU pass     */
/* (atg_flac_encode_frames_batch).  The streaming encode_flac uses it.   */
/* ------------------------------------------------------------------ */
typedef struct atg_service atg_service;
/* Connect to `device`'s service; with spawn != 0 start atgpu-encoderd when
   none listens (never from a process that has opened the GPU itself: it may
   not exec another program).  The service exits after an idle period. */
atg_status atg_service_connect(int device, int spawn, atg_service **out);
void atg_service_close(atg_service *svc);
const char *atg_service_last_error(void);
/* atg_flac_encode_frames' contract, encoded by the service */
atg_status atg_service_encode_frames(atg_service *svc, const atg_flac_options *opts,
                                     const void *pcm, atg_pcm_format format,
                                     uint64_t pcm_frames, const uint32_t *frame_sizes,
                                     uint64_t n_frame_sizes, uint32_t channels,
                                     uint32_t bits_per_sample, uint32_t sample_rate,
                                     uint64_t first_frame_number, uint8_t *out,
                                     uint64_t out_cap, uint64_t *out_bytes,
                                     uint32_t *frame_bytes);

/* PCM bytes per chunk of atg_flac_encode_host's pipeline (default 512 MiB):
   consecutive tracks are grouped into chunks of about this much PCM, and
   chunk c+1's upload, chunk c's encode and chunk c-1's download overlap. */
atg_status atg_engine_set_host_chunk_bytes(atg_engine *eng, uint64_t bytes);

/* Batches atg_flac_encode_device_async keeps in flight (slots in rotation,
   each its own device workspace, ~2 KB of tables per frame of the batch):
   3 .. 32, or 0 = automatic (the default).  Every track's MD5 is one serial
   hash (~12.5 ms per MiB of track on the GPU, whatever the batch width), so
   a narrow batch -- a rank's share of a strong-scaling job -- needs more
   batches in flight to keep the chains off its step.  From 4 on, the chains
   of all batches in flight advance together, one launch per enqueue on one
   stream, each batch's chain in n - 2 slices.  Automatic: the first device
   batch enqueued while nothing is in flight sets the depth from the ratio of
   its longest track's MD5 chain to its kernel time (12, 24 or 32; 3 when
   the chains are short or hashed on the host), and a host job sets it back
   to 3.  Lowering the depth frees the workspaces of the slots beyond it.
   Fails with ATG_ERR_INVALID while any batch or host job is unwaited. */
atg_status atg_engine_set_inflight(atg_engine *eng, uint32_t n);
/* The current depth D (the slots in rotation): a pipelined caller keeps up
   to D batches in flight and waits the oldest before enqueueing the next.
   With the automatic depth, read it after the pipeline's first enqueue. */
uint32_t atg_engine_inflight(atg_engine *eng);

/* Device-memory entry points run on the library's own non-blocking HIP
   streams: device inputs must be complete (e.g. the producing stream
   synchronized) when the call is made. */

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

/* The same batch encode, enqueued: returns once the work is queued, with a
   ticket for atg_flac_encode_wait.  The engine keeps D batches in flight
   (atg_engine_inflight: automatic unless atg_engine_set_inflight fixed it;
   each its own device workspace): batch k's MD5 chains and stream headers run on their own
   stream while batches k+1 .. k+D-1 are analysed, so a caller that waits
   for ticket k after enqueueing k+D-1 overlaps them.  d_pcm and d_out must
   stay untouched until the ticket is waited.  Enqueue number D+1 while D
   tickets are unwaited fails with ATG_ERR_INVALID (wait the oldest first);
   atg_flac_encode_device takes a slot too and fails the same way, and
   atg_flac_encode_host fails while any ticket is unwaited.  A waited
   ticket's results stay readable until its slot is reused D enqueues later, or
   until a streaming call (atg_flac_encode_frames[_batch]), which always
   takes slot 0. */
atg_status atg_flac_encode_device_async(atg_engine *eng, const atg_flac_options *opts,
                                        const void *d_pcm, atg_pcm_format format,
                                        const atg_track *tracks, uint32_t n_tracks,
                                        uint32_t channels, uint32_t bits_per_sample,
                                        uint32_t sample_rate, void *d_out, uint64_t out_cap,
                                        uint64_t *ticket);
/* wait for the batch of `ticket`; results as atg_flac_encode_device's */
atg_status atg_flac_encode_wait(atg_engine *eng, uint64_t ticket, atg_track_result *results);

/* Per-kernel device time of the engine's most recent encode, measured with
   HIP events recorded on the stream each kernel ran on.  names/ms arrays of
   capacity `cap`; returns the number of entries written. */
int atg_engine_kernel_times(atg_engine *eng, const char **names, float *ms, int cap);

/* Page-locked host memory: PCM and output buffers the host pipeline moves
   by DMA without staging (SURVEY 8(d)'s timer starts from pinned PCM). */
atg_status atg_host_alloc(uint64_t bytes, void **ptr);
void atg_host_free(void *ptr);

/* Device-memory helpers so callers without a GPU framework can stage data. */
atg_status atg_device_alloc(atg_engine *eng, uint64_t bytes, void **d_ptr);
atg_status atg_device_free(atg_engine *eng, void *d_ptr);
atg_status atg_copy_to_device(atg_engine *eng, void *d_dst, const void *src,
                              uint64_t bytes);
atg_status atg_copy_device(atg_engine *eng, void *d_dst, const void *d_src, uint64_t bytes);
/* Host-side gather: n host buffers (srcs[i], bytes[i]) copied back to back
   into dst on `threads` host threads (0 = the library's default, at most
   16) -- the reads of a batch of PCMReaders laid out in a (pinned) staging
   buffer in one call at memory bandwidth. */
atg_status atg_host_gather(void *dst, const void *const *srcs, const uint64_t *bytes,
                           uint64_t n, uint32_t threads);
atg_status atg_copy_to_host(atg_engine *eng, void *dst, const void *d_src,
                            uint64_t bytes);

/* ------------------------------------------------------------------ */
/* FLAC decoder (trackverify / FlacDecoder path).                     */
/* Replaces the body of the reference's audiotools.decoders.FlacDecoder */
/* (src/decoders/flac.c:28-98 init + flacdec_read_metadata :568-707,   */
/* read() :174-285 with its frame/subframe/residual readers :710-1269, */
/* offsets() :365-443, MD5 verify :446-493) for a batch of images.      */
/* ------------------------------------------------------------------ */

/* Decode status per track: the reference's flac_status values
   (src/decoders/flac.h:68-81) plus what read() raises itself. */
enum {
    ATG_FD_OK = 0, ATG_FD_ERROR = 1, ATG_FD_SYNC = 2, ATG_FD_RESERVED = 3,
    ATG_FD_BPS = 4, ATG_FD_RATE = 5, ATG_FD_HDR_CRC = 6,
    ATG_FD_RATE_MISMATCH = 7, ATG_FD_CH_MISMATCH = 8, ATG_FD_BPS_MISMATCH = 9,
    ATG_FD_MAXBS = 10, ATG_FD_CODING = 11, ATG_FD_FIXED_ORDER = 12,
    ATG_FD_SUBFRAME_TYPE = 13,
    ATG_FD_FRAME_CRC = 14, /* "invalid checksum in frame" (flac.c:251-255) */
    ATG_FD_EOF = 15,       /* IOError "EOF reading frame" (flac.c:259-264) */
    ATG_FD_MD5 = 16        /* "MD5 mismatch at end of stream" (:199-207) */
};

/* STREAMINFO and the parts of the other metadata blocks the reference
   decoder keeps (struct flac_STREAMINFO, src/decoders/flac.h:37-48). */
typedef struct {
    uint32_t min_block_size, max_block_size, min_frame_size, max_frame_size;
    uint32_t sample_rate, channels, bits_per_sample, channel_mask;
    uint64_t total_samples;
    uint8_t md5[16];
    uint64_t frames_offset; /* bytes from the image start to the first frame */
    uint32_t n_seekpoints;
    uint32_t reserved;
} atg_flac_streaminfo;

typedef struct {
    uint64_t sample_number, byte_offset;
    uint32_t samples, reserved;
} atg_flac_seekpoint;

/* flacdec_read_metadata (src/decoders/flac.c:568-707) over an in-memory
   image.  Returns 0 ok, 1 not a FLAC stream (ValueError), 2 EOF (IOError).
   Up to sp_cap SEEKTABLE points are stored into sp (may be NULL). */
int atg_flac_read_metadata(const uint8_t *data, uint64_t len, atg_flac_streaminfo *si,
                           atg_flac_seekpoint *sp, uint32_t sp_cap);

/* One stream of a decode batch: its frames occupy
   data[data_offset, data_offset + data_bytes) (data_offset = image start +
   frames_offset); the remaining fields are its STREAMINFO. */
typedef struct {
    uint64_t data_offset;
    uint64_t data_bytes;
    uint64_t total_samples;
    uint32_t sample_rate, channels, bits_per_sample, max_block_size;
    uint8_t md5[16];
} atg_flac_dec_track;

/* Per-track decode result.
   read() view (src/decoders/flac.c:174-285): the stream hands out n_frames
   FLAC frames = pcm_frames PCM frames (interleaved int32, FrameList layout,
   at PCM-frame index pcm_offset of the batch output) and then raises
   `status` (0 = end of stream with the MD5 verified); md5 = MD5 of those
   frames' little-endian PCM bytes.
   offsets() view (flac.c:365-443, which never checks CRC-16): walk_frames
   frames are walked (frame arrays first_frame .. first_frame+walk_frames-1,
   decoded PCM continuing after pcm_frames) before walk_status stops it.
   The two differ only when a frame fails its CRC-16.  walk_end = the byte
   (from the track's first frame) where the walk stopped: the frame that
   stopped it, or the end of the last frame once remaining reached 0 -- a
   streaming caller resumes a window there. */
typedef struct {
    uint64_t pcm_offset;
    uint64_t pcm_frames;
    uint32_t first_frame;
    uint32_t n_frames;
    int32_t status;
    uint32_t walk_frames;
    uint8_t md5[16];
    int32_t walk_status;
    uint32_t reserved;
    uint64_t walk_end;
} atg_flac_dec_result;

typedef struct atg_decoder atg_decoder;

atg_status atg_decoder_create(int device, atg_decoder **out);
void atg_decoder_destroy(atg_decoder *dec);
const char *atg_decoder_last_error(void);

/* Decode a batch held in host memory; the PCM stays in the decoder until
   atg_flac_decode_fetch.  total_samples = interleaved samples of the batch
   output, total_frames = FLAC frames decoded. */
atg_status atg_flac_decode_host(atg_decoder *dec, const uint8_t *data, uint64_t len,
                                const atg_flac_dec_track *tracks, uint32_t n_tracks,
                                atg_flac_dec_result *results, uint64_t *total_samples,
                                uint64_t *total_frames);

/* Copy the last decode's PCM (pcm_cap int32 samples) and, per FLAC frame,
   its byte offset from the track's first frame and its header block size
   (what FlacDecoder.offsets() reports, flac.c:365-443).  Any may be NULL. */
atg_status atg_flac_decode_fetch(atg_decoder *dec, int32_t *pcm, uint64_t pcm_cap,
                                 uint64_t *frame_offsets, uint32_t *frame_block_sizes,
                                 uint64_t frame_cap);

/* Decode a batch already in device memory (4-byte aligned, readable up to
   len rounded up to 4).  *d_pcm receives the decoder-owned device PCM
   (valid until the call after next). */
atg_status atg_flac_decode_device(atg_decoder *dec, const void *d_data, uint64_t len,
                                  const atg_flac_dec_track *tracks, uint32_t n_tracks,
                                  atg_flac_dec_result *results, const int32_t **d_pcm,
                                  uint64_t *total_samples);

/* Decode batches atg_flac_decode_device_async keeps in flight: 3 (default)
   .. 16.  A batch's STREAMINFO MD5 checks are serial hashes (~12 ms per 1 MB
   of decoded PCM whatever the batch width); from 4 on, the hashes of every
   batch in flight advance together, one launch per enqueue on one stream,
   each batch's in n - 2 slices.  Each slot holds its batch's PCM, restore
   scratch and MD5 byte image (~5 GB for a 1024-track config-2 batch);
   lowering the depth frees the slots past it.  Fails while a batch is
   unwaited; the last waited batch's buffers are no longer fetchable
   afterwards. */
atg_status atg_decoder_set_inflight(atg_decoder *dec, uint32_t n);

/* The parse's frame-end hypothesis (flac_decode.hip k_dec_spec): 1 (default)
   takes a frame's end from the next frame-header candidate whose bytes give
   a zero CRC-16 residue, so the parse does not walk the frame's last
   subframe; the restore checks every such frame on the subframe it walks
   anyway, and a batch with a failed check is redone with every subframe
   walked inside atg_flac_decode_wait -- results are those of the full parse
   (src/decoders/flac.c:174-285) either way; after four redone batches in a
   row the decoder switches itself to 0 (a stream of input the hypothesis
   keeps failing on would pay two decodes per batch) until the mode is set
   again.  0: every subframe walked by the parse.  2: as 1, and every batch
   redone (self-check of the redo path). */
atg_status atg_decoder_set_frame_hypothesis(atg_decoder *dec, int mode);

/* Batches this decoder redid with the full parse (mode 1: failed checks). */
uint64_t atg_decoder_frame_hypothesis_redos(atg_decoder *dec);

/* Asynchronous form of atg_flac_decode_device, D batches in flight (D = 3
   unless atg_decoder_set_inflight says otherwise, each slot with its own
   buffers): the scan, parse and frame walk run on the decoder's stream
   (two host round trips for the counts), then the restore, emit and
   per-track MD5 on the batch's slot stream, so batch k's back half runs
   under batch k+1's scan and parse.  Returns once everything is queued.
   d_data must stay valid and unchanged until the batch is waited: when a
   frame-end hypothesis fails its check, atg_flac_decode_wait re-reads
   d_data to redo the batch with the full parse.  The PCM pointer the wait
   returns stays valid until the slot is reused, D enqueues later.  An
   enqueue while D batches are unwaited fails with ATG_ERR_INVALID; an
   enqueue that fails leaves nothing of its batch queued. */
atg_status atg_flac_decode_device_async(atg_decoder *dec, const void *d_data, uint64_t len,
                                        const atg_flac_dec_track *tracks, uint32_t n_tracks,
                                        uint64_t *ticket);
atg_status atg_flac_decode_wait(atg_decoder *dec, uint64_t ticket,
                                atg_flac_dec_result *results, const int32_t **d_pcm,
                                uint64_t *total_samples);

/* Per-kernel device time of the decoder's most recently waited batch. */
int atg_decoder_kernel_times(atg_decoder *dec, const char **names, float *ms, int cap);

/* ------------------------------------------------------------------ */
/* Integer PCM converters (track2track --bits-per-sample / --channels). */
/* Replace the read() bodies of the reference's pcmconverter types:     */
/* BPSConverter (src/pcmconverter.c:667-747, dither src/dither.c:73-89),*/
/* Downmixer (:220-342) and Averager (:64-97), over whole tracks.       */
/* PCM is interleaved int32 (FrameList layout) in and out.              */
/* ------------------------------------------------------------------ */
enum {
    ATG_CONV_BPS = 0,     /* in_bps -> out_bps; dither bits when reducing */
    ATG_CONV_DOWNMIX = 1, /* -> 2 channels (channel_mask 0 = invented mask) */
    ATG_CONV_AVERAGE = 2  /* -> 1 channel */
};

const char *atg_pcm_convert_last_error(void);
uint32_t atg_pcm_convert_out_channels(int kind, uint32_t in_channels);

/* Device buffers; `stream` is a hipStream_t (NULL = default stream); the
   call returns after the launch.  Reducing bits reads one dither bit per
   sample from d_dither, starting at bit dither_bit0, MSB first, in the
   reference's order: per 4096-frame read(), channel by channel. */
atg_status atg_pcm_convert_device(int kind, const int32_t *d_in, int32_t *d_out,
                                  uint64_t frames, uint32_t channels, uint32_t channel_mask,
                                  uint32_t in_bps, uint32_t out_bps, const uint8_t *d_dither,
                                  uint64_t dither_bit0, void *stream);

/* Host buffers (staged through the device); out holds
   frames x atg_pcm_convert_out_channels() samples. */
atg_status atg_pcm_convert_host(int device, int kind, const int32_t *in, int32_t *out,
                                uint64_t frames, uint32_t channels, uint32_t channel_mask,
                                uint32_t in_bps, uint32_t out_bps, const uint8_t *dither,
                                uint64_t dither_bytes, uint64_t dither_bit0);

/* ------------------------------------------------------------------ */
/* ReplayGain analysis (tracktag/track2track --replay-gain).           */
/* Replaces ReplayGain(rate).title_gain(pcmreader) for every track of a */
/* batch and album_gain() per album (src/replaygain.c:115-322,         */
/* :566-807).  PCM is interleaved int32 (FrameList layout), 1 or 2      */
/* channels, 8/16/24 bits, one of the 20 supported sample rates.        */
/* ------------------------------------------------------------------ */
typedef struct {
    uint64_t pcm_offset; /* first PCM frame of the track in d_pcm */
    uint64_t pcm_frames;
    uint32_t channels, bits_per_sample, sample_rate;
    uint32_t album;      /* album index (tracks grouped by album) */
    /* host array: the frame counts pcmreader.read(4096) returned, one
       ReplayGain_analyze_samples call each (replaygain.c:210-305); they
       decide the fp64 summation order.  NULL = 4096-frame reads. */
    const uint32_t *chunk_frames;
    uint64_t n_chunks;
} atg_rg_track;

typedef struct {
    double title_gain;   /* dB; 0.0 when no 50 ms window completed */
    double title_peak;   /* max |x| / 2^(bps-1) */
    int32_t status;      /* 0 ok, 1 not enough samples */
    uint32_t reserved;
} atg_rg_result;

const char *atg_replaygain_last_error(void);

/* Title gains/peaks of all tracks; when n_albums > 0 also each album's
   12000-bin window histogram (the reference's B array) into d_album_hist
   (device, n_albums x 12000 uint32; NULL = internal) and album peaks into
   album_peaks (host, may be NULL).  Album gains follow from
   atg_replaygain_hist_gain -- after an RCCL all-reduce of the histograms
   when an album spans several GPUs. */
atg_status atg_replaygain_device(const int32_t *d_pcm, const atg_rg_track *tracks,
                                 uint32_t n_tracks, uint32_t n_albums, atg_rg_result *results,
                                 uint32_t *d_album_hist, double *album_peaks, void *stream);

/* The certification bound of the time-split title analysis for one sample
   rate (host computation, no GPU), out[6]: out[0] G = max over lags of the
   Butterworth output's l1 response to a unit error state, out[1] R_s and
   out[2] R_b the rounding sums into the state and the output, out[3]
   1 / (1 - ||A^L||_inf), out[4] L the segment length in frames, out[5] G_L
   = max over lags >= L (see replaygain.hip k_rg_seg).  A warm segment's
   outputs err by at most G m + G_L (m + R_s) out[3] + 1.5 R_b for the
   largest measured seam state difference m. */
atg_status atg_replaygain_bound(uint32_t sample_rate, double *out);
/* The multiple of R_b the kernels use in that bound: 1.5 -- R_b is two
   trajectories' rounding, and the bound counts three trajectories once
   each (warm, predecessor, and the serial one at disjoint times; the
   derivation is in replaygain.hip). */
double atg_replaygain_rb_factor(void);
/* windows whose histogram bin the host's log10 moved (lifetime count; a
   window within 1e-9 of a bin edge is binned with the C library's log10) */
uint64_t atg_replaygain_rebinned_windows(void);
/* Test hooks of the time-split analysis (replaygain.hip): the warm-up
   frames of every segment after a track's first (-1 = the rate-scaled
   default; 0 = none, so every track fails certification and is analysed
   again serially), and how many tracks the last atg_replaygain_device call
   analysed again serially. */
void atg_replaygain_set_warmup(int frames);
uint32_t atg_replaygain_fallback_tracks(void);

/* analyzeResult (replaygain.c:754-776) of n device histograms -> gains
   (host); NaN = not enough samples (album_gain raises ValueError). */
atg_status atg_replaygain_hist_gain(const uint32_t *d_hist, uint32_t n, double *gains,
                                    void *stream);

/* ReplayGainReader (src/replaygain.c:820-925): multiplier from (gain, peak)
   as ReplayGainReader_init computes it (long double pow; 1/peak when the
   gain would amplify), then per sample lround(x * multiplier), clamp to
   bits_per_sample, XOR one dither bit (consumed per read(chunk_frames)
   call, channel by channel, MSB first, starting at dither_bit0). */
double atg_replaygain_multiplier(double replaygain, double peak);
atg_status atg_pcm_apply_gain_device(const int32_t *d_in, int32_t *d_out, uint64_t frames,
                                     uint32_t channels, uint32_t bits_per_sample,
                                     double multiplier, uint32_t chunk_frames,
                                     const uint8_t *d_dither, uint64_t dither_bit0,
                                     void *stream);
atg_status atg_pcm_apply_gain_host(int device, const int32_t *in, int32_t *out,
                                   uint64_t frames, uint32_t channels,
                                   uint32_t bits_per_sample, double multiplier,
                                   uint32_t chunk_frames, const uint8_t *dither,
                                   uint64_t dither_bytes, uint64_t dither_bit0);

/* ------------------------------------------------------------------ */
/* ALAC encoder (E1-E7).  Replaces the body of the reference's          */
/* audiotools.encoders.encode_alac (src/encoders/alac.c:30-206:         */
/* ALACEncoder_encode_alac -> write_frameset / write_frame /            */
/* compute_coefficients / calculate_residuals / encode_residuals) for a */
/* batch of tracks; audiotools.m4a.ALACAudio.from_pcm wraps the mdat in */
/* the M4A atoms on the host.  Interlacing shift 2; leftweights        */
/* minimum..maximum_interlacing_leftweight (0..4 by default,            */
/* alac.c:57-72; 0 <= min <= max <= 255, others ATG_ERR_INVALID).       */
/* ------------------------------------------------------------------ */
typedef struct {
    uint32_t block_size;         /* PCM frames per frameset, 1..65535 */
    uint32_t initial_history;    /* encode_alac keyword arguments     */
    uint32_t history_multiplier;
    uint32_t maximum_k;
    uint32_t minimum_interlacing_leftweight;
    uint32_t maximum_interlacing_leftweight;
} atg_alac_options;

/* Per-track result: the mdat atom (32-bit size, "mdat", framesets) is
   `bytes` long at out + out_offset; frameset_bytes[first_frameset ..
   first_frameset + n_framesets) is the frame-size log encode_alac returns
   (alac.c:150-151, 1255-1290). */
typedef struct {
    uint64_t out_offset;
    uint64_t bytes;
    uint64_t pcm_frames;
    uint32_t first_frameset;
    uint32_t n_framesets;
    int32_t status;
    uint32_t reserved;
} atg_alac_track_result;

typedef struct atg_alac_encoder atg_alac_encoder;

const char *atg_alac_last_error(void);
atg_status atg_alac_encoder_create(int device, atg_alac_encoder **out);
void atg_alac_encoder_destroy(atg_alac_encoder *enc);
/* framesets and worst-case output bytes of a batch (tracks as for FLAC:
   block_size frames + a short last one, or explicit frame_sizes) */
atg_status atg_alac_batch_bounds(atg_alac_encoder *enc, const atg_alac_options *opts,
                                 const atg_track *tracks, uint32_t n_tracks, uint32_t channels,
                                 uint32_t bits_per_sample, uint64_t *total_framesets,
                                 uint64_t *out_bytes);
/* PCM and output in device memory (d_out 4-byte aligned, out_cap >= the
   bound); frameset_bytes (host, total_framesets entries) may be NULL */
atg_status atg_alac_encode_device(atg_alac_encoder *enc, const atg_alac_options *opts,
                                  const void *d_pcm, atg_pcm_format format,
                                  const atg_track *tracks, uint32_t n_tracks,
                                  uint32_t channels, uint32_t bits_per_sample, void *d_out,
                                  uint64_t out_cap, atg_alac_track_result *results,
                                  uint32_t *frameset_bytes);
/* the same for host buffers (staged through the device) */
atg_status atg_alac_encode_host(atg_alac_encoder *enc, const atg_alac_options *opts,
                                const void *pcm, atg_pcm_format format, const atg_track *tracks,
                                uint32_t n_tracks, uint32_t channels, uint32_t bits_per_sample,
                                uint8_t *out, uint64_t out_cap, atg_alac_track_result *results,
                                uint32_t *frameset_bytes);
int atg_alac_encoder_kernel_times(atg_alac_encoder *enc, const char **names, float *ms, int cap);

/* ------------------------------------------------------------------ */
/* ALAC decoder (D6).  Replaces the reference's                        */
/* audiotools.decoders.ALACDecoder (src/decoders/alac.c: init          */
/* :25-98 with parse_decoding_parameters :439-672 and seek_mdat        */
/* :953-971, read() :183-254, read_frame :818-951, read_residuals       */
/* :1017-1085, decode_subframe :1147-1235, decorrelate_channels         */
/* :1237-1259, alac_order_to_wave_order :709-816) for a batch of M4A    */
/* images.                                                             */
/* ------------------------------------------------------------------ */
/* status values: the reference's decoder status enum (decoders/alac.h)
   plus the conditions its Python methods raise */
enum {
    ATG_AD_OK = 0,
    ATG_AD_IO_ERROR = 1,           /* IOError ("I/O Errror" at init,
                                      "EOF during frame reading" in read) */
    ATG_AD_INVALID_UNUSED_BITS = 2,/* ValueError "invalid unused bits" */
    ATG_AD_INVALID_ALAC_ATOM = 3,
    ATG_AD_INVALID_MDHD_ATOM = 4,
    ATG_AD_MDIA_NOT_FOUND = 5,
    ATG_AD_STSD_NOT_FOUND = 6,
    ATG_AD_MDHD_NOT_FOUND = 7,
    ATG_AD_INVALID_SEEKTABLE = 8,
    ATG_AD_NO_MDAT = 9,            /* IOError "Unable to locate 'mdat' atom" */
    ATG_AD_CHANNEL_MISMATCH = 10   /* ValueError "channel length mismatch" */
};

/* the "alac" / "mdhd" fields the decoder keeps, and where "mdat" starts */
typedef struct {
    uint32_t max_samples_per_frame, bits_per_sample, history_multiplier, initial_history;
    uint32_t maximum_k, channels, sample_rate, total_frames;
    uint64_t mdat_offset;   /* byte (from the image start) of the first frameset */
    uint32_t n_seekpoints;  /* entries of the stts/stsc/stco seektable */
    uint32_t reserved;
} atg_alac_info;

typedef struct {
    uint64_t pcm_frames_offset, file_offset;
} atg_alac_seekpoint;

/* parse_decoding_parameters + seek_mdat over an in-memory image (host):
   returns an ATG_AD_* status.  Seekpoints (sp_cap) and the stsz frameset
   sizes (fs_cap, a decoding hint the reference does not read) are copied
   when the buffers are non-NULL. */
int atg_alac_read_info(const uint8_t *data, uint64_t len, atg_alac_info *info,
                       atg_alac_seekpoint *sp, uint32_t sp_cap, uint32_t *frame_sizes,
                       uint32_t fs_cap, uint32_t *n_frame_sizes);

/* One stream of a decode batch: the image at data[data_offset,
   data_offset + data_bytes) (4-byte aligned); reading starts at byte
   `start` of the image (the mdat offset, or a seekpoint's file offset) with
   remaining_frames = `remaining`.  frameset_bytes: the stsz sizes from
   `start` on (may be NULL: framesets are then found by the serial walk). */
typedef struct {
    uint64_t data_offset, data_bytes, start, remaining;
    uint32_t max_samples_per_frame, bits_per_sample, history_multiplier, initial_history;
    uint32_t maximum_k, channels;
    const uint32_t *frameset_bytes;
    uint64_t n_frameset_bytes;
} atg_alac_dec_track;

/* read() view: n_framesets framesets = pcm_frames PCM frames (interleaved
   int32 in wave channel order at sample index sample_offset of the batch
   output) are returned, then `status` ends the stream (0 = remaining_frames
   reached 0). */
typedef struct {
    uint64_t sample_offset;
    uint64_t pcm_frames;
    uint32_t first_frameset;
    uint32_t n_framesets;
    int32_t status;
    uint32_t channels;
} atg_alac_dec_result;

typedef struct atg_alac_decoder atg_alac_decoder;

const char *atg_alac_decoder_last_error(void);
atg_status atg_alac_decoder_create(int device, atg_alac_decoder **out);
void atg_alac_decoder_destroy(atg_alac_decoder *dec);
atg_status atg_alac_decode_host(atg_alac_decoder *dec, const uint8_t *data, uint64_t len,
                                const atg_alac_dec_track *tracks, uint32_t n_tracks,
                                atg_alac_dec_result *results, uint64_t *total_samples,
                                uint64_t *total_framesets);
/* the last decode's PCM and, per frameset, its PCM frames and its byte
   offset from the image start */
atg_status atg_alac_decode_fetch(atg_alac_decoder *dec, int32_t *pcm, uint64_t pcm_cap,
                                 uint32_t *frameset_frames, uint64_t *frameset_offsets,
                                 uint64_t fs_cap);
atg_status atg_alac_decode_device(atg_alac_decoder *dec, const void *d_data, uint64_t len,
                                  const atg_alac_dec_track *tracks, uint32_t n_tracks,
                                  atg_alac_dec_result *results, const int32_t **d_pcm,
                                  uint64_t *total_samples);
int atg_alac_decoder_kernel_times(atg_alac_decoder *dec, const char **names, float *ms,
                                  int cap);

/* ------------------------------------------------------------------ */
/* Sinc resampler (R1-R3, track2track --sample-rate).  Replaces the     */
/* reference's audiotools.pcmconverter.Resampler (src/pcmconverter.c    */
/* :370-495: src_new(SRC_SINC_BEST_QUALITY) + src_process per 4096-frame */
/* read, libsamplerate 0.1.8 src/samplerate/src_sinc.c) for whole       */
/* tracks.  Coefficients: the MEDIUM table (BEST's table is absent from */
/* the reference tree; parity is against oracle/resample_port.c).      */
/* PCM is interleaved int32 (FrameList layout), 1..8 channels, 1..24    */
/* bits, in and out (the output keeps bits_per_sample).                 */
/* ------------------------------------------------------------------ */
typedef struct {
    uint64_t pcm_offset;  /* first frame of the track in the input buffer */
    uint64_t pcm_frames;
    uint32_t in_rate, out_rate;
    /* frame counts the wrapped PCMReader's read(4096) calls returned (they
       sum to pcm_frames; NULL = 4096-frame reads).  They can move the end
       of the stream by one frame in rare ties (atg_resample_read_sizes). */
    const uint32_t *reads;
    uint64_t n_reads;
} atg_rs_track;

const char *atg_resample_last_error(void);
/* output frames of one track read in 4096-frame reads (the converter's
   termination rule) */
uint64_t atg_resample_output_frames(uint64_t in_frames, uint32_t channels, uint32_t in_rate,
                                    uint32_t out_rate);
/* Device buffers.  Track t's output is written at frame out_offsets[t]
   (host array, filled) of d_out, out_frames[t] frames; out_cap_samples
   >= the sum of atg_resample_output_frames() x channels.  Returns after
   the stream has drained. */
atg_status atg_resample_device(const atg_rs_track *tracks, uint32_t n, uint32_t channels,
                               uint32_t bits_per_sample, const int32_t *d_in, int32_t *d_out,
                               uint64_t out_cap_samples, uint64_t *out_offsets,
                               uint64_t *out_frames, void *stream);
/* Host buffers (staged through the device). */
atg_status atg_resample_host(int device, const atg_rs_track *tracks, uint32_t n,
                             uint32_t channels, uint32_t bits_per_sample, const int32_t *in,
                             uint64_t in_samples, int32_t *out, uint64_t out_cap_samples,
                             uint64_t *out_offsets, uint64_t *out_frames);
/* The frame counts successive Resampler.read() calls return (the last is
   the 0 that ends the stream), given the frame counts the wrapped reader's
   read(4096) calls returned (`reads`, its terminating 0 excluded).
   Returns the number of counts (written up to cap), or -1. */
int64_t atg_resample_read_sizes(uint64_t in_frames, uint32_t channels, uint32_t in_rate,
                                uint32_t out_rate, const uint32_t *reads, uint64_t n_reads,
                                uint32_t *sizes, uint64_t cap);
/* durations (ms) of the last atg_resample_device call's kernels on the
   calling thread's device: "rs_positions" (0 when every track had a closed
   form) and "rs_filter" */
int atg_resample_kernel_times(const char **names, float *ms, int cap);

#ifdef __cplusplus
}
#endif
#endif
