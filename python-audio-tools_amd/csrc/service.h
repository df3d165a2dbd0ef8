// service.h — wire format of the encoder service (atgpu-encoderd).
//
// track2track runs every conversion in a fresh process (ExecProgressQueue,
// reference audiotools/__init__.py:5494-5521).  With the encoder in each
// process, every track pays HIP init, engine creation and code-object
// loading (~0.3-0.5 s measured, against ~0.06 s for the reference encoder
// per 64-frame track), so encode_flac instead hands its segments
// to one process per GPU that owns the engine: atgpu-encoderd, reached over
// an abstract Unix socket, started on first use by whichever encoder
// process finds none, and gone after an idle period.  It encodes the
// segments of all waiting callers that share a format in one GPU batch
// (atg_flac_encode_frames_batch).
//
// Both sides are on one host and built together: native-endian structs.
#pragma once
#include <stdint.h>

#include "../../include/atgpu.h"

#define ATG_SVC_MAGIC 0x45475441u /* "ATGE" */
#define ATG_SVC_VERSION 1u
// bounds a request may not exceed (a malformed one is refused, not trusted)
#define ATG_SVC_MAX_FRAMES 65536u
#define ATG_SVC_MAX_PCM_BYTES (1ull << 31)
#define ATG_SVC_MAX_MSG 4096u

// request: this header, then uint32 frame_sizes[n_frame_sizes], then
// pcm_bytes of interleaved PCM (int16 for ATG_PCM_S16, int32 otherwise)
typedef struct {
    uint32_t magic, version;
    atg_flac_options opts;
    uint32_t format, channels, bits_per_sample, sample_rate;
    uint64_t pcm_frames, n_frame_sizes, first_frame_number, pcm_bytes;
} atg_svc_request;

// response: this header, then msg_len bytes of error text, then uint32
// frame_bytes[n_frames], then out_bytes of FLAC frames
typedef struct {
    int32_t status;
    uint32_t msg_len;
    uint64_t out_bytes, n_frames;
} atg_svc_response;

// the service's socket name for a device (abstract namespace: no file to
// clean up): "\0atgpu-encoderd.<uid>.<device>", or ATG_ENCODER_SOCKET's
// value when set.  An abstract name has no permissions, so both ends check
// the peer's uid (SO_PEERCRED) and drop a connection from another user; the
// client also checks every reply against its request (frame count, sizes,
// the segment's byte bound) and gives up on a reply that misses its
// deadline (ATG_SERVICE_TIMEOUT_MS + 1 ms per 50 KB of PCM)
#define ATG_SVC_NAME_FMT "atgpu-encoderd.%u.%d"
