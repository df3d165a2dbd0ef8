/*
 * flac_port.h — CPU restatement of python-audio-tools' FLAC encoder
 * (src/encoders/flac.c) and a FLAC decoder (semantics of src/decoders/flac.c).
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker and the
 * "port" CPU baseline; the product path (libatgpu.so) never links, loads or
 * calls it.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may use it.
 *
 * Parity pinning: checked byte-for-byte against the reference C encoder built
 * from /root/reference/src (oracle/_ref/flacenc, see oracle/Makefile) and
 * against the reference's own known-answer fixture test/tone.flac
 * (tests/golden/).
 */
#ifndef FLAC_PORT_H
#define FLAC_PORT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Encoder options, same meaning as the keyword arguments of
   audiotools.encoders.encode_flac (reference src/encoders/flac.c:52-108). */
typedef struct {
    uint32_t block_size;
    uint32_t max_lpc_order;
    uint32_t min_residual_partition_order; /* accepted, unused (as reference) */
    uint32_t max_residual_partition_order;
    int32_t mid_side;
    int32_t adaptive_mid_side;
    int32_t exhaustive_model_search;
    int32_t disable_verbatim_subframes;
    int32_t disable_constant_subframes;
    int32_t disable_fixed_subframes;
    int32_t disable_lpc_subframes;
    uint32_t padding_size;
} flacport_options;

/* Encode one whole stream.  pcm is interleaved int32 [pcm_frames][channels].
   Writes a complete .flac file image into out (capacity out_cap).
   frame_offsets / frame_lengths (optional, capacity max_frames) receive the
   (byte offset from first frame, pcm frames) list that encode_flac returns.
   Returns 0 on success, negative on error. */
int flacport_encode(const int32_t *pcm, uint64_t pcm_frames,
                    uint32_t channels, uint32_t bits_per_sample,
                    uint32_t sample_rate, const flacport_options *opts,
                    uint8_t *out, size_t out_cap, size_t *out_len,
                    uint64_t *frame_offsets, uint32_t *frame_lengths,
                    size_t max_frames, size_t *n_frames);

/* flacport_encode with the frame cut of a reader whose i-th read() returned
   read_sizes[i] frames (then block_size frames per read): each read is one
   frame (reference src/encoders/flac.c:244-274), a size other than the
   preset's block sizes takes block-size code 0x6/0x7 + an explicit size
   (flac.c:412-518), STREAMINFO's min/max block size stay the option
   (flac.c:193-194).  A listed 0 ends the stream there. */
int flacport_encode_sizes(const int32_t *pcm, uint64_t pcm_frames,
                          uint32_t channels, uint32_t bits_per_sample,
                          uint32_t sample_rate, const flacport_options *opts,
                          const uint32_t *read_sizes, size_t n_read_sizes,
                          uint8_t *out, size_t out_cap, size_t *out_len,
                          uint64_t *frame_offsets, uint32_t *frame_lengths,
                          size_t max_frames, size_t *n_frames);

/* Worst-case output size for flacport_encode / the GPU engine. */
size_t flacport_max_stream_bytes(uint64_t pcm_frames, uint32_t channels,
                                 uint32_t bits_per_sample, uint32_t block_size,
                                 uint32_t padding_size);

/* MD5 of the little-endian signed PCM bytes (STREAMINFO md5). */
void flacport_pcm_md5(const int32_t *pcm, uint64_t pcm_frames,
                      uint32_t channels, uint32_t bits_per_sample,
                      uint8_t digest[16]);

/* STREAMINFO + the parts of the other metadata blocks the reference decoder
   keeps (src/decoders/flac.c:568-707). */
typedef struct {
    uint32_t min_block_size, max_block_size, min_frame_size, max_frame_size;
    uint32_t sample_rate, channels, bits_per_sample, channel_mask;
    uint64_t total_samples;
    uint8_t md5[16];
    uint64_t frames_offset; /* byte offset of the first frame */
    uint32_t n_seekpoints;
    uint32_t reserved;
} flacport_streaminfo;

typedef struct {
    uint64_t sample_number, byte_offset;
    uint32_t samples, reserved;
} flacport_seekpoint;

/* 0 = ok, 1 = not a FLAC file (ValueError), 2 = EOF (IOError) */
int flacport_read_metadata(const uint8_t *data, size_t len, flacport_streaminfo *si,
                           flacport_seekpoint *sp, size_t sp_cap);

/* Decode frames from data (the first frame at data[0]) until `remaining`
   (uint64, decremented by each frame's block size with wrap-around, as the
   reference's remaining_samples) reaches 0 or an error ends the stream.
   Returns the FD_* code that ended decoding: 0 ok, 1..13 the reference's
   flac_status values, 14 frame CRC-16 mismatch, 15 EOF; -1 when pcm_cap or
   frame_cap is too small.  pcm receives the
   interleaved int32 samples of the frames decoded before the error. */
int flacport_decode_frames(const uint8_t *data, size_t len, const flacport_streaminfo *si,
                           uint64_t remaining, int check_crc, int32_t *pcm, size_t pcm_cap,
                           uint64_t *frame_offsets, uint32_t *frame_block_sizes,
                           size_t frame_cap, size_t *n_frames, uint64_t *pcm_frames);

/* Decode a .flac image.  On success returns 0 and fills the stream
   parameters; pcm (capacity pcm_cap samples, may be NULL to query) receives
   interleaved int32 samples.  Verifies CRC-8/CRC-16 and, when present,
   the STREAMINFO MD5 (returns -5 on MD5 mismatch). */
int flacport_decode(const uint8_t *flac, size_t len,
                    uint32_t *channels, uint32_t *bits_per_sample,
                    uint32_t *sample_rate, uint64_t *total_frames,
                    int32_t *pcm, size_t pcm_cap);

#ifdef __cplusplus
}
#endif
#endif
