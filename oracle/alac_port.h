/*
 * alac_port.h — CPU restatement of python-audio-tools' ALAC encoder
 * (src/encoders/alac.c) and decoder (src/decoders/alac.c).
 *
 * TEST INFRASTRUCTURE ONLY (see flac_port.h): the parity checker for the
 * GPU ALAC kernels; the product path never links, loads or calls it.
 */
#ifndef ALAC_PORT_H
#define ALAC_PORT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* encode_alac keyword arguments (src/encoders/alac.c:34-72); the
   interlacing leftweights are the reference's 0..4 */
typedef struct {
    uint32_t block_size, initial_history, history_multiplier, maximum_k;
    /* interlacing leftweights tried, min..max inclusive (alac.c:57-58,
       459-481: 0 and 4 unless the caller passes others) */
    uint32_t min_leftweight, max_leftweight;
} alacport_options;

/* the mdat atom (8-byte header + framesets) of a whole stream, as the
   reference's ALACEncoder_encode_alac writes it (alac.c:126-165).
   frame_sizes[i] = byte size of frameset i (the returned log).
   0 ok, 1 bad arguments, 2 out too small */
int alacport_encode(const int32_t *pcm, uint64_t frames, uint32_t channels, uint32_t bps,
                    const alacport_options *o, uint8_t *out, size_t cap, size_t *out_len,
                    uint32_t *frame_sizes, size_t fs_cap, size_t *n_framesets);
size_t alacport_max_mdat_bytes(uint64_t frames, uint32_t channels, uint32_t bps,
                               uint32_t block_size);
/* write_frameset's channel groups: pairs (c0, c1 or -1), returns count */
unsigned alacport_frameset_groups(unsigned channels, int32_t *groups);

/* decoder status: the reference's status values (decoders/alac.h) */
enum {
    ALACPORT_OK = 0,
    ALACPORT_IO_ERROR = 1,            /* IOError "I/O Errror" / EOF during frame reading */
    ALACPORT_INVALID_UNUSED_BITS = 2, /* ValueError "invalid unused bits" */
    ALACPORT_INVALID_ALAC_ATOM = 3,
    ALACPORT_INVALID_MDHD_ATOM = 4,
    ALACPORT_MDIA_NOT_FOUND = 5,
    ALACPORT_STSD_NOT_FOUND = 6,
    ALACPORT_MDHD_NOT_FOUND = 7,
    ALACPORT_INVALID_SEEKTABLE = 8,
    ALACPORT_NO_MDAT = 9,             /* IOError "Unable to locate 'mdat' atom" */
    ALACPORT_CHANNEL_MISMATCH = 10    /* ValueError "channel length mismatch" */
};

typedef struct {
    uint32_t max_samples_per_frame, bits_per_sample, history_multiplier, initial_history;
    uint32_t maximum_k, channels, sample_rate, total_frames;
    uint64_t mdat_offset; /* absolute byte of the first frameset */
    uint32_t n_seekpoints, reserved;
} alacport_info;

typedef struct {
    uint64_t pcm_frames_offset, file_offset;
} alacport_seekpoint;

/* parse_decoding_parameters + seek_mdat (alac.c:439-672, 953-971);
   seekpoints from stts/stsc/stco (the reference's seektable; empty when an
   atom is missing).  Returns an ALACPORT_* status. */
int alacport_read_info(const uint8_t *data, size_t len, alacport_info *info,
                       alacport_seekpoint *sp, size_t sp_cap);

/* read() loop from byte `start` (mdat_offset, or a seekpoint) with
   remaining_frames = `remaining`: interleaved wave-order int32 PCM of every
   frameset returned; fs_frames / fs_offsets = PCM frames and absolute byte
   offset of each.  Returns the status that ended it (0 = remaining hit 0),
   -1 when pcm_cap is too small. */
int alacport_decode(const uint8_t *data, size_t len, const alacport_info *info, uint64_t start,
                    uint64_t remaining, int32_t *pcm, size_t pcm_cap, uint64_t *pcm_frames,
                    uint32_t *fs_frames, uint64_t *fs_offsets, size_t fs_cap,
                    size_t *n_framesets);

#ifdef __cplusplus
}
#endif
#endif
