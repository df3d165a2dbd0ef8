// flac_dev.h — device-side data layout shared by the FLAC encoder kernels
// and the host engine.  All tables live in HBM for the whole batch:
//
//   pcm        interleaved S16/S32 samples of every track (caller's buffer)
//   FrameInfo  one per FLAC frame (pcm start, length, track, index)
//   windows    Tukey(0.5) windows, fp64, one per distinct block length,
//              computed on the host with glibc cos (bit-exact with the
//              reference's flacenc_window_signal, flac.c:1129-1167)
//   lpc table  per subframe candidate: quantised coefficient sets for
//              orders 1..max_lpc_order (triangular) + shifts
//   SubDesc    per subframe candidate: the chosen coding, exact bit count
//   FrameDesc  per frame: channel assignment, header bytes, frame size
//   TrackInfo  per track: output placement, STREAMINFO inputs
#pragma once

#include <stdint.h>

#define ATG_MAX_LPC 32        // widest LPC order accepted
#define ATG_FAST_ORDER 12     // orders <= this use the unrolled register path
#define ATG_MAX_PORDER 6      // partition orders the GPU search handles
#define ATG_MAX_BLOCK 4096    // block lengths the GPU search handles
#define ATG_RUN 64            // samples per lane (4096 / 64 lanes)
#define ATG_BIG_MAX_BLOCK 65535 // large-frame path (flac_big.hip): FLAC's 16-bit block field
#define ATG_BIG_MAX_PORDER 15   // large-frame path: the format's 4-bit partition order

enum { SF_CONSTANT = 0, SF_VERBATIM = 1, SF_FIXED = 2, SF_LPC = 3 };

struct FlacParams {
    uint32_t block_size;
    uint32_t max_lpc_order;
    uint32_t max_porder;     // min(max_residual_partition_order, ...)
    uint32_t qlp_precision;  // flac.c:165-178
    uint32_t max_rice;       // flac.c:180-184
    int32_t mid_side;
    int32_t adaptive_mid_side;
    int32_t exhaustive;
    int32_t try_verbatim;
    int32_t try_constant;
    int32_t try_fixed;
    int32_t try_lpc;
    uint32_t channels;
    uint32_t bps;
    uint32_t sample_rate;
    uint32_t n_cand;         // subframe candidates per frame (4 = L,R,avg,diff)
    uint32_t n_frames;
    uint32_t n_tracks;
    uint32_t coef_stride;    // int16 entries per candidate in the lpc table
    uint32_t coef_row;       // int16 entries per order row (even; zero past the order)
    uint32_t n_reg_frames;   // leading frames the register-staged packer takes (see K5)
    uint32_t padding_size;
    uint32_t header_bytes;   // bytes before the first frame of every track
    uint32_t frame_lds_words;// pack kernel frame buffer (32-bit words)
    uint32_t frame_bound;    // worst-case bytes of one frame (output slot = n_frames x this)
};

struct FrameInfo {
    uint64_t pcm_start;  // first PCM frame (index into interleaved array)
    uint32_t n;          // PCM frames in this FLAC frame
    uint32_t track;
    uint32_t index;      // frame number within the track
    uint32_t win_off;    // offset of this block length's window (doubles)
};

struct TrackInfo {
    uint64_t pcm_start;
    uint64_t pcm_frames;
    uint64_t out_base;   // byte offset of the track image in the output
    uint32_t first_pos;  // position of the track's first frame in the
                         // track-order frame list (frame ids are grouped
                         // by length, so a track's ids are not contiguous)
    uint32_t n_frames;
};

struct SubDesc {
    uint32_t bits;       // exact bits of the subframe (uint32, as bw counts)
    uint8_t type;
    uint8_t order;
    uint8_t wasted;
    uint8_t porder;
    uint8_t method;
    uint8_t precision;
    int8_t shift;
    uint8_t sbps;        // subframe bits per sample before wasted shift
    uint32_t amax;       // max |s >> wasted| of the candidate (FIXED/LPC/VERBATIM)
    int16_t coef[ATG_MAX_LPC];
    uint8_t rice[1 << ATG_MAX_PORDER];
};

struct FrameDesc {
    uint32_t bytes;      // whole frame incl. header and CRC-16
    uint32_t out_off;    // byte offset from the track's first frame
    uint8_t assign;      // FLAC channel assignment code
    uint8_t nsub;
    uint8_t hdr_len;
    uint8_t pad;
    uint8_t sub[8];      // candidate index of each written subframe
    uint8_t hdr[16];     // frame header bytes incl. CRC-8
};

struct TrackOut {
    uint64_t bytes;
    uint32_t min_fs;
    uint32_t max_fs;
    uint8_t md5[16];
};
