// launch.h — host-side launchers exported by each kernel translation unit.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "flac_dev.h"

// flac_lpc.hip
hipError_t launch_lpc_analyze(const FlacParams &p, const void *pcm, int fmt,
                              const FrameInfo *frames, const double *windows,
                              int16_t *coef_tab, int8_t *shift_tab,
                              uint8_t *est_tab, hipStream_t s);
// flac_search.hip
hipError_t launch_subframe_search(const FlacParams &p, const void *pcm, int fmt,
                                  const FrameInfo *frames,
                                  const int16_t *coef_tab,
                                  const int8_t *shift_tab,
                                  const uint8_t *est_tab, SubDesc *sub,
                                  uint32_t *err, hipStream_t s);
// the candidates flac_search16.hip handed over (list[0 .. *count))
hipError_t launch_subframe_search_list(const FlacParams &p, const void *pcm, int fmt,
                                       const FrameInfo *frames, const int16_t *coef_tab,
                                       const int8_t *shift_tab, const uint8_t *est_tab,
                                       SubDesc *sub, uint32_t *err, const uint32_t *list,
                                       const uint32_t *count, uint32_t grid, hipStream_t s);
// flac_search16.hip: full 4096-sample frames whose candidates fit int16;
// appends every other candidate to slow_list (count in *slow_count, zeroed
// by the caller)
hipError_t launch_subframe_search16(const FlacParams &p, const void *pcm, int fmt,
                                    const FrameInfo *frames, const int16_t *coef_tab,
                                    const int8_t *shift_tab, const uint8_t *est_tab,
                                    SubDesc *sub, uint32_t *slow_list, uint32_t *slow_count,
                                    hipStream_t s);
// flac_search16.hip: full 4096-sample frames of sources wider than 16 bits
// (hi/lo split images, |s| < 2^26), any channel layout; hand-over as above
hipError_t launch_subframe_search_hl(const FlacParams &p, const void *pcm, int fmt,
                                     const FrameInfo *frames, const int16_t *coef_tab,
                                     const int8_t *shift_tab, const uint8_t *est_tab,
                                     SubDesc *sub, uint32_t *slow_list, uint32_t *slow_count,
                                     hipStream_t s);
// flac_big.hip: frames longer than 4096 samples / partition orders > 6
hipError_t launch_subframe_search_big(const FlacParams &p, const void *pcm, int fmt,
                                      const FrameInfo *frames, const int16_t *coef_tab,
                                      const int8_t *shift_tab, const uint8_t *est_tab,
                                      SubDesc *sub, uint8_t *rice_big, uint32_t rice_stride,
                                      uint8_t *scratch, uint64_t slot_bytes, uint64_t row_bytes,
                                      uint32_t grid, hipStream_t s);
hipError_t launch_frame_pack_big(const FlacParams &p, const void *pcm, int fmt,
                                 const FrameInfo *frames, const TrackInfo *tracks,
                                 const SubDesc *sub, const uint8_t *rice_big,
                                 uint32_t rice_stride, const FrameDesc *fd, uint8_t *out,
                                 uint32_t *err, uint8_t *scratch, uint64_t slot_bytes,
                                 uint32_t grid, hipStream_t s);
// flac_frame.hip
hipError_t launch_frame_decide(const FlacParams &p, const FrameInfo *frames,
                               const SubDesc *sub, FrameDesc *fd, hipStream_t s);
hipError_t launch_track_scan(const FlacParams &p, const TrackInfo *tracks,
                             const uint32_t *order, FrameDesc *fd, TrackOut *tout,
                             hipStream_t s);
hipError_t launch_frame_pack(const FlacParams &p, const void *pcm, int fmt,
                             const FrameInfo *frames, const TrackInfo *tracks,
                             const SubDesc *sub, const FrameDesc *fd,
                             uint8_t *out, uint32_t *err, hipStream_t s);
// md5.hip: host-hashed digests into TrackOut (engine host-MD5 mode)
hipError_t launch_put_md5(TrackOut *tout, const uint8_t *md5, uint32_t n, hipStream_t s);
// md5.hip: the MD5 byte stream of n samples (low bb bytes of each int16 /
// int32 container) at dst, 16-byte aligned
hipError_t launch_md5_pack(const void *src, int s16, uint64_t n, uint32_t bb, uint8_t *dst,
                           hipStream_t s);
hipError_t launch_stream_header(const FlacParams &p, const TrackInfo *tracks,
                                const TrackOut *tout, uint8_t *out,
                                hipStream_t s);
// host pipeline: track images from their slots to dst + dst_off[t]
hipError_t launch_pack_images(const uint8_t *img, const TrackInfo *tracks, const TrackOut *tout,
                              const uint64_t *dst_off, uint32_t n, uint8_t *dst, hipStream_t s);
// CRC-16 chunk lengths 4q bytes (q = 1..kCrcQ) for frames up to 256 kCrcQ
// bytes: every lane of the pack kernel's CRC pass gets ceil(L / 256) words
constexpr int kCrcQ = 64;
hipError_t upload_crc_tables(const uint16_t *adv /*[24][16]*/,
                             const uint32_t *crc16_tab /*[4][256] slicing tables*/,
                             const uint32_t *crc8_tab /*[256]*/,
                             const uint16_t *advq /*[kCrcQ][6][16]: advance by 4q 2^s bytes*/);
// md5.hip
hipError_t launch_track_md5(const FlacParams &p, const void *pcm, int fmt,
                            const TrackInfo *tracks, TrackOut *tout, int part, hipStream_t s);
// rolled chains (engine rolled mode): one launch advances up to kRollMax
// batches' whole-block chains by their own slices (md5.hip k_track_md5_roll)
constexpr uint32_t kRollMax = 32;
struct MdRollBatch {
    const void *pcm;
    const TrackInfo *tracks;
    TrackOut *tout;
    uint32_t n_tracks, channels, bps, fmt; // fmt: 0 = ATG_PCM_S16, 1 = ATG_PCM_S32
    uint32_t wg0;                          // first workgroup of this batch
    uint32_t part, part_end, parts;        // slice [part, part_end) of `parts`
};
struct MdRollArgs {
    uint32_t n;
    MdRollBatch b[kRollMax];
};
bool track_md5_paired(const FlacParams &p, int fmt);
// the decoder's rolled byte-stream chains (md5.hip k_bytes_md5_roll)
struct MdBytesRoll {
    const uint8_t *base;
    const uint64_t *off, *len;
    uint8_t *md5;
    uint32_t n, wg0, part, part_end, parts;
};
struct MdBytesRollArgs {
    uint32_t n;
    MdBytesRoll b[kRollMax];
};
hipError_t launch_bytes_md5_roll(const MdBytesRollArgs &a, hipStream_t s);
hipError_t launch_bytes_md5_finish(const uint8_t *base, const uint64_t *off, const uint64_t *len,
                                   uint32_t n, uint8_t *md5, hipStream_t s);
hipError_t launch_track_md5_roll(const MdRollArgs &a, hipStream_t s);
hipError_t launch_track_md5_finish(const FlacParams &p, const void *pcm, int fmt,
                                   const TrackInfo *tracks, TrackOut *tout, hipStream_t s);
// MD5 of n byte streams base[off[t] .. off[t] + len[t]) (off 64-aligned),
// digests to md5[16 t] (the decoder's STREAMINFO check)
hipError_t launch_bytes_md5(const uint8_t *base, const uint64_t *off, const uint64_t *len,
                            uint32_t n, uint8_t *md5, hipStream_t s);
