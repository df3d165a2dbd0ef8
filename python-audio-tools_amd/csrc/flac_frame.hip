// flac_frame.hip — frame-level stages of the FLAC encoder.
//
//   K3 k_frame_decide   stereo decorrelation choice + frame header + size
//                       (reference flacenc_write_frame / _write_frame_header,
//                       src/encoders/flac.c:412-671)
//   K4 k_track_scan     per-track byte offsets of frames, STREAMINFO min/max
//                       frame size (flac.c:244-279)
//   K5 k_frame_pack     serialise the chosen subframes MSB-first into an LDS
//                       frame image, CRC-16 it, copy it to its final place
//                       (flac.c:813-1016, 1406-1434; bit writer semantics
//                       src/bitstream.c:1904-1945, 2234-2313)
//   K6 k_stream_header  "fLaC" + STREAMINFO + VORBIS_COMMENT + PADDING
//                       (flac.c:208-238, 376-409)
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "flac_dev.h"
#include "launch.h"
#include "pcm_read.h"
#include "residual.h"
#include "wave.h"


__constant__ uint16_t c_crc_adv[24][16]; // advance CRC-16 state by 2^m zero bytes
__constant__ uint32_t c_crc16[4][256]; // slicing tables: byte + k zero bytes
__constant__ uint32_t c_crc8[256];
__constant__ uint16_t c_crc_advq[kCrcQ][6][16]; // advance by 4q * 2^s zero bytes (q - 1, s)

#define VENDOR "Python Audio Tools 2.22alpha1"
#define VENDOR_LEN 29

hipError_t upload_crc_tables(const uint16_t *adv, const uint32_t *crc16_tab,
                             const uint32_t *crc8_tab, const uint16_t *advq)
{
    hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(c_crc_adv), adv, sizeof(uint16_t) * 24 * 16);
    if (e != hipSuccess)
        return e;
    e = hipMemcpyToSymbol(HIP_SYMBOL(c_crc_advq), advq, sizeof(uint16_t) * kCrcQ * 6 * 16);
    if (e != hipSuccess)
        return e;
    e = hipMemcpyToSymbol(HIP_SYMBOL(c_crc16), crc16_tab, sizeof(uint32_t) * 1024);
    if (e != hipSuccess)
        return e;
    return hipMemcpyToSymbol(HIP_SYMBOL(c_crc8), crc8_tab, sizeof(uint32_t) * 256);
}

// ---------------------------------------------------------------- K3
struct HdrWriter {
    uint8_t b[16];
    uint32_t pos;
    __device__ void put(uint32_t n, uint32_t v)
    {
        for (uint32_t i = n; i-- > 0;) {
            const uint32_t byte = pos >> 3;
            if ((pos & 7u) == 0u)
                b[byte] = 0;
            if ((v >> i) & 1u)
                b[byte] |= (uint8_t)(0x80u >> (pos & 7u));
            pos++;
        }
    }
};

__device__ uint32_t frame_header(uint8_t *out, uint32_t block, uint32_t rate, uint32_t bps,
                                 uint32_t assign, uint32_t number)
{
    uint32_t bsc, src, bpc;
    switch (block) {
    case 192: bsc = 1; break;
    case 576: bsc = 2; break;
    case 1152: bsc = 3; break;
    case 2304: bsc = 4; break;
    case 4608: bsc = 5; break;
    case 256: bsc = 8; break;
    case 512: bsc = 9; break;
    case 1024: bsc = 10; break;
    case 2048: bsc = 11; break;
    case 4096: bsc = 12; break;
    case 8192: bsc = 13; break;
    case 16384: bsc = 14; break;
    case 32768: bsc = 15; break;
    default: bsc = block <= 0xFFu ? 6u : (block <= 0xFFFFu ? 7u : 0u);
    }
    switch (rate) {
    case 88200: src = 1; break;
    case 176400: src = 2; break;
    case 192000: src = 3; break;
    case 8000: src = 4; break;
    case 16000: src = 5; break;
    case 22050: src = 6; break;
    case 24000: src = 7; break;
    case 32000: src = 8; break;
    case 44100: src = 9; break;
    case 48000: src = 10; break;
    case 96000: src = 11; break;
    default:
        if (rate <= 255000u && rate % 1000u == 0u)
            src = 12;
        else if (rate <= 655350u && rate % 10u == 0u)
            src = 14;
        else if (rate <= 0xFFFFu)
            src = 13;
        else
            src = 0;
    }
    switch (bps) {
    case 8: bpc = 1; break;
    case 12: bpc = 2; break;
    case 16: bpc = 4; break;
    case 20: bpc = 5; break;
    case 24: bpc = 6; break;
    default: bpc = 0;
    }
    HdrWriter w;
    w.pos = 0;
    w.put(14, 0x3FFE);
    w.put(2, 0);
    w.put(4, bsc);
    w.put(4, src);
    w.put(4, assign);
    w.put(3, bpc);
    w.put(1, 0);
    // UTF-8-style frame number (flac.c:1531-1566)
    if (number <= 0x7Fu) {
        w.put(8, number);
    } else {
        const uint32_t nb = number <= 0x7FFu ? 2 : number <= 0xFFFFu ? 3 : number <= 0x1FFFFFu ? 4
                          : number <= 0x3FFFFFFu ? 5 : 6;
        int shift = (int)(nb - 1) * 6;
        w.put(nb + 1, ((1u << nb) - 1u) << 1);
        w.put(7 - nb, number >> shift);
        for (shift -= 6; shift >= 0; shift -= 6) {
            w.put(2, 2);
            w.put(6, (number >> shift) & 0x3Fu);
        }
    }
    if (bsc == 6)
        w.put(8, block - 1);
    else if (bsc == 7)
        w.put(16, block - 1);
    if (src == 12)
        w.put(8, rate / 1000u);
    else if (src == 13)
        w.put(16, rate);
    else if (src == 14)
        w.put(16, rate / 10u);
    const uint32_t n = w.pos >> 3;
    uint32_t crc = 0;
    for (uint32_t i = 0; i < n; ++i)
        crc = c_crc8[crc ^ w.b[i]];
    w.put(8, crc);
    for (uint32_t i = 0; i <= n; ++i)
        out[i] = w.b[i];
    return n + 1;
}

__global__ void k_frame_decide(FlacParams p, const FrameInfo *__restrict__ frames,
                               const SubDesc *__restrict__ sub, FrameDesc *__restrict__ fd)
{
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= p.n_frames)
        return;
    const FrameInfo fi = frames[f];
    const SubDesc *s = sub + (size_t)f * p.n_cand;
    FrameDesc d;
    uint64_t bits = 0;
    if (p.n_cand == 4u && p.channels == 2u) {
        const uint32_t L = s[0].bits, R = s[1].bits, A = s[2].bits, D = s[3].bits;
        uint32_t assign, s0, s1;
        if (p.mid_side) {
            uint32_t m = L + D < D + R ? L + D : D + R;
            m = m < A + D ? m : A + D;
            if (L + R < m) {
                assign = 1; s0 = 0; s1 = 1;
            } else if (L < (R < A ? R : A)) {
                assign = 8; s0 = 0; s1 = 3;
            } else if (R < A) {
                assign = 9; s0 = 3; s1 = 1;
            } else {
                assign = 10; s0 = 2; s1 = 3;
            }
        } else if (L + R < A + D) {
            assign = 1; s0 = 0; s1 = 1;
        } else {
            assign = 10; s0 = 2; s1 = 3;
        }
        d.assign = (uint8_t)assign;
        d.nsub = 2;
        d.sub[0] = (uint8_t)s0;
        d.sub[1] = (uint8_t)s1;
        bits = (uint64_t)s[s0].bits + s[s1].bits;
    } else {
        d.assign = (uint8_t)(p.channels - 1u);
        d.nsub = (uint8_t)p.channels;
        for (uint32_t c = 0; c < p.channels; ++c) {
            d.sub[c] = (uint8_t)c;
            bits += s[c].bits;
        }
    }
    d.hdr_len = (uint8_t)frame_header(d.hdr, fi.n, p.sample_rate, p.bps, d.assign, fi.index);
    d.bytes = (uint32_t)(d.hdr_len + (bits + 7u) / 8u + 2u);
    d.out_off = 0;
    d.pad = 0;
    fd[f] = d;
}

// ---------------------------------------------------------------- K4
__global__ void k_track_scan(FlacParams p, const TrackInfo *__restrict__ tracks,
                             const uint32_t *__restrict__ order, FrameDesc *__restrict__ fd,
                             TrackOut *__restrict__ tout)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= p.n_tracks)
        return;
    const TrackInfo ti = tracks[t];
    uint64_t off = 0;
    uint32_t mn = 0xFFFFFFu, mx = 0;
    for (uint32_t i = 0; i < ti.n_frames; ++i) {
        const uint32_t f = order[ti.first_pos + i];
        const uint32_t b = fd[f].bytes;
        fd[f].out_off = (uint32_t)off;
        off += b;
        mn = b < mn ? b : mn;
        mx = b > mx ? b : mx;
    }
    tout[t].bytes = p.header_bytes + off;
    tout[t].min_fs = mn;
    tout[t].max_fs = mx;
}

// ---------------------------------------------------------------- K5
// One wave per frame.  The frame image is built MSB-first in a zeroed LDS
// buffer of big-endian words: lane l streams its own run of residual codes
// through a 64-bit register window and stores whole words (ds_write), only
// the first and last word of each run (shared with a neighbour) use ds_or.
// Residuals are recomputed with the search kernel's arithmetic
// (residual.h), so they are the same integers the bit counts came from.

// OR `n` (1..32) bits of v into the big-endian bit image at bit position pos
__device__ __forceinline__ void put_bits(uint32_t *fb, uint32_t pos, uint32_t n, uint32_t v)
{
    if (n == 0)
        return;
    const uint64_t val = (uint64_t)(n >= 32 ? v : (v & ((1u << n) - 1u)));
    const uint32_t w = pos >> 5, off = pos & 31u;
    const uint64_t x = val << (64u - off - n);
    const uint32_t hi = (uint32_t)(x >> 32), lo = (uint32_t)x;
    if (hi)
        atomicOr(&fb[w], hi);
    if (lo)
        atomicOr(&fb[w + 1], lo);
}

// LDS written by some lanes of a wave, then read by others of the same wave
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

// per-lane MSB-first bit stream into the zeroed LDS image.  A lane's bit
// range [begin, end) shares at most its first and last words with the
// neighbouring lanes: those two are OR-ed in by end() (the first is held
// in a register until then), every word in between is a plain store, so
// the word-crossing branch holds no atomics and no nested conditions.
struct LaneWriter {
    uint32_t *fb;
    uint64_t acc; // bits of words cw (high half) and cw + 1 (low half)
    uint32_t cw, w0, bp, first;

    __device__ __forceinline__ void begin(uint32_t *f, uint32_t pos)
    {
        fb = f;
        acc = 0;
        cw = pos >> 5;
        w0 = cw;
        bp = pos;
        first = 0;
    }
    // `zeros` 0-bits, then the low n (1..32) bits of v (v < 2^n)
    __device__ __forceinline__ void put(uint32_t zeros, uint32_t n, uint32_t v)
    {
        bp += zeros;
        const uint32_t nw = bp >> 5;
        if (nw != cw) {
            const uint32_t hi = (uint32_t)(acc >> 32), lo = (uint32_t)acc;
            if (cw == w0)
                first = hi;
            else
                fb[cw] = hi;
            const bool adj = nw == cw + 1u;
            if (!adj)
                fb[cw + 1u] = lo; // wholly this lane's: the run goes on past it
            acc = adj ? (uint64_t)lo << 32 : 0ull;
            cw = nw;
        }
        acc |= (uint64_t)v << (64u - (bp & 31u) - n);
        bp += n;
    }
    __device__ __forceinline__ void end()
    {
        const uint32_t hi = (uint32_t)(acc >> 32), lo = (uint32_t)acc;
        if (first)
            atomicOr(&fb[w0], first);
        if (hi)
            atomicOr(&fb[cw], hi);
        if (lo)
            atomicOr(&fb[cw + 1u], lo);
    }
};

__device__ __forceinline__ uint32_t fb_byte(const uint32_t *fb, uint32_t b)
{
    return (fb[b >> 2] >> (24u - 8u * (b & 3u))) & 0xFFu;
}

// big-endian 32 bits starting at image byte q (q >= 0) = alignbyte of two words
__device__ __forceinline__ uint32_t fb_be32(const uint32_t *fb, uint32_t q)
{
    const uint32_t hi = fb[q >> 2];
    const uint32_t r = q & 3u;
    if (r == 0u)
        return hi;
    return __builtin_amdgcn_alignbyte(hi, fb[(q >> 2) + 1u], 4u - r);
}

__device__ __forceinline__ uint32_t crc_adv(uint32_t c, int m)
{
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        r ^= ((c >> i) & 1u) ? (uint32_t)c_crc_adv[m][i] : 0u;
    return r;
}

// the same by 4 (q + 1) 2^s zero bytes
__device__ __forceinline__ uint32_t crc_advq(uint32_t c, uint32_t q, int s)
{
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        r ^= ((c >> i) & 1u) ? (uint32_t)c_crc_advq[q][s][i] : 0u;
    return r;
}

// rice-coded residual section of one lane from its kept zig-zag codes.
// FULL (the register-staged kernel: every lane holds a whole 64-sample run,
// hi = 64, and only lane 0 skips warm-up codes, lo <= 12): codes 12..63 are
// written unconditionally, so no per-code lane mask is formed for them
template <bool FULL>
__device__ __forceinline__ void emit_codes(LaneWriter &w, const uint32_t (&u)[ATG_RUN], int lo,
                                           int hi, uint32_t k)
{
    const uint32_t kmask = (1u << k) - 1u;
#pragma unroll
    for (int t = 0; t < ATG_RUN; ++t)
        if (FULL ? (t >= ATG_FAST_ORDER || t >= lo) : (t >= lo && t < hi))
            w.put(u[t] >> k, k + 1u, (1u << k) | (u[t] & kmask));
}

// REG = false: samples staged in LDS (any frame).  REG = true: the lane's
// 64-sample run (+16 predecessors) held in VGPRs, read as 16-bit stereo
// pairs with 16-byte loads: no sample LDS, twice the occupancy.  Used for
// the leading full-length (4096) frames of a 16-bit mid/side batch whose
// frame starts are 16-byte aligned (engine.hip counts them: n_reg_frames).
// NW waves per frame (REG: 1): wave w packs subframes w, w + NW, ... into
// the shared image, each from its own sample staging; a subframe's first bit
// is the header plus the searched sizes (SubDesc.bits) of the ones before
// it, and neighbouring subframes meet only in OR-ed words.  A 6-channel
// 24-bit frame's image (75 KB) leaves LDS for one frame per CU: one wave
// per CU before, three now.
// waves per SIMD the pack kernel's registers are budgeted for
constexpr int kK5WavesPerEu = 2;
template <typename T, bool REG, int NW>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(kK5WavesPerEu))) void k_frame_pack(
    FlacParams p, uint32_t f0, const T *__restrict__ pcm, const FrameInfo *__restrict__ frames,
    const TrackInfo *__restrict__ tracks, const SubDesc *__restrict__ sub,
    const FrameDesc *__restrict__ fdesc, uint8_t *__restrict__ out, uint32_t *__restrict__ err)
{
    static_assert(!REG || NW == 1, "the register-staged pack is one wave per frame");
    extern __shared__ __attribute__((aligned(16))) uint32_t fb[];
    __shared__ __attribute__((aligned(16))) int32_t sl_all[REG ? 4 : NW * SL_WORDS];
    __shared__ int32_t cfs_all[NW][ATG_MAX_LPC];
    __shared__ uint16_t crc_tab[4][256];

    const uint32_t f = f0 + blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = NW == 1 ? 0 : __builtin_amdgcn_readfirstlane(tid >> 6);
    int32_t *sl = sl_all + (REG ? 0 : wave * SL_WORDS);
    int32_t *cfs = cfs_all[wave];
    const FrameInfo fi = frames[f];
    const FrameDesc &fd = fdesc[f]; // by reference: hdr[]/sub[] indexed per lane
    const uint32_t N = fi.n;
    const bool ms = (p.n_cand == 4u) && (p.channels == 2u);
    const uint32_t words = (fd.bytes + 3u) / 4u + 1u;

    for (uint32_t i = tid; i < words; i += 64 * NW)
        fb[i] = 0;
    for (uint32_t i = tid; i < 1024u; i += 64 * NW)
        (&crc_tab[0][0])[i] = (uint16_t)(&c_crc16[0][0])[i];
    if (!REG)
        for (int i = lane; i < SL_PRE; i += 64)
            sl[i] = 0;
    __syncthreads();
    if (tid < fd.hdr_len)
        put_bits(fb, 8u * tid, 8, fd.hdr[tid]);
    // the sample staging and coefficients are the wave's own
    auto sync = [] {
        if (NW == 1)
            __syncthreads();
        else
            wave_lds_sync();
    };

    // lane run mapping (same as the search kernel; REG: N = 4096 -> 64l..64l+63)
    const uint32_t tz = N ? (uint32_t)__builtin_ctz(N) : 0u;
    uint32_t P = p.max_porder < tz ? p.max_porder : tz;
    P = P > ATG_MAX_PORDER ? ATG_MAX_PORDER : P;
    const uint32_t G = 64u >> P, S = N >> P, R = (S + G - 1u) / G;
    const uint32_t jf = (uint32_t)lane / G, qf = (uint32_t)lane % G;
    uint32_t ra = jf * S + qf * R, re = ra + R;
    re = re < (jf + 1u) * S ? re : (jf + 1u) * S;
    ra = ra < re ? ra : re;
    const int len = (int)(re - ra);

    for (uint32_t si = (uint32_t)wave; si < fd.nsub; si += NW) {
        uint32_t pos = 8u * fd.hdr_len;
        for (uint32_t s0 = 0; s0 < si; ++s0)
            pos += sub[(size_t)f * p.n_cand + fd.sub[s0]].bits;
        // REG: the frame's 16-bit stereo pairs for samples [ra - 16, ra + 64),
        // (re)loaded per subframe so they are not live across the emission
        uint32_t pr[80];
        if (REG) {
            const uint4 *q4 = (const uint4 *)((const uint32_t *)pcm + fi.pcm_start);
            const int b4 = ((int)ra - 16) / 4;
#pragma unroll
            for (int q = 0; q < 20; ++q) {
                const uint4 v = q4[max(b4 + q, 0)];
                const bool ok = b4 + q >= 0;
                pr[4 * q] = ok ? v.x : 0u;
                pr[4 * q + 1] = ok ? v.y : 0u;
                pr[4 * q + 2] = ok ? v.z : 0u;
                pr[4 * q + 3] = ok ? v.w : 0u;
            }
        }
        const uint32_t cand = fd.sub[si];
        const SubDesc &d = sub[(size_t)f * p.n_cand + cand];
        const uint32_t type = d.type, order = d.order, w = d.wasted, sbps = d.sbps;
        const uint32_t start = pos;
        // max |sample| of the candidate, from the search (picks the residual kernel)
        const uint32_t maxabs = d.amax;
        // REG: candidate sample (ra - 16 + i) from the staged pairs, computed
        // where used (one v_dot2 + one shift) instead of held in 80 VGPRs
        const uint32_t wts = cand == 0u ? 0x00000001u : cand == 1u ? 0x00010000u
                           : cand == 2u ? 0x00010001u : 0xFFFF0001u;
        int xsh = (cand == 2u ? 1 : 0) + (int)w;
        // the shift in a VGPR (a shift by an SGPR operand issues at half rate)
        asm volatile("v_mov_b32 %0, %0" : "+v"(xsh));
        auto xs = [&](int i) -> int { return dot2_z(pr[i], (int)wts) >> xsh; };
        if (!REG)
            stage_candidate_any(pcm, fi.pcm_start, N, p.channels, cand, ms, lane,
                                [&](uint32_t i, int32_t s) { sl[saddr((int)i)] = s >> w; });
        // sample i of this subframe (generic paths; REG reads PCM directly)
        auto sample = [&](int i) -> int32_t {
            if (REG)
                return i < 0 ? 0 : cand_sample(pcm, fi.pcm_start + (uint32_t)i, p.channels, cand, ms) >> w;
            return sl[saddr(i)];
        };
        if (lane < (int)order) {
            int c;
            if (type == SF_LPC)
                c = d.coef[lane];
            else // FIXED predictors as coefficient sets (flac.c:918-1016)
                c = order == 1 ? 1
                  : order == 2 ? (lane == 0 ? 2 : -1)
                  : order == 3 ? (lane == 0 ? 3 : lane == 1 ? -3 : 1)
                  : (lane == 0 ? 4 : lane == 1 ? -6 : lane == 2 ? 4 : -1);
            cfs[lane] = c;
        }
        sync();
        const uint32_t rb = sbps - w;
        const uint32_t rmask = rb >= 32u ? 0xFFFFFFFFu : (1u << rb) - 1u;
        if (type == SF_CONSTANT) {
            // 8 zero header bits, then the raw first sample (flac.c:813-830)
            const uint32_t s0 = REG ? (uint32_t)__builtin_amdgcn_readfirstlane(xs(16))
                                    : (uint32_t)sl[saddr(0)];
            if (lane == 0)
                put_bits(fb, pos + 8u, sbps, s0);
            pos += 8u + sbps;
        } else {
            const uint32_t code = type == SF_VERBATIM ? 1u
                                : type == SF_FIXED ? 8u + order : 32u + order - 1u;
            if (lane == 0) {
                put_bits(fb, pos, 7, code);
                if (w)
                    put_bits(fb, pos + 7u, w + 1u, (1u << w) | 1u);
            }
            const uint32_t hb = 7u + (w ? w + 1u : 1u);
            if (type == SF_VERBATIM) {
                LaneWriter wr;
                wr.begin(fb, pos + hb + ra * rb);
                if (REG) {
#pragma unroll
                    for (int t = 0; t < 64; ++t)
                        wr.put(0, rb, (uint32_t)xs(16 + t) & rmask);
                } else {
                    for (int t = 0; t < len; ++t)
                        wr.put(0, rb, (uint32_t)sl[saddr((int)ra + t)] & rmask);
                }
                wr.end();
                pos += hb + N * rb;
            } else {
                // warm-up samples
                if (REG) {
                    if (lane == 0) {
                        LaneWriter ww;
                        ww.begin(fb, pos + hb);
#pragma unroll
                        for (int j = 0; j < ATG_MAX_LPC; ++j)
                            if ((uint32_t)j < order)
                                ww.put(0, rb, (uint32_t)xs(16 + j) & rmask);
                        ww.end();
                    }
                } else if ((uint32_t)lane < order) {
                    put_bits(fb, pos + hb + lane * rb, rb, (uint32_t)sl[saddr(lane)]);
                }
                uint32_t q = pos + hb + order * rb;
                int shift = 0;
                if (type == SF_LPC) {
                    shift = d.shift;
                    if (lane == 0) {
                        put_bits(fb, q, 4, d.precision - 1u);
                        put_bits(fb, q + 4u, 5, (uint32_t)shift & 31u);
                    }
                    if ((uint32_t)lane < order)
                        put_bits(fb, q + 9u + lane * d.precision, d.precision,
                                 (uint32_t)cfs[lane]);
                    q += 9u + order * d.precision;
                }
                if (lane == 0) {
                    put_bits(fb, q, 2, d.method);
                    put_bits(fb, q + 2u, 4, d.porder);
                }
                const uint32_t rs = q + 6u;
                const uint32_t po = d.porder;
                const uint32_t pbits = d.method ? 5u : 4u;
                const bool degen = (N >> po) < order;
                const uint32_t jp = (uint32_t)lane >> (6u - po);
                const uint32_t k = degen ? d.rice[0] : d.rice[jp];
                const bool part_head = !degen && ((uint32_t)lane & ((64u >> po) - 1u)) == 0u;

                uint64_t csum = 0;
                for (uint32_t j = 0; j < order; ++j)
                    csum += (uint64_t)(cfs[j] < 0 ? -(int64_t)cfs[j] : cfs[j]);
                const int kind = residual_kernel(csum, maxabs, (int)order);
                // wide samples (24-bit): the hi/lo split, exact in 32 bits
                const bool hl = !REG && kind == RES_GENERIC && order <= ATG_FAST_ORDER &&
                                maxabs < (1u << 26) &&
                                csum * (uint64_t)((maxabs >> 12) + 1u) < (1ull << 31);
                uint32_t total, excl;
                LaneWriter wr;
                if (kind != RES_GENERIC || hl) {
                    int cf[ATG_FAST_ORDER];
#pragma unroll
                    for (int j = 0; j < ATG_FAST_ORDER; ++j)
                        cf[j] = uniform_i32(j < (int)order ? cfs[j] : 0);
                    uint32_t u[ATG_RUN];
                    int warm;
                    if (REG) {
                        if (kind == RES_DOT2)
                            lane_residuals_regs<true>(xs, cf, shift, u);
                        else
                            lane_residuals_regs<false>(xs, cf, shift, u);
                        warm = lane == 0 ? (int)order : 0;
#pragma unroll
                        for (int t = 0; t < ATG_FAST_ORDER; ++t)
                            u[t] = t < warm ? 0u : u[t];
                    } else if (hl) {
                        uint64_t asum;
                        const bool full = N == ATG_MAX_BLOCK;
                        if (shift >= 12)
                            asum = full ? lane_residuals_hl<true, true>(sl, (int)ra, len, cf, shift, u)
                                        : lane_residuals_hl<false, true>(sl, (int)ra, len, cf, shift, u);
                        else
                            asum = full ? lane_residuals_hl<true, false>(sl, (int)ra, len, cf, shift, u)
                                        : lane_residuals_hl<false, false>(sl, (int)ra, len, cf, shift, u);
                        warm = drop_warmup((int)ra, len, (int)order, u, asum);
                    } else {
                        uint64_t asum;
                        const bool full = N == ATG_MAX_BLOCK;
                        if (kind == RES_DOT2)
                            asum = full ? lane_residuals<true, true>(sl, (int)ra, len, cf, shift, u)
                                        : lane_residuals<true, false>(sl, (int)ra, len, cf, shift, u);
                        else
                            asum = full ? lane_residuals<false, true>(sl, (int)ra, len, cf, shift, u)
                                        : lane_residuals<false, false>(sl, (int)ra, len, cf, shift, u);
                        warm = drop_warmup((int)ra, len, (int)order, u, asum);
                    }
                    uint32_t cb = (uint32_t)(len - warm) * (1u + k);
#pragma unroll
                    for (int t = 0; t < ATG_RUN; ++t)
                        cb += u[t] >> k;
                    excl = wave_excl_scan_u32(cb, lane);
                    total = wave_sum_u32(cb);
                    wr.begin(fb, degen ? rs + pbits + excl
                                       : rs + pbits * (jp + (part_head ? 0u : 1u)) + excl);
                    if (part_head)
                        wr.put(0, pbits, k);
                    emit_codes<REG>(wr, u, warm, len, k);
                } else {
                    // any order <= 32 / wide samples: 64-bit accumulator
                    const int i0 = max((int)ra, (int)order);
                    uint32_t cb = 0;
                    for (int i = i0; i < (int)re; ++i) {
                        int64_t acc = 0;
                        for (uint32_t j = 0; j < order; ++j)
                            acc += (int64_t)cfs[j] * (int64_t)sample(i - 1 - (int)j);
                        const int r = (int)((uint32_t)sample(i) - (uint32_t)(int32_t)(acc >> shift));
                        cb += (zigzag(r) >> k) + 1u + k;
                    }
                    excl = wave_excl_scan_u32(cb, lane);
                    total = wave_sum_u32(cb);
                    wr.begin(fb, degen ? rs + pbits + excl
                                       : rs + pbits * (jp + (part_head ? 0u : 1u)) + excl);
                    if (part_head)
                        wr.put(0, pbits, k);
                    const uint32_t kmask = (1u << k) - 1u;
                    for (int i = i0; i < (int)re; ++i) {
                        int64_t acc = 0;
                        for (uint32_t j = 0; j < order; ++j)
                            acc += (int64_t)cfs[j] * (int64_t)sample(i - 1 - (int)j);
                        const int r = (int)((uint32_t)sample(i) - (uint32_t)(int32_t)(acc >> shift));
                        const uint32_t uu = zigzag(r);
                        wr.put(uu >> k, k + 1u, (1u << k) | (uu & kmask));
                    }
                }
                wr.end();
                if (degen) {
                    // partition 0 holds every residual; the others are empty
                    const uint32_t np = 1u << po;
                    for (uint32_t j = lane; j < np; j += 64)
                        put_bits(fb, j == 0 ? rs : rs + pbits + total + (j - 1u) * pbits,
                                 pbits, d.rice[j]);
                }
                pos = rs + (1u << po) * pbits + total;
            }
        }
        if (pos - start != d.bits && lane == 0)
            atomicOr(err, 2u);
        sync();
    }
    __syncthreads();

    // CRC-16 of bytes [0, L): 64 chunks of Lc bytes over a virtually
    // zero-prefixed image (leading zeros leave a zero-init CRC unchanged),
    // 4 bytes per step with slicing tables, tree-combined with "advance by
    // Lc 2^s zero bytes" matrices.  Lc = 4 ceil(L / 256) for frames up to
    // 256 kCrcQ bytes (fewer than 256 prefix bytes: every lane has work),
    // else the power of two 2^m >= L / 64
    const uint32_t L = fd.bytes - 2u;
    if (wave == 0) {
    const uint32_t cq = (L + 255u) >> 8;
    const bool qlen = cq >= 1u && cq <= (uint32_t)kCrcQ;
    uint32_t lc_log = 2;
    while ((64u << lc_log) < L)
        lc_log++;
    const uint32_t Lc = qlen ? 4u * cq : 1u << lc_log;
    const int z = (int)(64u * Lc) - (int)L;
    uint32_t crc = 0;
    {
        int q = lane * (int)Lc - z; // image byte of this lane's first group
        const int qe = q + (int)Lc;
        if (q < 0) {
            // groups wholly in the zero prefix leave crc = 0: skip them
            q += ((-q) >> 2) << 2; // now -4 < q <= 0
            if (q < 0 && q < qe) {
                const uint32_t t = fb[0] >> (8u * (uint32_t)(-q));
                crc = crc_tab[3][t >> 24] ^ crc_tab[2][(t >> 16) & 0xFFu] ^
                      crc_tab[1][(t >> 8) & 0xFFu] ^ crc_tab[0][t & 0xFFu];
                q += 4;
            }
        }
        for (; q < qe; q += 4) {
            const uint32_t t = fb_be32(fb, (uint32_t)q) ^ (crc << 16);
            crc = crc_tab[3][t >> 24] ^ crc_tab[2][(t >> 16) & 0xFFu] ^
                  crc_tab[1][(t >> 8) & 0xFFu] ^ crc_tab[0][t & 0xFFu];
        }
    }
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        const uint32_t other = (uint32_t)__shfl_down((int)crc, 1 << s, 64);
        if ((lane & ((2 << s) - 1)) == 0)
            crc = (qlen ? crc_advq(crc, cq - 1u, s) : crc_adv(crc, (int)lc_log + s)) ^ other;
    }
    if (lane == 0)
        put_bits(fb, 8u * L, 16, crc);
    }
    __syncthreads();

    // copy the image to its place: aligned dwords inside, bytes at the ends
    const TrackInfo ti = tracks[fi.track];
    uint8_t *dst = out + ti.out_base + p.header_bytes + fd.out_off;
    const uintptr_t d0 = (uintptr_t)dst;
    const uint32_t head = (uint32_t)((4u - (d0 & 3u)) & 3u);
    const uint32_t nb = fd.bytes;
    const uint32_t h = head < nb ? head : nb;
    if ((uint32_t)tid < h)
        dst[tid] = (uint8_t)fb_byte(fb, tid);
    const uint32_t body = (nb - h) / 4u;
    uint32_t *dw = (uint32_t *)(dst + h);
    for (uint32_t i = tid; i < body; i += 64 * NW)
        dw[i] = __builtin_bswap32(fb_be32(fb, h + 4u * i));
    const uint32_t tail0 = h + 4u * body;
    if (tid < 64 && tail0 + (uint32_t)tid < nb)
        dst[tail0 + tid] = (uint8_t)fb_byte(fb, tail0 + tid);
}

// ---------------------------------------------------------------- K6
__global__ __launch_bounds__(64) void k_stream_header(FlacParams p,
                                                      const TrackInfo *__restrict__ tracks,
                                                      const TrackOut *__restrict__ tout,
                                                      uint8_t *__restrict__ out)
{
    __shared__ uint8_t hdr[128];
    const uint32_t t = blockIdx.x;
    const int lane = threadIdx.x;
    const TrackInfo ti = tracks[t];
    const TrackOut to = tout[t];
    uint8_t *dst = out + ti.out_base;
    if (lane == 0) {
        uint32_t n = 0;
        hdr[n++] = 'f'; hdr[n++] = 'L'; hdr[n++] = 'a'; hdr[n++] = 'C';
        hdr[n++] = 0x00; hdr[n++] = 0; hdr[n++] = 0; hdr[n++] = 34;
        HdrWriter w; // reuse as a 34-byte STREAMINFO writer in two halves
        const uint32_t bs = p.block_size > 0xFFFFu ? 0xFFFFu : p.block_size;
        const uint32_t mn = to.min_fs > 0xFFFFFFu ? 0xFFFFFFu : to.min_fs;
        const uint32_t mx = to.max_fs > 0xFFFFFFu ? 0xFFFFFFu : to.max_fs;
        const uint32_t rate = p.sample_rate > 0xFFFFFu ? 0xFFFFFu : p.sample_rate;
        const uint64_t total = ti.pcm_frames;
        w.pos = 0;
        w.put(16, bs);
        w.put(16, bs);
        w.put(24, mn);
        w.put(24, mx);
        w.put(20, rate);
        w.put(3, p.channels - 1u > 7u ? 7u : p.channels - 1u);
        w.put(5, p.bps - 1u > 31u ? 31u : p.bps - 1u);
        w.put(4, (uint32_t)(total >> 32) & 0xFu);
        for (int i = 0; i < 14; ++i)
            hdr[n++] = w.b[i];
        const uint32_t lo = (uint32_t)total;
        hdr[n++] = (uint8_t)(lo >> 24); hdr[n++] = (uint8_t)(lo >> 16);
        hdr[n++] = (uint8_t)(lo >> 8); hdr[n++] = (uint8_t)lo;
        for (int i = 0; i < 16; ++i)
            hdr[n++] = to.md5[i];
        const uint32_t vc = 4u + VENDOR_LEN + 4u;
        hdr[n++] = 0x04; hdr[n++] = (uint8_t)(vc >> 16); hdr[n++] = (uint8_t)(vc >> 8);
        hdr[n++] = (uint8_t)vc;
        hdr[n++] = VENDOR_LEN; hdr[n++] = 0; hdr[n++] = 0; hdr[n++] = 0;
        const char *v = VENDOR;
        for (int i = 0; i < VENDOR_LEN; ++i)
            hdr[n++] = (uint8_t)v[i];
        hdr[n++] = 0; hdr[n++] = 0; hdr[n++] = 0; hdr[n++] = 0;
        hdr[n++] = 0x81; hdr[n++] = (uint8_t)(p.padding_size >> 16);
        hdr[n++] = (uint8_t)(p.padding_size >> 8); hdr[n++] = (uint8_t)p.padding_size;
    }
    __syncthreads();
    const uint32_t fixed = p.header_bytes - p.padding_size;
    for (uint32_t i = lane; i < fixed; i += 64)
        dst[i] = hdr[i];
    for (uint32_t i = fixed + lane; i < p.header_bytes; i += 64)
        dst[i] = 0;
}

// ---------------------------------------------------------------- launchers
hipError_t launch_frame_decide(const FlacParams &p, const FrameInfo *frames, const SubDesc *sub,
                               FrameDesc *fd, hipStream_t s)
{
    if (!p.n_frames)
        return hipSuccess;
    hipLaunchKernelGGL(k_frame_decide, dim3((p.n_frames + 255u) / 256u), dim3(256), 0, s, p,
                       frames, sub, fd);
    return hipGetLastError();
}

hipError_t launch_track_scan(const FlacParams &p, const TrackInfo *tracks,
                             const uint32_t *order, FrameDesc *fd, TrackOut *tout,
                             hipStream_t s)
{
    if (!p.n_tracks)
        return hipSuccess;
    hipLaunchKernelGGL(k_track_scan, dim3((p.n_tracks + 63u) / 64u), dim3(64), 0, s, p, tracks,
                       order, fd, tout);
    return hipGetLastError();
}

hipError_t launch_frame_pack(const FlacParams &p, const void *pcm, int fmt,
                             const FrameInfo *frames, const TrackInfo *tracks,
                             const SubDesc *sub, const FrameDesc *fd, uint8_t *out,
                             uint32_t *err, hipStream_t s)
{
    if (!p.n_frames)
        return hipSuccess;
    const size_t lds = (size_t)p.frame_lds_words * 4u;
    const uint32_t nreg = fmt == 0 ? p.n_reg_frames : 0u;
    if (nreg)
        hipLaunchKernelGGL((k_frame_pack<int16_t, true, 1>), dim3(nreg), dim3(64), lds, s, p, 0u,
                           (const int16_t *)pcm, frames, tracks, sub, fd, out, err);
    const uint32_t rest = p.n_frames - nreg;
    if (rest == 0)
        return hipGetLastError();
    // waves per frame: the subframes (one per channel) in as few rounds as
    // four waves take them, spread evenly (6 -> 3 x 2, 5 -> 3, 8 -> 4 x 2),
    // fewer while the image and the waves' staging exceed the CU's LDS
    const uint32_t nsub = p.channels > 8u ? 8u : (p.channels ? p.channels : 1u);
    const uint32_t rounds = (nsub + 3u) / 4u;
    uint32_t nw = (nsub + rounds - 1u) / rounds;
    const size_t per_wave = (size_t)(SL_WORDS + ATG_MAX_LPC) * 4u;
    while (nw > 1u && lds + 2048u + nw * per_wave > 160u * 1024u)
        --nw;
#define ATG_PACK(TT, W)                                                                            \
    hipLaunchKernelGGL((k_frame_pack<TT, false, W>), dim3(rest), dim3(64 * W), lds, s, p, nreg,    \
                       (const TT *)pcm, frames, tracks, sub, fd, out, err)
#define ATG_PACK_T(TT)                                                                             \
    switch (nw) {                                                                                  \
    case 4: ATG_PACK(TT, 4); break;                                                                \
    case 3: ATG_PACK(TT, 3); break;                                                                \
    case 2: ATG_PACK(TT, 2); break;                                                                \
    default: ATG_PACK(TT, 1); break;                                                               \
    }
    if (fmt == 0) {
        ATG_PACK_T(int16_t)
    } else {
        ATG_PACK_T(int32_t)
    }
#undef ATG_PACK_T
#undef ATG_PACK
    return hipGetLastError();
}

hipError_t launch_stream_header(const FlacParams &p, const TrackInfo *tracks,
                                const TrackOut *tout, uint8_t *out, hipStream_t s)
{
    if (!p.n_tracks)
        return hipSuccess;
    hipLaunchKernelGGL(k_stream_header, dim3(p.n_tracks), dim3(64), 0, s, p, tracks, tout, out);
    return hipGetLastError();
}

// ---------------------------------------------------------------- images
// The host pipeline's compaction: each track's finished image moves from
// its worst-case slot (tracks[t].out_base) to dst + dst_off[t] (16-byte
// aligned, tracks back to back), so one contiguous copy brings a chunk's
// images to host memory.  One workgroup per track, 16-byte moves; the
// rounded-up tail stays inside both 16-byte-aligned slots.
__global__ __launch_bounds__(256) void k_pack_images(const uint8_t *__restrict__ img,
                                                     const TrackInfo *__restrict__ tracks,
                                                     const TrackOut *__restrict__ tout,
                                                     const uint64_t *__restrict__ dst_off,
                                                     uint32_t n, uint8_t *__restrict__ dst)
{
    for (uint32_t t = blockIdx.x; t < n; t += gridDim.x) {
        const uint4 *__restrict__ s = (const uint4 *)(img + tracks[t].out_base);
        uint4 *__restrict__ d = (uint4 *)(dst + dst_off[t]);
        const uint64_t n16 = (tout[t].bytes + 15u) / 16u;
        for (uint64_t i = threadIdx.x; i < n16; i += blockDim.x)
            d[i] = s[i];
    }
}

hipError_t launch_pack_images(const uint8_t *img, const TrackInfo *tracks, const TrackOut *tout,
                              const uint64_t *dst_off, uint32_t n, uint8_t *dst, hipStream_t s)
{
    if (!n)
        return hipSuccess;
    hipLaunchKernelGGL(k_pack_images, dim3(n < 4096u ? n : 4096u), dim3(256), 0, s, img, tracks,
                       tout, dst_off, n, dst);
    return hipGetLastError();
}
