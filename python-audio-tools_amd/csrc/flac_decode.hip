// flac_decode.hip — MI355X batch FLAC decoder (SURVEY §8(a) rows D1–D5,
// §8(f) rank 1): the frame loop of the reference's FlacDecoder.read()
// (src/decoders/flac.c:174-285), its frame header / subframe / residual
// readers (flac.c:710-1209) and channel decorrelation (flac.c:1212-1269),
// error for error, for a whole batch of .flac images at once.
//
// A FLAC stream has no frame index, and a frame's length is only known once
// its residuals are parsed, so the serial loop is split into passes that are
// each parallel:
//
//   K1 k_dec_sync      thread per 16 input bytes: every byte that starts a
//      k_dec_hdr       sync code is listed, then gets a full frame-header
//                      parse (CRC-8 and STREAMINFO consistency,
//                      flac.c:710-851); survivors are "candidates"
//                      (cand_pos[i], cand_idx[byte] = i).
//   K2 k_dec_parse     lane per candidate (grid-stride): parse the subframes
//                      (Rice codes included) without reconstructing samples,
//                      CRC-16 the frame; record status, length, and the bit
//                      offset of every subframe.
//   K3 k_dec_chain     lane per track: walk first frame -> frame end -> ...
//                      exactly as the reference's read() loop (remaining
//                      samples, uint64 wrap); a position that is not a
//                      candidate, or a frame truncated by `remaining`, is
//                      parsed inline.  Pass 1 counts, pass 2 (after a host
//                      prefix over tracks) writes the frame and subframe jobs.
//   K4 k_dec_subframe  lane per (frame, channel): restart at the recorded bit
//                      offset, Rice-decode and restore FIXED/LPC samples with
//                      the predictor history in registers (one window
//                      predictor for all orders), one row per residual-loop
//                      iteration into a [row][lane] scratch (coalesced).
//   K5 k_dec_emit      block per 64-job slot: rows -> samples (gather),
//                      decorrelate (L-S, S-R, mid-side), interleave to the
//                      FrameList layout (int32), and the little-endian PCM
//                      byte stream the MD5 hashes, in one pass.
//   K6 k_bytes_md5     lane per track (md5.hip): STREAMINFO MD5 check input.
//
// Only K2 and K4 do real work; K1 and K5 are HBM passes.  Status codes are
// the FD_* values of include/atgpu.h (the reference's flac_status plus the
// conditions read() raises itself).
#include "handle_lock.h"
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/atgpu.h"
#include "launch.h"
#include "wave.h"

namespace {

enum {
    FD_OK = 0, FD_ERROR = 1, FD_SYNC = 2, FD_RESERVED = 3, FD_BPS = 4, FD_RATE = 5,
    FD_HDR_CRC = 6, FD_RATE_MISMATCH = 7, FD_CH_MISMATCH = 8, FD_BPS_MISMATCH = 9,
    FD_MAXBS = 10, FD_CODING = 11, FD_FIXED_ORDER = 12, FD_SUBFRAME_TYPE = 13,
    FD_FRAME_CRC = 14, FD_EOF = 15, FD_MD5 = 16
};

__constant__ uint8_t c_crc8[256];
__constant__ uint16_t c_crc16[4][256];
__constant__ uint16_t c_crc_adv[24][16]; // CRC-16 state advanced by 2^m zero bytes

struct DecTrack {
    uint64_t start;     // absolute byte of the first frame
    uint64_t end;       // absolute byte end of the track image
    uint64_t total;     // STREAMINFO total samples (remaining_samples)
    uint32_t rate, channels, bps, max_bs;
    uint64_t frame_base; // pass 2: first DecFrame slot
    uint64_t pcm_base;   // pass 2: first interleaved sample of the output
    uint64_t md5_base;   // pass 2: first byte of the track's PCM byte stream
    uint64_t job_base;   // pass 2: first (frame, channel) job
};

struct DecCount {
    uint64_t pcm_frames; // walked (offsets() view: CRC-16 not checked)
    uint32_t n_frames;
    int32_t status;      // what stopped the walk
    uint64_t crc_pcm;    // PCM frames before the first bad CRC-16 frame
    uint32_t crc_frame;  // index of that frame, ~0u if none
    uint32_t pad;
    uint64_t stop;       // byte where the walk stopped (from the track's start)
};

struct ParseRec {
    int32_t status;
    uint32_t bs;        // header block size
    uint32_t bytes;     // whole frame incl. CRC-16
    uint8_t assign, ch, bps, pad;
    uint32_t sub_bit[8]; // bit offset of each subframe from the frame start
};

struct DecFrame {
    uint64_t pos;       // absolute byte of the frame
    uint64_t pcm_start; // first interleaved sample of the frame in the output
    uint32_t n;         // samples per channel decoded (MIN(bs, remaining))
    uint32_t track;
    uint32_t bs;
    uint8_t assign, ch, bps, spec; // spec: length from the frame-end hypothesis
    uint32_t sub_bit[8];
    uint32_t bytes;     // whole frame incl. CRC-16
    uint32_t pad;
};

struct Hdr {
    uint32_t bs, rate, assign, ch, bps;
};

// what K4 leaves for the row transposer (K4b) per subframe job
struct JobMeta {
    uint8_t kind;   // 0 CONSTANT, 1 VERBATIM (rows = samples), 2 FIXED/LPC, 3 none
    uint8_t order;
    uint8_t porder;
    uint8_t pad;
    int32_t value;  // CONSTANT sample (already shifted by wasted bits)
    uint32_t iters; // rows written
    uint32_t pad2;
};

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// MSB-first random-access bit reader over the batch buffer (big-endian
// 32-bit words).  Position = 32-bit bit offset from a base word, so the
// decode loops do 32-bit arithmetic and carry no refill state: every peek
// loads the two words under the position (L1 hits: a lane walks its own
// frame sequentially).  Keeping the loops free of data-dependent branches is
// what matters here -- the lanes of a wave hold different frames, and a
// per-lane refill branch diverges on almost every code.  Reading past the
// track end is not trapped per bit: eof() compares the position with the
// end (any read past the end makes the reference report EOF, flac.c
// br_abort), and loads are clamped to the buffer.
struct BitR {
    const uint32_t *w;
    uint64_t last;  // last valid word index
    uint64_t bw;    // base word
    uint32_t pos;   // bits from 32 * bw
    uint32_t end;   // track end, bits from 32 * bw (saturated)

    __device__ __forceinline__ void init(const uint32_t *w_, uint64_t nw, uint64_t bit,
                                         uint64_t endbit)
    {
        w = w_;
        last = nw - 1;
        bw = bit >> 5;
        pos = (uint32_t)(bit & 31);
        const uint64_t e = endbit - bw * 32; // endbit >= bit - 31 for every caller
        end = endbit < bw * 32 ? 0u : (e > 0xF0000000ull ? 0xF0000000u : (uint32_t)e);
    }
    __device__ __forceinline__ uint64_t abspos() const { return bw * 32 + pos; }
    __device__ __forceinline__ bool eof() const { return pos > end; }
    // the two words under the position (raw, big-endian)
    __device__ __forceinline__ void words(uint32_t &a, uint32_t &b) const
    {
        const uint64_t i = bw + (pos >> 5);
        a = w[i < last ? i : last];
        b = w[i + 1 < last ? i + 1 : last];
    }
    __device__ __forceinline__ uint32_t window(uint32_t a, uint32_t b) const
    {
        a = bswap32(a);
        b = bswap32(b);
        const uint32_t sh = pos & 31;
        return sh ? (a << sh) | (b >> (32 - sh)) : a;
    }
    __device__ __forceinline__ uint32_t peek32() const
    {
        uint32_t a, b;
        words(a, b);
        return window(a, b);
    }
    __device__ __forceinline__ void skip(uint32_t n) { pos += n; }
    __device__ __forceinline__ void skip_far(uint64_t n)
    {
        const uint64_t p = (uint64_t)pos + n;
        pos = p > 0xF0000001ull ? 0xF0000001u : (uint32_t)p; // saturate past any end
    }
    __device__ __forceinline__ uint32_t get(uint32_t n) // n <= 32
    {
        const uint32_t v = n ? peek32() >> (32 - n) : 0u;
        pos += n;
        return v;
    }
    // br_read_signed_bits_be (src/bitstream.c:418-425)
    __device__ __forceinline__ int32_t get_signed(uint32_t n)
    {
        if (n == 0) { // asks for 2^32-1 magnitude bits: always EOF
            skip_far(1ull << 33);
            return 0;
        }
        if (n > 33) {
            skip_far(n);
            return 0;
        }
        const uint32_t sign = get(1);
        const uint32_t v = n > 1 ? get(n - 1) : 0u;
        return sign ? (int32_t)(v - (1u << ((n - 1) & 31))) : (int32_t)v;
    }
    // read_unary(stop=1): number of 0 bits before a 1
    __device__ __forceinline__ uint32_t zeros()
    {
        uint32_t q = 0;
        for (;;) {
            const uint32_t p = peek32();
            if (p) {
                const uint32_t z = __builtin_clz(p);
                pos += z + 1;
                return q + z;
            }
            q += 32;
            pos += 32;
            if (eof())
                return q;
        }
    }
};

__device__ __forceinline__ uint32_t byte_at(const uint32_t *w, uint64_t i)
{
    return (bswap32(w[i >> 2]) >> (24 - 8 * (uint32_t)(i & 3))) & 0xFFu;
}

#define RET(code) return r.eof() ? FD_EOF : (code)

// flacdec_read_frame_header (flac.c:710-851)
__device__ int dec_header(BitR &r, const DecTrack &t, Hdr &h)
{
    const uint64_t start = r.abspos();
    if (r.get(14) != 0x3FFEu) RET(FD_SYNC);
    if (r.get(1)) RET(FD_RESERVED);
    r.get(1); // blocking strategy
    const uint32_t bs_bits = r.get(4), sr_bits = r.get(4);
    h.assign = r.get(4);
    h.ch = (h.assign >= 8 && h.assign <= 10) ? 2u : h.assign + 1u;
    switch (r.get(3)) {
    case 0: h.bps = t.bps; break;
    case 1: h.bps = 8; break;
    case 2: h.bps = 12; break;
    case 4: h.bps = 16; break;
    case 5: h.bps = 20; break;
    case 6: h.bps = 24; break;
    default: RET(FD_BPS);
    }
    r.get(1);
    // read_utf8 (flac.c:1310-1320): leading 1 bits count the bytes
    uint32_t nbytes = __builtin_clz(~r.peek32() | 1u);
    if (nbytes > 7)
        return FD_EOF;
    r.skip(nbytes + 1);
    r.get(7 - nbytes);
    for (; nbytes > 1; nbytes--)
        r.get(8);
    switch (bs_bits) {
    case 0: h.bs = t.max_bs; break;
    case 6: h.bs = r.get(8) + 1; break;
    case 7: h.bs = r.get(16) + 1; break;
    case 1: h.bs = 192; break;
    case 2: case 3: case 4: case 5: h.bs = 576u << (bs_bits - 2); break;
    default: h.bs = 256u << (bs_bits - 8); break;
    }
    switch (sr_bits) {
    case 0: h.rate = t.rate; break;
    case 1: h.rate = 88200; break;
    case 2: h.rate = 176400; break;
    case 3: h.rate = 192000; break;
    case 4: h.rate = 8000; break;
    case 5: h.rate = 16000; break;
    case 6: h.rate = 22050; break;
    case 7: h.rate = 24000; break;
    case 8: h.rate = 32000; break;
    case 9: h.rate = 44100; break;
    case 10: h.rate = 48000; break;
    case 11: h.rate = 96000; break;
    case 12: h.rate = r.get(8) * 1000; break;
    case 13: h.rate = r.get(16); break;
    case 14: h.rate = r.get(16) * 10; break;
    default: RET(FD_RATE);
    }
    r.get(8);
    if (r.eof())
        return FD_EOF;
    uint32_t crc = 0;
    for (uint64_t i = start >> 3; i < (r.abspos() >> 3); ++i)
        crc = c_crc8[crc ^ byte_at(r.w, i)];
    if (crc)
        return FD_HDR_CRC;
    if (t.rate != h.rate) return FD_RATE_MISMATCH;
    if (t.channels != h.ch) return FD_CH_MISMATCH;
    if (t.bps != h.bps) return FD_BPS_MISMATCH;
    if (h.bs > t.max_bs) return FD_MAXBS;
    return FD_OK;
}

// Every FIXED and LPC subframe is restored by one W-tap window predictor
// (W = 12 for orders <= 12, 32 beyond): coefficients zero-padded past the
// order, FIXED orders as LPC coefficients with shift 0 (flac.c:1090-1132;
// the reference's wrapping int arithmetic equals the int64 sum truncated to
// 32 bits).  One code path for all orders keeps the lanes of a wave, which
// hold subframes of different orders, in lockstep.
//
// `fast`: the int64 sum of the reference is computed as int32 with
// v_mad_i32_i24 when that is exact -- Σ|c|·2^(bps-1) < 2^31, |c| and
// samples within 24 bits -- and every restored sample stays inside the
// bps range (checked per sample into `bad`; a lane that trips it re-decodes
// the subframe with the int64 path).
// v_mad_i32_i24: 24-bit signed multiply, 32-bit add, one full-rate op
__device__ __forceinline__ int32_t mad24(int32_t a, int32_t b, int32_t c)
{
    int32_t d;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

template <int W>
struct WinPred {
    int4 *row;      // the job's samples, [sample/4][lane][4]: lane column at row[.. * 64]
    int32_t q0, q1, q2, q3; // the 4 samples stored together
    uint32_t i, n, wasted, shift, half, porder;
    bool fast, bad;
    int32_t c[W];
    int32_t h[W]; // h[0] newest sample
    // sample i (warm-up or restored) into the job's column: one 16-byte
    // store per 4 samples (64 lanes of a wave store 1 KB contiguous); the
    // emitter reads 4 consecutive samples of a job with one 16-byte load
    __device__ __forceinline__ void put(int32_t v, bool on)
    {
        const uint32_t k = i & 3;
        q0 = on && k == 0 ? v : q0;
        q1 = on && k == 1 ? v : q1;
        q2 = on && k == 2 ? v : q2;
        q3 = on && k == 3 ? v : q3;
        if (on && k == 3)
            row[(uint64_t)(i >> 2) * 64] = make_int4(q0, q1, q2, q3);
        i += on ? 1u : 0u;
    }
    __device__ __forceinline__ void warm(int32_t s)
    {
#pragma unroll
        for (int j = W - 1; j > 0; --j)
            h[j] = h[j - 1];
        h[0] = s;
        put((int32_t)((uint32_t)s << wasted), true);
    }
    __device__ __forceinline__ void partition_order(uint32_t p) { porder = p; }
    // one residual-loop iteration (a partition header when !commit)
    __device__ __forceinline__ void step(int32_t rv, bool commit)
    {
        int32_t p;
        if (fast) {
            int32_t acc = 0;
#pragma unroll
            for (int j = 0; j < W; ++j)
                acc = mad24(c[j], h[j], acc);
            p = acc >> (shift < 31 ? shift : 31);
        } else {
            int64_t acc = 0;
#pragma unroll
            for (int j = 0; j < W; ++j)
                acc += (int64_t)c[j] * (int64_t)h[j];
            p = (int32_t)(acc >> shift);
        }
        const int32_t s = (int32_t)((uint32_t)p + (uint32_t)rv);
        bad |= commit && ((uint32_t)(s + (int32_t)half) >= 2u * half);
#pragma unroll
        for (int j = W - 1; j > 0; --j)
            h[j] = commit ? h[j - 1] : h[j];
        h[0] = commit ? s : h[0];
        put((int32_t)((uint32_t)s << wasted), commit);
    }
    __device__ __forceinline__ void flush()
    {
        if (i & 3)
            row[(uint64_t)(i >> 2) * 64] = make_int4(q0, q1, q2, q3);
    }
};

struct NullSink {
    __device__ __forceinline__ void step(int32_t, bool) {}
    __device__ __forceinline__ void partition_order(uint32_t) {}
};

// flacdec_read_residual (flac.c:1135-1209), residuals handed to `sink`.
// One flat loop whose iterations each consume either a partition header or
// one residual, both decoded from the same 32-bit peek and merged with
// selects: lanes holding different partition orders and Rice parameters
// never branch apart (long unary codes, > 32 bits with their LSBs, take a
// rare slow path).
// Residual-loop reads.  Lanes hold different subframes, so a lane's words
// are its own stream, and at one or two waves per SIMD (a lane per frame or
// per subframe: ~1-2 k waves for a config-2 batch) nothing hides a load's
// latency: with the next word fetched from global memory one iteration
// ahead, every word crossing waits an L2 round trip (the subframe kernel
// ran ~2,000 cycles per residual, and prediction cost nothing measurable,
// profiles/r04_h_dec_probe.jsonl).  Ring: a lane's words come from a
// 64-word LDS ring, refilled at wave-uniform points every kRingG
// iterations by two alternating 16-word buffers (four 16-byte loads each):
// a buffer issued at refill point k is committed to the ring at point k+2,
// so a load has 2 kRingG iterations to arrive and the loop itself reads only
// LDS.  A refill holds 16 words per kRingG = 16 iterations, one word per
// iteration: what the widest codes that stay on the fast path consume.  A
// lane that outruns its ring (long codes, the slow path's jumps) reads
// global memory directly until the ring catches up.
constexpr uint32_t kRing = 64;       // words per lane (power of 2)
constexpr uint32_t kRingStride = 68; // LDS words between lanes (16-byte rows)
constexpr uint32_t kRingG = 16;      // iterations per refill point
constexpr uint32_t kRingB = 16;      // words per refill buffer

// Refill loads: plain loads whose waits the compiler places.  With both
// buffers in fixed registers (the loop is unrolled over the two refill
// points, no phi moves them) and the window's first words waited for before
// the loop, the compiler's wait for a buffer at its commit is a counted
// vmcnt past the other buffer's four loads (checked in the ISA), and the
// residual steps in between wait only for LDS.
__device__ __forceinline__ void ring_load4(const uint4 *p, uint4 &q0, uint4 &q1, uint4 &q2,
                                           uint4 &q3)
{
    q0 = p[0];
    q1 = p[1];
    q2 = p[2];
    q3 = p[3];
}

// one refill point for buffer (q, addr, pend): commit what it loaded two
// points ago, then load the next 16 words (kept only if the ring has room
// for them).  The four loads are issued whether or not they are kept (a
// lane without room re-reads a block it already holds), so the compiler
// can wait for a buffer with a counted vmcnt(4) -- the other buffer's four
// loads stay in flight -- instead of vmcnt(0).
#define RING_REFILL(q0, q1, q2, q3, addr, pend)                                        \
    do {                                                                               \
        if (pend) {                                                                    \
            if (addr >= fill) { /* blocks arrive in address order; a gap restarts */   \
                if (addr > fill)                                                       \
                    rbeg = addr;                                                       \
                uint4 *d_ = (uint4 *)(ring + (addr & (kRing - 1)));                    \
                d_[0] = q0;                                                            \
                d_[1] = q1;                                                            \
                d_[2] = q2;                                                            \
                d_[3] = q3;                                                            \
                fill = addr + kRingB;                                                  \
                rbeg = fill > rbeg + kRing ? fill - kRing : rbeg;                      \
            }                                                                          \
        }                                                                              \
        const uint64_t a_ = nf > (S.cw & ~15ull) ? nf : (S.cw & ~15ull);               \
        pend = a_ + kRingB <= S.cw + kRing && a_ + kRingB <= r.last + 1;               \
        const uint4 *s_ = (const uint4 *)(r.w + (pend ? a_ : ((r.last + 1 - kRingB) & ~3ull))); \
        ring_load4(s_, q0, q1, q2, q3);                                                \
        addr = a_;                                                                     \
        nf = pend ? a_ + kRingB : nf;                                                  \
    } while (0)

// Register window of a lane's residual stream: hi:lo = words cw, cw+1 (byte-
// swapped), off = bits consumed of hi, nx = word cw+2 (raw), plus the
// partition state of flacdec_read_residual.
struct ResState {
    uint64_t cw;
    uint32_t off, hi, lo, nx;
    uint32_t k, hdrs, left, rice, esc;
};

struct ResShape {
    uint32_t total, parts, p0, plen, pbits, escv;
};

// One iteration of the flat residual loop: a partition header or one
// residual, both decoded from the same 32-bit peek and merged with selects
// (lanes holding different partition orders and Rice parameters never
// branch apart; long unary codes, > 32 bits with their LSBs, take a rare
// slow path).  The window moves at most one word (to nx); the caller loads
// the next nx.  Returns false when the lane is done (end or EOF in `st`).
template <class P>
__device__ __forceinline__ bool res_step(BitR &r, ResState &S, const ResShape &Z, P &sink, int &st)
{
    const uint32_t p = S.off ? (S.hi << S.off) | (S.lo >> (32 - S.off)) : S.hi;
    const bool hdr = S.left == 0;
    // partition header: Rice parameter (+ escape width)
    const uint32_t hr = p >> (32 - Z.pbits);
    const bool hesc = hr == Z.escv;
    const uint32_t hlen = Z.pbits + (hesc ? 5u : 0u);
    const uint32_t hbits = (p >> (27 - Z.pbits)) & 31u;
    // residual: Rice code (unary MSBs, stop bit, LSBs) or escaped raw
    const uint32_t z = __builtin_clz(p | 1u);
    const uint32_t clen = z + 1 + S.rice;
    const uint32_t lsb = __builtin_amdgcn_ubfe(p, 31 - z - S.rice, S.rice);
    const uint32_t value = (z << S.rice) | lsb;
    int32_t v = (int32_t)(value >> 1) ^ -(int32_t)(value & 1u);
    uint32_t len = clen;
    if (S.esc) {
        v = (int32_t)p >> (32 - S.esc);
        len = S.esc;
    }
    const uint32_t step = hdr ? hlen : len;
    if (!hdr && !S.esc && (p == 0 || clen > 32)) { // rare: long code
        r.pos = (uint32_t)((S.cw - r.bw) * 32) + S.off;
        const uint32_t msb = r.zeros();
        const uint32_t val = (msb << S.rice) | r.get(S.rice);
        v = (int32_t)(val >> 1) ^ -(int32_t)(val & 1u);
        S.cw = r.bw + (r.pos >> 5);
        S.off = r.pos & 31;
        S.hi = bswap32(r.w[S.cw < r.last ? S.cw : r.last]);
        S.lo = bswap32(r.w[S.cw + 1 < r.last ? S.cw + 1 : r.last]);
    } else {
        S.off += step;
        const bool need = S.off >= 32;
        S.hi = need ? S.lo : S.hi;
        S.lo = need ? bswap32(S.nx) : S.lo;
        S.cw += need ? 1u : 0u;
        S.off -= need ? 32u : 0u;
    }
    sink.step(v, !hdr);
    S.k += hdr ? 0u : 1u;
    S.left = hdr ? (S.hdrs == 0 ? Z.p0 : Z.plen) : S.left - 1u;
    S.rice = hdr ? hr : S.rice;
    S.esc = hdr ? (hesc ? hbits : 0u) : S.esc;
    S.hdrs += hdr ? 1u : 0u;
    if (hdr) {
        r.pos = (uint32_t)((S.cw - r.bw) * 32) + S.off;
        if (r.eof()) {
            st = FD_EOF;
            return false;
        }
    }
    return S.k < Z.total || S.hdrs < Z.parts;
}

// 16 iterations of the ring loop: the ring word for the next nx (ds_read),
// or, for a lane that outran its ring, the word from global memory, waited
// for inside the branch (a select of the two would become a flat load,
// which waits for every outstanding load -- the refills -- at its use)
#define RING_STEPS()                                                                       \
    for (uint32_t s_ = 0; s_ < kRingG; ++s_) {                                             \
        if (live) {                                                                        \
            live = res_step(r, S, Z, sink, st);                                            \
            const uint64_t nw_ = S.cw + 2;                                                 \
            S.nx = ring[nw_ & (kRing - 1)];                                                \
            if (nw_ < rbeg || nw_ >= fill) {                                               \
                const uint32_t g_ = r.w[nw_ < r.last ? nw_ : r.last];                      \
                asm volatile("" : : "v"(g_));                                              \
                S.nx = g_;                                                                 \
            }                                                                              \
        }                                                                                  \
    }

// flacdec_read_residual (flac.c:1135-1209), residuals handed to `sink`.
template <class P, bool RING = false>
__device__ __forceinline__ int dec_residual(BitR &r, uint32_t order, uint32_t N, P &sink,
                                            uint32_t *ring = nullptr)
{
    const uint32_t method = r.get(2);
    const uint32_t porder = r.get(4);
    sink.partition_order(porder);
    // a partition order that does not divide the block: rejected (the
    // reference would predict from a stale buffer), as the oracle does
    if (!r.eof() && method <= 1 && ((N >> porder) << porder) != N)
        return FD_ERROR;
    if (method > 1)
        RET(FD_CODING); // raised at the first partition (flac.c:1160-1170)
    ResShape Z;
    Z.plen = N >> porder;
    Z.p0 = Z.plen > order ? Z.plen - order : 0u;
    Z.parts = 1u << porder;
    Z.total = Z.p0 + (Z.parts - 1u) * Z.plen;
    Z.pbits = method ? 5u : 4u;
    Z.escv = method ? 0x1Fu : 0xFu;
    ResState S;
    S.k = S.hdrs = S.left = S.rice = S.esc = 0;
    S.cw = r.bw + (r.pos >> 5);
    S.off = r.pos & 31;
    S.hi = bswap32(r.w[S.cw < r.last ? S.cw : r.last]);
    S.lo = bswap32(r.w[S.cw + 1 < r.last ? S.cw + 1 : r.last]);
    int st = FD_OK;
    bool live = true; // parts >= 1: at least one header
    if (RING && (((uintptr_t)r.w) & 15u) == 0 && r.last >= 2 * kRingB) {
        // ring: words [rbeg, fill) are in the LDS ring, loads issued up to
        // nf; two blocks up front (the first refill lands 2 kRingG
        // iterations on); blocks sit at multiples of 16 words, so a block
        // never wraps the ring
        const uint64_t a0 = (S.cw & ~15ull) + 2 * kRingB <= r.last + 1
                                ? (S.cw & ~15ull) : ((r.last + 1 - 2 * kRingB) & ~15ull);
        {
            uint4 x0, x1, x2, x3, y0, y1, y2, y3;
            ring_load4((const uint4 *)(r.w + a0), x0, x1, x2, x3);
            ring_load4((const uint4 *)(r.w + a0 + kRingB), y0, y1, y2, y3);
            uint4 *d0 = (uint4 *)(ring + (a0 & (kRing - 1)));
            uint4 *d1 = (uint4 *)(ring + ((a0 + kRingB) & (kRing - 1)));
            d0[0] = x0;
            d0[1] = x1;
            d0[2] = x2;
            d0[3] = x3;
            d1[0] = y0;
            d1[1] = y1;
            d1[2] = y2;
            d1[3] = y3;
        }
        uint64_t rbeg = a0, fill = a0 + 2 * kRingB, nf = fill;
        {
            const uint64_t nw = S.cw + 2;
            S.nx = nw >= rbeg && nw < fill ? ring[nw & (kRing - 1)]
                                           : r.w[nw < r.last ? nw : r.last];
        }
        // the window's first words are waited for here: a load still in
        // flight into them at the loop entry would make the compiler wait
        // for every outstanding load (the refills) at each use in the loop
        asm volatile("" : : "v"(S.nx), "v"(S.hi), "v"(S.lo));
        uint4 qa0, qa1, qa2, qa3, qb0, qb1, qb2, qb3; // the two refill buffers
        uint64_t aa = 0, ab = 0;
        bool pa = false, pb = false;
        // every lane of the wave that runs this loop entered it together:
        // refill points are wave-uniform; a buffer's loads are committed two
        // points later (its registers never move, so the wait is a counted
        // vmcnt past the other buffer's loads)
        while (__ballot(live) != 0ull) {
            RING_STEPS();
            RING_REFILL(qa0, qa1, qa2, qa3, aa, pa);
            RING_STEPS();
            RING_REFILL(qb0, qb1, qb2, qb3, ab, pb);
        }
    } else {
        S.nx = r.w[S.cw + 2 < r.last ? S.cw + 2 : r.last];
        while (live) {
            live = res_step(r, S, Z, sink, st);
            S.nx = r.w[S.cw + 2 < r.last ? S.cw + 2 : r.last];
        }
    }
    if (st != FD_OK)
        return st;
    r.pos = (uint32_t)((S.cw - r.bw) * 32) + S.off;
    if (r.eof())
        return FD_EOF;
    return FD_OK;
}

// The residual walk on a 64-bit window (the parse kernel's and, with
// values, the restore kernel's loop).  W holds the stream's next `avail`
// bits MSB-first; cw indexes the next word to enter it, nx = that word (raw,
// read from the lane's LDS ring one iteration ahead).  An iteration consumes
// one partition header or one residual (at most 37 bits, after a refill of
// one word whenever fewer than 32 bits are left, so the window never runs
// dry on the fast path) with selects only: lanes in different partitions,
// Rice parameters or escapes stay in lockstep, ~25 VALU per residual
// against ~120 for the word-window step with its per-lane branches (the
// parse loop was instruction-issue bound at one wave per SIMD).  Codes
// longer than the window (> 32 zero bits, or LSBs past the window) and
// lanes whose ring does not hold cw take wave-uniform slow paths.
constexpr uint32_t kWalkInit = 3; // ring blocks loaded before the loop

template <bool VALUES, class P>
__device__ __forceinline__ int walk_residual(BitR &r, uint32_t order, uint32_t N, P &sink,
                                             uint32_t *ring)
{
    const uint32_t method = r.get(2);
    const uint32_t porder = r.get(4);
    sink.partition_order(porder);
    if (!r.eof() && method <= 1 && ((N >> porder) << porder) != N)
        return FD_ERROR;
    if (method > 1)
        RET(FD_CODING); // raised at the first partition (flac.c:1160-1170)
    const uint32_t plen = N >> porder;
    const uint32_t p0 = plen > order ? plen - order : 0u;
    const uint32_t parts = 1u << porder;
    const uint32_t pbits = method ? 5u : 4u, escv = method ? 0x1Fu : 0xFu;
    uint32_t units = p0 + (parts - 1u) * plen + parts; // headers + residuals left
    uint32_t left = 0, rice = 0, esc = 0, hdrs = 0;
    // ring: blocks of 16 words at multiples of 16; kWalkInit up front
    const uint64_t p_abs = r.abspos();
    uint64_t cw = p_abs >> 5;
    const uint64_t lastw = r.last;
    const uint64_t a0 = (cw & ~15ull) + kWalkInit * kRingB <= lastw + 1
                            ? (cw & ~15ull) : ((lastw + 1 - kWalkInit * kRingB) & ~15ull);
    {
        uint4 x0, x1, x2, x3, y0, y1, y2, y3, z0, z1, z2, z3;
        ring_load4((const uint4 *)(r.w + a0), x0, x1, x2, x3);
        ring_load4((const uint4 *)(r.w + a0 + kRingB), y0, y1, y2, y3);
        ring_load4((const uint4 *)(r.w + a0 + 2 * kRingB), z0, z1, z2, z3);
        uint4 *d0 = (uint4 *)(ring + (a0 & (kRing - 1)));
        uint4 *d1 = (uint4 *)(ring + ((a0 + kRingB) & (kRing - 1)));
        uint4 *d2 = (uint4 *)(ring + ((a0 + 2 * kRingB) & (kRing - 1)));
        d0[0] = x0; d0[1] = x1; d0[2] = x2; d0[3] = x3;
        d1[0] = y0; d1[1] = y1; d1[2] = y2; d1[3] = y3;
        d2[0] = z0; d2[1] = z1; d2[2] = z2; d2[3] = z3;
    }
    uint64_t rbeg = a0, fill = a0 + kWalkInit * kRingB, nf = fill;
    // the window: the bits from p_abs to the end of word cw + 1
    uint32_t avail;
    uint64_t W;
    {
        const uint32_t w0 = bswap32(r.w[cw < lastw ? cw : lastw]);
        const uint32_t w1 = bswap32(r.w[cw + 1 < lastw ? cw + 1 : lastw]);
        const uint32_t sh = (uint32_t)(p_abs & 31);
        W = (((uint64_t)w0 << 32) | w1) << sh;
        avail = 64 - sh;
        cw += 2;
    }
    uint32_t nx = cw >= rbeg && cw < fill ? ring[cw & (kRing - 1)] : r.w[cw < lastw ? cw : lastw];
    asm volatile("" : : "v"(nx), "v"(W)); // waited before the loop (see RING_STEPS)
    uint4 qa0, qa1, qa2, qa3, qb0, qb1, qb2, qb3;
    uint64_t aa = 0, ab = 0;
    bool pa = false, pb = false;
    bool live = units != 0, eof = false;
    struct Nop {
    } nop;
    (void)nop;
#define WALK_STEPS()                                                                       \
    for (uint32_t s_ = 0; s_ < kRingG; ++s_) {                                             \
        bool slow = false;                                                                 \
        if (live) {                                                                        \
            const bool need = avail < 32;                                                  \
            W = need ? W | ((uint64_t)bswap32(nx) << (32 - avail)) : W;                    \
            avail += need ? 32u : 0u;                                                      \
            cw += need ? 1u : 0u;                                                          \
            const uint32_t top = (uint32_t)(W >> 32);                                      \
            const bool hdr = left == 0;                                                    \
            const uint32_t hr = top >> (32 - pbits);                                       \
            const bool hesc = hr == escv;                                                  \
            const uint32_t hlen = pbits + (hesc ? 5u : 0u);                                \
            const uint32_t hbits = (top >> (27 - pbits)) & 31u;                            \
            const uint32_t z = __builtin_clz(top | 1u);                                    \
            const uint32_t clen = z + 1u + rice;                                           \
            const uint32_t len = hdr ? hlen : (esc ? esc : clen);                          \
            slow = !hdr && !esc && (top == 0u || clen > avail);                            \
            if (VALUES) {                                                                  \
                const uint32_t mid = (uint32_t)((W << (z + 1u)) >> 32);                    \
                const uint32_t value = (z << rice) | __builtin_amdgcn_ubfe(mid, 32u - rice, rice); \
                int32_t v = (int32_t)(value >> 1) ^ -(int32_t)(value & 1u);                \
                v = esc ? (int32_t)top >> (32u - esc) : v;                                 \
                if (!slow)                                                                 \
                    sink.step(v, !hdr);                                                    \
            }                                                                              \
            const uint32_t sl = slow ? 0u : len;                                           \
            W = sl >= 64u ? 0ull : W << sl;                                                \
            avail -= sl;                                                                   \
            left = hdr ? (hdrs == 0u ? p0 : plen) : left - (slow ? 0u : 1u);               \
            rice = hdr ? hr : rice;                                                        \
            esc = hdr ? (hesc ? hbits : 0u) : esc;                                         \
            hdrs += hdr ? 1u : 0u;                                                         \
            units -= slow ? 0u : 1u;                                                       \
            /* a header past the track end: the reference aborts (EOF) */                  \
            if (hdr && cw * 32 - avail > r.bw * 32 + r.end) {                              \
                eof = true;                                                                \
                slow = false;                                                              \
            }                                                                              \
            live = units != 0u && !eof;                                                    \
            nx = ring[cw & (kRing - 1)];                                                   \
        }                                                                                  \
        if (__ballot(slow || (live && (cw < rbeg || cw >= fill))) != 0ull) {               \
            if (slow) { /* a code the window cannot hold: the bit reader */                \
                r.pos = (uint32_t)(cw * 32 - avail - r.bw * 32);                           \
                const uint32_t msb = r.zeros();                                            \
                const uint32_t val = (msb << rice) | r.get(rice);                          \
                if (VALUES)                                                                \
                    sink.step((int32_t)(val >> 1) ^ -(int32_t)(val & 1u), true);           \
                const uint64_t pa_ = r.abspos();                                           \
                cw = pa_ >> 5;                                                             \
                const uint32_t w0 = bswap32(r.w[cw < lastw ? cw : lastw]);                 \
                const uint32_t w1 = bswap32(r.w[cw + 1 < lastw ? cw + 1 : lastw]);         \
                const uint32_t sh = (uint32_t)(pa_ & 31);                                  \
                W = (((uint64_t)w0 << 32) | w1) << sh;                                     \
                avail = 64 - sh;                                                           \
                cw += 2;                                                                   \
                left -= 1u;                                                                \
                units -= 1u;                                                               \
                eof = r.eof();                                                             \
                live = units != 0u && !eof;                                                \
            }                                                                              \
            if (live && (cw < rbeg || cw >= fill)) {                                       \
                const uint32_t g_ = r.w[cw < lastw ? cw : lastw];                          \
                asm volatile("" : : "v"(g_));                                              \
                nx = g_;                                                                   \
            } else if (live) {                                                             \
                nx = ring[cw & (kRing - 1)];                                               \
            }                                                                              \
        }                                                                                  \
    }
#define WALK_REFILL(q0, q1, q2, q3, addr, pend)                                            \
    do {                                                                                   \
        if (pend && addr >= fill) {                                                        \
            if (addr > fill)                                                               \
                rbeg = addr;                                                               \
            uint4 *d_ = (uint4 *)(ring + (addr & (kRing - 1)));                            \
            d_[0] = q0;                                                                    \
            d_[1] = q1;                                                                    \
            d_[2] = q2;                                                                    \
            d_[3] = q3;                                                                    \
            fill = addr + kRingB;                                                          \
            rbeg = fill > rbeg + kRing ? fill - kRing : rbeg;                              \
        }                                                                                  \
        const uint64_t a_ = nf > (cw & ~15ull) ? nf : (cw & ~15ull);                       \
        pend = a_ + kRingB <= cw + kRing && a_ + kRingB <= lastw + 1;                      \
        ring_load4((const uint4 *)(r.w + (pend ? a_ : ((lastw + 1 - kRingB) & ~3ull))), q0, q1, \
                   q2, q3);                                                                \
        addr = a_;                                                                         \
        nf = pend ? a_ + kRingB : nf;                                                      \
    } while (0)
    while (__ballot(live) != 0ull) {
        WALK_STEPS();
        WALK_REFILL(qa0, qa1, qa2, qa3, aa, pa);
        WALK_STEPS();
        WALK_REFILL(qb0, qb1, qb2, qb3, ab, pb);
    }
#undef WALK_STEPS
#undef WALK_REFILL
    if (eof)
        return FD_EOF;
    r.pos = (uint32_t)(cw * 32 - avail - r.bw * 32);
    if (r.eof())
        return FD_EOF;
    return FD_OK;
}

struct SubHdr {
    uint32_t kind, order, wasted;
};

// subframe header (flac.c:854-905)
__device__ __forceinline__ int dec_subhdr(BitR &r, SubHdr &s)
{
    r.get(1);
    const uint32_t t = r.get(6);
    if (t == 0) { s.kind = 0; s.order = 0; }
    else if (t == 1) { s.kind = 1; s.order = 0; }
    else if ((t & 0x38) == 0x08) { s.kind = 2; s.order = t & 7; }
    else if ((t & 0x20) == 0x20) { s.kind = 3; s.order = (t & 0x1F) + 1; }
    else RET(FD_SUBFRAME_TYPE);
    s.wasted = 0;
    if (r.get(1))
        s.wasted = r.zeros() + 1;
    if (r.eof())
        return FD_EOF;
    return FD_OK;
}

// parse-only subframe (K2 and the chain's inline path)
template <bool RING = false>
__device__ int parse_subframe(BitR &r, uint32_t N, uint32_t bps, uint32_t *ring = nullptr)
{
    SubHdr sh;
    int rc = dec_subhdr(r, sh);
    if (rc)
        return rc;
    bps -= sh.wasted; // unsigned, as the reference
    NullSink np;
    if (sh.kind == 0) {
        r.get_signed(bps);
    } else if (sh.kind == 1) {
        // VERBATIM: N raw samples of bps bits (0 bits asks for 2^32-1
        // magnitude bits per sample: EOF); the parse only skips them -- read
        // one by one, each a dependent load, they set the pace of every wave
        // holding a white-noise frame
        r.skip_far(bps ? (uint64_t)N * bps : (N ? 1ull << 33 : 0ull));
    } else {
        for (uint32_t i = 0; i < sh.order; ++i)
            r.get_signed(bps);
        if (sh.kind == 3) {
            const uint32_t prec = r.get(4) + 1;
            r.get_signed(5);
            for (uint32_t i = 0; i < sh.order; ++i)
                r.get_signed(prec);
        }
        rc = RING && (((uintptr_t)r.w) & 15u) == 0 && r.last >= kWalkInit * kRingB
                 ? walk_residual<false>(r, sh.order, N, np, ring)
                 : dec_residual<NullSink, false>(r, sh.order, N, np);
        if (rc)
            return rc;
        if (sh.kind == 2 && sh.order > 4)
            return FD_FIXED_ORDER;
    }
    if (r.eof())
        return FD_EOF;
    return FD_OK;
}

__device__ __forceinline__ uint32_t sub_bps(uint32_t assign, uint32_t c, uint32_t bps)
{
    return ((assign == 8 && c == 1) || (assign == 9 && c == 0) || (assign == 10 && c == 1))
               ? bps + 1 : bps;
}

// CRC-16 (0x8005) of bytes [b0, b1), slicing by 4 with tables in LDS
__device__ uint32_t crc16_range(const uint32_t *w, uint64_t b0, uint64_t b1,
                                const uint16_t (*T)[256])
{
    uint32_t crc = 0;
    uint64_t i = b0;
    for (; i < b1 && (i & 3); ++i)
        crc = ((crc << 8) & 0xFFFFu) ^ T[0][(crc >> 8) ^ byte_at(w, i)];
#pragma unroll 8
    for (; i + 4 <= b1; i += 4) {
        const uint32_t x = bswap32(w[i >> 2]) ^ (crc << 16);
        crc = (uint32_t)T[3][x >> 24] ^ T[2][(x >> 16) & 0xFF] ^ T[1][(x >> 8) & 0xFF] ^
              T[0][x & 0xFF];
    }
    for (; i < b1; ++i)
        crc = ((crc << 8) & 0xFFFFu) ^ T[0][(crc >> 8) ^ byte_at(w, i)];
    return crc;
}

// one frame of the reference's read() loop, parse only: header, subframes
// with N = MIN(block size, nlimit), byte align, CRC-16
// CRC = false: the frame's CRC-16 is left to k_dec_crc (status stays OK)
// spec_bytes != 0: the frame-end hypothesis (k_dec_spec) -- the last
// subframe is not walked when the ones before it end inside the frame; the
// record then carries the hypothesis (pad = 1, CRC-16 already checked)
template <bool RING = false, bool CRC = true>
__device__ void parse_frame(const uint32_t *w, uint64_t nw, uint64_t pos, const DecTrack &t,
                            uint64_t nlimit, const uint16_t (*T)[256], ParseRec &rec,
                            uint32_t *ring = nullptr, uint32_t spec_bytes = 0)
{
    BitR r;
    r.init(w, nw, pos * 8, t.end * 8);
    Hdr h;
    rec.bytes = 0;
    rec.pad = 0;
    rec.status = dec_header(r, t, h);
    if (rec.status)
        return;
    rec.bs = h.bs;
    rec.assign = (uint8_t)h.assign;
    rec.ch = (uint8_t)h.ch;
    rec.bps = (uint8_t)h.bps;
    const uint32_t N = (uint32_t)((uint64_t)h.bs < nlimit ? (uint64_t)h.bs : nlimit);
    for (uint32_t c = 0; c < h.ch; ++c) {
        rec.sub_bit[c] = (uint32_t)(r.abspos() - pos * 8);
        if (spec_bytes && c + 1u == h.ch && N == h.bs &&
            (uint64_t)rec.sub_bit[c] + 8u <= 8ull * (spec_bytes - 2u)) {
            rec.bytes = spec_bytes;
            rec.status = FD_OK;
            rec.pad = 1;
            return;
        }
        const int rc = parse_subframe<RING>(r, N, sub_bps(h.assign, c, h.bps), ring);
        if (rc) {
            rec.status = rc;
            return;
        }
    }
    const uint32_t a = (uint32_t)(r.abspos() & 7);
    if (a)
        r.skip(8 - a);
    r.get(16);
    if (r.eof()) {
        rec.status = FD_EOF;
        return;
    }
    const uint64_t endb = r.abspos() >> 3;
    rec.bytes = (uint32_t)(endb - pos);
    if (CRC)
        rec.status = crc16_range(w, pos, endb, T) ? FD_FRAME_CRC : FD_OK;
    else
        rec.status = FD_OK;
}

__device__ __forceinline__ void load_crc_lds(uint16_t (*T)[256])
{
    for (uint32_t i = threadIdx.x; i < 4 * 256; i += blockDim.x)
        T[i >> 8][i & 255] = c_crc16[i >> 8][i & 255];
    __syncthreads();
}

__device__ __forceinline__ uint32_t find_track(const DecTrack *tr, uint32_t nt, uint64_t p)
{
    // last track with start <= p (tracks sorted by start)
    uint32_t lo = 0, hi = nt;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (tr[mid].start <= p) lo = mid;
        else hi = mid;
    }
    return lo;
}

// K1: sync-code candidates.  A position needs byte 0xFF followed by
// 0xF8/0xF9 (14-bit sync 0x3FFE, reserved bit 0).  Grid-stride over 16-byte
// chunks: a lane takes one 16-byte load (plus the next chunk's first word
// for a sync code straddling the chunks), so the pass streams the buffer at
// a few TB/s instead of launching a wave per 256 bytes; the header parse
// runs only for the rare lanes holding a sync pattern.
__device__ __forceinline__ bool sync_at(uint32_t a, uint32_t b, int k)
{
    const uint64_t pair = ((uint64_t)a << 32) | b;
    return ((uint32_t)(pair >> (48 - 8 * k)) & 0xFFFEu) == 0xFFF8u;
}

// K1a: the sync-pattern positions, streamed: a lane takes one 16-byte load
// (plus the next chunk's first word for a pattern straddling the chunks)
// and appends its hits to the list -- the rare lanes with a hit do one
// atomic each; no header is parsed here, so the pass runs at streaming rate
// (the single-pass scan parsed each hit's header in place, serialising its
// dependent loads on the wave that found it: 1.0 ms per config-2 batch).
// Only the bytes inside tracks are read: the host lists them as segments of
// at most kSegChunks 16-byte chunks (a batch laid out in per-track output
// slots, as the encoder leaves it, is half gaps); a workgroup streams one
// segment at a time.
constexpr uint32_t kSegChunks = 4096; // 64 KB

struct ScanSeg {
    uint64_t c0; // first 16-byte chunk
    uint32_t n;  // chunks
    uint32_t pad;
};

__global__ __launch_bounds__(256) void k_dec_sync(const uint32_t *__restrict__ w, uint64_t nw,
                                                  uint64_t len, const ScanSeg *__restrict__ segs,
                                                  uint32_t nseg, uint32_t *__restrict__ nhit,
                                                  uint64_t hcap, uint64_t *__restrict__ hits)
{
    // the workgroup's hits gather in LDS and go out with one global atomic
    // per workgroup: one atomic per hit-holding wave (~80 k, one address)
    // held the pass at 0.87 ms whatever the bytes scanned
    constexpr uint32_t kLocal = 2048;
    __shared__ uint64_t lpos[kLocal];
    __shared__ uint32_t lcnt, lbase;
    if (threadIdx.x == 0)
        lcnt = 0;
    __syncthreads();
    const bool a16 = ((uintptr_t)w & 15u) == 0; // the API promises 4-byte alignment only
    for (uint32_t sg = blockIdx.x; sg < nseg; sg += gridDim.x)
    for (uint64_t c = segs[sg].c0 + threadIdx.x, ce = segs[sg].c0 + segs[sg].n; c < ce;
         c += blockDim.x) {
        uint32_t v[5];
        if (a16 && 4 * c + 4 <= nw) {
            const uint4 q = *(const uint4 *)(w + 4 * c);
            v[0] = q.x;
            v[1] = q.y;
            v[2] = q.z;
            v[3] = q.w;
        } else {
#pragma unroll
            for (int i = 0; i < 4; ++i)
                v[i] = 4 * c + i < nw ? w[4 * c + i] : 0u;
        }
        v[4] = 4 * c + 4 < nw ? w[4 * c + 4] : 0u;
        uint32_t m = 0; // bit 4j+k: a sync pattern at byte 4j+k of the chunk
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t a = bswap32(v[j]), b = bswap32(v[j + 1]);
#pragma unroll
            for (int k = 0; k < 4; ++k)
                m |= sync_at(a, b, k) ? 1u << (4 * j + k) : 0u;
        }
        while (m) {
            const int bit = __builtin_ctz(m);
            m &= m - 1;
            const uint64_t p = 16 * c + (uint64_t)bit;
            const uint64_t pp = p < len ? p : len; // (a pattern in the pad past len)
            const uint32_t i = atomicAdd(&lcnt, 1u);
            if (i < kLocal) {
                lpos[i] = pp;
            } else { // a dense run of patterns: straight to the list
                const uint32_t g = atomicAdd(nhit, 1u);
                if (g < hcap) // over capacity: the host re-scans with room for all
                    hits[g] = pp;
            }
        }
    }
    __syncthreads();
    const uint32_t nl = min(lcnt, kLocal);
    if (threadIdx.x == 0)
        lbase = nl ? atomicAdd(nhit, nl) : 0u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nl; i += blockDim.x)
        if (lbase + i < hcap)
            hits[lbase + i] = lpos[i];
}

// K1b: lane per sync position: the full frame-header parse (CRC-8 and the
// STREAMINFO checks, flac.c:710-851); survivors are the candidates
// (cand_pos[i], cand_idx[byte] = i)
__global__ __launch_bounds__(256) void k_dec_hdr(const uint32_t *__restrict__ w, uint64_t nw,
                                                 uint64_t len, const DecTrack *__restrict__ tr,
                                                 uint32_t nt, const uint32_t *__restrict__ nhit,
                                                 uint64_t hcap, const uint64_t *__restrict__ hits,
                                                 uint32_t *__restrict__ ncand, uint32_t cap,
                                                 uint64_t *__restrict__ cand_pos,
                                                 uint32_t *__restrict__ cand_idx,
                                                 uint32_t *__restrict__ cand_trk,
                                                 unsigned long long *__restrict__ cbits)
{
    const uint64_t n = min((uint64_t)*nhit, hcap);
    for (uint64_t h = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; h < n;
         h += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t p = hits[h];
        if (p + 1 >= len)
            continue;
        const uint32_t t = find_track(tr, nt, p);
        const DecTrack T = tr[t];
        if (p < T.start || p >= T.end)
            continue;
        BitR r;
        r.init(w, nw, p * 8, T.end * 8);
        Hdr hd;
        if (dec_header(r, T, hd) != FD_OK)
            continue;
        const uint32_t i = atomicAdd(ncand, 1u);
        if (i < cap) { // over capacity: the host re-scans with room for all
            cand_pos[i] = p;
            cand_idx[p] = i;
            cand_trk[i] = t;
        }
        if (cbits) // the candidate bitmap of the frame-end hypothesis (k_dec_spec)
            atomicOr(&cbits[p >> 6], 1ull << (p & 63u));
    }
}

// K2: parse every candidate frame (grid-stride; the count lives on device)
__global__ __launch_bounds__(64) void k_dec_parse(const uint32_t *__restrict__ w, uint64_t nw,
                                                  const DecTrack *__restrict__ tr, uint32_t nt,
                                                  const uint32_t *__restrict__ ncand,
                                                  const uint64_t *__restrict__ cand_pos,
                                                  const uint32_t *__restrict__ cand_trk,
                                                  const uint32_t *__restrict__ spec,
                                                  ParseRec *__restrict__ recs)
{
    __shared__ __align__(16) uint32_t ring[64 * kRingStride]; // the lanes' residual-word rings
    const uint32_t n = *ncand;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const uint64_t p = cand_pos[i];
        const DecTrack t = tr[cand_trk[i]];
        ParseRec rec;
        // (the frame's CRC-16 is k_dec_crc's)
        parse_frame<true, false>(w, nw, p, t, ~0ull, nullptr, rec, ring + threadIdx.x * kRingStride,
                                 spec ? spec[i] : 0u);
        recs[i] = rec;
    }
}

// CRC-16 advance: the state after 2^m more zero bytes (GF(2) matrix m)
__device__ __forceinline__ uint32_t dcrc_adv(uint32_t c, int m)
{
    uint32_t r = 0;
#pragma unroll
    for (int i = 0; i < 16; ++i)
        r ^= ((c >> i) & 1u) ? (uint32_t)c_crc_adv[m][i] : 0u;
    return r;
}

// big-endian 32 bits at absolute byte b of the buffer (two aligned loads)
__device__ __forceinline__ uint32_t be32_at(const uint32_t *w, uint64_t last, uint64_t b)
{
    const uint64_t i = b >> 2;
    const uint32_t x = bswap32(w[i < last ? i : last]);
    const uint32_t r = (uint32_t)(b & 3u);
    if (!r)
        return x;
    const uint32_t y = bswap32(w[i + 1 < last ? i + 1 : last]);
    return (x << (8u * r)) | (y >> (32u - 8u * r));
}

// CRC-16 residue of bytes [pos, pos + L) on one wave (0 for an intact
// frame: header to CRC bytes): 64 chunks of Lc = 2^m bytes of a virtually
// zero-prefixed image (leading zeros leave a zero-init CRC unchanged),
// slicing by 4 from LDS tables, tree-combined with the advance matrices.
// Wave-uniform arguments; the result is returned in every lane.
__device__ uint32_t wave_crc16(const uint32_t *__restrict__ w, uint64_t nw, uint64_t pos, uint32_t L,
                               const uint16_t (*T)[256], uint32_t lane)
{
    if (L > (64u << 17)) { // beyond any real frame (the matrices reach 2^23)
        const uint32_t c = lane == 0 ? crc16_range(w, pos, pos + L, T) : 0u;
        return (uint32_t)__shfl((int)c, 0, 64);
    }
    uint32_t lc_log = 2;
    while ((64u << lc_log) < L)
        lc_log++;
    const uint32_t Lc = 1u << lc_log;
    const int64_t z = (int64_t)(64u << lc_log) - (int64_t)L;
    uint32_t crc = 0;
    int64_t q = (int64_t)lane * Lc - z; // image byte of this lane's first group
    const int64_t qe = q + Lc;
    if (q < 0) { // groups in the zero prefix leave crc = 0
        q += ((-q) >> 2) << 2; // now -4 < q <= 0
        if (q < 0 && q < qe) {
            const uint32_t t = be32_at(w, nw - 1, pos) >> (8u * (uint32_t)(-q));
            crc = (uint32_t)T[3][t >> 24] ^ T[2][(t >> 16) & 0xFFu] ^ T[1][(t >> 8) & 0xFFu] ^
                  T[0][t & 0xFFu];
            q += 4;
        }
    }
    // 256 bytes at a time: the 65 aligned words under them loaded at once
    // (one memory latency per 256 bytes of the lane's chunk -- the wave
    // spent 94 % of its cycles waiting with a latency per 64 bytes,
    // profiles/r04_k_dec_pmc.txt), then the 64 big-endian words
    for (; q + 256 <= qe; q += 256) {
        const uint64_t b0 = pos + (uint64_t)q, i0 = b0 >> 2;
        const uint32_t sb = 8u * (uint32_t)(b0 & 3);
        uint32_t x[65];
#pragma unroll
        for (int u = 0; u < 65; ++u)
            x[u] = bswap32(w[i0 + u < nw - 1 ? i0 + u : nw - 1]);
#pragma unroll
        for (int u = 0; u < 64; ++u) {
            const uint32_t wd = sb ? (x[u] << sb) | (x[u + 1] >> (32u - sb)) : x[u];
            const uint32_t t = wd ^ (crc << 16);
            crc = (uint32_t)T[3][t >> 24] ^ T[2][(t >> 16) & 0xFFu] ^
                  T[1][(t >> 8) & 0xFFu] ^ T[0][t & 0xFFu];
        }
    }
    for (; q + 64 <= qe; q += 64) {
        uint32_t x[16];
#pragma unroll
        for (int u = 0; u < 16; ++u)
            x[u] = be32_at(w, nw - 1, pos + (uint64_t)(q + 4 * u));
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const uint32_t t = x[u] ^ (crc << 16);
            crc = (uint32_t)T[3][t >> 24] ^ T[2][(t >> 16) & 0xFFu] ^
                  T[1][(t >> 8) & 0xFFu] ^ T[0][t & 0xFFu];
        }
    }
    for (; q < qe; q += 4) {
        const uint32_t t = be32_at(w, nw - 1, pos + (uint64_t)q) ^ (crc << 16);
        crc = (uint32_t)T[3][t >> 24] ^ T[2][(t >> 16) & 0xFFu] ^ T[1][(t >> 8) & 0xFFu] ^
              T[0][t & 0xFFu];
    }
#pragma unroll
    for (int k = 0; k < 6; ++k) {
        const uint32_t other = (uint32_t)__shfl_down((int)crc, 1 << k, 64);
        if ((lane & ((2u << k) - 1u)) == 0)
            crc = dcrc_adv(crc, (int)lc_log + k) ^ other;
    }
    return (uint32_t)__shfl((int)crc, 0, 64);
}

// K2b: CRC-16 of every parsed candidate frame whose length the parse walked
// (a wave per frame, wave_crc16; frames the speculative pass measured are
// checked already).  The serial per-lane CRC in k_dec_parse cost 0.8 of its
// 4.7 ms (profiles/r04_h_dec_probe.jsonl).
__global__ __launch_bounds__(256) void k_dec_crc(const uint32_t *__restrict__ w, uint64_t nw,
                                                 const uint32_t *__restrict__ ncand,
                                                 const uint64_t *__restrict__ cand_pos,
                                                 ParseRec *__restrict__ recs)
{
    __shared__ uint16_t T[4][256];
    load_crc_lds(T);
    const uint32_t n = *ncand;
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6); i < n; i += gridDim.x * 4u) {
        const int st = recs[i].status;
        const uint32_t L = recs[i].bytes;
        if (st != FD_OK || L < 2u || recs[i].pad) // wave-uniform: one candidate per wave
            continue;
        if (wave_crc16(w, nw, cand_pos[i], L, T, lane) && lane == 0)
            recs[i].status = FD_FRAME_CRC;
    }
}

// The frame-end hypothesis (K2s, before the parse): for candidate p, the
// next candidates q (the bitmap k_dec_hdr set, bounded by the track end) in
// turn, up to three: the first whose bytes [p, q) carry a zero CRC-16 residue
// is taken as the frame, so the parse need not walk the frame's last
// subframe -- its start is the end of the one before, its end is q.  A
// frame with no such q (corrupt, cut by the window, or followed by bytes no
// candidate starts) gets 0: the parse walks every subframe and k_dec_crc
// checks the walked length, as before.  The restore checks every taken
// hypothesis on the subframe it walks anyway (k_dec_subframe: no error,
// aligned end + 16 bits == q); a failed check makes decode_wait redo the
// batch with the full parse, so the results are the walked parse's.
constexpr uint32_t kSpecTries = 3;
constexpr uint32_t kSpecMaxBytes = 1u << 22;

__device__ __forceinline__ uint64_t next_cand(const unsigned long long *__restrict__ cbits,
                                              uint64_t nwords, uint64_t from, uint64_t te,
                                              uint32_t lane)
{
    uint64_t wi = from >> 6;
    bool first = true;
    while (wi * 64u < te) {
        const uint64_t k = wi + lane;
        unsigned long long x = k < nwords && k * 64u < te ? cbits[k] : 0ull;
        if (first && lane == 0)
            x &= ~0ull << (from & 63u);
        first = false;
        const unsigned long long b = __ballot(x != 0ull);
        if (b) {
            const uint32_t f = (uint32_t)__builtin_ctzll(b);
            const unsigned long long xf = (unsigned long long)__shfl((long long)x, (int)f, 64);
            const uint64_t q = (wi + f) * 64u + (uint64_t)__builtin_ctzll(xf);
            return q < te ? q : te;
        }
        wi += 64u;
    }
    return te;
}

__global__ __launch_bounds__(256) void k_dec_spec(const uint32_t *__restrict__ w, uint64_t nw,
                                                  const DecTrack *__restrict__ tr, uint32_t nt,
                                                  const uint32_t *__restrict__ ncand,
                                                  const uint64_t *__restrict__ cand_pos,
                                                  const uint32_t *__restrict__ cand_trk,
                                                  const unsigned long long *__restrict__ cbits,
                                                  uint64_t nwords, uint32_t *__restrict__ spec)
{
    __shared__ uint16_t T[4][256];
    load_crc_lds(T);
    const uint32_t n = *ncand;
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t i = blockIdx.x * 4u + (threadIdx.x >> 6); i < n; i += gridDim.x * 4u) {
        const uint64_t p = cand_pos[i];
        const uint64_t te = tr[cand_trk[i]].end;
        uint32_t out = 0;
        uint64_t from = p + 1u;
        for (uint32_t k = 0; k < kSpecTries && !out; ++k) {
            const uint64_t q = next_cand(cbits, nwords, from, te, lane);
            if (q <= p + 2u || q - p > kSpecMaxBytes)
                break;
            if (wave_crc16(w, nw, p, (uint32_t)(q - p), T, lane) == 0u)
                out = (uint32_t)(q - p);
            if (q >= te)
                break;
            from = q + 1u;
        }
        if (lane == 0)
            spec[i] = out;
    }
}

// K3: the read() loop per track (flac.c:196-258); pass 1 counts, pass 2
// writes frames and subframe jobs
__global__ __launch_bounds__(64) void k_dec_chain(const uint32_t *__restrict__ w, uint64_t nw,
                                                  const DecTrack *__restrict__ tr, uint32_t nt,
                                                  const uint32_t *__restrict__ ncand,
                                                  const uint64_t *__restrict__ cand_pos,
                                                  const uint32_t *__restrict__ cand_idx,
                                                  const ParseRec *__restrict__ recs,
                                                  DecCount *__restrict__ counts, int pass,
                                                  DecFrame *__restrict__ frames,
                                                  uint2 *__restrict__ jobs)
{
    __shared__ uint16_t T[4][256];
    load_crc_lds(T);
    const uint32_t ti = blockIdx.x * blockDim.x + threadIdx.x;
    if (ti >= nt)
        return;
    const DecTrack t = tr[ti];
    const uint32_t nc = *ncand;
    uint64_t pos = t.start, remaining = t.total, pcm = 0, crc_pcm = 0;
    uint32_t nf = 0, crc_frame = 0xFFFFFFFFu;
    int status = FD_OK;
    while (remaining != 0) {
        ParseRec rec;
        uint32_t ci = 0xFFFFFFFFu;
        if (pos < t.end) {
            const uint32_t c = cand_idx[pos];
            if (c < nc && cand_pos[c] == pos)
                ci = c;
        }
        if (ci != 0xFFFFFFFFu && (uint64_t)recs[ci].bs <= remaining)
            rec = recs[ci];
        else // not a candidate (its header fails), or truncated by remaining
            parse_frame(w, nw, pos, t, remaining, T, rec);
        // a bad CRC-16 does not change the frame's length: read() raises at
        // it (flac.c:251-255), offsets() never checks it (flac.c:413-415)
        if (rec.status == FD_FRAME_CRC) {
            if (crc_frame == 0xFFFFFFFFu) {
                crc_frame = nf;
                crc_pcm = pcm;
            }
        } else if (rec.status) {
            status = rec.status;
            break;
        }
        const uint32_t N = (uint32_t)((uint64_t)rec.bs < remaining ? (uint64_t)rec.bs : remaining);
        if (pass == 2) {
            const uint64_t slot = t.frame_base + nf;
            DecFrame f;
            f.pos = pos;
            f.pcm_start = t.pcm_base + pcm * t.channels;
            f.n = N;
            f.track = ti;
            f.bs = rec.bs;
            f.assign = rec.assign;
            f.ch = rec.ch;
            f.bps = rec.bps;
            f.spec = rec.pad;
            f.bytes = rec.bytes;
            f.pad = 0;
            for (int c = 0; c < 8; ++c)
                f.sub_bit[c] = rec.sub_bit[c];
            frames[slot] = f;
            for (uint32_t c = 0; c < rec.ch; ++c)
                jobs[t.job_base + (uint64_t)nf * rec.ch + c] = make_uint2((uint32_t)slot, c);
        }
        ++nf;
        pcm += N;
        pos += rec.bytes;
        remaining -= rec.bs; // uint64, wraps as the reference's
    }
    if (pass == 1) {
        DecCount dc;
        dc.pcm_frames = pcm;
        dc.n_frames = nf;
        dc.status = status;
        dc.crc_pcm = crc_pcm;
        dc.crc_frame = crc_frame;
        dc.pad = 0;
        dc.stop = pos - t.start;
        counts[ti] = dc;
    }
}

template <int W>
__device__ __forceinline__ bool restore_win(BitR &r, uint32_t N, uint32_t bps, uint32_t wasted,
                                            uint32_t kind, uint32_t order, int32_t *out,
                                            int4 *row, JobMeta &m, bool allow_fast,
                                            uint32_t *ring, int &rc)
{
    WinPred<W> p;
    p.row = row;
    p.q0 = p.q1 = p.q2 = p.q3 = 0;
    p.porder = 0;
    p.n = N;
    p.i = 0;
    p.wasted = wasted;
    p.shift = 0;
    p.bad = false;
#pragma unroll
    for (int j = 0; j < W; ++j) {
        p.c[j] = 0;
        p.h[j] = 0;
    }
    for (uint32_t j = 0; j < order; ++j) // warm-up samples enter the window
        p.warm(r.get_signed(bps));
    uint32_t sum_abs = 0;
    if (kind == 3) {
        const uint32_t prec = r.get(4) + 1;
        p.shift = (uint32_t)r.get_signed(5) & 63u;
        for (uint32_t k = 0; k < order; ++k) {
            const int32_t v = r.get_signed(prec);
            sum_abs += (uint32_t)(v < 0 ? -v : v);
#pragma unroll
            for (int j = 0; j < W; ++j)
                p.c[j] = (uint32_t)j == k ? v : p.c[j];
        }
    } else { // FIXED order 0..4: coefficients of the difference polynomial
        const int32_t o = (int32_t)(order < 5 ? order : 4);
        p.c[0] = o;                                  // 0, 1, 2, 3, 4
        p.c[1] = o == 2 ? -1 : o == 3 ? -3 : o == 4 ? -6 : 0;
        p.c[2] = o == 3 ? 1 : o == 4 ? 4 : 0;
        p.c[3] = o == 4 ? -1 : 0;
        sum_abs = o == 4 ? 15u : o == 3 ? 7u : o == 2 ? 3u : (uint32_t)o;
    }
    // int32 is exact while every sample is inside the bps range (see WinPred)
    p.half = bps >= 1 && bps <= 24 ? 1u << (bps - 1) : 0u;
    p.fast = allow_fast && p.half && (uint64_t)sum_abs * p.half < 0x80000000ull;
    if ((((uintptr_t)r.w) & 15u) == 0 && r.last >= kWalkInit * kRingB)
        rc = walk_residual<true>(r, order, N, p, ring);
    else
        rc = dec_residual<WinPred<W>, false>(r, order, N, p);
    p.flush();
    m.porder = (uint8_t)p.porder;
    m.iters = p.i;
    return p.fast && p.bad;
}

// K4: one subframe per lane.  Every sample (warm-up, restored or verbatim)
// goes to the job's column of the wave's [sample/4][lane][4] scratch
// (coalesced 16-byte stores); K5 gathers 4 samples of a job per load.
__global__ __launch_bounds__(64) void k_dec_subframe(const uint32_t *__restrict__ w, uint64_t nw,
                                                     const DecTrack *__restrict__ tr,
                                                     const DecFrame *__restrict__ frames,
                                                     const uint2 *__restrict__ jobs,
                                                     uint64_t njobs, int32_t *__restrict__ warm,
                                                     int32_t *__restrict__ rows, uint32_t nrows,
                                                     JobMeta *__restrict__ meta,
                                                     uint32_t *__restrict__ spec_bad)
{
    __shared__ __align__(16) uint32_t rings[64 * kRingStride]; // the lanes' residual-word rings
    uint32_t *ring = rings + threadIdx.x * kRingStride;
    const uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= njobs)
        return;
    const uint2 jb = jobs[j];
    const DecFrame &f = frames[jb.x];
    const uint32_t c = jb.y;
    BitR r;
    r.init(w, nw, f.pos * 8 + f.sub_bit[c], tr[f.track].end * 8);
    const uint32_t N = f.n;
    int32_t *out = warm + j * 32u; // warm-up samples (orders <= 32)
    // [row/4][lane][4] scratch: this lane's 16-byte cells, every 64th int4
    int4 *row = (int4 *)(rows + (uint64_t)blockIdx.x * nrows * 64) + threadIdx.x;
    JobMeta m;
    m.kind = 3;
    m.order = 0;
    m.porder = 0;
    m.pad = 0;
    m.value = 0;
    m.iters = 0;
    m.pad2 = 0;
    SubHdr sh;
    int rc = dec_subhdr(r, sh);
    if (rc == FD_OK) {
        const uint32_t bps = sub_bps(f.assign, c, f.bps) - sh.wasted;
        const uint32_t ws = sh.wasted;
        if (sh.kind == 0) {
            m.kind = 0;
            m.value = (int32_t)((uint32_t)r.get_signed(bps) << ws);
        } else if (sh.kind == 1) {
            m.kind = 1;
            m.iters = N;
            if (bps >= 1 && bps <= 32) {
                // sample i sits at a known bit offset: the loads of a group
                // of four are independent (no chain through the reader)
                const uint64_t b0 = r.abspos();
                for (uint32_t i = 0; i < N; i += 4) {
                    int32_t v[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const uint64_t b = b0 + (uint64_t)(i + q) * bps;
                        const uint64_t wi = b >> 5;
                        const uint32_t a = bswap32(w[wi < r.last ? wi : r.last]);
                        const uint32_t c = bswap32(w[wi + 1 < r.last ? wi + 1 : r.last]);
                        const uint32_t sb = (uint32_t)(b & 31);
                        const uint32_t x = sb ? (a << sb) | (c >> (32 - sb)) : a;
                        v[q] = (int32_t)((uint32_t)((int32_t)x >> (32 - bps)) << ws);
                    }
                    row[(uint64_t)(i >> 2) * 64] = make_int4(v[0], v[1], v[2], v[3]);
                }
                r.skip_far((uint64_t)N * bps);
            } else {
                for (uint32_t i = 0; i < N; ++i)
                    ((int32_t *)(row + (uint64_t)(i >> 2) * 64))[i & 3] =
                        (int32_t)((uint32_t)r.get_signed(bps) << ws);
            }
        } else {
            m.kind = 2;
            m.order = (uint8_t)sh.order;
            if (sh.order <= 12) {
                const uint32_t at = r.pos;
                if (restore_win<12>(r, N, bps, ws, sh.kind, sh.order, out, row, m, true, ring,
                                    rc)) {
                    r.pos = at; // a sample left the bps range: redo with int64 sums
                    restore_win<12>(r, N, bps, ws, sh.kind, sh.order, out, row, m, false, ring,
                                    rc);
                }
            } else {
                restore_win<32>(r, N, bps, ws, sh.kind, sh.order, out, row, m, false, ring, rc);
            }
            if (sh.kind == 2 && sh.order > 4)
                rc = FD_FIXED_ORDER;
        }
    }
    meta[j] = m;
    // the frame-end hypothesis (k_dec_spec) on the subframe the parse did
    // not walk: the walk the parse would have made must end, byte-aligned,
    // 16 bits before the hypothesised end, without an error
    if (f.spec && c + 1u == f.ch) {
        const uint64_t e = r.abspos() - f.pos * 8u;
        if (rc != FD_OK || r.eof() || ((e + 7u) >> 3) + 2u != (uint64_t)f.bytes)
            *spec_bad = 1u;
    }
}

// K5: rows -> samples -> flacdec_decorrelate_channels (flac.c:1212-1269) ->
// the interleaved FrameList int32 and the little-endian byte stream of
// FrameList.to_bytes (MD5 input), in one pass.  Block = the frames whose
// first (frame, channel) job lies in 64-job slot blockIdx.x (their other
// channels' jobs may run into the next slot).  The block's frame and job
// descriptors are read once into LDS.  Per tile of kEmitTile samples: lane
// l of every wave gathers job l's samples (x = wave, wave + 4, ...) from the
// K4 row scratch -- adjacent lanes read adjacent 16-byte cells -- or the
// warm-up cell into an LDS tile; then each wave writes whole frames (frame
// k on wave k mod 4), channel-interleaved and contiguous.
constexpr uint32_t kEmitTile = 64;
constexpr uint32_t kEmitJobs = 64 + 7;

__global__ __launch_bounds__(256) void k_dec_emit(const DecTrack *__restrict__ tr,
                                                  const DecFrame *__restrict__ frames,
                                                  const uint2 *__restrict__ jobs, uint64_t njobs,
                                                  const JobMeta *__restrict__ meta,
                                                  const int32_t *__restrict__ rows, uint32_t nrows,
                                                  const int32_t *__restrict__ warm,
                                                  int32_t *__restrict__ pcm,
                                                  uint8_t *__restrict__ bytes)
{
    __shared__ int32_t tile[kEmitJobs][kEmitTile + 1];
    __shared__ JobMeta jm[kEmitJobs];
    // the block's frames: first job (slot-relative), samples, channels,
    // assignment, bytes per MD5 sample, the bps clamp, output positions
    __shared__ uint32_t fj[64], fn[64], fch[64], fas[64], fbb[64];
    __shared__ int32_t fhi[64];
    __shared__ uint64_t fpcm[64], fmd5[64];
    __shared__ uint32_t nfr, nj, maxn;
    const uint64_t j0 = (uint64_t)blockIdx.x * 64;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    if (tid < 64) {
        const uint64_t j = j0 + tid;
        const bool start = j < njobs && jobs[j].y == 0u;
        const uint64_t bal = __ballot(start);
        const uint32_t nf = (uint32_t)__popcll(bal);
        uint32_t jend = 0, n = 0;
        if (start) {
            const uint32_t k = (uint32_t)__popcll(bal & ((1ull << tid) - 1ull));
            const DecFrame f = frames[jobs[j].x];
            const DecTrack t = tr[f.track];
            const uint32_t bb = (t.bps + 7u) / 8u;
            fj[k] = tid;
            fn[k] = f.n;
            fch[k] = f.ch;
            fas[k] = f.assign;
            fbb[k] = bb;
            // FrameList.to_bytes saturates samples outside the bps range
            // (src/pcm.c:1826-1948): only a corrupt stream can produce them
            fhi[k] = t.bps >= 1 && t.bps <= 31 ? (int32_t)((1u << (t.bps - 1)) - 1u) : 0x7FFFFFFF;
            fpcm[k] = f.pcm_start;
            fmd5[k] = t.md5_base + (f.pcm_start - t.pcm_base) * bb;
            jend = tid + (uint32_t)f.ch;
            n = f.n;
        }
        jend = wave_max_u32(jend);
        n = wave_max_u32(n);
        if (tid == 0) {
            nfr = nf;
            nj = jend;
            maxn = n;
        }
    }
    __syncthreads();
    const uint32_t NJ = min(nj, kEmitJobs), NF = nfr;
    if (tid < NJ) {
        const uint64_t j = j0 + tid;
        JobMeta m;
        m.kind = 3;
        m.order = 0;
        m.porder = 0;
        m.iters = 0;
        m.value = 0;
        if (j < njobs)
            m = meta[j];
        jm[tid] = m;
    }
    __syncthreads();
    for (uint32_t i0 = 0; i0 < maxn; i0 += kEmitTile) {
        // gather: lane = job; K4 left every FIXED/LPC/VERBATIM job's samples
        // (warm-up included) in sample order, [sample / 4][lane][4] per 64-job
        // slot, so wave wv's 16 samples [16 wv, 16 wv + 16) of a job are four
        // 16-byte loads (adjacent lanes: adjacent cells)
        for (uint32_t l = lane; l < NJ; l += 64) {
            const JobMeta m = jm[l];
            const uint64_t j = j0 + l;
            const int4 *__restrict__ cell =
                (const int4 *)(rows + (j >> 6) * nrows * 64u) + (j & 63u);
            const uint32_t xa = 16u * wv, ia = i0 + xa;
            int4 q[4];
            if (m.kind == 1 || m.kind == 2) {
#pragma unroll
                for (int c4 = 0; c4 < 4; ++c4)
                    q[c4] = cell[(uint64_t)((ia >> 2) + c4) * 64];
            } else {
                const int32_t v = m.kind == 0 ? m.value : 0;
#pragma unroll
                for (int c4 = 0; c4 < 4; ++c4)
                    q[c4] = make_int4(v, v, v, v);
            }
#pragma unroll
            for (int c4 = 0; c4 < 4; ++c4) {
                tile[l][xa + 4 * c4] = q[c4].x;
                tile[l][xa + 4 * c4 + 1] = q[c4].y;
                tile[l][xa + 4 * c4 + 2] = q[c4].z;
                tile[l][xa + 4 * c4 + 3] = q[c4].w;
            }
        }
        __syncthreads();
        // write: wave wv takes frames wv, wv + 4, ...; lane = sample of the
        // tile, all its channels (stereo: one 8-byte PCM store and one
        // 4-byte MD5 store per lane, 512 + 256 contiguous bytes per wave)
        for (uint32_t k = wv; k < NF; k += 4) {
            const uint32_t n = fn[k];
            const uint32_t left = n > i0 ? min(n - i0, kEmitTile) : 0u;
            if (lane >= left)
                continue;
            const uint32_t ch = fch[k], as = fas[k], l = fj[k], bb = fbb[k], x = lane;
            const int32_t hi = fhi[k], lo = -hi - 1;
            int32_t *__restrict__ dst = pcm + fpcm[k] + (uint64_t)(i0 + x) * ch;
            uint8_t *__restrict__ bdst = bytes + fmd5[k] + (uint64_t)(i0 + x) * ch * bb;
            if (ch == 2) {
                const int32_t a = tile[l][x], b = tile[l + 1][x];
                int32_t o0 = a, o1 = b;
                if (as == 8) {
                    o1 = (int32_t)((uint32_t)a - (uint32_t)b);
                } else if (as == 9) {
                    o0 = (int32_t)((uint32_t)a + (uint32_t)b);
                } else if (as == 10) {
                    const int64_t mid = (int64_t)((uint64_t)(int64_t)a << 1) | (b & 1);
                    o0 = (int32_t)((mid + b) >> 1);
                    o1 = (int32_t)((mid - b) >> 1);
                }
                *(int2 *)dst = make_int2(o0, o1);
                // FrameList.to_bytes saturates samples outside the bps range
                // (src/pcm.c:1826-1948): only a corrupt stream can produce them
                const int32_t v0 = o0 > hi ? hi : (o0 < lo ? lo : o0);
                const int32_t v1 = o1 > hi ? hi : (o1 < lo ? lo : o1);
                if (bb == 2) {
                    *(uint32_t *)bdst = ((uint32_t)v0 & 0xFFFFu) | ((uint32_t)v1 << 16);
                } else {
                    for (uint32_t q = 0; q < bb; ++q) {
                        bdst[q] = (uint8_t)((uint32_t)v0 >> (8 * q));
                        bdst[bb + q] = (uint8_t)((uint32_t)v1 >> (8 * q));
                    }
                }
            } else {
                for (uint32_t c = 0; c < ch; ++c) {
                    const int32_t o = tile[l + c][x];
                    dst[c] = o;
                    const int32_t v = o > hi ? hi : (o < lo ? lo : o);
                    if (bb == 2)
                        *(int16_t *)(bdst + 2u * c) = (int16_t)v;
                    else
                        for (uint32_t q = 0; q < bb; ++q)
                            bdst[c * bb + q] = (uint8_t)((uint32_t)v >> (8 * q));
                }
            }
        }
        __syncthreads();
    }
}

const int kDecTimed = 7;
const char *kDecNames[kDecTimed] = {"dec_scan",     "dec_parse", "dec_chain", "dec_subframe",
                                    "dec_emit",     "dec_md5",   "dec_total"};

} // namespace

thread_local std::string g_dec_err;

static atg_status dfail(atg_status s, const std::string &m)
{
    g_dec_err = m;
    return s;
}

#define DHIP(expr)                                                                         \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return dfail(ATG_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

struct DBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes)
    {
        if (bytes <= cap && p)
            return hipSuccess;
        if (p)
            (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes, 256);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess)
            cap = want;
        return e;
    }
    void release()
    {
        if (p)
            (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

// One batch in flight: its PCM / MD5 byte buffers, the MD5 stream, and the
// host copies its results are computed from.  Three slots let batch k's
// restore, emit and per-track MD5 (on the slot's stream, with the slot's
// frame table, jobs and row scratch) run beside batch k+1's scan, parse and
// chain on the decoder stream: a batch's MD5 chains (~12 ms per 1 MB track,
// whatever the batch width) outlast its scan-to-emit path, and a slot is
// free again only after them (config 2, 30 steps: 14.4 ms per step with
// two slots, 11.1 with three, 13.4 with four -- more batches in flight only
// add contention; profiles/r03_f_decode_slots.txt).
//
// atg_decoder_set_inflight raises the rotation up to kDecMaxSlots: from 4
// slots on the batches' MD5 chains are rolled (as the encoder's, md5.hip
// k_bytes_md5_roll): every batch in flight advances by one slice per
// enqueue, in ONE launch on the decoder's MD5 stream, so more batches in
// flight no longer queue their chains behind one another on shared hardware
// queues (the 13.4 ms at four slots above).
constexpr int kDecSlots = 3;
constexpr uint32_t kSpecStreak = 4; // redone batches in a row before mode 0
constexpr int kDecMaxSlots = 16;
struct DecSlot {
    DBuf pcm, bytes, md5, md5meta;
    DBuf tracks, frames, jobs, warm, rows, meta; // the restore's tables and scratch
    hipStream_t s_md5 = nullptr;       // the slot's stream: restore, emit, MD5
    hipEvent_t ev[kDecTimed + 1] = {}; // phase events (emit end = ev[5])
    hipEvent_t ev_chain = nullptr;     // the chain's second pass is done (decoder stream)
    hipEvent_t ev_done = nullptr;
    uint8_t *md5_h = nullptr;          // pinned
    size_t md5_cap = 0;
    std::vector<DecTrack> tr;
    std::vector<DecCount> cnt;
    std::vector<uint64_t> md5_meta;    // offsets then lengths (upload source)
    std::vector<atg_flac_dec_track> want; // the caller's tracks (STREAMINFO MD5)
    uint64_t total_samples = 0, total_frames = 0;
    uint64_t ticket = 0;
    bool busy = false;
    // rolled mode: the chains in roll_parts slices on d->s_roll
    bool rolled = false;
    uint32_t roll_parts = 0, roll_done = 0;
    uint32_t n_md5 = 0; // streams hashed (the batch's track count)
    // the batch's input (decode_wait redoes it with the full parse when a
    // frame-end hypothesis fails the restore's check)
    const uint8_t *data = nullptr;
    uint64_t len = 0;
    bool spec = false; // k_dec_spec ran for this batch
};

struct atg_decoder {
    std::recursive_mutex mu; // held by every public entry point (handle_lock.h)
    int device = 0;
    hipStream_t s = nullptr;
    float times[kDecTimed] = {};
    bool have_times = false;
    DBuf data, tracks, counts, ncand, cand_pos, cand_idx, recs, hits, segs;
    DBuf cand_trk;    // each candidate's track (k_dec_hdr)
    DBuf cbits, spec; // the frame-end hypothesis: candidate bitmap, lengths
    int spec_mode = 1; // atg_decoder_set_frame_hypothesis
    uint64_t spec_redos = 0; // batches redone with the full parse
    uint32_t spec_streak = 0; // consecutive batches redone
    bool spec_off = false; // set while a batch is redone with the full parse
    std::vector<ScanSeg> segs_h; // the scan's segments (upload source)
    DecSlot slot[kDecMaxSlots];
    int depth = kDecSlots;          // slots in rotation (atg_decoder_set_inflight)
    hipStream_t s_roll = nullptr;   // rolled mode: every batch's MD5 slices and tails
    std::vector<DecSlot *> roll_q;  // rolled batches with slices to run, oldest first
    uint64_t next_ticket = 1;
    int last = -1; // slot of the last waited batch (decode_fetch)
};

static void build_dec_adv(const uint16_t t16[4][256], uint16_t adv[24][16])
{
    // adv[0]: one zero byte; adv[m] = adv[m-1] applied twice
    for (int i = 0; i < 16; ++i) {
        uint32_t c = 1u << i;
        c = ((c << 8) ^ t16[0][(c >> 8) & 0xFFu]) & 0xFFFFu;
        adv[0][i] = (uint16_t)c;
    }
    for (int m = 1; m < 24; ++m)
        for (int i = 0; i < 16; ++i) {
            uint32_t v = adv[m - 1][i], r = 0;
            for (int j = 0; j < 16; ++j)
                if ((v >> j) & 1u)
                    r ^= adv[m - 1][j];
            adv[m][i] = (uint16_t)r;
        }
}

static void build_dec_tables(uint8_t *t8, uint16_t t16[4][256])
{
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t c8 = b;
        for (int i = 0; i < 8; ++i)
            c8 = (c8 & 0x80) ? ((c8 << 1) ^ 0x07) : (c8 << 1);
        t8[b] = (uint8_t)c8;
        uint32_t c = b << 8;
        for (int i = 0; i < 8; ++i)
            c = (c & 0x8000) ? ((c << 1) ^ 0x8005) : (c << 1);
        t16[0][b] = (uint16_t)c;
    }
    for (int k = 1; k < 4; ++k)
        for (uint32_t b = 0; b < 256; ++b) {
            const uint32_t p = t16[k - 1][b];
            t16[k][b] = (uint16_t)(((p << 8) & 0xFFFF) ^ t16[0][p >> 8]);
        }
}

static const uint32_t kMasks[9] = {0, 0x4, 0x3, 0x7, 0x33, 0x37, 0x3F, 0x70F, 0x63F};

extern "C" {

const char *atg_decoder_last_error(void) { return g_dec_err.c_str(); }

int atg_flac_read_metadata(const uint8_t *data, uint64_t len, atg_flac_streaminfo *si,
                           atg_flac_seekpoint *sp, uint32_t sp_cap)
{
    // flacdec_read_metadata (src/decoders/flac.c:568-707) over an in-memory
    // image: STREAMINFO, SEEKTABLE, the VORBIS_COMMENT channel-mask tag
    if (!si || (!data && len))
        return 1;
    std::memset(si, 0, sizeof(*si));
    uint64_t pos = 0; // bits
    const uint64_t lb = len * 8;
    bool eof = false;
    auto get = [&](unsigned n) -> uint32_t {
        uint32_t v = 0;
        for (unsigned i = 0; i < n; ++i) {
            if (pos >= lb) {
                eof = true;
                return 0;
            }
            v = (v << 1) | ((data[pos >> 3] >> (7 - (pos & 7))) & 1u);
            ++pos;
        }
        return v;
    };
    const uint32_t magic = get(32);
    if (eof)
        return 2;
    if (magic != 0x664C6143u)
        return 1;
    unsigned last;
    do {
        last = get(1);
        const unsigned type = get(7);
        const uint32_t blen = get(24);
        if (eof)
            return 2;
        const uint64_t body = pos;
        if (type == 0) {
            si->min_block_size = get(16);
            si->max_block_size = get(16);
            si->min_frame_size = get(24);
            si->max_frame_size = get(24);
            si->sample_rate = get(20);
            si->channels = get(3) + 1;
            si->bits_per_sample = get(5) + 1;
            si->total_samples = ((uint64_t)get(4) << 32);
            si->total_samples |= get(32);
            for (int i = 0; i < 16; ++i)
                si->md5[i] = (uint8_t)get(8);
            si->channel_mask = si->channels <= 8 ? kMasks[si->channels] : 0;
        } else if (type == 3) {
            const uint32_t n = blen / 18;
            for (uint32_t k = 0; k < n; ++k) {
                atg_flac_seekpoint p;
                p.sample_number = (uint64_t)get(32) << 32;
                p.sample_number |= get(32);
                p.byte_offset = (uint64_t)get(32) << 32;
                p.byte_offset |= get(32);
                p.samples = get(16);
                p.reserved = 0;
                if (sp && k < sp_cap)
                    sp[k] = p;
            }
            si->n_seekpoints = n;
        } else if (type == 4) {
            // flacdec_read_vorbis_comment (flac.c:508-566): little-endian
            // lengths; a read error inside the block is swallowed
            if (body + (uint64_t)blen * 8 > lb)
                return 2;
            const uint8_t *c = data + (body >> 3);
            const size_t cl = blen;
            size_t i = 0;
            auto le32 = [](const uint8_t *q) {
                return (uint32_t)q[0] | ((uint32_t)q[1] << 8) | ((uint32_t)q[2] << 16) |
                       ((uint32_t)q[3] << 24);
            };
            if (i + 4 <= cl) {
                const uint32_t vl = le32(c + i);
                i += 4;
                if (vl <= cl - i) {
                    i += vl;
                    if (i + 4 <= cl) {
                        uint32_t lines = le32(c + i);
                        i += 4;
                        static const char pre[] = "WAVEFORMATEXTENSIBLE_CHANNEL_MASK=";
                        for (; lines > 0; --lines) {
                            if (i + 4 > cl)
                                break;
                            const uint32_t ll = le32(c + i);
                            i += 4;
                            if (ll > cl - i)
                                break;
                            char buf[256];
                            const size_t keep = ll < 255 ? ll : 255;
                            for (size_t k = 0; k < keep; ++k) {
                                const char ch = (char)c[i + k];
                                buf[k] = (ch >= 'a' && ch <= 'z') ? (char)(ch - 32) : ch;
                            }
                            buf[keep] = 0;
                            if (std::strncmp(buf, pre, sizeof(pre) - 1) == 0) {
                                const unsigned long m =
                                    std::strtoul(buf + sizeof(pre) - 1, nullptr, 16);
                                const unsigned mask = (unsigned)m;
                                unsigned bits = 0;
                                for (unsigned mm = mask; mm; mm >>= 1)
                                    bits += mm & 1u;
                                if (bits == si->channels)
                                    si->channel_mask = mask;
                            }
                            i += ll;
                        }
                    }
                }
            }
        }
        if (type != 0 && type != 3)
            pos = body + (uint64_t)blen * 8;
        if (pos > lb)
            return 2;
        if (eof)
            return 2;
    } while (!last);
    si->frames_offset = pos >> 3;
    return 0;
}

atg_status atg_decoder_create(int device, atg_decoder **out)
{
    if (!out)
        return dfail(ATG_ERR_INVALID, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return dfail(ATG_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= n)
        return dfail(ATG_ERR_INVALID, "device index out of range");
    DHIP(hipSetDevice(device));
    static uint8_t t8[256];
    static uint16_t t16[4][256];
    build_dec_tables(t8, t16);
    DHIP(hipMemcpyToSymbol(HIP_SYMBOL(c_crc8), t8, sizeof(t8)));
    DHIP(hipMemcpyToSymbol(HIP_SYMBOL(c_crc16), t16, sizeof(t16)));
    static uint16_t adv[24][16];
    build_dec_adv(t16, adv);
    DHIP(hipMemcpyToSymbol(HIP_SYMBOL(c_crc_adv), adv, sizeof(adv)));
    atg_decoder *d = new atg_decoder();
    d->device = device;
    DHIP(hipStreamCreateWithFlags(&d->s, hipStreamNonBlocking));
    for (DecSlot &sl : d->slot) {
        // the default rotation's streams; rolled mode runs the restores of
        // every slot on these in turn and the chains on s_roll
        if (&sl - d->slot < kDecSlots)
            DHIP(hipStreamCreateWithFlags(&sl.s_md5, hipStreamNonBlocking));
        for (auto &e : sl.ev)
            DHIP(hipEventCreate(&e));
        DHIP(hipEventCreateWithFlags(&sl.ev_chain, hipEventDisableTiming));
        DHIP(hipEventCreateWithFlags(&sl.ev_done, hipEventDisableTiming));
    }
    *out = d;
    return ATG_OK;
}

void atg_decoder_destroy(atg_decoder *d)
{
    if (!d)
        return;
    (void)hipSetDevice(d->device);
    (void)hipStreamSynchronize(d->s);
    for (DBuf *b : {&d->data, &d->tracks, &d->counts, &d->ncand, &d->cand_pos, &d->cand_idx,
                    &d->recs, &d->hits, &d->segs, &d->cbits, &d->spec, &d->cand_trk})
        b->release();
    if (d->s_roll)
        (void)hipStreamSynchronize(d->s_roll);
    for (DecSlot &sl : d->slot) {
        if (sl.s_md5)
            (void)hipStreamSynchronize(sl.s_md5);
        for (DBuf *b : {&sl.pcm, &sl.bytes, &sl.md5, &sl.md5meta, &sl.tracks, &sl.frames, &sl.jobs,
                        &sl.warm, &sl.rows, &sl.meta})
            b->release();
        for (auto &e : sl.ev)
            (void)hipEventDestroy(e);
        (void)hipEventDestroy(sl.ev_chain);
        (void)hipEventDestroy(sl.ev_done);
        if (sl.md5_h)
            (void)hipHostFree(sl.md5_h);
        if (sl.s_md5)
            (void)hipStreamDestroy(sl.s_md5);
    }
    if (d->s_roll)
        (void)hipStreamDestroy(d->s_roll);
    (void)hipStreamDestroy(d->s);
    delete d;
}

} // extern "C"

// the digests and the restore's hypothesis check word to the host, as two
// copies: one copy of 16 n + 16 bytes (16,400 at 1024 tracks) instead of the
// 16,384-byte digest copy put ~1 ms on every config-2 decode step
// (profiles/r05_zz_dec_spec.txt) -- past 16 KiB the copy takes another path
static hipError_t dec_results_d2h(DecSlot &sl, uint32_t n, hipStream_t q)
{
    if (!n)
        return hipSuccess;
    hipError_t e = hipMemcpyAsync(sl.md5_h, sl.md5.p, 16 * (size_t)n, hipMemcpyDeviceToHost, q);
    if (e == hipSuccess)
        e = hipMemcpyAsync(sl.md5_h + 16 * (size_t)n, (uint8_t *)sl.md5.p + 16 * (size_t)n, 16,
                           hipMemcpyDeviceToHost, q);
    return e;
}

// a batch whose enqueue failed part-way: nothing of it may run on or be
// waited for -- out of the rolled queue (its slices would otherwise keep
// advancing a stale entry, and a reuse of the slot would queue it twice),
// its streams drained, the slot free
static void dec_abort(atg_decoder *d, DecSlot &sl)
{
    auto it = std::find(d->roll_q.begin(), d->roll_q.end(), &sl);
    if (it != d->roll_q.end())
        d->roll_q.erase(it);
    sl.roll_done = sl.roll_parts = 0;
    (void)hipStreamSynchronize(d->s);
    if (d->s_roll)
        (void)hipStreamSynchronize(d->s_roll);
    if (sl.s_md5)
        (void)hipStreamSynchronize(sl.s_md5);
    sl.busy = false;
}

// the tail of a rolled batch on s_roll: tails + padding + digests, the
// digests to the host, done
static atg_status dec_roll_tail(atg_decoder *d, DecSlot &sl)
{
    const uint32_t n = sl.n_md5;
    DHIP(launch_bytes_md5_finish((const uint8_t *)sl.bytes.p, (const uint64_t *)sl.md5meta.p,
                                 (const uint64_t *)sl.md5meta.p + n, n, (uint8_t *)sl.md5.p,
                                 d->s_roll));
    DHIP(hipEventRecord(sl.ev[7], d->s_roll));
    DHIP(dec_results_d2h(sl, n, d->s_roll));
    DHIP(hipEventRecord(sl.ev_done, d->s_roll));
    return ATG_OK;
}

// one rolled launch on s_roll after `after`: every rolled batch in flight
// advances by one slice; finished batches get their tails
static atg_status dec_roll_step(atg_decoder *d, hipEvent_t after)
{
    MdBytesRollArgs a;
    std::memset(&a, 0, sizeof(a));
    std::vector<DecSlot *> starting, finished;
    uint32_t wg = 0;
    for (DecSlot *sl : d->roll_q) {
        MdBytesRoll &b = a.b[a.n++];
        b.base = (const uint8_t *)sl->bytes.p;
        b.off = (const uint64_t *)sl->md5meta.p;
        b.len = (const uint64_t *)sl->md5meta.p + sl->n_md5;
        b.md5 = (uint8_t *)sl->md5.p;
        b.n = sl->n_md5;
        b.wg0 = wg;
        b.parts = sl->roll_parts;
        b.part = sl->roll_done;
        b.part_end = sl->roll_done + 1u;
        wg += (sl->n_md5 + 63u) / 64u;
        if (b.part == 0)
            starting.push_back(sl);
        sl->roll_done = b.part_end;
        if (sl->roll_done == sl->roll_parts)
            finished.push_back(sl);
    }
    if (!a.n)
        return ATG_OK;
    if (after)
        DHIP(hipStreamWaitEvent(d->s_roll, after, 0));
    for (DecSlot *sl : starting)
        DHIP(hipEventRecord(sl->ev[6], d->s_roll));
    DHIP(launch_bytes_md5_roll(a, d->s_roll));
    for (DecSlot *sl : finished) {
        d->roll_q.erase(std::find(d->roll_q.begin(), d->roll_q.end(), sl));
        const atg_status st = dec_roll_tail(d, *sl);
        if (st != ATG_OK)
            return st;
    }
    return ATG_OK;
}

// Enqueue the device-resident decode of a batch on slot `sl`: scan ->
// parse -> chain (two host round trips for the counts) on the decoder
// stream, then restore -> emit -> per-track MD5 on the slot's stream, so the
// next batch's scan and parse start while this one restores.  Returns once
// everything is queued; finish_decode waits.
static atg_status enqueue_decode(atg_decoder *d, DecSlot &sl, const uint8_t *d_data,
                                 uint64_t len, const atg_flac_dec_track *tracks, uint32_t n)
{
    hipStream_t s = d->s;
    std::vector<DecTrack> &tr = sl.tr;
    tr.assign(n, DecTrack());
    for (uint32_t t = 0; t < n; ++t) {
        const atg_flac_dec_track &a = tracks[t];
        DecTrack &b = tr[t];
        if (a.data_offset > len || a.data_bytes > len - a.data_offset)
            return dfail(ATG_ERR_INVALID, "track data range outside the buffer");
        if (t && a.data_offset < tracks[t - 1].data_offset)
            return dfail(ATG_ERR_INVALID, "tracks must be ordered by data_offset");
        if (a.channels < 1 || a.channels > 8)
            return dfail(ATG_ERR_UNSUPPORTED, "channels must be 1..8");
        b.start = a.data_offset;
        b.end = a.data_offset + a.data_bytes;
        b.total = a.total_samples;
        b.rate = a.sample_rate;
        b.channels = a.channels;
        b.bps = a.bits_per_sample;
        b.max_bs = a.max_block_size;
    }
    sl.want.assign(tracks, tracks + n);
    sl.data = d_data;
    sl.len = len;
    const uint64_t nw = std::max<uint64_t>(1, (len + 3) / 4);
    // the frame-end hypothesis (k_dec_spec): a bit per byte of the buffer
    const bool use_spec = d->spec_mode != 0 && !d->spec_off && n && len;
    const uint64_t nbw = (len >> 6) + 2;
    if (use_spec)
        DHIP(d->cbits.ensure(sizeof(uint64_t) * nbw));
    DHIP(d->tracks.ensure(sizeof(DecTrack) * std::max<uint32_t>(n, 1)));
    DHIP(d->counts.ensure(sizeof(DecCount) * std::max<uint32_t>(n, 1)));
    DHIP(d->ncand.ensure(2 * sizeof(uint32_t)));
    // candidate scratch: a real frame is >= 10 bytes, but the true count is
    // close to the frame count, so start at one slot per 16 bytes and re-scan
    // with the exact count in the rare batch that needs more
    uint64_t cap = std::min<uint64_t>(len / 16 + 4096, 0xFFFFFFFFull);
    DHIP(d->cand_idx.ensure(sizeof(uint32_t) * (len + 4)));
    DHIP(hipMemcpyAsync(d->tracks.p, tr.data(), sizeof(DecTrack) * n, hipMemcpyHostToDevice, s));
    const uint32_t *w = (const uint32_t *)d_data;
    DecTrack *dtr = (DecTrack *)d->tracks.p;
    hipEvent_t *ev = sl.ev;
    DHIP(hipEventRecord(ev[0], s));
    // the segments of the scan: the tracks' byte ranges (merged where they
    // touch) in 16-byte chunks, cut at kSegChunks-chunk boundaries
    {
        std::vector<ScanSeg> &sg = d->segs_h;
        sg.clear();
        const uint64_t nchunk = (nw + 3) / 4;
        uint64_t c0 = 0, c1 = 0; // the pending range [c0, c1)
        auto flush = [&](uint64_t a, uint64_t b) {
            for (uint64_t x = a; x < b; x += kSegChunks) {
                ScanSeg g;
                g.c0 = x;
                g.n = (uint32_t)std::min<uint64_t>(b - x, kSegChunks);
                g.pad = 0;
                sg.push_back(g);
            }
        };
        for (uint32_t t = 0; t < n; ++t) {
            const uint64_t a = tr[t].start / 16, b = std::min(nchunk, (tr[t].end + 15) / 16);
            if (a >= b)
                continue;
            if (c1 > c0 && a <= c1) {
                c1 = std::max(c1, b);
            } else {
                if (c1 > c0)
                    flush(c0, c1);
                c0 = a;
                c1 = b;
            }
        }
        if (c1 > c0)
            flush(c0, c1);
    }
    const uint64_t nseg = d->segs_h.size();
    DHIP(d->segs.ensure(sizeof(ScanSeg) * std::max<uint64_t>(nseg, 1)));
    if (nseg)
        DHIP(hipMemcpyAsync(d->segs.p, d->segs_h.data(), sizeof(ScanSeg) * nseg,
                            hipMemcpyHostToDevice, s));
    // counters: [0] candidates, [1] sync positions
    uint32_t cnt_h[2] = {0, 0};
    uint32_t &found = cnt_h[0];
    uint64_t hcap = cap;
    for (int pass = 0; pass < 3; ++pass) {
        DHIP(d->cand_pos.ensure(sizeof(uint64_t) * cap));
        DHIP(d->cand_trk.ensure(sizeof(uint32_t) * cap));
        DHIP(d->hits.ensure(sizeof(uint64_t) * hcap));
        DHIP(hipMemsetAsync(d->ncand.p, 0, 2 * sizeof(uint32_t), s));
        if (use_spec)
            DHIP(hipMemsetAsync(d->cbits.p, 0, sizeof(uint64_t) * nbw, s));
        // grid-stride: at most 8 workgroups of 256 per CU (2048 over 256 CUs)
        if (n && len) {
            hipLaunchKernelGGL(k_dec_sync, dim3((unsigned)std::min<uint64_t>(nseg, 2048)),
                               dim3(256), 0, s, w, nw, len, (const ScanSeg *)d->segs.p,
                               (uint32_t)nseg, (uint32_t *)d->ncand.p + 1, hcap,
                               (uint64_t *)d->hits.p);
            hipLaunchKernelGGL(k_dec_hdr, dim3((unsigned)std::min<uint64_t>((hcap + 255) / 256, 1024)),
                               dim3(256), 0, s, w, nw, len, dtr, n,
                               (const uint32_t *)d->ncand.p + 1, hcap, (const uint64_t *)d->hits.p,
                               (uint32_t *)d->ncand.p, (uint32_t)cap, (uint64_t *)d->cand_pos.p,
                               (uint32_t *)d->cand_idx.p, (uint32_t *)d->cand_trk.p,
                               use_spec ? (unsigned long long *)d->cbits.p : nullptr);
        }
        DHIP(hipGetLastError());
        DHIP(hipMemcpyAsync(cnt_h, d->ncand.p, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, s));
        DHIP(hipStreamSynchronize(s));
        if (cnt_h[1] > hcap) { // every sync position of the buffer is now known
            hcap = cnt_h[1];
            continue;
        }
        if (found > cap) {
            cap = found;
            continue;
        }
        break;
    }
    DHIP(d->recs.ensure(sizeof(ParseRec) * std::max<uint64_t>(found, 1)));
    DHIP(hipEventRecord(ev[1], s));
    sl.spec = use_spec && found;
    if (sl.spec) {
        DHIP(d->spec.ensure(sizeof(uint32_t) * found));
        hipLaunchKernelGGL(k_dec_spec, dim3((unsigned)std::min<uint64_t>((found + 3) / 4, 8192)),
                           dim3(256), 0, s, w, nw, dtr, n, (const uint32_t *)d->ncand.p,
                           (const uint64_t *)d->cand_pos.p, (const uint32_t *)d->cand_trk.p,
                           (const unsigned long long *)d->cbits.p, nbw, (uint32_t *)d->spec.p);
        DHIP(hipGetLastError());
    }
    hipLaunchKernelGGL(k_dec_parse, dim3(4096), dim3(64), 0, s, w, nw, dtr, n,
                       (const uint32_t *)d->ncand.p, (const uint64_t *)d->cand_pos.p,
                       (const uint32_t *)d->cand_trk.p,
                       sl.spec ? (const uint32_t *)d->spec.p : nullptr, (ParseRec *)d->recs.p);
    DHIP(hipGetLastError());
    if (found)
        hipLaunchKernelGGL(k_dec_crc, dim3((unsigned)std::min<uint64_t>((found + 3) / 4, 8192)),
                           dim3(256), 0, s, w, nw, (const uint32_t *)d->ncand.p,
                           (const uint64_t *)d->cand_pos.p, (ParseRec *)d->recs.p);
    DHIP(hipGetLastError());
    DHIP(hipEventRecord(ev[2], s));
    const dim3 tg((n + 63) / 64);
    if (n)
        hipLaunchKernelGGL(k_dec_chain, tg, dim3(64), 0, s, w, nw, dtr, n,
                           (const uint32_t *)d->ncand.p, (const uint64_t *)d->cand_pos.p,
                           (const uint32_t *)d->cand_idx.p, (const ParseRec *)d->recs.p,
                           (DecCount *)d->counts.p, 1, (DecFrame *)nullptr, (uint2 *)nullptr);
    DHIP(hipGetLastError());
    sl.cnt.assign(n, DecCount());
    DHIP(hipMemcpyAsync(sl.cnt.data(), d->counts.p, sizeof(DecCount) * n, hipMemcpyDeviceToHost,
                        s));
    DHIP(hipStreamSynchronize(s));
    // host prefix over tracks: frame slots, PCM placement, MD5 byte streams
    uint64_t fb = 0, pb = 0, mb = 0, jb = 0;
    for (uint32_t t = 0; t < n; ++t) {
        DecTrack &b = tr[t];
        b.frame_base = fb;
        b.pcm_base = pb;
        b.md5_base = mb;
        b.job_base = jb;
        fb += sl.cnt[t].n_frames;
        jb += (uint64_t)sl.cnt[t].n_frames * b.channels;
        const uint64_t ns = sl.cnt[t].pcm_frames * b.channels;
        pb += ns;
        mb += (ns * ((b.bps + 7) / 8) + 63) & ~63ull;
    }
    sl.total_samples = pb;
    sl.total_frames = fb;
    // the slot's buffers: its previous batch was waited (take_dec_slot)
    DHIP(sl.frames.ensure(sizeof(DecFrame) * std::max<uint64_t>(fb, 1)));
    DHIP(sl.jobs.ensure(sizeof(uint2) * std::max<uint64_t>(jb, 1)));
    DHIP(sl.warm.ensure(sizeof(int32_t) * 32 * std::max<uint64_t>(jb, 1)));
    uint32_t max_bs = 1;
    for (uint32_t t = 0; t < n; ++t)
        if (sl.cnt[t].n_frames)
            max_bs = std::max(max_bs, tr[t].max_bs);
    // sample rows (warm-up samples included: at least 32), whole 64-row tiles
    const uint32_t nrows = (std::max(max_bs, 32u) + 63) & ~63u;
    const uint64_t nslots = (jb + 63) / 64;
    DHIP(sl.rows.ensure(sizeof(int32_t) * std::max<uint64_t>(nslots, 1) * nrows * 64));
    DHIP(sl.meta.ensure(sizeof(JobMeta) * std::max<uint64_t>(jb, 1)));
    DHIP(sl.pcm.ensure(sizeof(int32_t) * std::max<uint64_t>(pb, 1)));
    DHIP(sl.bytes.ensure(std::max<uint64_t>(mb, 64)));
    // the digests, then the restore's hypothesis check word (16 n)
    DHIP(sl.md5.ensure(16 * (size_t)n + 16));
    // the placed track table: the slot's own copy (the next batch re-uploads
    // the decoder's while this one restores)
    DHIP(sl.tracks.ensure(sizeof(DecTrack) * std::max<uint32_t>(n, 1)));
    DecTrack *str = (DecTrack *)sl.tracks.p;
    DHIP(hipMemcpyAsync(str, tr.data(), sizeof(DecTrack) * n, hipMemcpyHostToDevice, s));
    if (n)
        hipLaunchKernelGGL(k_dec_chain, tg, dim3(64), 0, s, w, nw, (const DecTrack *)str, n,
                           (const uint32_t *)d->ncand.p, (const uint64_t *)d->cand_pos.p,
                           (const uint32_t *)d->cand_idx.p, (const ParseRec *)d->recs.p,
                           (DecCount *)d->counts.p, 2, (DecFrame *)sl.frames.p,
                           (uint2 *)sl.jobs.p);
    DHIP(hipGetLastError());
    DHIP(hipEventRecord(sl.ev_chain, s));
    // the restore / emit stream: the slot's own, or in rolled mode the
    // default slots' streams in turn
    sl.rolled = d->depth > kDecSlots;
    hipStream_t ss = sl.rolled ? d->slot[sl.ticket % kDecSlots].s_md5 : sl.s_md5;
    DHIP(hipStreamWaitEvent(ss, sl.ev_chain, 0));
    uint32_t *spec_bad = (uint32_t *)((uint8_t *)sl.md5.p + 16 * (size_t)n);
    DHIP(hipMemsetAsync(spec_bad, 0, 16, ss));
    DHIP(hipEventRecord(ev[3], ss));
    if (jb)
        hipLaunchKernelGGL(k_dec_subframe, dim3((unsigned)((jb + 63) / 64)), dim3(64), 0, ss, w,
                           nw, (const DecTrack *)str, (const DecFrame *)sl.frames.p,
                           (const uint2 *)sl.jobs.p, jb, (int32_t *)sl.warm.p,
                           (int32_t *)sl.rows.p, nrows, (JobMeta *)sl.meta.p, spec_bad);
    DHIP(hipGetLastError());
    DHIP(hipEventRecord(ev[4], ss));
    if (jb)
        hipLaunchKernelGGL(k_dec_emit, dim3((unsigned)nslots), dim3(256), 0, ss,
                           (const DecTrack *)str, (const DecFrame *)sl.frames.p,
                           (const uint2 *)sl.jobs.p, jb, (const JobMeta *)sl.meta.p,
                           (const int32_t *)sl.rows.p, nrows, (const int32_t *)sl.warm.p,
                           (int32_t *)sl.pcm.p, (uint8_t *)sl.bytes.p);
    DHIP(hipGetLastError());
    DHIP(hipEventRecord(ev[5], ss));
    // MD5 of the decoded bytes on the slot's stream: the next batch's scan,
    // parse and restore run on the decoder stream meanwhile
    sl.md5_meta.assign(2 * (size_t)n, 0);
    for (uint32_t t = 0; t < n; ++t) {
        sl.md5_meta[t] = tr[t].md5_base;
        const uint64_t vis = sl.cnt[t].crc_frame != 0xFFFFFFFFu ? sl.cnt[t].crc_pcm
                                                                : sl.cnt[t].pcm_frames;
        sl.md5_meta[n + t] = vis * tr[t].channels * ((tr[t].bps + 7) / 8);
    }
    DHIP(sl.md5meta.ensure(sizeof(uint64_t) * 2 * std::max<uint32_t>(n, 1)));
    if (sl.md5_cap < 16 * (size_t)n + 16) {
        if (sl.md5_h)
            (void)hipHostFree(sl.md5_h);
        sl.md5_h = nullptr;
        sl.md5_cap = 0;
        DHIP(hipHostMalloc((void **)&sl.md5_h, 16 * (size_t)n + 16, hipHostMallocDefault));
        sl.md5_cap = 16 * (size_t)n + 16;
    }
    if (n)
        DHIP(hipMemcpyAsync(sl.md5meta.p, sl.md5_meta.data(), sizeof(uint64_t) * 2 * n,
                            hipMemcpyHostToDevice, ss));
    sl.n_md5 = n;
    if (sl.rolled) {
        // the chain in depth - 2 slices, one per enqueue, all batches' in one
        // launch on s_roll once this batch's bytes are written
        DHIP(hipEventRecord(ev[5], ss));
        if (!d->s_roll) {
            int prio_lo = 0, prio_hi = 0;
            DHIP(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
            DHIP(hipStreamCreateWithPriority(&d->s_roll, hipStreamNonBlocking, prio_hi));
        }
        sl.roll_parts = (uint32_t)d->depth - 2u;
        sl.roll_done = 0;
        d->roll_q.push_back(&sl);
        return dec_roll_step(d, ev[5]);
    }
    DHIP(hipEventRecord(ev[6], sl.s_md5));
    DHIP(launch_bytes_md5((const uint8_t *)sl.bytes.p, (const uint64_t *)sl.md5meta.p,
                          (const uint64_t *)sl.md5meta.p + n, n, (uint8_t *)sl.md5.p, sl.s_md5));
    DHIP(hipEventRecord(ev[7], sl.s_md5));
    DHIP(dec_results_d2h(sl, n, sl.s_md5));
    DHIP(hipEventRecord(sl.ev_done, sl.s_md5));
    return ATG_OK;
}

// wait for slot `sl`'s batch and fill its results
static atg_status finish_decode(atg_decoder *d, DecSlot &sl, atg_flac_dec_result *res)
{
    // a rolled batch with slices left: advance every rolled batch together
    while (sl.rolled && sl.roll_done < sl.roll_parts) {
        const atg_status st = dec_roll_step(d, nullptr);
        if (st != ATG_OK)
            return st;
    }
    DHIP(hipEventSynchronize(sl.ev_done));
    const size_t nt = sl.tr.size();
    if (sl.spec && nt && (*(const uint32_t *)(sl.md5_h + 16 * nt) || d->spec_mode == 2)) {
        // a frame-end hypothesis failed the restore's check (or the
        // self-check mode): the batch again with every subframe walked
        const std::vector<atg_flac_dec_track> want = sl.want;
        d->spec_off = true;
        atg_status st = enqueue_decode(d, sl, sl.data, sl.len, want.data(), (uint32_t)want.size());
        d->spec_off = false;
        if (st != ATG_OK) {
            dec_abort(d, sl);
            return st;
        }
        while (sl.rolled && sl.roll_done < sl.roll_parts)
            if ((st = dec_roll_step(d, nullptr)) != ATG_OK) {
                dec_abort(d, sl);
                return st;
            }
        DHIP(hipEventSynchronize(sl.ev_done));
        ++d->spec_redos;
        // a stream of inputs the hypothesis keeps failing on (junk after
        // frames, damaged files) would pay two decodes per batch: after
        // kSpecStreak redone batches in a row the parse walks every
        // subframe (mode 0) until the caller sets the mode again
        if (++d->spec_streak >= kSpecStreak && d->spec_mode == 1)
            d->spec_mode = 0;
    } else if (sl.spec) {
        d->spec_streak = 0;
    }
    // timings: scan, parse, chain (both passes + the host prefix), subframe,
    // emit, md5, total (scan start -> md5 end)
    const int map[kDecTimed][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 4}, {4, 5}, {6, 7}, {0, 7}};
    for (int k = 0; k < kDecTimed; ++k)
        if (hipEventElapsedTime(&d->times[k], sl.ev[map[k][0]], sl.ev[map[k][1]]) != hipSuccess)
            d->times[k] = 0.f;
    d->have_times = true;
    static const uint8_t zero[16] = {0};
    uint64_t fbase = 0;
    const uint32_t n = (uint32_t)sl.tr.size();
    for (uint32_t t = 0; t < n; ++t) {
        atg_flac_dec_result &r = res[t];
        const DecCount &c = sl.cnt[t];
        r.pcm_offset = sl.tr[t].pcm_base / sl.tr[t].channels;
        r.first_frame = (uint32_t)fbase;
        r.walk_frames = c.n_frames;
        r.walk_status = c.status;
        fbase += c.n_frames;
        std::memcpy(r.md5, &sl.md5_h[16 * (size_t)t], 16);
        if (c.crc_frame != 0xFFFFFFFFu) { // read() stops at the bad frame
            r.pcm_frames = c.crc_pcm;
            r.n_frames = c.crc_frame;
            r.status = FD_FRAME_CRC;
        } else {
            r.pcm_frames = c.pcm_frames;
            r.n_frames = c.n_frames;
            r.status = c.status;
            // FlacDecoder_verify_okay (flac.c:479-493) once remaining reaches 0
            if (r.status == FD_OK && std::memcmp(sl.want[t].md5, zero, 16) != 0 &&
                std::memcmp(sl.want[t].md5, r.md5, 16) != 0)
                r.status = FD_MD5;
        }
        r.reserved = 0;
        r.walk_end = c.stop;
    }
    sl.busy = false;
    d->last = (int)(&sl - d->slot);
    return ATG_OK;
}

// the slot for a new batch: the oldest, which must have been waited
static atg_status take_dec_slot(atg_decoder *d, DecSlot **out)
{
    DecSlot *sl = &d->slot[0];
    for (int k = 1; k < d->depth; ++k)
        if (d->slot[k].ticket < sl->ticket)
            sl = &d->slot[k];
    if (sl->busy)
        return dfail(ATG_ERR_INVALID, "every decode slot holds a batch in flight: wait for one");
    sl->ticket = d->next_ticket++;
    *out = sl;
    return ATG_OK;
}

static DecSlot *find_dec_ticket(atg_decoder *d, uint64_t ticket)
{
    for (DecSlot &sl : d->slot)
        if (sl.ticket == ticket && sl.busy)
            return &sl;
    return nullptr;
}

extern "C" {

atg_status atg_flac_decode_device_async(atg_decoder *d, const void *d_data, uint64_t len,
                                        const atg_flac_dec_track *tracks, uint32_t n,
                                        uint64_t *ticket)
{
    ATG_HANDLE_LOCK(d);
    if (!d || (!tracks && n) || !ticket || (!d_data && len))
        return dfail(ATG_ERR_INVALID, "NULL argument");
    if (((uintptr_t)d_data) & 3)
        return dfail(ATG_ERR_INVALID, "d_data must be 4-byte aligned");
    DHIP(hipSetDevice(d->device));
    DecSlot *sl = nullptr;
    atg_status st = take_dec_slot(d, &sl);
    if (st != ATG_OK)
        return st;
    st = enqueue_decode(d, *sl, (const uint8_t *)d_data, len, tracks, n);
    if (st != ATG_OK) {
        dec_abort(d, *sl);
        return st;
    }
    sl->busy = true;
    *ticket = sl->ticket;
    return ATG_OK;
}

atg_status atg_flac_decode_wait(atg_decoder *d, uint64_t ticket, atg_flac_dec_result *results,
                                const int32_t **d_pcm, uint64_t *total_samples)
{
    ATG_HANDLE_LOCK(d);
    if (!d)
        return dfail(ATG_ERR_INVALID, "NULL decoder");
    DecSlot *sl = find_dec_ticket(d, ticket);
    if (!sl)
        return dfail(ATG_ERR_INVALID, "unknown or already waited decode ticket");
    if (!results && !sl->tr.empty())
        return dfail(ATG_ERR_INVALID, "NULL results");
    DHIP(hipSetDevice(d->device));
    atg_status st = finish_decode(d, *sl, results);
    if (st != ATG_OK)
        return st;
    if (d_pcm)
        *d_pcm = (const int32_t *)sl->pcm.p;
    if (total_samples)
        *total_samples = sl->total_samples;
    return ATG_OK;
}

atg_status atg_flac_decode_device(atg_decoder *d, const void *d_data, uint64_t len,
                                  const atg_flac_dec_track *tracks, uint32_t n,
                                  atg_flac_dec_result *results, const int32_t **d_pcm,
                                  uint64_t *total_samples)
{
    ATG_HANDLE_LOCK(d);
    if (!d || (!tracks && n) || (!results && n) || (!d_data && len))
        return dfail(ATG_ERR_INVALID, "NULL argument");
    uint64_t ticket = 0;
    atg_status st = atg_flac_decode_device_async(d, d_data, len, tracks, n, &ticket);
    if (st != ATG_OK)
        return st;
    return atg_flac_decode_wait(d, ticket, results, d_pcm, total_samples);
}

atg_status atg_flac_decode_host(atg_decoder *d, const uint8_t *data, uint64_t len,
                                const atg_flac_dec_track *tracks, uint32_t n,
                                atg_flac_dec_result *results, uint64_t *total_samples,
                                uint64_t *total_frames)
{
    ATG_HANDLE_LOCK(d);
    if (!d || (!tracks && n) || (!results && n) || (!data && len))
        return dfail(ATG_ERR_INVALID, "NULL argument");
    DHIP(hipSetDevice(d->device));
    // the staging buffer is read by the decoder stream: no batch in flight
    for (DecSlot &sl : d->slot)
        if (sl.busy)
            return dfail(ATG_ERR_INVALID, "a device decode is in flight: wait for it first");
    DHIP(d->data.ensure(len + 64));
    DHIP(hipMemsetAsync((uint8_t *)d->data.p + (len & ~3ull), 0, 64, d->s));
    if (len)
        DHIP(hipMemcpyAsync(d->data.p, data, len, hipMemcpyHostToDevice, d->s));
    uint64_t ticket = 0;
    atg_status st = atg_flac_decode_device_async(d, d->data.p, len, tracks, n, &ticket);
    if (st != ATG_OK)
        return st;
    uint64_t ts = 0;
    st = atg_flac_decode_wait(d, ticket, results, nullptr, &ts);
    if (st != ATG_OK)
        return st;
    if (total_samples)
        *total_samples = ts;
    if (total_frames)
        *total_frames = d->slot[d->last].total_frames;
    return ATG_OK;
}

atg_status atg_flac_decode_fetch(atg_decoder *d, int32_t *pcm, uint64_t pcm_cap,
                                 uint64_t *frame_offsets, uint32_t *frame_block_sizes,
                                 uint64_t frame_cap)
{
    ATG_HANDLE_LOCK(d);
    if (!d)
        return dfail(ATG_ERR_INVALID, "NULL decoder");
    if (d->last < 0)
        return dfail(ATG_ERR_INVALID, "no decoded batch");
    DecSlot &sl = d->slot[d->last];
    const bool want_frames = frame_offsets || frame_block_sizes;
    // the slot's buffers hold the last waited batch until a newer batch takes
    // the slot
    if (sl.busy)
        return dfail(ATG_ERR_INVALID, "the last waited batch's slot holds a newer batch: fetch "
                                      "before enqueueing three more");
    if ((pcm && pcm_cap < sl.total_samples) || (want_frames && frame_cap < sl.total_frames))
        return dfail(ATG_ERR_CAPACITY, "output buffer too small for the decoded batch");
    DHIP(hipSetDevice(d->device));
    if (pcm && sl.total_samples)
        DHIP(hipMemcpyAsync(pcm, sl.pcm.p, sizeof(int32_t) * sl.total_samples,
                            hipMemcpyDeviceToHost, d->s));
    std::vector<DecFrame> fr;
    if (want_frames && sl.total_frames) {
        fr.resize(sl.total_frames);
        DHIP(hipMemcpyAsync(fr.data(), sl.frames.p, sizeof(DecFrame) * sl.total_frames,
                            hipMemcpyDeviceToHost, d->s));
    }
    DHIP(hipStreamSynchronize(d->s));
    for (uint64_t i = 0; i < fr.size(); ++i) {
        const DecTrack &t = sl.tr[fr[i].track];
        if (frame_offsets)
            frame_offsets[i] = fr[i].pos - t.start;
        if (frame_block_sizes)
            frame_block_sizes[i] = fr[i].bs;
    }
    return ATG_OK;
}

atg_status atg_decoder_set_inflight(atg_decoder *d, uint32_t n)
{
    ATG_HANDLE_LOCK(d);
    if (!d || n < (uint32_t)kDecSlots || n > (uint32_t)kDecMaxSlots)
        return dfail(ATG_ERR_INVALID, "decode batches in flight must be 3..16");
    for (DecSlot &sl : d->slot)
        if (sl.busy)
            return dfail(ATG_ERR_INVALID, "a decode batch is in flight: wait for it first");
    // a lower depth gives the workspaces of the slots past it back (a
    // config-2 slot holds ~5 GB: PCM, rows, byte image)
    for (int k = (int)n; k < kDecMaxSlots; ++k) {
        DecSlot &sl = d->slot[k];
        if (sl.s_md5)
            (void)hipStreamSynchronize(sl.s_md5);
        for (DBuf *b : {&sl.pcm, &sl.bytes, &sl.md5, &sl.md5meta, &sl.tracks, &sl.frames, &sl.jobs,
                        &sl.warm, &sl.rows, &sl.meta})
            b->release();
    }
    d->depth = (int)n;
    d->last = -1; // the oldest-slot rotation starts over
    return ATG_OK;
}

atg_status atg_decoder_set_frame_hypothesis(atg_decoder *d, int mode)
{
    ATG_HANDLE_LOCK(d);
    if (!d || mode < 0 || mode > 2)
        return dfail(ATG_ERR_INVALID, "frame hypothesis mode must be 0, 1 or 2");
    d->spec_mode = mode;
    d->spec_streak = 0;
    return ATG_OK;
}

uint64_t atg_decoder_frame_hypothesis_redos(atg_decoder *d)
{
    ATG_HANDLE_LOCK(d);
    return d ? d->spec_redos : 0;
}

int atg_decoder_kernel_times(atg_decoder *d, const char **names, float *ms, int cap)
{
    ATG_HANDLE_LOCK(d);
    if (!d || !d->have_times)
        return 0;
    const int n = cap < kDecTimed ? cap : kDecTimed;
    for (int k = 0; k < n; ++k) {
        if (names)
            names[k] = kDecNames[k];
        if (ms)
            ms[k] = d->times[k];
    }
    return n;
}

} // extern "C"
