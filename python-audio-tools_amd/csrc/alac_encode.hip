// alac_encode.hip — MI355X batch ALAC encoder (SURVEY §8(a) rows E1–E7):
// the reference's ALACEncoder_encode_alac / write_frameset / write_frame /
// compute_coefficients / calculate_residuals / encode_residuals
// (src/encoders/alac.c:126-1116) for a whole batch of tracks at once,
// byte-identical output.
//
// A frameset is one block of PCM frames; its channels are grouped into
// "elements" of one or two channels exactly as write_frameset does
// (alac.c:299-366).  What the reference tries one after the other, the GPU
// runs side by side:
//
//   K1 k_alac_lpc      lane per (element, signal): the distinct signals a
//                      stereo element's leftweights need -- ch0, ch1
//                      (leftweight 0), ch0-ch1 (the second channel of every
//                      leftweight > 0) and ch1 + ((ch0-ch1)*lw >> 2) for
//                      each lw > 0 tried (minimum..maximum_interlacing_
//                      leftweight, 0..4 by default) -- or the one channel of
//                      a mono element.
//                      Tukey window (host glibc cos table), 9-lag
//                      autocorrelation as one left-to-right fp64 sum per lag,
//                      Levinson, quantisation at orders 4 and 8
//                      (alac.c:714-905); fp contraction off.
//   K2 k_alac_chain    lane per (signal, order 4 | 8): the sign-LMS adaptive
//                      residual recurrence (alac.c:932-1005) and the exact
//                      bit count of the adaptive Golomb coder with its
//                      zero-run mode run as one streaming state machine
//                      (alac.c:1020-1100), plus the residual-overflow flag
//                      the reference longjmps on.
//   K3 k_alac_decide   lane per frameset: per element the order (bits4 <
//                      bits8 + 64), the leftweight (strict <, in order), the
//                      uncompressed fallback (< 10 samples or any overflow);
//                      frameset bytes.
//   K4 k_alac_scan     lane per track: frameset byte offsets, mdat header.
//   K5 k_alac_pack     lane per element: re-runs the chosen recurrences and
//                      writes the element's bits MSB-first into its bit
//                      range (whole words stored, the two shared edge words
//                      OR-ed atomically), the frameset's trailing '111'.
#include "handle_lock.h"
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/atgpu.h"
#include "alac_common.h"

#pragma clang fp contract(off)

namespace {

constexpr uint32_t kMaxBlock = 65535; // frameset lengths handled (32-bit size field)
constexpr uint32_t kMaxLw = 255;      // leftweights 0..255 (an 8-bit header field)
constexpr uint32_t kMaxStSig = kMaxLw + 3; // signals of a stereo element: ch0, ch1, diff, 255 mixes

struct AlacParams {
    uint32_t block_size, initial_history, history_multiplier, maximum_k;
    uint32_t channels, bps, lshift; // lshift = 8 * uncompressed LSB bytes (24-bit: 8)
    uint32_t n_elem;                // elements per frameset
    uint32_t n_sig;                 // signals per frameset
    int32_t elem_ch[8][2];          // element -> channels (second -1 for mono)
    uint32_t elem_sig[8];           // element -> first signal within the frameset
    uint32_t n_fs, n_tracks;
    // interlacing leftweights tried, lw_lo..lw_hi (alac.c:459-481); a stereo
    // element's n_st signals are, in order: ch0 and ch1 (when 0 is in the
    // range), ch0 - ch1 and the mix of every leftweight > 0 in the range
    uint32_t lw_lo, lw_hi, n_st;
    uint32_t sig_first_mix;         // index of leftweight max(lo, 1)'s mix within the element
    uint16_t st_kind[kMaxStSig];    // stereo signal index -> kind (see sig_at)
};

struct FsInfo {
    uint64_t pcm_start; // first PCM frame
    uint32_t n;         // PCM frames
    uint32_t track;
    uint32_t win_off;   // window table offset (doubles)
    uint32_t pad;
};

struct TrackInfoA {
    uint64_t out_base; // byte offset of the track's mdat atom
    uint32_t first_fs, n_fs;
};

struct SigLpc {
    int32_t q4[4];
    int32_t q8[8];
    uint32_t zero; // autocorrelation R[0] == 0: order 4, zero coefficients
    uint32_t pad;
};

struct ChainOut {
    uint32_t bits;
    uint32_t overflow;
};

struct ElemDesc {
    uint32_t bits;        // element bits incl. the 3-bit channel count
    uint8_t compressed;   // 0 = write_uncompressed_frame
    uint8_t lw;           // interlacing leftweight (stereo)
    uint8_t order[2];     // chosen order of each channel's signal
    uint16_t sig[2];      // chosen signal (within the frameset) of each channel
};

struct FsDesc {
    uint32_t bytes;   // frameset bytes (byte-aligned after '111')
    uint32_t pad;
    uint64_t out_off; // byte offset of the frameset from the track's mdat start
};

__constant__ AlacParams c_p;

// ------------------------------------------------------------------ signals
template <typename T>
__device__ __forceinline__ int32_t msb_at(const T *__restrict__ pcm, uint64_t frame, uint32_t c)
{
    const int32_t v = (int32_t)pcm[frame * c_p.channels + c];
    return c_p.lshift ? (v >> c_p.lshift) : v;
}

// signal `kind` of an element at PCM frame `frame` (see the header comment)
template <typename T>
__device__ __forceinline__ int32_t sig_at(const T *__restrict__ pcm, uint64_t frame, int32_t ca,
                                          int32_t cb, uint32_t kind)
{
    const int32_t a = msb_at(pcm, frame, (uint32_t)ca);
    if (cb < 0)
        return a;
    const int32_t b = msb_at(pcm, frame, (uint32_t)cb);
    if (kind == 0)
        return a;
    if (kind == 1)
        return b;
    if (kind == 2)
        return a - b;
    int64_t t = (int64_t)(a - b);
    t *= (int64_t)(kind - 2);
    t >>= ALAC_SHIFT;
    return b + (int32_t)t;
}

// signal index within the frameset -> (element, kind)
__device__ __forceinline__ void sig_decode(uint32_t s, uint32_t &elem, uint32_t &kind)
{
    uint32_t e = 0;
    for (uint32_t k = 1; k < c_p.n_elem; ++k)
        e = s >= c_p.elem_sig[k] ? k : e;
    elem = e;
    kind = c_p.elem_ch[e][1] >= 0 ? (uint32_t)c_p.st_kind[s - c_p.elem_sig[e]] : 0u;
}

// sample size of an element's signals (alac.c:570-573, 629-641)
__device__ __forceinline__ uint32_t elem_ss(uint32_t e)
{
    return c_p.bps - c_p.lshift + (c_p.elem_ch[e][1] >= 0 ? 1u : 0u);
}

// ------------------------------------------------------------------ K1
template <typename T>
__global__ __launch_bounds__(64) void k_alac_lpc(const T *__restrict__ pcm,
                                                 const FsInfo *__restrict__ fs,
                                                 const double *__restrict__ win,
                                                 SigLpc *__restrict__ out)
{
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (uint64_t)c_p.n_fs * c_p.n_sig)
        return;
    const uint32_t f = (uint32_t)(gid / c_p.n_sig), s = (uint32_t)(gid % c_p.n_sig);
    uint32_t e, kind;
    sig_decode(s, e, kind);
    const FsInfo F = fs[f];
    const int32_t ca = c_p.elem_ch[e][0], cb = c_p.elem_ch[e][1];
    const double *w = win + F.win_off;
    // autocorrelate (alac.c:818-836): R[lag] = sum_i x[i] x[i+lag], left to
    // right in i; accumulated as x[j-lag] x[j] in increasing j (same order)
    double R[ALAC_MAX_ORDER + 1], h[ALAC_MAX_ORDER];
#pragma unroll
    for (int l = 0; l <= ALAC_MAX_ORDER; ++l)
        R[l] = 0.0;
#pragma unroll
    for (int l = 0; l < ALAC_MAX_ORDER; ++l)
        h[l] = 0.0;
    const uint32_t N = F.n;
    for (uint32_t j = 0; j < N; ++j) {
        const double x = (double)sig_at(pcm, F.pcm_start + j, ca, cb, kind) * w[j];
        R[0] = R[0] + x * x;
#pragma unroll
        for (int l = 1; l <= ALAC_MAX_ORDER; ++l)
            if (j >= (uint32_t)l)
                R[l] = R[l] + h[l - 1] * x;
#pragma unroll
        for (int l = ALAC_MAX_ORDER - 1; l > 0; --l)
            h[l] = h[l - 1];
        h[0] = x;
    }
    SigLpc o;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        o.q4[i] = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i)
        o.q8[i] = 0;
    o.zero = R[0] == 0.0 ? 1u : 0u;
    o.pad = 0;
    if (!o.zero) {
        // compute_lp_coefficients (alac.c:838-881)
        double lp[ALAC_MAX_ORDER][ALAC_MAX_ORDER], err[ALAC_MAX_ORDER];
        double k = R[1] / R[0];
        lp[0][0] = k;
        err[0] = R[0] * (1.0 - (k * k));
#pragma unroll
        for (int i = 1; i < ALAC_MAX_ORDER; ++i) {
            double q = R[i + 1];
#pragma unroll
            for (int j = 0; j < i; ++j)
                q = q - (lp[i - 1][j] * R[i - j]);
            k = q / err[i - 1];
#pragma unroll
            for (int j = 0; j < i; ++j)
                lp[i][j] = lp[i - 1][j] - (k * lp[i - 1][i - j - 1]);
            lp[i][i] = k;
            err[i] = err[i - 1] * (1.0 - (k * k));
        }
        // quantize_coefficients (alac.c:883-905)
#pragma unroll
        for (int pass = 0; pass < 2; ++pass) {
            const int order = pass ? 8 : 4;
            double e2 = 0.0;
#pragma unroll
            for (int i = 0; i < order; ++i) {
                e2 = e2 + (lp[order - 1][i] * (double)(1 << 9));
                const int ei = (int)round(e2);
                const int c = ei < -(1 << 15) ? -(1 << 15) : (ei > (1 << 15) - 1 ? (1 << 15) - 1 : ei);
                if (pass)
                    o.q8[i] = c;
                else
                    o.q4[i] = c;
                e2 = e2 - (double)ei;
            }
        }
    }
    out[gid] = o;
}

// ------------------------------------------------------------------ LMS + Golomb
// the sign-LMS recurrence of calculate_residuals (alac.c:932-1005) with an
// ORDER-sample history in registers; residual() returns r[i] for i in order
struct GolombCount {
    // encode_residuals (alac.c:1020-1079) as a streaming state machine: the
    // zero-run lookahead becomes "count zeros until the next non-zero
    // residual (or the end), then emit the run"
    int32_t history;
    uint32_t sign_mod, in_run, zeros, kz, bits, overflow, max_unsigned, ss;
    __device__ void init(uint32_t sample_size)
    {
        history = (int32_t)c_p.initial_history;
        sign_mod = 0;
        in_run = 0;
        zeros = 0;
        kz = 0;
        bits = 0;
        overflow = 0;
        ss = sample_size;
        max_unsigned = sample_size >= 32 ? 0xFFFFFFFFu : (1u << sample_size);
    }
    __device__ __forceinline__ void push(int32_t r, bool has_next)
    {
        if (in_run) {
            if (r == 0) {
                ++zeros;
                return;
            }
            bits += alac_code_bits(zeros, kz, 16);
            sign_mod = zeros < 0xFFFFu ? 1u : 0u;
            history = 0;
            in_run = 0;
        }
        const uint32_t u = r >= 0 ? (uint32_t)r << 1 : ((uint32_t)(-r) << 1) - 1u;
        overflow |= u >= max_unsigned ? 1u : 0u;
        uint32_t k = alac_log2((uint32_t)(history >> 9) + 3u);
        k = k < c_p.maximum_k ? k : c_p.maximum_k;
        bits += alac_code_bits(u - sign_mod, k, ss);
        sign_mod = 0;
        if (u <= 0xFFFFu) {
            history += (int32_t)(u * c_p.history_multiplier) -
                       ((history * (int32_t)c_p.history_multiplier) >> 9);
            if (history < 128 && has_next) {
                // LOG2(0) is never reached on encoder residuals (history > 0
                // here), kept as the NDEBUG build's UINT_MAX for safety
                const uint32_t lg = history > 0 ? alac_log2((uint32_t)history) : 0xFFFFFFFFu;
                uint32_t kk = 7u - lg + (uint32_t)((history + 16) >> 6);
                kz = kk < c_p.maximum_k ? kk : c_p.maximum_k;
                in_run = 1;
                zeros = 0;
            }
        } else {
            history = 0xFFFF;
        }
    }
    __device__ __forceinline__ void finish()
    {
        if (in_run)
            bits += alac_code_bits(zeros, kz, 16);
    }
};

// the residuals of one signal with ORDER coefficients, handed to sink(r, i)
template <int ORDER, typename T, typename Sink>
__device__ __forceinline__ void lms_run(const T *__restrict__ pcm, const FsInfo &F, int32_t ca,
                                        int32_t cb, uint32_t kind, const int32_t *coef_in,
                                        uint32_t ss, Sink &sink)
{
    const uint32_t N = F.n;
    int32_t c[ORDER], h[ORDER + 1]; // h[0] newest .. h[ORDER] oldest
#pragma unroll
    for (int j = 0; j < ORDER; ++j)
        c[j] = coef_in[j];
#pragma unroll
    for (int j = 0; j <= ORDER; ++j)
        h[j] = 0;
    for (uint32_t i = 0; i < N; ++i) {
        const int32_t s = sig_at(pcm, F.pcm_start + i, ca, cb, kind);
        int32_t r;
        if (i == 0) {
            r = s;
        } else if (i < ORDER + 1u) {
            r = alac_trunc(s - h[0], ss);
        } else {
            const int32_t base = h[ORDER];
            int64_t sum = 1 << 8;
#pragma unroll
            for (int j = 0; j < ORDER; ++j)
                sum += (int64_t)c[j] * (int64_t)(h[j] - base);
            sum >>= 9;
            r = alac_trunc(s - base - (int32_t)sum, ss);
            // sign-LMS update, branch-free over the early exits: step j
            // touches c[ORDER-1-j] with diff = base - s[i-ORDER+j]
            int32_t e = r;
            const bool pos = r > 0;
            bool live = r != 0;
#pragma unroll
            for (int j = 0; j < ORDER; ++j) {
                const int32_t diff = base - h[ORDER - 1 - j];
                const int32_t sg = alac_sgn(diff);
                const int32_t step = pos ? sg : -sg;
                c[ORDER - 1 - j] -= live ? step : 0;
                e -= live ? ((diff * step) >> 9) * (j + 1) : 0;
                live = live && (pos ? e > 0 : e < 0);
            }
        }
        sink(r, i);
#pragma unroll
        for (int j = ORDER; j > 0; --j)
            h[j] = h[j - 1];
        h[0] = s;
    }
}

// ------------------------------------------------------------------ K2
struct CountSink {
    GolombCount g;
    uint32_t N;
    __device__ __forceinline__ void operator()(int32_t r, uint32_t i) { g.push(r, i + 1 < N); }
};

template <int ORDER, typename T>
__global__ __launch_bounds__(64) void k_alac_chain(const T *__restrict__ pcm,
                                                   const FsInfo *__restrict__ fs,
                                                   const SigLpc *__restrict__ lpc,
                                                   ChainOut *__restrict__ out)
{
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (uint64_t)c_p.n_fs * c_p.n_sig)
        return;
    const uint32_t f = (uint32_t)(gid / c_p.n_sig), s = (uint32_t)(gid % c_p.n_sig);
    uint32_t e, kind;
    sig_decode(s, e, kind);
    const FsInfo F = fs[f];
    const SigLpc L = lpc[gid];
    ChainOut o;
    o.bits = 0;
    o.overflow = 0;
    if (ORDER == 8 && L.zero) { // the all-zero case encodes order 4 only
        out[gid] = o;
        return;
    }
    int32_t coef[ORDER];
#pragma unroll
    for (int j = 0; j < ORDER; ++j)
        coef[j] = ORDER == 4 ? (L.zero ? 0 : L.q4[j]) : L.q8[j];
    CountSink sink;
    const uint32_t ss = elem_ss(e);
    sink.g.init(ss);
    sink.N = F.n;
    lms_run<ORDER>(pcm, F, c_p.elem_ch[e][0], c_p.elem_ch[e][1], kind, coef, ss, sink);
    sink.g.finish();
    o.bits = sink.g.bits;
    o.overflow = sink.g.overflow;
    out[gid] = o;
}

// ------------------------------------------------------------------ K3
__device__ __forceinline__ uint32_t frame_head_bits(uint32_t N)
{
    return 16u + 1u + 2u + 1u + (N != c_p.block_size ? 32u : 0u);
}

__global__ __launch_bounds__(64) void k_alac_decide(const FsInfo *__restrict__ fs,
                                                    const SigLpc *__restrict__ lpc,
                                                    const ChainOut *__restrict__ c4,
                                                    const ChainOut *__restrict__ c8,
                                                    ElemDesc *__restrict__ ed,
                                                    FsDesc *__restrict__ fd)
{
    const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= c_p.n_fs)
        return;
    const uint32_t N = fs[f].n;
    uint32_t total = 0;
    for (uint32_t e = 0; e < c_p.n_elem; ++e) {
        const uint32_t nch = c_p.elem_ch[e][1] >= 0 ? 2u : 1u;
        const uint64_t s0 = (uint64_t)f * c_p.n_sig + c_p.elem_sig[e];
        // a signal's chosen order and residual bits (compute_coefficients)
        auto pick = [&](uint32_t s, uint32_t &ord, uint32_t &rb) {
            const SigLpc &L = lpc[s0 + s];
            const ChainOut a = c4[s0 + s], b = c8[s0 + s];
            if (L.zero || a.bits < b.bits + 64u) {
                ord = 4;
                rb = a.bits;
            } else {
                ord = 8;
                rb = b.bits;
            }
        };
        // any residual overflow of a signal the leftweights use makes the
        // reference longjmp to write_uncompressed_frame (alac.c:426-436)
        uint32_t overflow = 0;
        const uint32_t nsig = nch == 2 ? c_p.n_st : 1u;
        for (uint32_t s = 0; s < nsig; ++s) {
            const SigLpc &L = lpc[s0 + s];
            overflow |= c4[s0 + s].overflow | (L.zero ? 0u : c8[s0 + s].overflow);
        }
        ElemDesc d;
        const uint32_t lsb_bits = N * nch * c_p.lshift;
        if (N >= 10 && !overflow) {
            d.compressed = 1;
            if (nch == 1) {
                uint32_t o0, r0;
                pick(0, o0, r0);
                d.lw = 0;
                d.sig[0] = (uint16_t)c_p.elem_sig[e];
                d.sig[1] = 0;
                d.order[0] = (uint8_t)o0;
                d.order[1] = 0;
                d.bits = frame_head_bits(N) + 16u + 16u + 16u * o0 + lsb_bits + r0;
            } else {
                // write_compressed_frame: leftweights lo..hi in order, the
                // smallest frame kept (strict <, alac.c:459-481); leftweight
                // 0 codes (ch0, ch1), lw > 0 (mix(lw), ch0 - ch1)
                const uint32_t diff = c_p.lw_lo == 0 ? 2u : 0u;
                uint32_t best = 0xFFFFFFFFu, best_a = 0, best_b = 1, best_lw = 0;
                uint32_t oa = 0, ob = 0;
                for (uint32_t lw = c_p.lw_lo; lw <= c_p.lw_hi; ++lw) {
                    const uint32_t a = lw ? c_p.sig_first_mix + lw - max(c_p.lw_lo, 1u) : 0u;
                    const uint32_t b = lw ? diff : 1u;
                    uint32_t o1, r1, o2, r2;
                    pick(a, o1, r1);
                    pick(b, o2, r2);
                    const uint32_t bits = frame_head_bits(N) + 16u + 2u * 16u + 16u * o1 +
                                          16u * o2 + lsb_bits + r1 + r2;
                    if (bits < best) {
                        best = bits;
                        best_lw = lw;
                        best_a = a;
                        best_b = b;
                        oa = o1;
                        ob = o2;
                    }
                }
                d.lw = (uint8_t)best_lw;
                d.sig[0] = (uint16_t)(c_p.elem_sig[e] + best_a);
                d.sig[1] = (uint16_t)(c_p.elem_sig[e] + best_b);
                d.order[0] = (uint8_t)oa;
                d.order[1] = (uint8_t)ob;
                d.bits = best;
            }
        } else {
            d.compressed = 0;
            d.lw = 0;
            d.sig[0] = d.sig[1] = 0;
            d.order[0] = d.order[1] = 0;
            d.bits = frame_head_bits(N) + N * nch * c_p.bps;
        }
        d.bits += 3u; // channel count
        ed[(uint64_t)f * c_p.n_elem + e] = d;
        total += d.bits;
    }
    total += 3u; // trailing '111'
    FsDesc o;
    o.bytes = (total + 7u) >> 3;
    o.pad = 0;
    o.out_off = 0;
    fd[f] = o;
}

// ------------------------------------------------------------------ K4
__global__ __launch_bounds__(64) void k_alac_scan(const TrackInfoA *__restrict__ tr,
                                                  FsDesc *__restrict__ fd, uint8_t *__restrict__ out,
                                                  uint64_t *__restrict__ mdat_bytes)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= c_p.n_tracks)
        return;
    const TrackInfoA T = tr[t];
    uint64_t off = 8;
    for (uint32_t k = 0; k < T.n_fs; ++k) {
        FsDesc &d = fd[T.first_fs + k];
        d.out_off = off;
        off += d.bytes;
    }
    uint8_t *o = out + T.out_base;
    const uint32_t sz = (uint32_t)off;
    o[0] = (uint8_t)(sz >> 24);
    o[1] = (uint8_t)(sz >> 16);
    o[2] = (uint8_t)(sz >> 8);
    o[3] = (uint8_t)sz;
    o[4] = 'm';
    o[5] = 'd';
    o[6] = 'a';
    o[7] = 't';
    mdat_bytes[t] = off;
}

// ------------------------------------------------------------------ K5
// MSB-first bit writer over a bit range that may share its first and last
// 32-bit words with the neighbouring ranges: those two are OR-ed atomically,
// the words in between are stored whole.
struct BitW {
    uint32_t *w;      // word array (big-endian byte order in memory)
    uint64_t pos;     // absolute bit position
    uint64_t first_w; // first word of the range
    uint64_t acc;     // pending bits, MSB-aligned at bit 63
    uint32_t n;       // pending bit count (< 32 after each put)
    __device__ void init(uint32_t *words, uint64_t bit0)
    {
        w = words;
        pos = bit0;
        first_w = bit0 >> 5;
        const uint32_t lead = (uint32_t)(bit0 & 31u);
        acc = 0;
        n = lead; // leading bits of the first word belong to the neighbour (zeros)
    }
    __device__ __forceinline__ void emit(uint32_t word, uint64_t wi)
    {
        const uint32_t be = __builtin_bswap32(word);
        if (wi == first_w)
            atomicOr(w + wi, be);
        else
            w[wi] = be;
    }
    __device__ __forceinline__ void put(uint32_t nbits, uint32_t v)
    {
        // nbits <= 32
        if (!nbits)
            return;
        const uint64_t vv = nbits >= 32 ? (uint64_t)v : ((uint64_t)v & ((1ull << nbits) - 1ull));
        acc |= vv << (64u - n - nbits);
        n += nbits;
        pos += nbits;
        if (n >= 32) {
            emit((uint32_t)(acc >> 32), (pos - n) >> 5);
            acc <<= 32;
            n -= 32;
        }
    }
    __device__ __forceinline__ void put_ones(uint32_t count) // count <= 8
    {
        put(count, (1u << count) - 1u);
    }
    __device__ void finish() // the last partial word is shared
    {
        if (n) {
            const uint64_t wi = (pos - n) >> 5;
            atomicOr(w + wi, __builtin_bswap32((uint32_t)(acc >> 32)));
        }
    }
};

// write_residual (alac.c:1081-1100)
__device__ __forceinline__ void put_code(BitW &bw, uint32_t value, uint32_t k, uint32_t ss)
{
    const uint32_t m = (1u << k) - 1u;
    if (value >= 9u * m) {
        bw.put(9, 0x1FFu);
        bw.put(ss, value);
        return;
    }
    uint32_t msb = 0;
#pragma unroll
    for (uint32_t t = 1; t <= 8; ++t)
        msb += value >= t * m ? 1u : 0u;
    const uint32_t lsb = value - msb * m;
    bw.put(msb + 1u, ((1u << msb) - 1u) << 1); // msb ones, then the 0 stop bit
    if (k > 1u) {
        if (lsb > 0u)
            bw.put(k, lsb + 1u);
        else
            bw.put(k - 1u, 0u);
    }
}

struct WriteSink {
    BitW *bw;
    uint32_t N, ss;
    int32_t history;
    uint32_t sign_mod, in_run, zeros, kz;
    __device__ void init(BitW *b, uint32_t n, uint32_t sample_size)
    {
        bw = b;
        N = n;
        ss = sample_size;
        history = (int32_t)c_p.initial_history;
        sign_mod = in_run = zeros = kz = 0;
    }
    __device__ __forceinline__ void operator()(int32_t r, uint32_t i)
    {
        if (in_run) {
            if (r == 0) {
                ++zeros;
                return;
            }
            put_code(*bw, zeros, kz, 16);
            sign_mod = zeros < 0xFFFFu ? 1u : 0u;
            history = 0;
            in_run = 0;
        }
        const uint32_t u = r >= 0 ? (uint32_t)r << 1 : ((uint32_t)(-r) << 1) - 1u;
        uint32_t k = alac_log2((uint32_t)(history >> 9) + 3u);
        k = k < c_p.maximum_k ? k : c_p.maximum_k;
        put_code(*bw, u - sign_mod, k, ss);
        sign_mod = 0;
        if (u <= 0xFFFFu) {
            history += (int32_t)(u * c_p.history_multiplier) -
                       ((history * (int32_t)c_p.history_multiplier) >> 9);
            if (history < 128 && i + 1 < N) {
                const uint32_t lg = history > 0 ? alac_log2((uint32_t)history) : 0xFFFFFFFFu;
                uint32_t kk = 7u - lg + (uint32_t)((history + 16) >> 6);
                kz = kk < c_p.maximum_k ? kk : c_p.maximum_k;
                in_run = 1;
                zeros = 0;
            }
        } else {
            history = 0xFFFF;
        }
    }
    __device__ void finish()
    {
        if (in_run)
            put_code(*bw, zeros, kz, 16);
    }
};

template <typename T>
__device__ void pack_signal(BitW &bw, const T *__restrict__ pcm, const FsInfo &F, uint32_t e,
                            uint32_t kind, uint32_t order, const SigLpc &L)
{
    const uint32_t ss = elem_ss(e);
    WriteSink sink;
    sink.init(&bw, F.n, ss);
    if (order == 8) {
        lms_run<8>(pcm, F, c_p.elem_ch[e][0], c_p.elem_ch[e][1], kind, L.q8, ss, sink);
    } else {
        int32_t c4[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
            c4[j] = L.zero ? 0 : L.q4[j];
        lms_run<4>(pcm, F, c_p.elem_ch[e][0], c_p.elem_ch[e][1], kind, c4, ss, sink);
    }
    sink.finish();
}

template <typename T>
__global__ __launch_bounds__(64) void k_alac_pack(const T *__restrict__ pcm,
                                                  const FsInfo *__restrict__ fs,
                                                  const TrackInfoA *__restrict__ tr,
                                                  const SigLpc *__restrict__ lpc,
                                                  const ElemDesc *__restrict__ ed,
                                                  const FsDesc *__restrict__ fd,
                                                  uint8_t *__restrict__ out)
{
    const uint64_t gid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= (uint64_t)c_p.n_fs * c_p.n_elem)
        return;
    const uint32_t f = (uint32_t)(gid / c_p.n_elem), e = (uint32_t)(gid % c_p.n_elem);
    const FsInfo F = fs[f];
    const uint64_t base = tr[F.track].out_base + fd[f].out_off; // 4-byte aligned track base
    uint64_t bit0 = base * 8;
    const ElemDesc *row = ed + (uint64_t)f * c_p.n_elem;
    for (uint32_t k = 0; k < e; ++k)
        bit0 += row[k].bits;
    const ElemDesc d = row[e];
    const uint32_t N = F.n;
    const int32_t ca = c_p.elem_ch[e][0], cb = c_p.elem_ch[e][1];
    const uint32_t nch = cb >= 0 ? 2u : 1u;
    BitW bw;
    bw.init((uint32_t *)out, bit0);
    bw.put(3, nch - 1u);
    if (!d.compressed) { // write_uncompressed_frame (alac.c:402-430)
        bw.put(16, 0);
        bw.put(1, N == c_p.block_size ? 0u : 1u);
        bw.put(2, 0);
        bw.put(1, 1);
        if (N != c_p.block_size)
            bw.put(32, N);
        const uint32_t mask = c_p.bps >= 32 ? 0xFFFFFFFFu : (1u << c_p.bps) - 1u;
        for (uint32_t i = 0; i < N; ++i) {
            bw.put(c_p.bps, (uint32_t)(int32_t)pcm[(F.pcm_start + i) * c_p.channels + ca] & mask);
            if (nch == 2)
                bw.put(c_p.bps,
                       (uint32_t)(int32_t)pcm[(F.pcm_start + i) * c_p.channels + cb] & mask);
        }
    } else {
        const uint32_t lsbs = c_p.lshift / 8;
        bw.put(16, 0);
        bw.put(1, N == c_p.block_size ? 0u : 1u);
        bw.put(2, lsbs);
        bw.put(1, 0);
        if (N != c_p.block_size)
            bw.put(32, N);
        bw.put(8, nch == 2 ? ALAC_SHIFT : 0u);
        bw.put(8, d.lw);
        const uint64_t s0 = (uint64_t)f * c_p.n_sig;
        SigLpc L[2];
        for (uint32_t c = 0; c < nch; ++c) {
            L[c] = lpc[s0 + d.sig[c]];
            // write_subframe_header (alac.c:1103-1116)
            bw.put(4, 0);
            bw.put(4, 9);
            bw.put(3, 4);
            bw.put(5, d.order[c]);
            for (uint32_t j = 0; j < d.order[c]; ++j) {
                const int32_t q = d.order[c] == 8 ? L[c].q8[j] : (L[c].zero ? 0 : L[c].q4[j]);
                bw.put(16, (uint32_t)q & 0xFFFFu);
            }
        }
        if (lsbs) {
            const uint32_t lm = (1u << c_p.lshift) - 1u;
            for (uint32_t i = 0; i < N; ++i) {
                bw.put(c_p.lshift,
                       (uint32_t)(int32_t)pcm[(F.pcm_start + i) * c_p.channels + ca] & lm);
                if (nch == 2)
                    bw.put(c_p.lshift,
                           (uint32_t)(int32_t)pcm[(F.pcm_start + i) * c_p.channels + cb] & lm);
            }
        }
        for (uint32_t c = 0; c < nch; ++c) {
            const uint32_t k = d.sig[c] - c_p.elem_sig[e];
            const uint32_t kind = nch == 2 ? (uint32_t)c_p.st_kind[k] : 0u;
            pack_signal(bw, pcm, F, e, kind, d.order[c], L[c]);
        }
    }
    if (e + 1 == c_p.n_elem) { // trailing '111' (alac.c:368-369); padding stays 0
        bw.put(3, 7);
    }
    bw.finish();
}

// ------------------------------------------------------------------ host
thread_local std::string g_alac_err;

atg_status afail(atg_status s, const std::string &m)
{
    g_alac_err = m;
    return s;
}

#define AHIP(expr)                                                                         \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return afail(ATG_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

struct ABuf {
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

const int kATimed = 6;
const char *kANames[kATimed] = {"alac_lpc", "alac_chain", "alac_decide", "alac_scan",
                                "alac_pack", "alac_total"};

// Tukey(0.5) exactly as window_signal (alac.c:778-816), glibc cos
void alac_window(unsigned N, double *w)
{
    const double alpha = 0.5;
    const unsigned w1 = (unsigned)(alpha * (N - 1)) / 2;
    const unsigned w2 = (unsigned)((N - 1) * (1.0 - (alpha / 2.0)));
    for (unsigned n = 0; n < N; n++) {
        if (n <= w1)
            w[n] = 0.5 * (1.0 + std::cos(M_PI * (((2 * n) / (alpha * (N - 1))) - 1.0)));
        else if (n <= w2)
            w[n] = 1.0;
        else
            w[n] = 0.5 * (1.0 + std::cos(M_PI * (((2.0 * n) / (alpha * (N - 1))) -
                                                 (2.0 / alpha) + 1.0)));
    }
}

// write_frameset's channel groups (alac.c:299-366)
uint32_t alac_groups(uint32_t nch, int32_t g[8][2])
{
    static const int T[9][6][2] = {
        {{0, -1}},
        {{0, -1}},
        {{0, 1}},
        {{2, -1}, {0, 1}},
        {{2, -1}, {0, 1}, {3, -1}},
        {{2, -1}, {0, 1}, {3, 4}},
        {{2, -1}, {0, 1}, {4, 5}, {3, -1}},
        {{2, -1}, {0, 1}, {4, 5}, {6, -1}, {3, -1}},
        {{2, -1}, {6, 7}, {0, 1}, {4, 5}, {3, -1}},
    };
    static const uint32_t n[9] = {0, 1, 1, 2, 3, 3, 4, 5, 5};
    for (uint32_t i = 0; i < n[nch]; ++i) {
        g[i][0] = T[nch][i][0];
        g[i][1] = T[nch][i][1];
    }
    return n[nch];
}

uint64_t fs_bound(uint32_t N, uint32_t nch, uint32_t bps)
{
    // worst case per sample: an escape (9 + 25 bits) plus a zero-run code
    // (<= 9 + 16 bits); headers + coefficients per element
    return (uint64_t)N * nch * 8u + (uint64_t)(bps / 8) * N * nch + 64u * nch + 16u;
}

} // namespace

struct atg_alac_encoder {
    std::recursive_mutex mu; // held by every public entry point (handle_lock.h)
    int device = 0;
    hipStream_t s = nullptr;
    hipEvent_t ev[kATimed] = {};
    float times[kATimed] = {};
    bool have_times = false;
    ABuf fs, tracks, win, lpc, c4, c8, ed, fd, mdat, h_pcm, h_out;
    std::vector<double> win_host;
    std::map<uint32_t, uint32_t> win_off;
    size_t win_uploaded = 0;
};

namespace {

struct APlan {
    AlacParams p;
    std::vector<FsInfo> fs;
    std::vector<TrackInfoA> tracks;
    std::vector<uint64_t> slot; // per track output slot bytes
    uint64_t out_bytes = 0;
};

atg_status alac_plan(atg_alac_encoder *enc, const atg_alac_options *o, const atg_track *tracks,
                     uint32_t n, uint32_t channels, uint32_t bps, APlan &P)
{
    if (!o)
        return afail(ATG_ERR_INVALID, "options is NULL");
    if (bps != 16 && bps != 24)
        return afail(ATG_ERR_INVALID, "bits per sample must be 16 or 24");
    if (channels < 1 || channels > 8)
        return afail(ATG_ERR_UNSUPPORTED, "channels must be 1..8");
    if (o->block_size < 1 || o->block_size > kMaxBlock)
        return afail(ATG_ERR_UNSUPPORTED, "block_size must be 1..65535");
    if (o->maximum_k < 1 || o->maximum_k > 24)
        return afail(ATG_ERR_UNSUPPORTED, "maximum_k must be 1..24");
    // the reference writes the leftweight in 8 bits and, with min > max,
    // copies a stale recorder as the frame (alac.c:459-481): both refused
    if (o->minimum_interlacing_leftweight > o->maximum_interlacing_leftweight ||
        o->maximum_interlacing_leftweight > kMaxLw)
        return afail(ATG_ERR_INVALID, "interlacing leftweights must satisfy 0 <= min <= max <= 255");
    AlacParams &p = P.p;
    std::memset(&p, 0, sizeof(p));
    p.block_size = o->block_size;
    p.initial_history = o->initial_history;
    p.history_multiplier = o->history_multiplier;
    p.maximum_k = o->maximum_k;
    p.channels = channels;
    p.bps = bps;
    p.lshift = bps <= 16 ? 0u : ((bps - 16) / 8) * 8;
    p.lw_lo = o->minimum_interlacing_leftweight;
    p.lw_hi = o->maximum_interlacing_leftweight;
    {
        uint32_t k = 0;
        if (p.lw_lo == 0) {
            p.st_kind[k++] = 0; // ch0
            p.st_kind[k++] = 1; // ch1
        }
        if (p.lw_hi > 0) {
            p.st_kind[k++] = 2; // ch0 - ch1
            p.sig_first_mix = k;
            for (uint32_t lw = std::max(p.lw_lo, 1u); lw <= p.lw_hi; ++lw)
                p.st_kind[k++] = (uint16_t)(2u + lw); // ch1 + ((ch0 - ch1) lw >> 2)
        }
        p.n_st = k;
    }
    int32_t g[8][2];
    p.n_elem = alac_groups(channels, g);
    uint32_t ns = 0;
    for (uint32_t e = 0; e < p.n_elem; ++e) {
        p.elem_ch[e][0] = g[e][0];
        p.elem_ch[e][1] = g[e][1];
        p.elem_sig[e] = ns;
        ns += g[e][1] >= 0 ? p.n_st : 1;
    }
    p.n_sig = ns;
    P.fs.clear();
    P.tracks.assign(n, TrackInfoA());
    P.slot.assign(n, 0);
    uint64_t out = 0;
    for (uint32_t t = 0; t < n; ++t) {
        const atg_track &T = tracks[t];
        TrackInfoA &ti = P.tracks[t];
        ti.first_fs = (uint32_t)P.fs.size();
        uint64_t bound = 8;
        auto add = [&](uint64_t start, uint32_t len) {
            FsInfo f;
            f.pcm_start = T.pcm_offset + start;
            f.n = len;
            f.track = t;
            f.pad = 0;
            auto it = enc->win_off.find(len);
            if (it == enc->win_off.end()) {
                const uint32_t off = (uint32_t)enc->win_host.size();
                enc->win_host.resize(off + len);
                alac_window(len, enc->win_host.data() + off);
                it = enc->win_off.emplace(len, off).first;
            }
            f.win_off = it->second;
            P.fs.push_back(f);
            bound += fs_bound(len, channels, bps);
        };
        if (T.frame_sizes) {
            uint64_t pos = 0;
            for (uint64_t k = 0; k < T.n_frame_sizes; ++k) {
                const uint32_t len = T.frame_sizes[k];
                if (len < 1 || len > kMaxBlock)
                    return afail(ATG_ERR_INVALID, "frame sizes must be 1..65535");
                add(pos, len);
                pos += len;
            }
            if (pos != T.pcm_frames)
                return afail(ATG_ERR_INVALID, "frame sizes must sum to pcm_frames");
        } else {
            for (uint64_t pos = 0; pos < T.pcm_frames; pos += o->block_size)
                add(pos, (uint32_t)std::min<uint64_t>(o->block_size, T.pcm_frames - pos));
        }
        ti.n_fs = (uint32_t)P.fs.size() - ti.first_fs;
        ti.out_base = out;
        P.slot[t] = (bound + 15) & ~15ull;
        out += P.slot[t];
    }
    p.n_fs = (uint32_t)P.fs.size();
    p.n_tracks = n;
    P.out_bytes = out;
    return ATG_OK;
}

template <typename T>
atg_status alac_run(atg_alac_encoder *enc, const APlan &P, const T *d_pcm, uint8_t *d_out,
                    atg_alac_track_result *res, uint32_t *fs_bytes)
{
    hipStream_t s = enc->s;
    const AlacParams &p = P.p;
    const uint64_t nfs = p.n_fs, nsig = nfs * p.n_sig, nel = nfs * p.n_elem;
    const uint32_t n = p.n_tracks;
    AHIP(hipMemcpyToSymbolAsync(HIP_SYMBOL(c_p), &p, sizeof(p), 0, hipMemcpyHostToDevice, s));
    AHIP(enc->fs.ensure(sizeof(FsInfo) * std::max<uint64_t>(nfs, 1)));
    AHIP(enc->tracks.ensure(sizeof(TrackInfoA) * std::max<uint32_t>(n, 1)));
    AHIP(enc->lpc.ensure(sizeof(SigLpc) * std::max<uint64_t>(nsig, 1)));
    AHIP(enc->c4.ensure(sizeof(ChainOut) * std::max<uint64_t>(nsig, 1)));
    AHIP(enc->c8.ensure(sizeof(ChainOut) * std::max<uint64_t>(nsig, 1)));
    AHIP(enc->ed.ensure(sizeof(ElemDesc) * std::max<uint64_t>(nel, 1)));
    AHIP(enc->fd.ensure(sizeof(FsDesc) * std::max<uint64_t>(nfs, 1)));
    AHIP(enc->mdat.ensure(sizeof(uint64_t) * std::max<uint32_t>(n, 1)));
    if (enc->win_host.size() > enc->win_uploaded || !enc->win.p) {
        AHIP(enc->win.ensure(sizeof(double) * std::max<size_t>(enc->win_host.size(), 1)));
        if (!enc->win_host.empty())
            AHIP(hipMemcpyAsync(enc->win.p, enc->win_host.data(),
                                sizeof(double) * enc->win_host.size(), hipMemcpyHostToDevice, s));
        enc->win_uploaded = enc->win_host.size();
    }
    if (nfs)
        AHIP(hipMemcpyAsync(enc->fs.p, P.fs.data(), sizeof(FsInfo) * nfs, hipMemcpyHostToDevice,
                            s));
    if (n)
        AHIP(hipMemcpyAsync(enc->tracks.p, P.tracks.data(), sizeof(TrackInfoA) * n,
                            hipMemcpyHostToDevice, s));
    // the frames are OR-ed into place: clear every track's slot
    if (P.out_bytes)
        AHIP(hipMemsetAsync(d_out, 0, P.out_bytes, s));
    const FsInfo *dfs = (const FsInfo *)enc->fs.p;
    AHIP(hipEventRecord(enc->ev[0], s));
    if (nsig)
        hipLaunchKernelGGL(k_alac_lpc<T>, dim3((unsigned)((nsig + 63) / 64)), dim3(64), 0, s,
                           d_pcm, dfs, (const double *)enc->win.p, (SigLpc *)enc->lpc.p);
    AHIP(hipGetLastError());
    AHIP(hipEventRecord(enc->ev[1], s));
    if (nsig) {
        hipLaunchKernelGGL((k_alac_chain<4, T>), dim3((unsigned)((nsig + 63) / 64)), dim3(64), 0,
                           s, d_pcm, dfs, (const SigLpc *)enc->lpc.p, (ChainOut *)enc->c4.p);
        hipLaunchKernelGGL((k_alac_chain<8, T>), dim3((unsigned)((nsig + 63) / 64)), dim3(64), 0,
                           s, d_pcm, dfs, (const SigLpc *)enc->lpc.p, (ChainOut *)enc->c8.p);
    }
    AHIP(hipGetLastError());
    AHIP(hipEventRecord(enc->ev[2], s));
    if (nfs)
        hipLaunchKernelGGL(k_alac_decide, dim3((unsigned)((nfs + 63) / 64)), dim3(64), 0, s, dfs,
                           (const SigLpc *)enc->lpc.p, (const ChainOut *)enc->c4.p,
                           (const ChainOut *)enc->c8.p, (ElemDesc *)enc->ed.p,
                           (FsDesc *)enc->fd.p);
    AHIP(hipGetLastError());
    AHIP(hipEventRecord(enc->ev[3], s));
    if (n)
        hipLaunchKernelGGL(k_alac_scan, dim3((n + 63) / 64), dim3(64), 0, s,
                           (const TrackInfoA *)enc->tracks.p, (FsDesc *)enc->fd.p, d_out,
                           (uint64_t *)enc->mdat.p);
    AHIP(hipGetLastError());
    AHIP(hipEventRecord(enc->ev[4], s));
    if (nel)
        hipLaunchKernelGGL(k_alac_pack<T>, dim3((unsigned)((nel + 63) / 64)), dim3(64), 0, s,
                           d_pcm, dfs, (const TrackInfoA *)enc->tracks.p,
                           (const SigLpc *)enc->lpc.p, (const ElemDesc *)enc->ed.p,
                           (const FsDesc *)enc->fd.p, d_out);
    AHIP(hipGetLastError());
    AHIP(hipEventRecord(enc->ev[5], s));
    std::vector<uint64_t> mdat(n);
    std::vector<FsDesc> fd(nfs);
    if (n)
        AHIP(hipMemcpyAsync(mdat.data(), enc->mdat.p, sizeof(uint64_t) * n,
                            hipMemcpyDeviceToHost, s));
    if (nfs)
        AHIP(hipMemcpyAsync(fd.data(), enc->fd.p, sizeof(FsDesc) * nfs, hipMemcpyDeviceToHost,
                            s));
    AHIP(hipStreamSynchronize(s));
    for (int k = 0; k < kATimed - 1; ++k)
        (void)hipEventElapsedTime(&enc->times[k], enc->ev[k], enc->ev[k + 1]);
    (void)hipEventElapsedTime(&enc->times[kATimed - 1], enc->ev[0], enc->ev[kATimed - 1]);
    enc->have_times = true;
    for (uint32_t t = 0; t < n; ++t) {
        atg_alac_track_result &r = res[t];
        r.out_offset = P.tracks[t].out_base;
        r.bytes = mdat[t];
        r.first_frameset = P.tracks[t].first_fs;
        r.n_framesets = P.tracks[t].n_fs;
        r.pcm_frames = 0;
        for (uint32_t k = 0; k < P.tracks[t].n_fs; ++k)
            r.pcm_frames += P.fs[P.tracks[t].first_fs + k].n;
        r.status = r.bytes > P.slot[t] ? ATG_ERR_CAPACITY : 0;
        r.reserved = 0;
    }
    if (fs_bytes)
        for (uint64_t k = 0; k < nfs; ++k)
            fs_bytes[k] = fd[k].bytes;
    return ATG_OK;
}

} // namespace

extern "C" {

const char *atg_alac_last_error(void) { return g_alac_err.c_str(); }

atg_status atg_alac_encoder_create(int device, atg_alac_encoder **out)
{
    if (!out)
        return afail(ATG_ERR_INVALID, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return afail(ATG_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= n)
        return afail(ATG_ERR_INVALID, "device index out of range");
    AHIP(hipSetDevice(device));
    atg_alac_encoder *e = new atg_alac_encoder();
    e->device = device;
    AHIP(hipStreamCreateWithFlags(&e->s, hipStreamNonBlocking));
    for (auto &ev : e->ev)
        AHIP(hipEventCreate(&ev));
    *out = e;
    return ATG_OK;
}

void atg_alac_encoder_destroy(atg_alac_encoder *e)
{
    if (!e)
        return;
    (void)hipSetDevice(e->device);
    (void)hipStreamSynchronize(e->s);
    for (ABuf *b : {&e->fs, &e->tracks, &e->win, &e->lpc, &e->c4, &e->c8, &e->ed, &e->fd,
                    &e->mdat, &e->h_pcm, &e->h_out})
        b->release();
    for (auto &ev : e->ev)
        (void)hipEventDestroy(ev);
    (void)hipStreamDestroy(e->s);
    delete e;
}

atg_status atg_alac_batch_bounds(atg_alac_encoder *e, const atg_alac_options *o,
                                 const atg_track *tracks, uint32_t n, uint32_t channels,
                                 uint32_t bps, uint64_t *total_framesets, uint64_t *out_bytes)
{
    ATG_HANDLE_LOCK(e);
    if (!e || (!tracks && n))
        return afail(ATG_ERR_INVALID, "NULL argument");
    APlan P;
    atg_status st = alac_plan(e, o, tracks, n, channels, bps, P);
    if (st != ATG_OK)
        return st;
    if (total_framesets)
        *total_framesets = P.fs.size();
    if (out_bytes)
        *out_bytes = P.out_bytes;
    return ATG_OK;
}

atg_status atg_alac_encode_device(atg_alac_encoder *e, const atg_alac_options *o,
                                  const void *d_pcm, atg_pcm_format fmt, const atg_track *tracks,
                                  uint32_t n, uint32_t channels, uint32_t bps, void *d_out,
                                  uint64_t out_cap, atg_alac_track_result *results,
                                  uint32_t *frameset_bytes)
{
    ATG_HANDLE_LOCK(e);
    if (!e || (!tracks && n) || (!results && n))
        return afail(ATG_ERR_INVALID, "NULL argument");
    if (((uintptr_t)d_out) & 3)
        return afail(ATG_ERR_INVALID, "d_out must be 4-byte aligned");
    if (fmt == ATG_PCM_S16 && bps > 16)
        return afail(ATG_ERR_INVALID, "S16 PCM holds at most 16-bit samples");
    AHIP(hipSetDevice(e->device));
    APlan P;
    atg_status st = alac_plan(e, o, tracks, n, channels, bps, P);
    if (st != ATG_OK)
        return st;
    if (P.out_bytes > out_cap)
        return afail(ATG_ERR_CAPACITY, "output buffer smaller than atg_alac_batch_bounds");
    if (fmt == ATG_PCM_S16)
        return alac_run(e, P, (const int16_t *)d_pcm, (uint8_t *)d_out, results, frameset_bytes);
    return alac_run(e, P, (const int32_t *)d_pcm, (uint8_t *)d_out, results, frameset_bytes);
}

atg_status atg_alac_encode_host(atg_alac_encoder *e, const atg_alac_options *o, const void *pcm,
                                atg_pcm_format fmt, const atg_track *tracks, uint32_t n,
                                uint32_t channels, uint32_t bps, uint8_t *out, uint64_t out_cap,
                                atg_alac_track_result *results, uint32_t *frameset_bytes)
{
    ATG_HANDLE_LOCK(e);
    if (!e || (!tracks && n) || (!results && n) || (!pcm && n))
        return afail(ATG_ERR_INVALID, "NULL argument");
    AHIP(hipSetDevice(e->device));
    APlan P;
    atg_status st = alac_plan(e, o, tracks, n, channels, bps, P);
    if (st != ATG_OK)
        return st;
    if (P.out_bytes > out_cap)
        return afail(ATG_ERR_CAPACITY, "output buffer smaller than atg_alac_batch_bounds");
    uint64_t frames = 0;
    for (uint32_t t = 0; t < n; ++t)
        frames = std::max<uint64_t>(frames, tracks[t].pcm_offset + tracks[t].pcm_frames);
    const size_t es = fmt == ATG_PCM_S16 ? 2 : 4;
    const uint64_t in_bytes = frames * channels * es;
    AHIP(e->h_pcm.ensure(std::max<uint64_t>(in_bytes, 4)));
    AHIP(e->h_out.ensure(std::max<uint64_t>(P.out_bytes, 4)));
    if (in_bytes)
        AHIP(hipMemcpyAsync(e->h_pcm.p, pcm, in_bytes, hipMemcpyHostToDevice, e->s));
    st = fmt == ATG_PCM_S16
             ? alac_run(e, P, (const int16_t *)e->h_pcm.p, (uint8_t *)e->h_out.p, results,
                        frameset_bytes)
             : alac_run(e, P, (const int32_t *)e->h_pcm.p, (uint8_t *)e->h_out.p, results,
                        frameset_bytes);
    if (st != ATG_OK)
        return st;
    if (P.out_bytes)
        AHIP(hipMemcpyAsync(out, e->h_out.p, P.out_bytes, hipMemcpyDeviceToHost, e->s));
    AHIP(hipStreamSynchronize(e->s));
    return ATG_OK;
}

int atg_alac_encoder_kernel_times(atg_alac_encoder *e, const char **names, float *ms, int cap)
{
    ATG_HANDLE_LOCK(e);
    if (!e || !e->have_times)
        return 0;
    const int k = cap < kATimed ? cap : kATimed;
    for (int i = 0; i < k; ++i) {
        if (names)
            names[i] = kANames[i];
        if (ms)
            ms[i] = e->times[i];
    }
    return k;
}

} // extern "C"
