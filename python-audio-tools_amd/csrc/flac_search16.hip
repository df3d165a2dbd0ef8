// flac_search16.hip — K2 fast path: the subframe search for full 4096-sample
// frames of sources whose samples fit int16.  Same decisions and the same
// uint32 bit counts as k_subframe_search (flac_search.hip; reference
// flacenc_write_subframe, src/encoders/flac.c:673-1016, 1326-1505,
// 1578-1631); any candidate it cannot take is handed to that kernel through
// a list.
//
// Two kernels:
//   k_frame_search_ms   stereo with mid/side (the FLAC-8 case): one
//                       256-thread workgroup per frame, wave c searches
//                       candidate c.  The frame's PCM is read once and LDS
//                       holds L, R and M = (L + R) >> 1 as packed int16
//                       pairs (28 KB per frame: 4 frames per CU); the side
//                       channel S = L - R (17 bits) is never stored: its
//                       predictor takes one v_dot2 per tap on (L, R) words
//                       (one v_perm of the L and R images per sample) with
//                       taps (c, -c) (exact, linear).
//   k_subframe_search16 any other layout: one wave per candidate with its
//                       own packed array (candidates outside int16 are
//                       handed over).
//
// Residual arithmetic (lane l owns samples [64l, 64l + 64)).  With
// O_t = (s[t-1], s[t]) as an int16 pair (an LDS word for odd t, one
// v_alignbit of two words for even t, shared by every tap pair), tap pairs
// (c0, -2^sh), (c2, c1), (c4, c3), ... and an accumulator that starts at
// -2^(sh + w) (w = wasted bits, samples unshifted):
//     acc >> (sh + w) = floor(pred') - s' - 1 = ~r       (s' = s >> w)
// exactly -- the reference's r = s' - (sum c s' >> sh), flac.c:1060-1126 --
// whenever the true sum fits int32 (checked per predictor, wave-uniform;
// otherwise a 64-bit loop runs).  v = n ^ (n >> 31) is the same for n and
// ~n, so the loop has no subtraction and no sample unpacking: floor(order /
// 2) + 1 v_dot2 + 4 VALU per residual, wasted bits included for free.
// v = |r| - [r < 0] is kept per sample (u >> k = v >> (k - 1) for the
// zig-zag code u = 2v + [r < 0], k >= 1); #neg = 64 + sum (n >> 31).
// The seed also carries + 2^31: a logical
// shift gives x = n + 2^(31 - sh - w), sum |r| is one v_sad_u32 per sample
// (2 VALU per residual after the v_dot2s), and x is kept instead of v.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "flac_dev.h"
#include "launch.h"
#include "partsel.h"
#include "pcm_read.h"
#include "residual.h"
#include "rice.h"
#include "wave.h"

// waves per SIMD the register allocation targets
constexpr int kK2fWavesPerEu = 4;

#define PK_PRE 16
#define PK_WORDS (PK_PRE + ATG_MAX_BLOCK / 2 + 4 * (ATG_MAX_BLOCK / 64) + 16)

// word m of a packed candidate; 4 pad words after every 32 words, so lane
// runs (32 words apart) start 36 words apart: 16-byte aligned and
// conflict-free for ds_read_b128 (36 l mod 64 hits every 4-bank group of a
// 16-lane access group once).  Words -8..-1 (lane 0's history) are zeros.
__device__ __forceinline__ int paddr(int m) { return PK_PRE + m + 4 * (m >> 5); }

// low / high sample of a packed word
__device__ __forceinline__ int lo16(uint32_t w) { return (int32_t)(int16_t)(w & 0xFFFFu); }
__device__ __forceinline__ int hi16(uint32_t w) { return (int32_t)w >> 16; }

// sample i of a packed image (i >= -16), sign-extended
__device__ __forceinline__ int32_t pk_sample(const uint32_t *__restrict__ pk, int i)
{
    const uint32_t w = pk[paddr(i >> 1)];
    return (i & 1) ? hi16(w) : lo16(w);
}

// candidate sample i: a packed image (TWO = false), or L - R with the L
// image at img and the R image right after it (TWO = true, the side channel)
template <int MODE>
__device__ __forceinline__ int32_t cand_pk(const uint32_t *__restrict__ img, int i)
{
    // MODE 2: s = hi * 4096 + lo from the hi image and the lo image after it
    if (MODE == 2)
        return (pk_sample(img, i) << 12) + pk_sample(img + PK_WORDS, i);
    return MODE ? pk_sample(img, i) - pk_sample(img + PK_WORDS, i) : pk_sample(img, i);
}

__device__ __forceinline__ uint32_t align16(uint32_t hi_word, uint32_t lo_word)
{
    return __builtin_amdgcn_alignbit(hi_word, lo_word, 16);
}

__device__ __forceinline__ int dot2(uint32_t a, int b_uniform, int c)
{
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, a),
                                  __builtin_bit_cast(short2_t, b_uniform), c, false);
}

// First tap of a residual: VOP3 v_dot2 with the tap pair in a VGPR and the
// accumulator start in an SGPR (one SGPR operand per VALU instruction on
// gfx950), so no v_mov seeds an accumulator per sample.
__device__ __forceinline__ int dot2_first(uint32_t a, int tap_v, int acc_s)
{
    int d;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(tap_v), "s"(acc_s));
    return d;
}

// sa += v + s31 as one v_add3_u32 the compiler cannot re-associate (it
// otherwise defers the sums and keeps every s31 live: register pressure)
__device__ __forceinline__ void add3_acc(uint32_t &sa, uint32_t v, uint32_t s31)
{
    asm("v_add3_u32 %0, %0, %1, %2" : "+v"(sa) : "v"(v), "v"(s31));
}

// Pass-1 post-processing with a biased accumulator: the
// fold's seed carries + 2^31, so x = acc >>> shv (a full-rate logical
// shift) is n + B with n = ~r and B = 2^(31 - shv) (acc + 2^31 is the true
// int32 sum offset into [0, 2^32), and 2^31 is a multiple of 2^shv); the
// run's sum |r| = sum |x - (B - 1)| is one v_sad_u32 per sample.  Two VALU
// per residual instead of four; pass 2 recovers n = x - B.  The split and
// hi/lo folds keep their arithmetic n and store x = n ^ 2^31 (B = 2^31).
// A/B (profiles/r04_af_k2_bias_ab.jsonl): K2 6.75 -> 6.65 ms live, 7.52 ->
// 7.63 M frames/s; 0 selects the previous four-VALU form.
__device__ __forceinline__ void sad_acc(uint32_t &sa, uint32_t x, uint32_t b)
{
    asm("v_sad_u32 %0, %1, %2, %0" : "+v"(sa) : "v"(x), "v"(b));
}

// the lane index from an opaque instruction pair: a value the compiler can
// neither hoist nor share with the kernel's own, so the rare paths (split
// fold) derive their run addresses where they run instead of keeping them
// live -- or spilled to scratch, one write per thread -- across the job loop
__device__ __forceinline__ int opaque_lane()
{
    int l;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
    return l;
}

// Where pass 1 puts its per-sample x (every pass-1 form below takes one).
// PkStore keeps x's low 16 bits, two samples per register (v_perm): the
// low 16 bits of n = x - B (B's low half is 0 for shv <= 15), which are n
// itself whenever |r| < 2^15 -- checked after pass 1 from the lane sums
// (every |r| <= sum |r|).  32 registers instead of 64: what pass 1 and the
// partition search keep live no longer spills.  ReSum is pass 2 by
// recomputation, for a wave with a larger residual: the same tap chains,
// summing v >> kv (v = n ^ (n >> 31)) per sample instead of keeping x; its
// chunk loop is rolled (rare path, small code).
struct PkStore {
    static constexpr bool kStore = true;
    static constexpr int kUnroll = ATG_RUN / 8;
    uint32_t up[ATG_RUN / 2];
    uint32_t sel; // v_perm selector: bits 0..15 of both x (quiet lane) or 8..23 (loud)
    __device__ __forceinline__ void put2(int i, uint32_t x0, uint32_t x1)
    {
        up[i >> 1] = __builtin_amdgcn_perm(x1, x0, sel);
    }
};
// a lane whose last finished job of the candidate coded with k >= 9 keeps
// bits 8..23 of x instead (the same v_perm, another selector): n >> 8,
// exact for |r| < 2^23, and v >> kv = (v >> 8) >> (kv - 8) for kv >= 8
constexpr uint32_t kSelQuiet = 0x05040100u, kSelLoud = 0x06050201u;
struct ReSum {
    static constexpr bool kStore = false;
    static constexpr int kUnroll = 1;
    uint32_t kv, bias, s;
    __device__ __forceinline__ void put2(int, uint32_t x0, uint32_t x1)
    {
        const int n0 = (int)(x0 - bias), n1 = (int)(x1 - bias);
        s = s + (uint32_t)((n0 >> kv) ^ (n0 >> 31)) + (uint32_t)((n1 >> kv) ^ (n1 >> 31));
    }
};

// the chunk index a pass-1 loop addresses its next words with: in a rolled
// (ReSum) loop an opaque copy, so no address of the loop is strength-reduced
// into a value live -- or spilled, one scratch write per thread -- across
// the whole job loop
template <class Sink>
__device__ __forceinline__ int chunk_index(int c)
{
    int cc = c;
    if constexpr (!Sink::kStore)
        asm volatile("" : "+s"(cc));
    return cc;
}

typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));

// Pass 2 on PkStore's words: sum over the run of v >> kv, two samples per
// word: n = q - B_lo (v_pk_sub_u16), v = n ^ (n >> 15), v >> kv (kv >= 15
// gives 0 as v < 2^15; the 16-bit shift reads 4 bits of its amount), both
// halves summed by one v_dot2_u32_u16 -- 5 VALU per two samples where the
// 32-bit form takes 9.
__device__ __forceinline__ uint32_t packed_vsum(const uint32_t (&up)[ATG_RUN / 2], uint32_t kv,
                                                uint32_t b_lo)
{
    const unsigned short kk = (unsigned short)(kv < 15u ? kv : 15u);
    const ushort2_t kk2 = {kk, kk};
    const ushort2_t bb = {(unsigned short)b_lo, (unsigned short)b_lo};
    const ushort2_t one = {1, 1};
    uint32_t s = 0;
#pragma unroll
    for (int t = 0; t < ATG_RUN / 2; ++t) {
        const ushort2_t q = __builtin_bit_cast(ushort2_t, up[t]) - bb;
        const short2_t sg = __builtin_bit_cast(short2_t, q) >> (short)15;
        const uint32_t v = __builtin_bit_cast(uint32_t, q) ^ __builtin_bit_cast(uint32_t, sg);
        s = __builtin_amdgcn_udot2(__builtin_bit_cast(ushort2_t, v) >> kk2, one, s, false);
    }
    return s;
}

// packed int16 L - R per half word (v_pk_sub_u16): the side channel's
// packed words, exact when every |L - R| fits int16
__device__ __forceinline__ uint32_t pk_sub16(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2_t, a) - __builtin_bit_cast(short2_t, b));
}
__device__ __forceinline__ uint4 load_run4(const uint32_t *__restrict__ p, bool subr)
{
    uint4 a = *(const uint4 *)p;
    if (subr) {
        const uint4 b = *(const uint4 *)(p + PK_WORDS);
        a.x = pk_sub16(a.x, b.x);
        a.y = pk_sub16(a.y, b.y);
        a.z = pk_sub16(a.z, b.z);
        a.w = pk_sub16(a.w, b.w);
    }
    return a;
}

// A lane's window over one packed image: words -8..15 of the current
// 16-sample chunk (W) and their v_alignbit pairs (E).
struct Win {
    uint32_t W[16], E[16];
};

__device__ __forceinline__ void win_init(const uint32_t *__restrict__ run, Win &x, bool subr)
{
    const uint4 h0 = load_run4(run - 12, subr);
    const uint4 h1 = load_run4(run - 8, subr);
    x.W[8] = h0.x; x.W[9] = h0.y; x.W[10] = h0.z; x.W[11] = h0.w;
    x.W[12] = h1.x; x.W[13] = h1.y; x.W[14] = h1.z; x.W[15] = h1.w;
#pragma unroll
    for (int k = 9; k < 16; ++k)
        x.E[k] = align16(x.W[k], x.W[k - 1]);
    x.E[8] = 0;
}

// slide by one chunk: a0, a1 = words 8c .. 8c + 7 of the run
__device__ __forceinline__ void win_next(const uint4 &a0, const uint4 &a1, Win &x)
{
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        x.W[k] = x.W[8 + k];
        x.E[k] = x.E[8 + k];
    }
    x.W[8] = a0.x; x.W[9] = a0.y; x.W[10] = a0.z; x.W[11] = a0.w;
    x.W[12] = a1.x; x.W[13] = a1.y; x.W[14] = a1.z; x.W[15] = a1.w;
#pragma unroll
    for (int k = 8; k < 16; ++k)
        x.E[k] = align16(x.W[k], x.W[k - 1]);
}

// O_{t - 2j} for sample ii of the chunk
__device__ __forceinline__ uint32_t win_pair(const Win &x, int ii, int j)
{
    return (ii & 1) ? x.W[8 + (ii - 1) / 2 - j] : x.E[8 + ii / 2 - j];
}

// Pass 1 of one predictor over the lane's 64 samples, D tap pairs cp on a
// packed image.  Keeps v per sample in u[] and returns the run's sum |r| =
// sum (v + [r < 0]) = 64 + sum (v + (n >> 31)) (n >= 0 <=> r < 0); lane 0's
// warm-up samples (lane0 && i < order) are forced to n = -1 (v = 0,
// |r| = 0).  shv: the total shift sh + w, in a VGPR (a shift by an SGPR
// operand issues at half the rate on gfx950, tools/int_rate.hip).
// subr: run is the L image and the samples are L - R (the side channel
// of a frame whose |S| fits int16), packed on the fly from the R image
template <int D, class Sink>
__device__ __forceinline__ void pass1(const uint32_t *__restrict__ run, const int (&cp)[14],
                                      int c0acc, int shv, bool lane0, int order, Sink &u,
                                      uint32_t &sabs, bool subr)
{
    int tap0 = cp[0];
    asm volatile("v_mov_b32 %0, %0" : "+v"(tap0)); // the first tap pair in a VGPR
    const uint32_t bm1 = (0x80000000u >> shv) - 1u; // B - 1
    Win A;
    win_init(run, A, subr);
    // chunk c + 1's words are read while chunk c is computed
    uint4 n0 = load_run4(run, subr), n1 = load_run4(run + 4, subr);
    uint32_t sa = 0;
#pragma unroll Sink::kUnroll
    for (int c = 0; c < ATG_RUN / 16; ++c) {
        // keep each chunk's loads inside the chunk (bounds live registers)
        asm volatile("" ::: "memory");
        const int cc = chunk_index<Sink>(c);
        const uint4 a0 = n0, a1 = n1;
        if (c + 1 < ATG_RUN / 16) {
            n0 = load_run4(run + 8 * (cc + 1), subr);
            n1 = load_run4(run + 8 * (cc + 1) + 4, subr);
        }
        win_next(a0, a1, A);
        // two samples' tap chains interleaved: no dependent-issue bubble
        // after each chain
#pragma unroll
        for (int ii = 0; ii < 16; ii += 2) {
            int acc[2];
#pragma unroll
            for (int h = 0; h < 2; ++h)
                acc[h] = dot2_first(win_pair(A, ii + h, 0), tap0, c0acc);
#pragma unroll
            for (int j = 1; j < D; ++j)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    acc[h] = dot2(win_pair(A, ii + h, j), cp[j], acc[h]);
            uint32_t x[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 16 * c + ii + h;
                x[h] = (uint32_t)acc[h] >> shv;
                if (i < ATG_FAST_ORDER)
                    x[h] = (lane0 && i < order) ? bm1 : x[h];
                if (Sink::kStore)
                    sad_acc(sa, x[h], bm1);
            }
            u.put2(16 * c + ii, x[0], x[1]);
        }
    }
    sabs = sa;
}

// The same for the side channel S = L - R (17 bits): tap k of sample t is
// v_dot2((L, R)[t - k], (c_(k-1), -c_(k-1))), tap 0 the fold (-2^sh, 2^sh),
// on (L, R) words built with one v_perm per sample from the packed L and
// R images (runL, runL + PK_WORDS); TAPS = min(2D, 13) covers order
// <= 2D - 1.  Chunks of 8 samples (window: 12 history + 8 words).
__device__ __forceinline__ void lr_words(const uint4 &l, const uint4 &r, uint32_t *w)
{
    const uint32_t lw[4] = {l.x, l.y, l.z, l.w}, rw[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        w[2 * q] = __builtin_amdgcn_perm(rw[q], lw[q], 0x05040100u);     // (L[2m], R[2m])
        w[2 * q + 1] = __builtin_amdgcn_perm(rw[q], lw[q], 0x07060302u); // (L[2m+1], R[2m+1])
    }
}

// DBL (shift 15): the fold tap 2^15 does not fit int16, so tap 0 is
// (-2^14, 2^14) and is applied twice
template <int D, bool DBL, class Sink>
__device__ __forceinline__ void pass1_lr(const uint32_t *__restrict__ run, const int (&cl)[14],
                                         int c0acc, int shv, bool lane0, int order, Sink &u,
                                         uint32_t &sabs)
{
    constexpr int TAPS = 2 * D < 13 ? 2 * D : 13;
    const uint32_t *__restrict__ runR = run + PK_WORDS;
    int tap0 = cl[0];
    asm volatile("v_mov_b32 %0, %0" : "+v"(tap0)); // the first tap in a VGPR
    const uint32_t bm1 = (0x80000000u >> shv) - 1u; // B - 1
    uint32_t W[20]; // (L, R) words of samples t0 - 12 .. t0 + 7 of the current chunk
    {
        // packed words -8..-1 = samples a-16 .. a-1; keep a-12 .. a-1
        uint32_t h[16];
        lr_words(*(const uint4 *)(run - 12), *(const uint4 *)(runR - 12), h);
        lr_words(*(const uint4 *)(run - 8), *(const uint4 *)(runR - 8), h + 8);
#pragma unroll
        for (int k = 0; k < 12; ++k)
            W[8 + k] = h[4 + k];
    }
    // chunk c + 1's words are read while chunk c is computed
    uint4 nl = *(const uint4 *)run, nr = *(const uint4 *)runR;
    uint32_t sa = 0;
#pragma unroll Sink::kUnroll
    for (int c = 0; c < ATG_RUN / 8; ++c) {
        asm volatile("" ::: "memory");
        const int cc = chunk_index<Sink>(c);
#pragma unroll
        for (int k = 0; k < 12; ++k)
            W[k] = W[8 + k];
        lr_words(nl, nr, W + 12);
        if (c + 1 < ATG_RUN / 8) {
            nl = *(const uint4 *)(run + 4 * (cc + 1));
            nr = *(const uint4 *)(runR + 4 * (cc + 1));
        }
#pragma unroll
        for (int ii = 0; ii < 8; ii += 2) {
            int accs[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                accs[h] = dot2_first(W[12 + ii + h], tap0, c0acc);
                if constexpr (DBL)
                    accs[h] = dot2(W[12 + ii + h], tap0, accs[h]);
            }
#pragma unroll
            for (int k = 1; k < TAPS; ++k)
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    accs[h] = dot2(W[12 + ii + h - k], cl[k], accs[h]);
            uint32_t x[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 8 * c + ii + h;
                x[h] = (uint32_t)accs[h] >> shv;
                if (i < ATG_FAST_ORDER)
                    x[h] = (lane0 && i < order) ? bm1 : x[h];
                if (Sink::kStore)
                    sad_acc(sa, x[h], bm1);
            }
            u.put2(8 * c + ii, x[0], x[1]);
        }
    }
    sabs = sa;
}

// A lower bound on the Rice-coded bits of the wave's residuals under any
// partitioning: a lane's cnt codes with parameter k cost cnt (1 + k) +
// sum floor(u / 2^k) >= cnt k + (U + cnt) / 2^k (U = sum u), whose minimum
// over real k is cnt log2((U + cnt) ln2 / cnt) + cnt / ln2 (k = 0 when that
// log is negative: U + cnt); a coarser partition shares one k between lanes
// and costs at least the lanes' minima.  U >= 2 sum|r| - cnt (u = 2|r| or
// 2|r| - 1).  fp32 with a 4-bit margin per lane (sum|r| < 2^25 rounds by at
// most 2 in U).  Jobs are compared on exact bits; this only skips the
// partition search of a predictor that cannot win (flac.c:1326-1505 picks
// the smallest exact total, so one whose bound exceeds a finished total
// cannot be chosen).
#define K2F_PRUNED 0x3FFFFFFFu
__device__ __forceinline__ uint32_t residual_lb(uint32_t lane_sum, uint32_t cnt)
{
    const float cf = (float)cnt;
    const float U = fmaxf(2.0f * (float)lane_sum - cf, 0.0f);
    const float x = (U + cf) * 0.69314718f / cf;
    // (the integer-k minimum, two exp2 evaluations, pruned no more jobs per
    // ms of K2 than this: 6.23 vs 6.14 ms)
    const float lb = x >= 1.0f ? cf * __log2f(x) + cf * 1.44269504f : U + cf;
    const uint32_t lbi = (uint32_t)fmaxf(lb - 4.0f, 0.0f);
    return dpp_wave_sum<uint32_t>(lbi);
}

struct Eval16 {
    uint32_t bits; // residual section bits
    PartSel sel;
};

// After pass 1 (every predictor form): the lower-bound pruning and the
// partition search; false: pruned (ev says so)
template <bool RICE2 = false>
__device__ __forceinline__ bool eval_select(uint32_t lane_sum, const RunCtx &c, int order, int warm,
                                            uint32_t thr, Eval16 &ev)
{
    if (thr != 0xFFFFFFFFu && residual_lb(lane_sum, (uint32_t)(ATG_RUN - warm)) > thr) {
        // cannot beat a finished LPC job: no partition search, no exact bits
        ev.bits = K2F_PRUNED;
        ev.sel.porder = 0;
        ev.sel.method = 0;
        ev.sel.k_lane = 0;
        ev.sel.k_own = 0;
        ev.sel.hdr_bits = 0;
        return false;
    }
    if (wave_all(lane_sum < (1u << 25)))
        ev.sel = select_fast32<RICE2>(lane_sum, (uint32_t)order, c);
    else
        ev.sel = select_partitions((uint64_t)lane_sum, (uint32_t)order, c, false);
    return true;
}

// the exact residual-section bits from sh2 = sum of v >> (k - 1) (sum v
// for k = 0) over the lane's codes
__device__ __forceinline__ uint32_t eval_bits(const Eval16 &ev, uint32_t lane_sum, uint32_t sh2,
                                              int warm)
{
    const uint32_t k = ev.sel.k_lane;
    const uint32_t cnt = (uint32_t)(ATG_RUN - warm);
    // k = 0: sum u = 2 sum v + #neg = sum v + sum |r| (sh2 = sum v)
    const uint32_t lb = cnt * (1u + k) + (k ? sh2 : sh2 + lane_sum);
    return dpp_wave_sum<uint32_t>(lb) + ev.sel.hdr_bits;
}

// pass 2: the sum of v >> kv over the run, from PkStore's words when every
// |r| of the wave fits 15 bits, else by recomputation (redo fills a ReSum)
template <class Redo>
__device__ __forceinline__ uint32_t pass2_sum(const PkStore &st, uint32_t lane_sum, uint32_t kv,
                                              uint32_t bias, Redo &&redo)
{
    // loud lanes: |r| < 2^23, kv >= 8, and B (2^(31 - shv)) a multiple of 2^8
    const bool loud = st.sel == kSelLoud;
    const bool ok = loud ? lane_sum < (1u << 23) && kv >= 8u && (bias & 0xFFu) == 0u
                         : lane_sum < 32768u;
    if (wave_all(ok)) {
        const uint32_t s0 = loud ? 8u : 0u;
        return packed_vsum(st.up, kv - s0, (bias >> s0) & 0xFFFFu);
    }
    ReSum rs{kv, bias, 0u};
    redo(rs);
    return rs.s;
}

// the lanes whose next job of the candidate should keep bits 8..23 (a
// hint; any choice is exact or falls back to ReSum)
__device__ __forceinline__ void set_loud_hint(uint64_t *hint, int lane, uint32_t kv)
{
    const uint64_t m = __ballot(kv >= 9u);
    if (lane == 0)
        __atomic_store_n(hint, m, __ATOMIC_RELAXED);
}

// the same after a pass 1 that kept every x in 32 bits (the hi/lo kernel)
__device__ __forceinline__ Eval16 eval_tail(uint32_t lane_sum, const uint32_t (&u)[ATG_RUN],
                                            const RunCtx &c, int order, int warm, uint32_t thr,
                                            uint32_t bias)
{
    Eval16 ev;
    if (!eval_select<true>(lane_sum, c, order, warm, thr, ev)) // wide samples: RICE2
        return ev;
    const uint32_t kv = ev.sel.k_lane ? ev.sel.k_lane - 1u : 0u;
    uint32_t sh2 = 0;
    // v >> kv = (n >> kv) ^ (n >> 31) for n = x - B (arithmetic shifts)
#pragma unroll
    for (int t = 0; t < ATG_RUN; t += 2) {
        const int n0 = (int)(u[t] - bias), n1 = (int)(u[t + 1] - bias);
        sh2 = sh2 + (uint32_t)((n0 >> kv) ^ (n0 >> 31)) + (uint32_t)((n1 >> kv) ^ (n1 >> 31));
    }
    ev.bits = eval_bits(ev, lane_sum, sh2, warm);
    return ev;
}


// One predictor with the folded 32-bit arithmetic (caller checked the
// bounds): pass 1, partition search, exact bits.  run: the lane's run in a
// packed image, or in the (L, R) word image (TWO).
// cw: the predictor's taps as the LPC table stores them, int16 pairs
// (c_2m, c_2m+1) per dword, zero past the order (cw[6] = 0); wave-uniform.
// The tap words of one predictor: on packed words the pairs (c0, -2^sh),
// (c2, c1), (c4, c3), ... (halves of adjacent table dwords); on (L, R)
// words (lr, the side channel of a frame whose |S| exceeds int16) the fold
// (-2^sh, 2^sh), applied as (-2^14, 2^14) twice when sh = 15 (dbl), then
// (c_k, -c_k).  cw: the table's int16 pairs (c_2m, c_2m+1), zero past the
// order (cw[6] = 0).
__device__ __forceinline__ void make_taps(const uint32_t (&cw)[7], int sh, bool lr, bool dbl,
                                          int (&cq)[14])
{
    if (lr) {
        // (L, R) taps: (-2^sh, 2^sh), then (c_k, -c_k)
        const int t0 = dbl ? 1 << 14 : 1 << sh;
        cq[0] = (int)(((uint32_t)(-t0) & 0xFFFFu) | ((uint32_t)t0 << 16));
#pragma unroll
        for (int k = 1; k < 14; ++k) {
            const uint32_t d = cw[(k - 1) >> 1];
            const int ck = ((k - 1) & 1) ? hi16(d) : lo16(d);
            cq[k] = (int)(((uint32_t)ck & 0xFFFFu) | ((uint32_t)(-ck) << 16));
        }
    } else {
        // pairs (c0, -2^sh), (c2, c1), (c4, c3), ...: halves of adjacent
        // table dwords (s_pack_lh)
        cq[0] = (int)((cw[0] & 0xFFFFu) | ((uint32_t)(-(1 << sh)) << 16));
#pragma unroll
        for (int j = 1; j < 7; ++j)
            cq[j] = (int)((cw[j] & 0xFFFFu) | (cw[j - 1] & 0xFFFF0000u));
#pragma unroll
        for (int j = 7; j < 14; ++j)
            cq[j] = 0;
    }
}

// pass 1 of one predictor on the folded 32-bit arithmetic, any form
template <bool TWO, class Sink>
__device__ __forceinline__ void pass1_fold_any(const uint32_t *__restrict__ run, const int (&cq)[14],
                                               int c0acc, int shv, bool lane0, int order, bool lr,
                                               bool dbl, Sink &u, uint32_t &lane_sum)
{
    if (lr) {
        if (dbl) {
            switch (order / 2 + 1) {
            case 1: pass1_lr<1, true>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
            case 2: pass1_lr<2, true>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
            case 3: pass1_lr<3, true>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
            case 4: pass1_lr<4, true>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
            case 5: pass1_lr<5, true>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
            case 6: pass1_lr<6, true>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
            default: pass1_lr<7, true>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
            }
        } else
        switch (order / 2 + 1) {
        case 1: pass1_lr<1, false>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
        case 2: pass1_lr<2, false>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
        case 3: pass1_lr<3, false>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
        case 4: pass1_lr<4, false>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
        case 5: pass1_lr<5, false>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
        case 6: pass1_lr<6, false>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
        default: pass1_lr<7, false>(run, cq, c0acc, shv, lane0, order, u, lane_sum); break;
        }
    } else {
        switch (order / 2 + 1) {
        case 1: pass1<1>(run, cq, c0acc, shv, lane0, order, u, lane_sum, TWO); break;
        case 2: pass1<2>(run, cq, c0acc, shv, lane0, order, u, lane_sum, TWO); break;
        case 3: pass1<3>(run, cq, c0acc, shv, lane0, order, u, lane_sum, TWO); break;
        case 4: pass1<4>(run, cq, c0acc, shv, lane0, order, u, lane_sum, TWO); break;
        case 5: pass1<5>(run, cq, c0acc, shv, lane0, order, u, lane_sum, TWO); break;
        case 6: pass1<6>(run, cq, c0acc, shv, lane0, order, u, lane_sum, TWO); break;
        default: pass1<7>(run, cq, c0acc, shv, lane0, order, u, lane_sum, TWO); break;
        }
    }
}

// One predictor with the folded 32-bit arithmetic from its tap words
// (make_taps): pass 1, partition search, exact bits
template <bool TWO>
__device__ __forceinline__ Eval16 eval_fold_q(const uint32_t *__restrict__ run, const RunCtx &c,
                                              const int (&cq)[14], int order, int sh, uint32_t w,
                                              uint32_t thr, bool lr, bool dbl, uint64_t *hint)
{
    const int c0acc = (int)(0x80000000u - (1u << (sh + (int)w)));
    int shv = sh + (int)w;
    asm volatile("v_mov_b32 %0, %0" : "+v"(shv)); // keep the shift in a VGPR
    // lane 0's first `order` samples are warm-up: (lane0 && i < order) is a
    // lane mask and a scalar compare, so one v_cndmask per masked sample
    const bool lane0 = c.lane == 0;
    const int warm = lane0 ? order : 0;
    PkStore st;
    st.sel = ((__atomic_load_n(hint, __ATOMIC_RELAXED) >> c.lane) & 1u) ? kSelLoud : kSelQuiet;
    uint32_t lane_sum; // sum |r| of the run
    pass1_fold_any<TWO>(run, cq, c0acc, shv, lane0, order, lr, dbl, st, lane_sum);
    Eval16 ev;
    if (!eval_select(lane_sum, c, order, warm, thr, ev))
        return ev;
    const uint32_t kv = ev.sel.k_lane ? ev.sel.k_lane - 1u : 0u;
    set_loud_hint(hint, c.lane, kv);
    const uint32_t sh2 = pass2_sum(st, lane_sum, kv, 0x80000000u >> shv, [&](ReSum &rs) {
        uint32_t unused;
        pass1_fold_any<TWO>(run, cq, c0acc, shv, lane0, order, lr, dbl, rs, unused);
    });
    ev.bits = eval_bits(ev, lane_sum, sh2, warm);
    return ev;
}

template <bool TWO>
__device__ __forceinline__ Eval16 eval_fold(const uint32_t *__restrict__ run, const RunCtx &c,
                                            const uint32_t (&cw)[7], int order, int sh,
                                            uint32_t w, uint32_t thr, bool s16, uint64_t *hint)
{
    // s16 (side channel, every |S| <= 32767): the packed path on L - R
    // words formed on the fly -- 2 taps per v_dot2 instead of 1
    const bool lr = TWO && !s16;
    const bool dbl = lr && sh == 15; // tap 0 (-2^14, 2^14) twice
    int cq[14];
    make_taps(cw, sh, lr, dbl, cq);
    return eval_fold_q<TWO>(run, c, cq, order, sh, w, thr, lr, dbl, hint);
}

// ---- split fold: the 32-bit fold for predictors whose worst-case sum
// could leave int32 (loud side channels, large coefficient sums).  Each
// int16 sample is s = 256 h + l (h = s >> 8 signed, l = s & 255), split
// per packed word with one v_pk_ashrrev_i16 and one v_and; the same tap
// pairs run on the h words into A and on the l words into B (|A| < 2^24,
// |B| < 2^26: exact), and the shifted prediction of the 64-bit sum is
//     shv >= 8:  (A + (B >> 8)) >> (shv - 8)
//     shv <  8:  (A << (8 - shv)) + (B >> shv)
// with the -2^shv seed in A or B, so the result is ~r exactly as the fold
// gives it and everything after pass 1 is shared.  Linear, so the side
// channel's (L, R) words with taps (c, -c) split the same way.
__device__ __forceinline__ uint32_t pk_hi8(uint32_t w)
{
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(short2_t, w) >> (short)8);
}
__device__ __forceinline__ uint32_t pk_lo8(uint32_t w) { return w & 0x00FF00FFu; }
__device__ __forceinline__ uint4 split4(const uint4 &a, bool hi)
{
    return hi ? make_uint4(pk_hi8(a.x), pk_hi8(a.y), pk_hi8(a.z), pk_hi8(a.w))
              : make_uint4(pk_lo8(a.x), pk_lo8(a.y), pk_lo8(a.z), pk_lo8(a.w));
}

template <bool BIG>
__device__ __forceinline__ int split_n(int a, int b, int sa_v, int sb_v)
{
    return BIG ? (a + (b >> 8)) >> sa_v : (a << sa_v) + (b >> sb_v);
}

template <int D, bool BIG, class Sink>
__device__ __forceinline__ void pass1_split(const uint32_t *__restrict__ run, const int (&cp)[14],
                                            int seed_h, int seed_l, int sa_v, int sb_v,
                                            bool lane0, int order, Sink &u,
                                            uint32_t &sabs, bool subr)
{
    int tap0 = cp[0];
    asm volatile("v_mov_b32 %0, %0" : "+v"(tap0));
    uint32_t bm1 = 0x7FFFFFFFu; // B - 1 for B = 2^31
    asm volatile("v_mov_b32 %0, %0" : "+v"(bm1));
    Win A, B;
    {
        const uint4 h0 = load_run4(run - 12, subr), h1 = load_run4(run - 8, subr);
        const uint4 g[2] = {h0, h1};
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint4 hh = split4(g[q], true), ll = split4(g[q], false);
            A.W[8 + 4 * q] = hh.x; A.W[9 + 4 * q] = hh.y; A.W[10 + 4 * q] = hh.z; A.W[11 + 4 * q] = hh.w;
            B.W[8 + 4 * q] = ll.x; B.W[9 + 4 * q] = ll.y; B.W[10 + 4 * q] = ll.z; B.W[11 + 4 * q] = ll.w;
        }
#pragma unroll
        for (int k = 9; k < 16; ++k) {
            A.E[k] = align16(A.W[k], A.W[k - 1]);
            B.E[k] = align16(B.W[k], B.W[k - 1]);
        }
        A.E[8] = B.E[8] = 0;
    }
    uint4 n0 = load_run4(run, subr), n1 = load_run4(run + 4, subr);
    uint32_t sa = 0;
#pragma unroll Sink::kUnroll
    for (int c = 0; c < ATG_RUN / 16; ++c) {
        asm volatile("" ::: "memory");
        const int cc = chunk_index<Sink>(c);
        const uint4 a0 = n0, a1 = n1;
        if (c + 1 < ATG_RUN / 16) {
            n0 = load_run4(run + 8 * (cc + 1), subr);
            n1 = load_run4(run + 8 * (cc + 1) + 4, subr);
        }
        win_next(split4(a0, true), split4(a1, true), A);
        win_next(split4(a0, false), split4(a1, false), B);
#pragma unroll
        for (int ii = 0; ii < 16; ii += 2) {
            int ah[2], al[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                ah[h] = dot2_first(win_pair(A, ii + h, 0), tap0, seed_h);
                al[h] = dot2_first(win_pair(B, ii + h, 0), tap0, seed_l);
            }
#pragma unroll
            for (int j = 1; j < D; ++j)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    ah[h] = dot2(win_pair(A, ii + h, j), cp[j], ah[h]);
                    al[h] = dot2(win_pair(B, ii + h, j), cp[j], al[h]);
                }
            uint32_t x[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 16 * c + ii + h;
                int n = split_n<BIG>(ah[h], al[h], sa_v, sb_v);
                if (i < ATG_FAST_ORDER)
                    n = (lane0 && i < order) ? -1 : n;
                x[h] = (uint32_t)n ^ 0x80000000u;
                if (Sink::kStore)
                    sad_acc(sa, x[h], bm1);
            }
            u.put2(16 * c + ii, x[0], x[1]);
        }
    }
    sabs = sa;
}

// the side channel on (L, R) words, split: TAPS = min(2D, 13) as pass1_lr
template <int D, bool BIG, bool DBL, class Sink>
__device__ __forceinline__ void pass1_lr_split(const uint32_t *__restrict__ run, const int (&cl)[14],
                                               int seed_h, int seed_l, int sa_v, int sb_v,
                                               bool lane0, int order, Sink &u,
                                               uint32_t &sabs)
{
    constexpr int TAPS = 2 * D < 13 ? 2 * D : 13;
    const uint32_t *__restrict__ runR = run + PK_WORDS;
    int tap0 = cl[0];
    asm volatile("v_mov_b32 %0, %0" : "+v"(tap0));
    uint32_t bm1 = 0x7FFFFFFFu; // B - 1 for B = 2^31
    asm volatile("v_mov_b32 %0, %0" : "+v"(bm1));
    uint32_t WH[20], WL[20];
    {
        uint32_t h[16];
        lr_words(*(const uint4 *)(run - 12), *(const uint4 *)(runR - 12), h);
        lr_words(*(const uint4 *)(run - 8), *(const uint4 *)(runR - 8), h + 8);
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            WH[8 + k] = pk_hi8(h[4 + k]);
            WL[8 + k] = pk_lo8(h[4 + k]);
        }
    }
    uint4 nl = *(const uint4 *)run, nr = *(const uint4 *)runR;
    uint32_t sa = 0;
#pragma unroll Sink::kUnroll
    for (int c = 0; c < ATG_RUN / 8; ++c) {
        asm volatile("" ::: "memory");
        const int cc = chunk_index<Sink>(c);
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            WH[k] = WH[8 + k];
            WL[k] = WL[8 + k];
        }
        {
            uint32_t w8[8];
            lr_words(nl, nr, w8);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                WH[12 + k] = pk_hi8(w8[k]);
                WL[12 + k] = pk_lo8(w8[k]);
            }
        }
        if (c + 1 < ATG_RUN / 8) {
            nl = *(const uint4 *)(run + 4 * (cc + 1));
            nr = *(const uint4 *)(runR + 4 * (cc + 1));
        }
#pragma unroll
        for (int ii = 0; ii < 8; ii += 2) {
            int ah[2], al[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                ah[h] = dot2_first(WH[12 + ii + h], tap0, seed_h);
                al[h] = dot2_first(WL[12 + ii + h], tap0, seed_l);
                if constexpr (DBL) {
                    ah[h] = dot2(WH[12 + ii + h], tap0, ah[h]);
                    al[h] = dot2(WL[12 + ii + h], tap0, al[h]);
                }
            }
#pragma unroll
            for (int k = 1; k < TAPS; ++k)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    ah[h] = dot2(WH[12 + ii + h - k], cl[k], ah[h]);
                    al[h] = dot2(WL[12 + ii + h - k], cl[k], al[h]);
                }
            uint32_t x[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 8 * c + ii + h;
                int n = split_n<BIG>(ah[h], al[h], sa_v, sb_v);
                if (i < ATG_FAST_ORDER)
                    n = (lane0 && i < order) ? -1 : n;
                x[h] = (uint32_t)n ^ 0x80000000u;
                if (Sink::kStore)
                    sad_acc(sa, x[h], bm1);
            }
            u.put2(8 * c + ii, x[0], x[1]);
        }
    }
    sabs = sa;
}

template <bool BIG, class Sink>
__device__ __forceinline__ void pass1_split_any(const uint32_t *__restrict__ run, bool lr,
                                                const int (&cq)[14], int seed_h, int seed_l,
                                                int sa_v, int sb_v, bool lane0, int order,
                                                Sink &u, uint32_t &sabs, bool subr,
                                                bool dbl)
{
    if (lr && dbl) {
        switch (order / 2 + 1) {
        case 1: pass1_lr_split<1, BIG, true>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        case 2: pass1_lr_split<2, BIG, true>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        case 3: pass1_lr_split<3, BIG, true>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        case 4: pass1_lr_split<4, BIG, true>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        case 5: pass1_lr_split<5, BIG, true>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        case 6: pass1_lr_split<6, BIG, true>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        default: pass1_lr_split<7, BIG, true>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        }
    } else if (lr) {
        switch (order / 2 + 1) {
        case 1: pass1_lr_split<1, BIG, false>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        case 2: pass1_lr_split<2, BIG, false>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        case 3: pass1_lr_split<3, BIG, false>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        case 4: pass1_lr_split<4, BIG, false>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        case 5: pass1_lr_split<5, BIG, false>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        case 6: pass1_lr_split<6, BIG, false>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        default: pass1_lr_split<7, BIG, false>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs); break;
        }
    } else {
        switch (order / 2 + 1) {
        case 1: pass1_split<1, BIG>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs, subr); break;
        case 2: pass1_split<2, BIG>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs, subr); break;
        case 3: pass1_split<3, BIG>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs, subr); break;
        case 4: pass1_split<4, BIG>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs, subr); break;
        case 5: pass1_split<5, BIG>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs, subr); break;
        case 6: pass1_split<6, BIG>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs, subr); break;
        default: pass1_split<7, BIG>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs, subr); break;
        }
    }
}

// One predictor on the split fold (caller checked split_ok); run: the
// lane's run in the packed image, or in the L image (TWO)
template <bool TWO>
__device__ __forceinline__ Eval16 eval_split_q(const uint32_t *__restrict__ run, const RunCtx &c,
                                               const int (&cq)[14], int order, int sh, uint32_t w,
                                               uint32_t thr, bool lr, bool dbl, uint64_t *hint)
{
    const int shv = sh + (int)w;
    const bool big = shv >= 8;
    const int seed_h = big ? -(1 << (shv - 8)) : 0;
    const int seed_l = big ? 0 : -(1 << shv);
    int sa_v = big ? shv - 8 : 8 - shv, sb_v = shv;
    asm volatile("v_mov_b32 %0, %0" : "+v"(sa_v)); // shift amounts in VGPRs
    asm volatile("v_mov_b32 %0, %0" : "+v"(sb_v));
    const bool lane0 = c.lane == 0;
    const int warm = lane0 ? order : 0;
    PkStore st;
    st.sel = ((__atomic_load_n(hint, __ATOMIC_RELAXED) >> c.lane) & 1u) ? kSelLoud : kSelQuiet;
    uint32_t lane_sum;
    if (big)
        pass1_split_any<true>(run, lr, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, st, lane_sum,
                              TWO, dbl);
    else
        pass1_split_any<false>(run, lr, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, st, lane_sum,
                               TWO, dbl);
    Eval16 ev;
    if (!eval_select(lane_sum, c, order, warm, thr, ev))
        return ev;
    const uint32_t kv = ev.sel.k_lane ? ev.sel.k_lane - 1u : 0u;
    set_loud_hint(hint, c.lane, kv);
    const uint32_t sh2 = pass2_sum(st, lane_sum, kv, 0x80000000u, [&](ReSum &rs) {
        uint32_t unused;
        if (big)
            pass1_split_any<true>(run, lr, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, rs,
                                  unused, TWO, dbl);
        else
            pass1_split_any<false>(run, lr, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, rs,
                                   unused, TWO, dbl);
    });
    ev.bits = eval_bits(ev, lane_sum, sh2, warm);
    return ev;
}

template <bool TWO>
__device__ __forceinline__ Eval16 eval_split(const uint32_t *__restrict__ run, const RunCtx &c,
                                             const uint32_t (&cw)[7], int order, int sh, uint32_t w,
                                             uint32_t thr, bool s16, uint64_t *hint)
{
    const bool lr = TWO && !s16;
    const bool dbl = lr && sh == 15; // tap 0 (-2^14, 2^14) twice
    int cq[14];
    make_taps(cw, sh, lr, dbl, cq);
    return eval_split_q<TWO>(run, c, cq, order, sh, w, thr, lr, dbl, hint);
}

// Any predictor (order <= 12): 64-bit accumulation on the shifted samples,
// residuals recomputed for the exact bits.  TWO: 0 packed, 1 L - R, 2 hi/lo.
template <int TWO>
__device__ __forceinline__ Eval16 eval_wide(const uint32_t *__restrict__ img, const RunCtx &c,
                                            const uint32_t (&cw)[7], int order, int shift,
                                            uint32_t w)
{
    int cf[ATG_FAST_ORDER];
#pragma unroll
    for (int k = 0; k < ATG_FAST_ORDER; ++k)
        cf[k] = (k & 1) ? hi16(cw[k >> 1]) : lo16(cw[k >> 1]);
    uint64_t sum = 0;
    const int start = max(c.a, order);
    const int end = c.a + c.len;
    for (int i = start; i < end; ++i) {
        int64_t acc = 0;
        for (int k = 0; k < order; ++k)
            acc += (int64_t)cf[k] * (int64_t)(cand_pk<TWO>(img, i - 1 - k) >> w);
        const int r = (int)((uint32_t)(cand_pk<TWO>(img, i) >> w) -
                            (uint32_t)(int32_t)(acc >> shift));
        sum += iabs_u(r);
    }
    Eval16 ev;
    ev.sel = select_partitions(sum, (uint32_t)order, c);
    const uint32_t k = ev.sel.k_lane;
    uint32_t lb = 0;
    for (int i = start; i < end; ++i) {
        int64_t acc = 0;
        for (int k2 = 0; k2 < order; ++k2)
            acc += (int64_t)cf[k2] * (int64_t)(cand_pk<TWO>(img, i - 1 - k2) >> w);
        const int r = (int)((uint32_t)(cand_pk<TWO>(img, i) >> w) -
                            (uint32_t)(int32_t)(acc >> shift));
        lb += (zigzag(r) >> k) + 1u + k;
    }
    ev.bits = dpp_wave_sum<uint32_t>(lb) + ev.sel.hdr_bits;
    return ev;
}

// Sums of |x|, |d1| .. |d4| over the lane's run, unshifted samples (every
// term is a multiple of 2^w, so their order and ties are those of the
// shifted sums the reference compares, flac.c:856-916); samples 0..3 are
// outside the sums.  |d_k| < 2^(17 + k): 64 terms per lane < 2^28, the
// frame's sums < 2^31.  run: packed image, or (L, R) words (TWO).
template <bool TWO>
__device__ __forceinline__ uint32_t fixed_order_of(const uint32_t *__restrict__ run, int lane)
{
    uint32_t a5[5] = {0, 0, 0, 0, 0};
    int x1, x2, x3, x4;
    {
        uint4 h = *(const uint4 *)(run - 8); // packed words -4..-1: samples a-8 .. a-1
        if (TWO) {
            const uint4 g = *(const uint4 *)(run + PK_WORDS - 8);
            x1 = hi16(h.w) - hi16(g.w);
            x2 = lo16(h.w) - lo16(g.w);
            x3 = hi16(h.z) - hi16(g.z);
            x4 = lo16(h.z) - lo16(g.z);
        } else {
            x1 = hi16(h.w);
            x2 = lo16(h.w);
            x3 = hi16(h.z);
            x4 = lo16(h.z);
        }
    }
    int d1p = x1 - x2, d2p = d1p - (x2 - x3);
    int d3p = d2p - ((x2 - x3) - (x3 - x4));
    // chunks rolled: nothing here needs static indexing across chunks, and
    // an unrolled schedule computes all 64 difference chains at once
#pragma unroll 1
    for (int chn = 0; chn < ATG_RUN / 16; ++chn) {
        int x[16];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint4 a = *(const uint4 *)(run + 8 * chn + 4 * q);
            const uint32_t wa[4] = {a.x, a.y, a.z, a.w};
            uint32_t wb[4] = {0, 0, 0, 0};
            if (TWO) {
                const uint4 b = *(const uint4 *)(run + PK_WORDS + 8 * chn + 4 * q);
                wb[0] = b.x; wb[1] = b.y; wb[2] = b.z; wb[3] = b.w;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                x[8 * q + 2 * k] = lo16(wa[k]) - (TWO ? lo16(wb[k]) : 0);
                x[8 * q + 2 * k + 1] = hi16(wa[k]) - (TWO ? hi16(wb[k]) : 0);
            }
        }
        // |a - b| + acc as one v_sad_u32 on sign-flipped operands (x ^ 2^31
        // orders signed values as unsigned): |x0| = sad(x0', 2^31), |d_k| =
        // sad(d_(k-1)', d_(k-1)p') -- 12 VALU per sample instead of ~19
#pragma unroll
        for (int tt = 0; tt < 16; ++tt) {
            const int x0 = x[tt];
            const int d1 = x0 - x1, d2 = d1 - d1p, d3 = d2 - d2p;
            const bool v = chn > 0 || tt >= 4 || lane > 0;
            const uint32_t xb = (uint32_t)x0 ^ 0x80000000u, x1b = (uint32_t)x1 ^ 0x80000000u;
            const uint32_t d1b = (uint32_t)d1 ^ 0x80000000u, d1pb = (uint32_t)d1p ^ 0x80000000u;
            const uint32_t d2b = (uint32_t)d2 ^ 0x80000000u, d2pb = (uint32_t)d2p ^ 0x80000000u;
            const uint32_t d3b = (uint32_t)d3 ^ 0x80000000u, d3pb = (uint32_t)d3p ^ 0x80000000u;
            auto sad = [](uint32_t a, uint32_t b, uint32_t acc) {
                return acc + (a > b ? a - b : b - a);
            };
            const uint32_t s0 = sad(xb, 0x80000000u, a5[0]), s1 = sad(xb, x1b, a5[1]);
            const uint32_t s2 = sad(d1b, d1pb, a5[2]), s3 = sad(d2b, d2pb, a5[3]);
            const uint32_t s4 = sad(d3b, d3pb, a5[4]);
            a5[0] = v ? s0 : a5[0];
            a5[1] = v ? s1 : a5[1];
            a5[2] = v ? s2 : a5[2];
            a5[3] = v ? s3 : a5[3];
            a5[4] = v ? s4 : a5[4];
            x1 = x0;
            d1p = d1;
            d2p = d2;
            d3p = d3;
        }
    }
    uint32_t s5[5];
#pragma unroll
    for (int k = 0; k < 5; ++k)
        s5[k] = dpp_wave_sum<uint32_t>(a5[k]);
    uint32_t best = s5[0], order = 0;
#pragma unroll
    for (int k = 1; k < 5; ++k)
        if (s5[k] < best) {
            best = s5[k];
            order = (uint32_t)k;
        }
    return uniform_u32(order);
}

// Candidate extrema over the frame (unshifted), wave-uniform
struct CandStats {
    int32_t mn, mx;
    uint32_t orv;
};

// Per-candidate state a workgroup's waves share (LDS)
struct CandInfo {
    uint32_t active;      // not CONSTANT: its predictors are evaluated
    uint32_t w;           // wasted bits
    uint32_t amax;        // max |s|, unshifted
    uint32_t fixed_order; // FIXED order chosen from the difference sums
    uint32_t lo, hi;      // LPC orders evaluated
    uint32_t sbps;
};

#define K2F_MAXPRED (1 + ATG_FAST_ORDER)
// Per-(candidate, predictor) results (LDS): residual-section bits
// (partition header included), partition order, coding method and every
// lane's Rice parameter
struct PredRes {
    uint64_t loud;     // lanes that coded with k >= 9 in a finished job (PkStore hint)
    uint32_t best_lpc; // smallest LPC subframe total of the finished jobs
    uint32_t bits[K2F_MAXPRED];
    uint8_t porder[K2F_MAXPRED];
    uint8_t method[K2F_MAXPRED];
    uint8_t k[K2F_MAXPRED][64];
};

__device__ __forceinline__ uint32_t n_pred_of(const FlacParams &p, const CandInfo &ci)
{
    return (p.try_fixed ? 1u : 0u) + (p.try_lpc ? ci.hi - ci.lo + 1u : 0u);
}

__device__ __forceinline__ const uint32_t *run_of(const uint32_t *__restrict__ img, int lane)
{
    return img + PK_PRE + 36 * lane;
}


// Phase 1 of a candidate (one wave): CONSTANT (written here), wasted bits,
// the FIXED order (flac.c:856-916, 1578-1620) and the LPC orders to try
// (flac.c:1034-1126).  img: packed image, or (L, R) words (TWO).
__device__ __forceinline__ uint32_t fixed_order_hl(const uint32_t *__restrict__ run, int lane);

// Next job of the workgroup's LDS queue for the whole wave: ds_append adds
// the wave's active-lane count (64: every lane is active here) to the
// counter in one LDS operation and returns the old value, so old >> 6 is the
// job index.  (An atomicAdd from all 64 lanes on one address serialises 64
// read-modify-writes; one under `if (lane == 0)` made the loop exit
// divergent to the compiler, which then re-entered with a stale index.)
__device__ __forceinline__ uint32_t next_job(uint32_t *q)
{
    const int old = __builtin_amdgcn_ds_append((__attribute__((address_space(3))) int *)q);
    return uniform_u32((uint32_t)old) >> 6;
}

template <bool TWO, bool HL = false>
__device__ __forceinline__ void cand_prepare(const FlacParams &p, uint32_t unit, uint32_t sbps,
                                             const uint32_t *__restrict__ img, CandStats cs,
                                             int lane, const uint8_t *__restrict__ est_tab,
                                             SubDesc *__restrict__ d, CandInfo *__restrict__ ci)
{
    if (p.try_constant && cs.mn == cs.mx) {
        if (lane == 0) {
            d->bits = 8u + sbps;
            d->type = SF_CONSTANT;
            d->order = 0;
            d->wasted = 0;
            d->porder = 0;
            d->method = 0;
            d->precision = 0;
            d->shift = 0;
            d->sbps = (uint8_t)sbps;
            ci->active = 0;
        }
        return;
    }
    const uint32_t w = cs.orv ? (uint32_t)__builtin_ctz(cs.orv) : 0u;
    const uint32_t fixed_order = !p.try_fixed ? 0u
                               : HL ? fixed_order_hl(run_of(img, lane), lane)
                                    : fixed_order_of<TWO>(run_of(img, lane), lane);
    uint32_t lo = 1, hi = 0;
    if (p.try_lpc) {
        if (p.exhaustive) {
            lo = 1;
            hi = p.max_lpc_order;
        } else {
            lo = hi = est_tab[unit];
        }
    }
    if (lane == 0) {
        ci->active = 1;
        ci->w = w;
        ci->amax = max(iabs_u(cs.mn), iabs_u(cs.mx));
        ci->fixed_order = fixed_order;
        ci->lo = lo;
        ci->hi = hi;
        ci->sbps = sbps;
    }
}

__device__ __forceinline__ CandInfo load_info(const CandInfo *ci)
{
    CandInfo r;
    r.active = uniform_u32(ci->active);
    r.w = uniform_u32(ci->w);
    r.amax = uniform_u32(ci->amax);
    r.fixed_order = uniform_u32(ci->fixed_order);
    r.lo = uniform_u32(ci->lo);
    r.hi = uniform_u32(ci->hi);
    r.sbps = uniform_u32(ci->sbps);
    return r;
}

// The constants of predictor pi of a candidate (pi = 0 is FIXED when FIXED
// is tried, then LPC orders lo, lo + 1, ...): order, quantisation shift,
// tap words, the subframe header bits, and which residual path is exact.
// lq / ls: the candidate's LPC table rows and shifts, staged in LDS.
struct JobSetup {
    uint32_t o;
    int shift;
    uint32_t cw[7];
    bool is_fixed;
    uint32_t hdr, hdr_f; // LPC / FIXED header bits (residual section excluded)
    bool fold, split;    // the 32-bit fold / the split fold is exact (else 64-bit)
};

template <bool TWO>
__device__ __forceinline__ JobSetup job_setup(const FlacParams &p, const CandInfo &ci, uint32_t pi,
                                              const int16_t *__restrict__ lq,
                                              const int8_t *__restrict__ ls)
{
    JobSetup j;
    j.is_fixed = p.try_fixed && pi == 0;
    const uint32_t o = j.is_fixed ? ci.fixed_order : ci.lo + pi - (p.try_fixed ? 1u : 0u);
    j.o = o;
    int shift = 0;
    uint32_t *cw = j.cw;
    if (j.is_fixed) {
        // FIXED predictor of order o as taps (flac.c:918-1016)
        switch (o) {
        case 1: cw[0] = 1u; cw[1] = 0u; break;
        case 2: cw[0] = 2u | 0xFFFF0000u; cw[1] = 0u; break;                  // 2, -1
        case 3: cw[0] = 3u | 0xFFFD0000u; cw[1] = 1u; break;                  // 3, -3, 1
        case 4: cw[0] = 4u | 0xFFFA0000u; cw[1] = 4u | 0xFFFF0000u; break;    // 4, -6, 4, -1
        default: cw[0] = 0u; cw[1] = 0u; break;
        }
#pragma unroll
        for (int m = 2; m < 7; ++m)
            cw[m] = 0u;
    } else {
        shift = ls[o - 1u];
        const uint32_t *__restrict__ rw = (const uint32_t *)(lq + (o - 1u) * p.coef_row);
#pragma unroll
        for (int m = 0; m < 6; ++m)
            cw[m] = 2u * (uint32_t)m < p.coef_row ? rw[m] : 0u;
        cw[6] = 0u;
    }
    j.shift = shift;
    uint32_t csum = 0; // sum |c| < 12 * 2^14
#pragma unroll
    for (int m = 0; m < 6; ++m) {
        const int a = lo16(cw[m]), b = hi16(cw[m]);
        csum += (uint32_t)(a < 0 ? -a : a) + (uint32_t)(b < 0 ? -b : b);
    }
    // folded int32 sum exact: |sum c s| + 2^sh |s| + 2^(sh + w) < 2^31 on
    // unshifted samples (TWO on (L, R) words, shift 15: the fold tap
    // (-2^15, 2^15) does not fit int16 and runs as (-2^14, 2^14) twice);
    // 32-bit run sums: codes < 2^26
    const uint64_t mu = ci.amax, ms = ci.amax >> ci.w;
    const bool fold_ok = (uint64_t)csum * mu + (mu << shift) + (1ull << (shift + (int)ci.w)) <
                             (1ull << 31) &&
                         shift <= 15;
    const uint64_t rbound = ms + (((uint64_t)csum * ms) >> shift) + 1u;
    // LPC jobs: the subframe total is hdr + the residual section; a job
    // whose residual bound exceeds (best finished total - hdr) is skipped
    const uint32_t wf = ci.w ? ci.w + 1u : 1u;
    j.hdr = 7u + wf + o * (ci.sbps - ci.w) + 9u + o * p.qlp_precision;
    // FIXED too: it wins only below every LPC total
    // (flac.c:727-809, strict <), so a bound above a finished LPC total
    // rules it out the same way; its header is 7 + wf + o (sbps - w)
    j.hdr_f = 7u + wf + o * (ci.sbps - ci.w);
    // split fold (eval_split): the partial sums stay within int32 whatever
    // the coefficients (|h| <= 128 (255 for L - R), l <= 255); shv < 8
    // shifts A left, which must stay inside int32
    const uint64_t hsum = ((uint64_t)csum + (1ull << shift)) * (TWO ? 510ull : 255ull);
    const int shv = shift + (int)ci.w;
    const bool split_ok = shift <= 15 && hsum + (1ull << shv) < (1ull << 30) &&
                          (shv >= 8 || (hsum << (8 - shv)) < (1ull << 30));
    const bool codes_ok = 2u * rbound + 1u < (1ull << 26);
    j.fold = fold_ok && codes_ok;
    j.split = !j.fold && split_ok && codes_ok;
    return j;
}

// the pruning threshold of a job from the candidate's best finished LPC total
__device__ __forceinline__ uint32_t job_threshold(const PredRes *__restrict__ res, uint32_t hh)
{
    const uint32_t best = uniform_u32(__atomic_load_n(&res->best_lpc, __ATOMIC_RELAXED));
    return best == 0xFFFFFFFFu ? 0xFFFFFFFFu : best > hh ? best - hh : 0u;
}

__device__ __forceinline__ RunCtx job_ctx(const FlacParams &p, uint32_t N, int lane)
{
    RunCtx c;
    c.lane = lane;
    c.a = ATG_RUN * lane;
    c.len = ATG_RUN;
    c.N = N;
    c.max_rice = p.max_rice;
    c.P = (int)(p.max_porder < (uint32_t)ATG_MAX_PORDER ? p.max_porder : (uint32_t)ATG_MAX_PORDER);
    return c;
}

__device__ __forceinline__ void job_store(PredRes *__restrict__ res, uint32_t pi, int lane,
                                          bool is_fixed, uint32_t hdr, const Eval16 &ev)
{
    if (!is_fixed && ev.bits != K2F_PRUNED && lane == 0)
        atomicMin(&res->best_lpc, hdr + ev.bits);
    res->k[pi][lane] = (uint8_t)ev.sel.k_own;
    if (lane == 0) {
        res->bits[pi] = ev.bits;
        res->porder[pi] = (uint8_t)ev.sel.porder;
        res->method[pi] = (uint8_t)ev.sel.method;
    }
}

// One predictor of one candidate (one wave, any wave of the workgroup):
// residual-section bits and partition choice into res[pi]
template <bool TWO>
__device__ __forceinline__ void pred_job(const FlacParams &p, uint32_t N,
                                         const uint32_t *__restrict__ img, const CandInfo &ci,
                                         uint32_t pi, int lane, const int16_t *__restrict__ lq,
                                         const int8_t *__restrict__ ls,
                                         PredRes *__restrict__ res)
{
    const JobSetup j = job_setup<TWO>(p, ci, pi, lq, ls);
    const RunCtx c = job_ctx(p, N, lane);
    const uint32_t thr = job_threshold(res, j.is_fixed ? j.hdr_f : j.hdr);
    Eval16 ev;
    if (j.fold)
        ev = eval_fold<TWO>(run_of(img, lane), c, j.cw, (int)j.o, j.shift, ci.w, thr,
                            TWO && ci.amax <= 32767u, &res->loud);
    else if (j.split)
        ev = eval_split<TWO>(run_of(img, lane), c, j.cw, (int)j.o, j.shift, ci.w, thr,
                             TWO && ci.amax <= 32767u, &res->loud);
    else
        ev = eval_wide<TWO>(img, c, j.cw, (int)j.o, j.shift, ci.w);
    job_store(res, pi, lane, j.is_fixed, j.hdr, ev);
}

// k_frame_search_ms: every job's constants are formed once per frame, in
// phase 1, by the candidate's wave with one lane per predictor (vector
// arithmetic for all 13 at once), and kept in LDS as a descriptor: the tap
// words ready for v_dot2, the path, the header bits.  A job then reads
// its descriptor instead of re-deriving the bounds in scalar code (DESIGN
// 4a'' ledger: ~190 SALU per job went to that).
struct JobDesc {
    int cq[14];
    uint32_t meta; // o | shift << 4 | path << 9 | fixed << 11 | lr << 12 | dbl << 13 | w << 14
    uint32_t hh;   // header bits the pruning threshold subtracts
    uint32_t hdr;  // LPC header bits (the candidate's best total)
    uint32_t pad;
};
#define K2F_NOJOB 0xFFFFFFFFu

template <bool TWO>
__device__ __forceinline__ void jobs_prepare(const FlacParams &p, const CandInfo &ci, int lane,
                                             const int16_t *__restrict__ lq,
                                             const int8_t *__restrict__ ls,
                                             JobDesc *__restrict__ jd)
{
    if (lane >= K2F_MAXPRED)
        return;
    const uint32_t n_pred = ci.active ? n_pred_of(p, ci) : 0u;
    JobDesc *d = jd + lane;
    if ((uint32_t)lane >= n_pred) {
        d->meta = K2F_NOJOB;
        return;
    }
    const JobSetup j = job_setup<TWO>(p, ci, (uint32_t)lane, lq, ls);
    const bool lr = TWO && ci.amax > 32767u;
    const bool dbl = lr && j.shift == 15;
    int cq[14];
    make_taps(j.cw, j.shift, lr, dbl, cq);
#pragma unroll
    for (int m = 0; m < 14; ++m)
        d->cq[m] = cq[m];
    const uint32_t path = j.fold ? 0u : (j.split ? 1u : 2u);
    d->meta = j.o | ((uint32_t)j.shift << 4) | (path << 9) | ((uint32_t)j.is_fixed << 11) |
              ((uint32_t)lr << 12) | ((uint32_t)dbl << 13) | (ci.w << 14);
    d->hh = j.is_fixed ? j.hdr_f : j.hdr;
    d->hdr = j.hdr;
}

// one job from its descriptor (k_frame_search_ms); the 64-bit path, which
// needs the table words, takes them again from the candidate's rows
template <bool TWO>
__device__ __forceinline__ void pred_job_d(const FlacParams &p, uint32_t N,
                                           const uint32_t *__restrict__ img, const JobDesc *jd,
                                           uint32_t meta, uint32_t pi, int lane,
                                           const CandInfo *__restrict__ info,
                                           const int16_t *__restrict__ lq,
                                           const int8_t *__restrict__ ls,
                                           PredRes *__restrict__ res)
{
    const int o = (int)(meta & 15u), shift = (int)((meta >> 4) & 31u);
    const uint32_t path = (meta >> 9) & 3u, w = (meta >> 14) & 31u;
    const bool is_fixed = (meta >> 11) & 1u, lr = (meta >> 12) & 1u, dbl = (meta >> 13) & 1u;
    const RunCtx c = job_ctx(p, N, lane);
    const uint32_t thr = job_threshold(res, uniform_u32(jd->hh));
    Eval16 ev;
    if (path < 2u) {
        int cq[14];
#pragma unroll
        for (int m = 0; m < 7; ++m)
            cq[m] = (int)uniform_u32((uint32_t)jd->cq[m]);
        if (lr) {
#pragma unroll
            for (int m = 7; m < 14; ++m)
                cq[m] = (int)uniform_u32((uint32_t)jd->cq[m]);
        } else {
#pragma unroll
            for (int m = 7; m < 14; ++m)
                cq[m] = 0;
        }
        if (path == 0u)
            ev = eval_fold_q<TWO>(run_of(img, lane), c, cq, o, shift, w, thr, lr, dbl, &res->loud);
        else
            ev = eval_split_q<TWO>(run_of(img, opaque_lane()), c, cq, o, shift, w, thr, lr, dbl,
                                   &res->loud);
    } else {
        const JobSetup j = job_setup<TWO>(p, load_info(info), pi, lq, ls);
        ev = eval_wide<TWO>(img, c, j.cw, o, shift, w);
    }
    job_store(res, pi, lane, is_fixed, uniform_u32(jd->hdr), ev);
}

// Phase 3 of a candidate (one wave): the subframe choice (flac.c:727-809)
// from the predictor results, its SubDesc.
__device__ __forceinline__ void cand_finish(const FlacParams &p, uint32_t N, const CandInfo &ci,
                                            const PredRes *__restrict__ res, int lane,
                                            const int16_t *__restrict__ lq,
                                            const int8_t *__restrict__ ls, SubDesc *__restrict__ d)
{
    if (!ci.active)
        return;
    const uint32_t w = ci.w;
    const uint32_t wf = w ? w + 1u : 1u;
    const uint32_t rb = ci.sbps - w; // bits per warm-up / verbatim sample
    const uint32_t n_pred = n_pred_of(p, ci);
    uint32_t fixed_bits = 0;
    if (p.try_fixed)
        fixed_bits = 7u + wf + ci.fixed_order * rb + res->bits[0];
    uint32_t lpc_bits = 0xFFFFFFFFu, lpc_order = 0, lpc_pi = 0;
    int lpc_shift = 0;
    for (uint32_t pi = p.try_fixed ? 1u : 0u; pi < n_pred; ++pi) {
        const uint32_t o = ci.lo + pi - (p.try_fixed ? 1u : 0u);
        const uint32_t bits = 7u + wf + o * rb + 4u + 5u + o * p.qlp_precision + res->bits[pi];
        if (bits < lpc_bits) {
            lpc_bits = bits;
            lpc_order = o;
            lpc_pi = pi;
        }
    }
    if (lpc_order)
        lpc_shift = ls[lpc_order - 1u];
    const uint32_t verbatim_cmp = p.try_verbatim ? rb * N : 0x7FFFFFFFu;
    int pick;
    const bool F = p.try_fixed, L = p.try_lpc, V = p.try_verbatim;
    if (F && L && V) {
        const uint32_t m = lpc_bits < verbatim_cmp ? lpc_bits : verbatim_cmp;
        pick = fixed_bits < m ? SF_FIXED : (lpc_bits < verbatim_cmp ? SF_LPC : SF_VERBATIM);
    } else if (!F && !L) {
        pick = SF_VERBATIM;
    } else if (F && !L && !V) {
        pick = SF_FIXED;
    } else if (!F && L && !V) {
        pick = SF_LPC;
    } else if (F && L && !V) {
        pick = fixed_bits < lpc_bits ? SF_FIXED : SF_LPC;
    } else if (F && !L && V) {
        pick = fixed_bits < verbatim_cmp ? SF_FIXED : SF_VERBATIM;
    } else {
        pick = lpc_bits < verbatim_cmp ? SF_LPC : SF_VERBATIM;
    }
    const uint32_t spi = pick == SF_FIXED ? 0u : lpc_pi;
    const uint32_t po = res->porder[spi];
    if (pick != SF_VERBATIM) {
        // rice parameter of partition j is held by its first lane
        const uint32_t mask = (64u >> po) - 1u;
        if (((uint32_t)lane & mask) == 0u)
            d->rice[(uint32_t)lane >> (6u - po)] = res->k[spi][lane];
    }
    if (pick == SF_LPC) {
        if (lane < (int)lpc_order)
            d->coef[lane] = lq[(lpc_order - 1u) * p.coef_row + lane];
    }
    if (lane == 0) {
        d->type = (uint8_t)pick;
        d->wasted = (uint8_t)w;
        d->sbps = (uint8_t)ci.sbps;
        d->amax = ci.amax >> w; // exact: the low w bits of every sample are 0
        d->method = res->method[spi];
        d->porder = (uint8_t)po;
        if (pick == SF_FIXED) {
            d->bits = fixed_bits;
            d->order = (uint8_t)ci.fixed_order;
            d->precision = 0;
            d->shift = 0;
        } else if (pick == SF_LPC) {
            d->bits = lpc_bits;
            d->order = (uint8_t)lpc_order;
            d->precision = (uint8_t)p.qlp_precision;
            d->shift = (int8_t)lpc_shift;
        } else {
            d->bits = 7u + wf + rb * N;
            d->order = 0;
            d->precision = 0;
            d->shift = 0;
            d->method = 0;
            d->porder = 0;
        }
    }
}


// wave-uniform min / max / OR of per-lane values
__device__ __forceinline__ CandStats wave_stats(int32_t mn, int32_t mx, uint32_t orv)
{
    CandStats s;
    s.orv = dpp_wave_or_u32(orv);
    // through the biased unsigned order
    s.mx = (int32_t)(dpp_wave_max_u32((uint32_t)mx ^ 0x80000000u) ^ 0x80000000u);
    s.mn = (int32_t)(~dpp_wave_max_u32(~((uint32_t)mn ^ 0x80000000u)) ^ 0x80000000u);
    return s;
}

__device__ __forceinline__ void stats_add(const int32_t (&s)[4], int32_t &mn, int32_t &mx,
                                          uint32_t &orv)
{
    mn = min(mn, min(min(s[0], s[1]), min(s[2], s[3])));
    mx = max(mx, max(max(s[0], s[1]), max(s[2], s[3])));
    orv |= (uint32_t)s[0] | (uint32_t)s[1] | (uint32_t)s[2] | (uint32_t)s[3];
}

__device__ __forceinline__ uint2 pack4(const int32_t (&s)[4])
{
    uint2 w;
    w.x = __builtin_amdgcn_perm((uint32_t)s[1], (uint32_t)s[0], 0x05040100u);
    w.y = __builtin_amdgcn_perm((uint32_t)s[3], (uint32_t)s[2], 0x05040100u);
    return w;
}

// ---------------------------------------------------------------------------
// stereo with mid/side: one workgroup (4 waves) per frame

// 4 stereo PCM frames starting at j0: left / right samples
template <bool A16, typename T>
__device__ __forceinline__ void load_lr4(const T *__restrict__ src, uint32_t j0, int32_t (&l)[4],
                                         int32_t (&r)[4])
{
    if constexpr (sizeof(T) == 2 && A16) {
        const uint4 v = *(const uint4 *)((const uint32_t *)src + j0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            l[q] = lo16(w[q]);
            r[q] = hi16(w[q]);
        }
    } else {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            l[q] = (int32_t)src[2u * (j0 + q)];
            r[q] = (int32_t)src[2u * (j0 + q) + 1u];
        }
    }
}

template <bool A16, typename T>
__device__ __forceinline__ void stage_ms(const T *__restrict__ src, int tid, uint32_t *__restrict__ img,
                                         int32_t (&mn)[4], int32_t (&mx)[4], uint32_t (&orv)[4])
{
#pragma unroll
    for (int m = 0; m < ATG_MAX_BLOCK / 1024; ++m) {
        const uint32_t q0 = (uint32_t)(tid + 256 * m); // 4-frame group
        int32_t s[4][4];
        load_lr4<A16>(src, 4u * q0, s[0], s[1]);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            s[2][q] = (int32_t)((uint32_t)s[0][q] + (uint32_t)s[1][q]) >> 1;
            s[3][q] = (int32_t)((uint32_t)s[0][q] - (uint32_t)s[1][q]);
        }
#pragma unroll
        for (int cnd = 0; cnd < 4; ++cnd)
            stats_add(s[cnd], mn[cnd], mx[cnd], orv[cnd]);
#pragma unroll
        for (int cnd = 0; cnd < 3; ++cnd)
            *(uint2 *)&img[cnd * PK_WORDS + paddr(2 * (int)q0)] = pack4(s[cnd]);

    }
}


template <typename T>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kK2fWavesPerEu))) void k_frame_search_ms(
    FlacParams p, const T *__restrict__ pcm, const FrameInfo *__restrict__ frames,
    const int16_t *__restrict__ coef_tab, const int8_t *__restrict__ shift_tab,
    const uint8_t *__restrict__ est_tab, SubDesc *__restrict__ out,
    uint32_t *__restrict__ slow_list, uint32_t *__restrict__ slow_count)
{
    __shared__ __attribute__((aligned(16))) uint32_t img[3 * PK_WORDS]; // L, R, M packed
    __shared__ int32_t red[4][4][3];                                      // [wave][cand][mn,mx,or]
    __shared__ CandInfo info[4];
    __shared__ PredRes res[4];
    __shared__ JobDesc jdesc[4][K2F_MAXPRED];
    __shared__ uint32_t qnext;
    // the frame's LPC tables (4 candidates x M rows) and shifts
    __shared__ __attribute__((aligned(16))) uint32_t lq32[4 * ATG_FAST_ORDER * ATG_FAST_ORDER / 2];
    __shared__ uint32_t ls32[ATG_FAST_ORDER];

    const uint32_t f = blockIdx.x;
    if (f >= p.n_frames)
        return;
    const int tid = threadIdx.x;
    // the wave index in an SGPR: the candidate's table addresses are scalar
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const FrameInfo fi = frames[f];
    const uint32_t N = fi.n;
    if (N != ATG_MAX_BLOCK) {
        if (tid < 4) {
            const uint32_t slot = atomicAdd(slow_count, 1u);
            slow_list[slot] = f * 4u + (uint32_t)tid;
        }
        return;
    }
    if (tid < 3 * PK_PRE)
        img[(tid / PK_PRE) * PK_WORDS + (tid % PK_PRE)] = 0u;
    else if (tid == 255)
        qnext = 0u;
    {
        // the 4 candidates' tables are contiguous (unit = 4 f + cand)
        const uint32_t nq = 2u * p.coef_stride, ns = p.max_lpc_order;
        const uint32_t *__restrict__ gq = (const uint32_t *)(coef_tab + (size_t)f * 4u * p.coef_stride);
        const uint32_t *__restrict__ gs = (const uint32_t *)(shift_tab + (size_t)f * 4u * p.max_lpc_order);
        for (uint32_t i = (uint32_t)tid; i < nq; i += 256u)
            lq32[i] = gq[i];
        if ((uint32_t)tid < ns)
            ls32[tid] = gs[tid];
    }
    int32_t mn[4], mx[4];
    uint32_t orv[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        mn[k] = INT32_MAX;
        mx[k] = INT32_MIN;
        orv[k] = 0;
    }
    {
        const T *__restrict__ src = pcm + fi.pcm_start * 2u;
        if ((((uintptr_t)src) & 15u) == 0u)
            stage_ms<true>(src, tid, img, mn, mx, orv);
        else
            stage_ms<false>(src, tid, img, mn, mx, orv);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const CandStats s = wave_stats(mn[k], mx[k], orv[k]);
        if (lane == 0) {
            red[wave][k][0] = s.mn;
            red[wave][k][1] = s.mx;
            red[wave][k][2] = (int32_t)s.orv;
        }
    }
    __syncthreads();
    // L, R and M fit int16 for any source of <= 16 bits; S is L - R
    bool fits = true;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const int32_t a = min(min(red[0][k][0], red[1][k][0]), min(red[2][k][0], red[3][k][0]));
        const int32_t b = max(max(red[0][k][1], red[1][k][1]), max(red[2][k][1], red[3][k][1]));
        fits = fits && a >= -32768 && b <= 32767;
    }
    if (!fits) {
        if (tid < 4) {
            const uint32_t slot = atomicAdd(slow_count, 1u);
            slow_list[slot] = f * 4u + (uint32_t)tid;
        }
        return;
    }

    // phase 1: wave c prepares candidate c
    const uint32_t cand = (uint32_t)wave;
    const uint32_t unit = f * 4u + cand;
    {
        CandStats cs;
        cs.mn = min(min(red[0][cand][0], red[1][cand][0]), min(red[2][cand][0], red[3][cand][0]));
        cs.mx = max(max(red[0][cand][1], red[1][cand][1]), max(red[2][cand][1], red[3][cand][1]));
        cs.orv = (uint32_t)(red[0][cand][2] | red[1][cand][2] | red[2][cand][2] | red[3][cand][2]);
        cs.mn = uniform_i32(cs.mn);
        cs.mx = uniform_i32(cs.mx);
        cs.orv = uniform_u32(cs.orv);
        const uint32_t sbps = p.bps + (cand == 3u ? 1u : 0u);
        if (cand == 3u)
            cand_prepare<true>(p, unit, sbps, img, cs, lane, est_tab, out + unit, &info[3]);
        else
            cand_prepare<false>(p, unit, sbps, img + cand * PK_WORDS, cs, lane, est_tab,
                                out + unit, &info[cand]);
        if (lane == 0) {
            res[cand].best_lpc = 0xFFFFFFFFu;
            res[cand].loud = 0u;
        }
    }
    __syncthreads();
    // phase 1b: wave c forms candidate c's job descriptors, a lane per job
    {
        const CandInfo ci = load_info(&info[cand]);
        const int16_t *lq = (const int16_t *)lq32 + cand * p.coef_stride;
        const int8_t *ls = (const int8_t *)ls32 + cand * p.max_lpc_order;
        if (cand == 3u)
            jobs_prepare<true>(p, ci, lane, lq, ls, jdesc[3]);
        else
            jobs_prepare<false>(p, ci, lane, lq, ls, jdesc[cand]);
    }
    __syncthreads();

    // phase 2: the (candidate, predictor) jobs, dynamically shared by the 4
    // waves, the costliest first (highest orders, side channel first): the
    // waves finish together although a side-channel residual costs up to
    // twice a packed one
    const uint32_t jmax = (p.try_fixed ? 1u : 0u) +
                          (p.try_lpc ? (p.exhaustive ? p.max_lpc_order : 1u) : 0u);
    const uint32_t njobs = 4u * jmax;
    for (;;) {
        const uint32_t j = next_job(&qnext);
        if (j >= njobs)
            break;
        const uint32_t jc = (j + 3u) & 3u; // 3, 0, 1, 2
        const uint32_t pi = jmax - 1u - (j >> 2);
        const JobDesc *jd = &jdesc[jc][pi];
        const uint32_t meta = uniform_u32(jd->meta);
        if (meta == K2F_NOJOB)
            continue;
        const int16_t *lq = (const int16_t *)lq32 + jc * p.coef_stride;
        const int8_t *ls = (const int8_t *)ls32 + jc * p.max_lpc_order;
        if (jc == 3u)
            pred_job_d<true>(p, N, img, jd, meta, pi, lane, &info[3], lq, ls, &res[3]);
        else
            pred_job_d<false>(p, N, img + jc * PK_WORDS, jd, meta, pi, lane, &info[jc], lq, ls,
                              &res[jc]);
    }
    __syncthreads();

    // phase 3: wave c writes candidate c
    cand_finish(p, N, load_info(&info[cand]), &res[cand], lane,
                (const int16_t *)lq32 + cand * p.coef_stride,
                (const int8_t *)ls32 + cand * p.max_lpc_order, out + unit);
}

// ---------------------------------------------------------------------------
// any other layout: one wave per candidate

// 4 consecutive candidate samples starting at PCM frame j0
enum { CS_L = 0, CS_R = 1, CS_AVG = 2, CS_DIF = 3, CS_CH = 4 };
template <int CS, typename T>
__device__ __forceinline__ void load4(const T *__restrict__ src, uint32_t j0, uint32_t ch,
                                      uint32_t cand, int32_t (&s)[4])
{
    if constexpr (CS == CS_CH) {
#pragma unroll
        for (int q = 0; q < 4; ++q)
            s[q] = (int32_t)src[(size_t)(j0 + q) * ch + cand];
    } else {
        int32_t l[4], r[4];
        load_lr4<false>(src, j0, l, r);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (CS == CS_L) s[q] = l[q];
            else if (CS == CS_R) s[q] = r[q];
            else if (CS == CS_AVG) s[q] = (int32_t)((uint32_t)l[q] + (uint32_t)r[q]) >> 1;
            else s[q] = (int32_t)((uint32_t)l[q] - (uint32_t)r[q]);
        }
    }
}

template <int CS, typename T>
__device__ __forceinline__ void stage16(const T *__restrict__ src, uint32_t ch, uint32_t cand,
                                        int lane, uint32_t *__restrict__ pk, int32_t &mn,
                                        int32_t &mx, uint32_t &orv)
{
#pragma unroll 4
    for (int m = 0; m < ATG_MAX_BLOCK / 256; ++m) {
        const uint32_t q0 = (uint32_t)(lane + 64 * m); // 4-sample group
        int32_t s[4];
        load4<CS>(src, 4u * q0, ch, cand, s);
        stats_add(s, mn, mx, orv);
        *(uint2 *)&pk[paddr(2 * (int)q0)] = pack4(s);
    }
}

template <typename T>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kK2fWavesPerEu))) void k_subframe_search16(
    FlacParams p, const T *__restrict__ pcm, const FrameInfo *__restrict__ frames,
    const int16_t *__restrict__ coef_tab, const int8_t *__restrict__ shift_tab,
    const uint8_t *__restrict__ est_tab, SubDesc *__restrict__ out,
    uint32_t *__restrict__ slow_list, uint32_t *__restrict__ slow_count)
{
    __shared__ __attribute__((aligned(16))) uint32_t pk[PK_WORDS];
    __shared__ CandInfo info;
    __shared__ PredRes res;
    __shared__ __attribute__((aligned(16))) uint32_t lq32[ATG_FAST_ORDER * ATG_FAST_ORDER / 2];
    __shared__ uint32_t ls32[ATG_FAST_ORDER / 4];

    uint32_t f, cand;
    xcd_unit_map(blockIdx.x, p.n_cand, &f, &cand);
    if (f >= p.n_frames)
        return;
    const int lane = threadIdx.x;
    const FrameInfo fi = frames[f];
    const uint32_t N = fi.n;
    const bool ms = (p.n_cand == 4u) && (p.channels == 2u);
    const uint32_t sbps = p.bps + ((ms && cand == 3u) ? 1u : 0u);
    const uint32_t unit = f * p.n_cand + cand;

    auto hand_over = [&]() {
        if (lane == 0) {
            const uint32_t slot = atomicAdd(slow_count, 1u);
            slow_list[slot] = unit;
        }
    };
    if (N != ATG_MAX_BLOCK) {
        hand_over();
        return;
    }
    if (lane < PK_PRE)
        pk[lane] = 0u;
    {
        // this candidate's table rows and shifts (alignment: coef_stride is
        // even, M shifts per unit are read bytewise)
        const uint32_t *__restrict__ gq = (const uint32_t *)(coef_tab + (size_t)unit * p.coef_stride);
        for (uint32_t i = (uint32_t)lane; i < p.coef_stride / 2u; i += 64u)
            lq32[i] = gq[i];
        if ((uint32_t)lane < p.max_lpc_order)
            ((int8_t *)ls32)[lane] = shift_tab[(size_t)unit * p.max_lpc_order + lane];
    }
    int32_t mn = INT32_MAX, mx = INT32_MIN;
    uint32_t orv = 0;
    {
        const T *__restrict__ src = pcm + fi.pcm_start * p.channels;
        if (!ms) {
            stage16<CS_CH>(src, p.channels, cand, lane, pk, mn, mx, orv);
        } else {
            switch (cand) {
            case 0: stage16<CS_L>(src, 2u, cand, lane, pk, mn, mx, orv); break;
            case 1: stage16<CS_R>(src, 2u, cand, lane, pk, mn, mx, orv); break;
            case 2: stage16<CS_AVG>(src, 2u, cand, lane, pk, mn, mx, orv); break;
            default: stage16<CS_DIF>(src, 2u, cand, lane, pk, mn, mx, orv); break;
            }
        }
    }
    const CandStats cs = wave_stats(mn, mx, orv);
    const bool constant = p.try_constant && cs.mn == cs.mx;
    if (!constant && (cs.mn < -32768 || cs.mx > 32767)) {
        hand_over();
        return;
    }
    __syncthreads();
    cand_prepare<false>(p, unit, sbps, pk, cs, lane, est_tab, out + unit, &info);
    if (lane == 0) {
        res.best_lpc = 0xFFFFFFFFu;
        res.loud = 0u;
    }
    __syncthreads();
    const CandInfo ci = load_info(&info);
    if (!ci.active)
        return;
    const uint32_t n_pred = n_pred_of(p, ci);
    // highest orders first: their totals prune the lower orders
    for (uint32_t pi = n_pred; pi-- > 0;)
        pred_job<false>(p, N, pk, ci, pi, lane, (const int16_t *)lq32, (const int8_t *)ls32, &res);
    __syncthreads();
    cand_finish(p, N, ci, &res, lane, (const int16_t *)lq32, (const int8_t *)ls32, out + unit);
}

// ---------------------------------------------------------------------------
// Samples wider than int16 (24-bit sources; the 25-bit side channel of
// 24-bit stereo): s = hi * 4096 + lo with hi = s >> 12 and lo = s & 4095, two
// packed int16 images (hi, then lo PK_WORDS later).  A predictor runs the
// 16-bit tap chain on both images with the same tap pairs -- the fold
// (c0, -2^sh) included -- into two int32 accumulators A (hi) and B (lo), and
// the shifted prediction of the reference's 64-bit sum (flac.c:999-1008),
// floor((4096 A + B) / 2^shv), comes from 32-bit operations:
//     shv >= 12:  (A + (B >> 12)) >> (shv - 12)
//     shv <  12:  (A << (12 - shv)) + (B >> shv)
// with the -2^shv seed in A or B, so the result is ~r as on the 16-bit path
// and everything after pass 1 is shared.  |s| < 2^26 keeps A and B exact.
// One 128-thread workgroup (two waves sharing the predictor jobs) per
// candidate, any channel layout.

__device__ __forceinline__ uint2 pack4_hi(const int32_t (&s)[4])
{
    const int32_t h[4] = {s[0] >> 12, s[1] >> 12, s[2] >> 12, s[3] >> 12};
    return pack4(h);
}

__device__ __forceinline__ uint2 pack4_lo(const int32_t (&s)[4])
{
    const int32_t l[4] = {s[0] & 4095, s[1] & 4095, s[2] & 4095, s[3] & 4095};
    return pack4(l);
}

// CHK: the codes' range is not bounded in advance; the biased ~r (x) are
// kept in [xmn, xmx] for the caller's check (max3 / min3, one op a sample)
template <int D, bool BIG, bool CHK>
__device__ __forceinline__ void pass1_hl(const uint32_t *__restrict__ run, const int (&cp)[14],
                                         int seed_h, int seed_l, int sa_v, int sb_v, bool lane0,
                                         int order, uint32_t (&u)[ATG_RUN], uint32_t &sabs,
                                         uint32_t &xmx, uint32_t &xmn)
{
    int tap0 = cp[0];
    asm volatile("v_mov_b32 %0, %0" : "+v"(tap0));
    uint32_t bm1 = 0x7FFFFFFFu; // B - 1 for B = 2^31
    asm volatile("v_mov_b32 %0, %0" : "+v"(bm1));
    Win A, B;
    win_init(run, A, false);
    win_init(run + PK_WORDS, B, false);
    uint4 n0 = load_run4(run, false), n1 = load_run4(run + 4, false);
    uint4 m0 = load_run4(run + PK_WORDS, false), m1 = load_run4(run + PK_WORDS + 4, false);
    uint32_t sa = 0;
#pragma unroll
    for (int c = 0; c < ATG_RUN / 16; ++c) {
        asm volatile("" ::: "memory");
        const uint4 a0 = n0, a1 = n1, b0 = m0, b1 = m1;
        if (c + 1 < ATG_RUN / 16) {
            n0 = load_run4(run + 8 * (c + 1), false);
            n1 = load_run4(run + 8 * (c + 1) + 4, false);
            m0 = load_run4(run + PK_WORDS + 8 * (c + 1), false);
            m1 = load_run4(run + PK_WORDS + 8 * (c + 1) + 4, false);
        }
        win_next(a0, a1, A);
        win_next(b0, b1, B);
#pragma unroll
        for (int ii = 0; ii < 16; ii += 2) {
            int ah[2], al[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                ah[h] = dot2_first(win_pair(A, ii + h, 0), tap0, seed_h);
                al[h] = dot2_first(win_pair(B, ii + h, 0), tap0, seed_l);
            }
#pragma unroll
            for (int j = 1; j < D; ++j)
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    ah[h] = dot2(win_pair(A, ii + h, j), cp[j], ah[h]);
                    al[h] = dot2(win_pair(B, ii + h, j), cp[j], al[h]);
                }
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int i = 16 * c + ii + h;
                int n = BIG ? (ah[h] + (al[h] >> 12)) >> sa_v : (ah[h] << sa_v) + (al[h] >> sb_v);
                if (i < ATG_FAST_ORDER)
                    n = (lane0 && i < order) ? -1 : n;
                const uint32_t x = (uint32_t)n ^ 0x80000000u;
                u[i] = x;
                sad_acc(sa, x, bm1);
            }
            if (CHK) {
                const int i = 16 * c + ii;
                xmx = max(xmx, max(u[i], u[i + 1]));
                xmn = min(xmn, min(u[i], u[i + 1]));
            }
        }
    }
    sabs = sa;
}

template <bool BIG, bool CHK>
__device__ __forceinline__ void pass1_hl_any(const uint32_t *__restrict__ run, const int (&cq)[14],
                                             int seed_h, int seed_l, int sa_v, int sb_v,
                                             bool lane0, int order, uint32_t (&u)[ATG_RUN],
                                             uint32_t &sabs, uint32_t &xmx, uint32_t &xmn)
{
#define ATG_P1HL(D)                                                                                \
    pass1_hl<D, BIG, CHK>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, sabs, xmx, xmn)
    switch (order / 2 + 1) {
    case 1: ATG_P1HL(1); break;
    case 2: ATG_P1HL(2); break;
    case 3: ATG_P1HL(3); break;
    case 4: ATG_P1HL(4); break;
    case 5: ATG_P1HL(5); break;
    case 6: ATG_P1HL(6); break;
    default: ATG_P1HL(7); break;
    }
#undef ATG_P1HL
}

// one predictor on the hi/lo images (caller checked that A and B are
// exact).  CHK: the caller could not bound the codes below 2^26 in advance
// (loud 24-bit audio: the bound |s| (1 + sum|c| / 2^sh) is far above the
// residuals a predictor leaves); pass 1 checks every ~r instead, and
// *wide = true (nothing evaluated) when one lies outside [-2^25, 2^25)
template <bool CHK>
__device__ __forceinline__ Eval16 eval_fold_hl(const uint32_t *__restrict__ run, const RunCtx &c,
                                               const uint32_t (&cw)[7], int order, int sh,
                                               uint32_t w, uint32_t thr, bool *wide)
{
    int cq[14];
    cq[0] = (int)((cw[0] & 0xFFFFu) | ((uint32_t)(-(1 << sh)) << 16));
#pragma unroll
    for (int j = 1; j < 7; ++j)
        cq[j] = (int)((cw[j] & 0xFFFFu) | (cw[j - 1] & 0xFFFF0000u));
#pragma unroll
    for (int j = 7; j < 14; ++j)
        cq[j] = 0;
    const int shv = sh + (int)w;
    const bool big = shv >= 12;
    const int seed_h = big ? -(1 << (shv - 12)) : 0;
    const int seed_l = big ? 0 : -(1 << shv);
    int sa_v = big ? shv - 12 : 12 - shv, sb_v = shv;
    asm volatile("v_mov_b32 %0, %0" : "+v"(sa_v)); // shift amounts in VGPRs
    asm volatile("v_mov_b32 %0, %0" : "+v"(sb_v));
    const bool lane0 = c.lane == 0;
    const int warm = lane0 ? order : 0;
    uint32_t u[ATG_RUN];
    uint32_t lane_sum, xmx = 0u, xmn = 0xFFFFFFFFu;
    if (big)
        pass1_hl_any<true, CHK>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, lane_sum,
                                xmx, xmn);
    else
        pass1_hl_any<false, CHK>(run, cq, seed_h, seed_l, sa_v, sb_v, lane0, order, u, lane_sum,
                                 xmx, xmn);
    // x = ~r + 2^31: ~r in [-2^25, 2^25) <=> x - (2^31 - 2^25) < 2^26, so
    // every zig-zag code is below 2^26 as eval_tail's sums need
    if (CHK && __ballot(xmx - 0x7E000000u >= (1u << 26) || xmn < 0x7E000000u) != 0ull) {
        *wide = true;
        Eval16 ev;
        return ev;
    }
    return eval_tail(lane_sum, u, c, order, warm, thr, 0x80000000u);
}

// FIXED order (flac.c:856-916) on the hi/lo images: differences in int32
// (|d4| < 2^30 for |s| < 2^26), sums in 64 bits
__device__ __forceinline__ uint32_t fixed_order_hl(const uint32_t *__restrict__ run, int lane)
{
    uint64_t a5[5] = {0, 0, 0, 0, 0};
    int x1, x2, x3, x4;
    {
        const uint4 h = *(const uint4 *)(run - 8), g = *(const uint4 *)(run + PK_WORDS - 8);
        x1 = (hi16(h.w) << 12) + hi16(g.w);
        x2 = (lo16(h.w) << 12) + lo16(g.w);
        x3 = (hi16(h.z) << 12) + hi16(g.z);
        x4 = (lo16(h.z) << 12) + lo16(g.z);
    }
    int d1p = x1 - x2, d2p = d1p - (x2 - x3);
    int d3p = d2p - ((x2 - x3) - (x3 - x4));
#pragma unroll 1
    for (int chn = 0; chn < ATG_RUN / 16; ++chn) {
        int x[16];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
            const uint4 a = *(const uint4 *)(run + 8 * chn + 4 * q);
            const uint4 b = *(const uint4 *)(run + PK_WORDS + 8 * chn + 4 * q);
            const uint32_t wa[4] = {a.x, a.y, a.z, a.w}, wb[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                x[8 * q + 2 * k] = (lo16(wa[k]) << 12) + lo16(wb[k]);
                x[8 * q + 2 * k + 1] = (hi16(wa[k]) << 12) + hi16(wb[k]);
            }
        }
#pragma unroll
        for (int tt = 0; tt < 16; ++tt) {
            const int x0 = x[tt];
            const int d1 = x0 - x1, d2 = d1 - d1p, d3 = d2 - d2p, d4 = d3 - d3p;
            if (chn > 0 || tt >= 4 || lane > 0) {
                a5[0] += iabs_u(x0);
                a5[1] += iabs_u(d1);
                a5[2] += iabs_u(d2);
                a5[3] += iabs_u(d3);
                a5[4] += iabs_u(d4);
            }
            x1 = x0;
            d1p = d1;
            d2p = d2;
            d3p = d3;
        }
    }
    uint64_t s5[5];
#pragma unroll
    for (int k = 0; k < 5; ++k)
        s5[k] = dpp_wave_sum<uint64_t>(a5[k]);
    uint64_t best = s5[0];
    uint32_t order = 0;
#pragma unroll
    for (int k = 1; k < 5; ++k)
        if (s5[k] < best) {
            best = s5[k];
            order = (uint32_t)k;
        }
    return uniform_u32(order);
}

// one predictor of a hi/lo candidate (pred_job's wide-sample form)
__device__ __forceinline__ void pred_job_hl(const FlacParams &p, uint32_t N,
                                            const uint32_t *__restrict__ img, const CandInfo &ci,
                                            uint32_t pi, int lane, const int16_t *__restrict__ lq,
                                            const int8_t *__restrict__ ls,
                                            PredRes *__restrict__ res)
{
    const bool is_fixed = p.try_fixed && pi == 0;
    const uint32_t o = is_fixed ? ci.fixed_order : ci.lo + pi - (p.try_fixed ? 1u : 0u);
    int shift = 0;
    uint32_t cw[7];
    if (is_fixed) {
        switch (o) {
        case 1: cw[0] = 1u; cw[1] = 0u; break;
        case 2: cw[0] = 2u | 0xFFFF0000u; cw[1] = 0u; break;
        case 3: cw[0] = 3u | 0xFFFD0000u; cw[1] = 1u; break;
        case 4: cw[0] = 4u | 0xFFFA0000u; cw[1] = 4u | 0xFFFF0000u; break;
        default: cw[0] = 0u; cw[1] = 0u; break;
        }
#pragma unroll
        for (int m = 2; m < 7; ++m)
            cw[m] = 0u;
    } else {
        shift = uniform_i32(ls[o - 1u]);
        const uint32_t *__restrict__ rw = (const uint32_t *)(lq + (o - 1u) * p.coef_row);
#pragma unroll
        for (int m = 0; m < 6; ++m)
            cw[m] = 2u * (uint32_t)m < p.coef_row ? uniform_u32(rw[m]) : 0u;
        cw[6] = 0u;
    }
    uint32_t csum = 0;
#pragma unroll
    for (int m = 0; m < 6; ++m) {
        const int a = lo16(cw[m]), b = hi16(cw[m]);
        csum += (uint32_t)(a < 0 ? -a : a) + (uint32_t)(b < 0 ? -b : b);
    }
    RunCtx c;
    c.lane = lane;
    c.a = ATG_RUN * lane;
    c.len = ATG_RUN;
    c.N = N;
    c.max_rice = p.max_rice;
    c.P = (int)(p.max_porder < (uint32_t)ATG_MAX_PORDER ? p.max_porder : (uint32_t)ATG_MAX_PORDER);
    // A and B exact in int32: (sum|c| + 2^sh) (max|hi| + 1) + 2^(shv - 12)
    // and (sum|c| + 2^sh) 4095 + 2^shv below 2^31; codes below 2^26
    const uint64_t mu = ci.amax, ms = ci.amax >> ci.w;
    const uint64_t hmax = (mu >> 12) + 1u, tsum = (uint64_t)csum + (1ull << shift);
    const uint32_t shv = (uint32_t)shift + ci.w;
    const bool fold_ok = tsum * hmax + (1ull << (shv > 12 ? shv - 12 : 0)) < (1ull << 31) &&
                         tsum * 4095u + (shv < 12 ? (1ull << shv) : 0ull) < (1ull << 31);
    const uint64_t rbound = ms + (((uint64_t)csum * ms) >> shift) + 1u;
    const uint32_t wf = ci.w ? ci.w + 1u : 1u;
    const uint32_t hdr = 7u + wf + o * (ci.sbps - ci.w) + 9u + o * p.qlp_precision;
    // FIXED too: it wins only below every LPC total
    // (flac.c:727-809, strict <), so a bound above a finished LPC total
    // rules it out the same way; its header is 7 + wf + o (sbps - w)
    const uint32_t hdr_f = 7u + wf + o * (ci.sbps - ci.w);
    uint32_t thr = 0xFFFFFFFFu;
    {
        const uint32_t best = uniform_u32(__atomic_load_n(&res->best_lpc, __ATOMIC_RELAXED));
        const uint32_t hh = is_fixed ? hdr_f : hdr;
        if (best != 0xFFFFFFFFu)
            thr = best > hh ? best - hh : 0u;
    }
    Eval16 ev;
    bool wide = !fold_ok;
    if (fold_ok && 2u * rbound + 1u < (1ull << 26))
        ev = eval_fold_hl<false>(run_of(img, lane), c, cw, (int)o, shift, ci.w, thr, &wide);
    else if (fold_ok)
        ev = eval_fold_hl<true>(run_of(img, lane), c, cw, (int)o, shift, ci.w, thr, &wide);
    if (wide)
        ev = eval_wide<2>(img, c, cw, (int)o, shift, ci.w);
    if (!is_fixed && ev.bits != K2F_PRUNED && lane == 0)
        atomicMin(&res->best_lpc, hdr + ev.bits);
    res->k[pi][lane] = (uint8_t)ev.sel.k_own;
    if (lane == 0) {
        res->bits[pi] = ev.bits;
        res->porder[pi] = (uint8_t)ev.sel.porder;
        res->method[pi] = (uint8_t)ev.sel.method;
    }
}

template <int CS, typename T>
__device__ __forceinline__ void stage_hl(const T *__restrict__ src, uint32_t ch, uint32_t cand,
                                         int tid, uint32_t *__restrict__ pk, int32_t &mn,
                                         int32_t &mx, uint32_t &orv)
{
#pragma unroll 4
    for (int m = 0; m < ATG_MAX_BLOCK / 512; ++m) {
        const uint32_t q0 = (uint32_t)(tid + 128 * m); // 4-sample group
        int32_t s[4];
        load4<CS>(src, 4u * q0, ch, cand, s);
        stats_add(s, mn, mx, orv);
        *(uint2 *)&pk[paddr(2 * (int)q0)] = pack4_hi(s);
        *(uint2 *)&pk[PK_WORDS + paddr(2 * (int)q0)] = pack4_lo(s);
    }
}

template <typename T>
__global__ __launch_bounds__(128) void k_subframe_search_hl(
    FlacParams p, const T *__restrict__ pcm, const FrameInfo *__restrict__ frames,
    const int16_t *__restrict__ coef_tab, const int8_t *__restrict__ shift_tab,
    const uint8_t *__restrict__ est_tab, SubDesc *__restrict__ out,
    uint32_t *__restrict__ slow_list, uint32_t *__restrict__ slow_count)
{
    __shared__ __attribute__((aligned(16))) uint32_t pk[2 * PK_WORDS]; // hi, lo images
    __shared__ int32_t red[2][3];
    __shared__ CandInfo info;
    __shared__ PredRes res;
    __shared__ uint32_t qnext;
    __shared__ __attribute__((aligned(16))) uint32_t lq32[ATG_FAST_ORDER * ATG_FAST_ORDER / 2];
    __shared__ uint32_t ls32[ATG_FAST_ORDER / 4];

    uint32_t f, cand;
    xcd_unit_map(blockIdx.x, p.n_cand, &f, &cand);
    if (f >= p.n_frames)
        return;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const FrameInfo fi = frames[f];
    const uint32_t N = fi.n;
    const bool ms = (p.n_cand == 4u) && (p.channels == 2u);
    const uint32_t sbps = p.bps + ((ms && cand == 3u) ? 1u : 0u);
    const uint32_t unit = f * p.n_cand + cand;
    if (N != ATG_MAX_BLOCK) {
        if (tid == 0)
            slow_list[atomicAdd(slow_count, 1u)] = unit;
        return;
    }
    if (tid < 2 * PK_PRE)
        pk[(tid / PK_PRE) * PK_WORDS + (tid % PK_PRE)] = 0u;
    else if (tid == 127)
        qnext = 0u;
    {
        const uint32_t *__restrict__ gq = (const uint32_t *)(coef_tab + (size_t)unit * p.coef_stride);
        for (uint32_t i = (uint32_t)tid; i < p.coef_stride / 2u; i += 128u)
            lq32[i] = gq[i];
        if ((uint32_t)tid < p.max_lpc_order)
            ((int8_t *)ls32)[tid] = shift_tab[(size_t)unit * p.max_lpc_order + tid];
    }
    int32_t mn = INT32_MAX, mx = INT32_MIN;
    uint32_t orv = 0;
    {
        const T *__restrict__ src = pcm + fi.pcm_start * p.channels;
        if (!ms) {
            stage_hl<CS_CH>(src, p.channels, cand, tid, pk, mn, mx, orv);
        } else {
            switch (cand) {
            case 0: stage_hl<CS_L>(src, 2u, cand, tid, pk, mn, mx, orv); break;
            case 1: stage_hl<CS_R>(src, 2u, cand, tid, pk, mn, mx, orv); break;
            case 2: stage_hl<CS_AVG>(src, 2u, cand, tid, pk, mn, mx, orv); break;
            default: stage_hl<CS_DIF>(src, 2u, cand, tid, pk, mn, mx, orv); break;
            }
        }
    }
    {
        const CandStats w = wave_stats(mn, mx, orv);
        if (lane == 0) {
            red[wave][0] = w.mn;
            red[wave][1] = w.mx;
            red[wave][2] = (int32_t)w.orv;
        }
    }
    __syncthreads();
    CandStats cs;
    cs.mn = uniform_i32(min(red[0][0], red[1][0]));
    cs.mx = uniform_i32(max(red[0][1], red[1][1]));
    cs.orv = uniform_u32((uint32_t)(red[0][2] | red[1][2]));
    const bool constant = p.try_constant && cs.mn == cs.mx;
    if (!constant && (cs.mn < -(1 << 26) || cs.mx >= (1 << 26))) {
        if (tid == 0)
            slow_list[atomicAdd(slow_count, 1u)] = unit;
        return;
    }
    if (wave == 0) {
        cand_prepare<false, true>(p, unit, sbps, pk, cs, lane, est_tab, out + unit, &info);
        if (lane == 0) {
            res.best_lpc = 0xFFFFFFFFu;
            res.loud = 0u;
        }
    }
    __syncthreads();
    const CandInfo ci = load_info(&info);
    if (!ci.active)
        return;
    const uint32_t n_pred = n_pred_of(p, ci);
    // the two waves share the predictor jobs, highest orders first (their
    // totals prune the lower orders); see k_frame_search_ms for the counter
    for (;;) {
        const uint32_t j = next_job(&qnext);
        if (j >= n_pred)
            break;
        pred_job_hl(p, N, pk, ci, n_pred - 1u - j, lane, (const int16_t *)lq32,
                    (const int8_t *)ls32, &res);
    }
    __syncthreads();
    if (wave == 0)
        cand_finish(p, N, ci, &res, lane, (const int16_t *)lq32, (const int8_t *)ls32,
                    out + unit);
}

hipError_t launch_subframe_search_hl(const FlacParams &p, const void *pcm, int fmt,
                                     const FrameInfo *frames, const int16_t *coef_tab,
                                     const int8_t *shift_tab, const uint8_t *est_tab,
                                     SubDesc *sub, uint32_t *slow_list, uint32_t *slow_count,
                                     hipStream_t s)
{
    if (p.n_frames == 0)
        return hipSuccess;
    const uint32_t f8 = (p.n_frames + 7u) / 8u * 8u;
    dim3 grid(f8 * p.n_cand);
    if (fmt == 0)
        hipLaunchKernelGGL((k_subframe_search_hl<int16_t>), grid, dim3(128), 0, s, p,
                           (const int16_t *)pcm, frames, coef_tab, shift_tab, est_tab, sub,
                           slow_list, slow_count);
    else
        hipLaunchKernelGGL((k_subframe_search_hl<int32_t>), grid, dim3(128), 0, s, p,
                           (const int32_t *)pcm, frames, coef_tab, shift_tab, est_tab, sub,
                           slow_list, slow_count);
    return hipGetLastError();
}

hipError_t launch_subframe_search16(const FlacParams &p, const void *pcm, int fmt,
                                    const FrameInfo *frames, const int16_t *coef_tab,
                                    const int8_t *shift_tab, const uint8_t *est_tab,
                                    SubDesc *sub, uint32_t *slow_list, uint32_t *slow_count,
                                    hipStream_t s)
{
    if (p.n_frames == 0)
        return hipSuccess;
    const bool ms = (p.n_cand == 4u) && (p.channels == 2u);
    if (ms) {
        dim3 grid(p.n_frames);
        if (fmt == 0)
            hipLaunchKernelGGL((k_frame_search_ms<int16_t>), grid, dim3(256), 0, s, p,
                               (const int16_t *)pcm, frames, coef_tab, shift_tab, est_tab, sub,
                               slow_list, slow_count);
        else
            hipLaunchKernelGGL((k_frame_search_ms<int32_t>), grid, dim3(256), 0, s, p,
                               (const int32_t *)pcm, frames, coef_tab, shift_tab, est_tab, sub,
                               slow_list, slow_count);
        return hipGetLastError();
    }
    const uint32_t f8 = (p.n_frames + 7u) / 8u * 8u;
    dim3 grid(f8 * p.n_cand);
    if (fmt == 0)
        hipLaunchKernelGGL((k_subframe_search16<int16_t>), grid, dim3(64), 0, s, p,
                           (const int16_t *)pcm, frames, coef_tab, shift_tab, est_tab, sub,
                           slow_list, slow_count);
    else
        hipLaunchKernelGGL((k_subframe_search16<int32_t>), grid, dim3(64), 0, s, p,
                           (const int32_t *)pcm, frames, coef_tab, shift_tab, est_tab, sub,
                           slow_list, slow_count);
    return hipGetLastError();
}


