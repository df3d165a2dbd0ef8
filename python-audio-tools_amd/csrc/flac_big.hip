// flac_big.hip — the FLAC encoder's large-frame path: block lengths up to
// FLAC's 65535 and residual partition orders up to 15.  The reference takes
// both (the partition-order loop of src/encoders/flac.c:1362-1402 runs while
// the block divides by 2^p; test/test_formats.py:3798-3844 encodes 32768-
// and 65535-sample blocks).  The 4096-sample kernels hold a frame in LDS
// with one finest partition per lane (K2 flac_search.hip, K5
// flac_frame.hip); here a 256-thread workgroup walks a candidate held in an
// HBM scratch row, and the partition sums of every order form a pyramid in
// scratch.  Same arithmetic as K2's generic path (64-bit predictor
// accumulator, flac.c:1060-1126 / 918-1016), same decisions, same bits.
//
//   KB2 k_subframe_search_big  one workgroup per subframe candidate
//                              (persistent grid): constant / wasted bits,
//                              FIXED order, every LPC order, partition
//                              search, exact bits, subframe choice
//   KB5 k_frame_pack_big       one workgroup per frame (persistent grid):
//                              the frame written MSB-first straight into
//                              the zeroed output with 32-bit atomic ORs,
//                              residual bit offsets from a workgroup scan,
//                              CRC-16 in 256 chunks combined on one lane
//
// Thread ranges: the thread's contiguous run of samples lies inside one
// finest partition (F <= 256 partitions: 256/F threads share one), or
// covers F/256 whole partitions, so partition sums need no global atomics.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "flac_dev.h"
#include "launch.h"
#include "pcm_read.h"
#include "residual.h"
#include "rice.h"
#include "wave.h"

namespace {

constexpr uint32_t BT = 256;       // threads per workgroup
constexpr uint32_t NW = BT / 64;   // waves per workgroup

// ---- workgroup reductions (every thread calls; two barriers each)
__device__ __forceinline__ uint64_t wg_sum_u64(uint64_t v, uint64_t *red)
{
    v = dpp_wave_sum<uint64_t>(v);
    __syncthreads();
    if ((threadIdx.x & 63u) == 0u)
        red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (red[0] + red[1]) + (red[2] + red[3]);
}

// modulo 2^32, as the reference's uint32 bit counters
__device__ __forceinline__ uint32_t wg_sum_u32(uint32_t v, uint64_t *red)
{
    v = dpp_wave_sum<uint32_t>(v);
    __syncthreads();
    if ((threadIdx.x & 63u) == 0u)
        red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (uint32_t)((red[0] + red[1]) + (red[2] + red[3]));
}

__device__ __forceinline__ uint32_t wg_or_u32(uint32_t v, uint64_t *red)
{
    v = dpp_wave_or_u32(v);
    __syncthreads();
    if ((threadIdx.x & 63u) == 0u)
        red[threadIdx.x >> 6] = v;
    __syncthreads();
    return (uint32_t)(red[0] | red[1] | red[2] | red[3]);
}

// exclusive scan of one value per thread over the workgroup (plus total)
__device__ __forceinline__ uint32_t wg_excl_scan_u32(uint32_t v, uint32_t *tmp, uint32_t &total)
{
    const int lane = (int)(threadIdx.x & 63u);
    const uint32_t wex = wave_excl_scan_u32(v, lane);
    __syncthreads();
    if (lane == 63)
        tmp[threadIdx.x >> 6] = wex + v;
    __syncthreads();
    uint32_t off = 0;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w)
        off += tmp[w];
    total = tmp[0] + tmp[1] + tmp[2] + tmp[3];
    return off + wex;
}

// residual of sample i >= order (flac_search.hip eval_generic arithmetic)
__device__ __forceinline__ int32_t residual_at(const int32_t *__restrict__ s, int i,
                                               const int *__restrict__ cf, int order, int shift)
{
    int64_t acc = 0;
    for (int k = 0; k < order; ++k)
        acc += (int64_t)cf[k] * (int64_t)s[i - 1 - k];
    return (int)((uint32_t)s[i] - (uint32_t)(int32_t)(acc >> shift));
}

// FIXED predictor of order o as LPC taps (flac.c:918-1016)
__device__ __forceinline__ int fixed_tap_big(uint32_t o, uint32_t j)
{
    switch (o) {
    case 1: return j == 0 ? 1 : 0;
    case 2: return j == 0 ? 2 : j == 1 ? -1 : 0;
    case 3: return j == 0 ? 3 : j == 1 ? -3 : j == 2 ? 1 : 0;
    case 4: return j == 0 ? 4 : j == 1 ? -6 : j == 2 ? 4 : j == 3 ? -1 : 0;
    default: return 0;
    }
}

// the finest usable partition order and this thread's run of samples
struct BigRun {
    uint32_t N, P, F, Sp;  // block, finest order, 2^P partitions of Sp samples
    uint32_t ra, re;       // this thread's samples [ra, re)
    uint32_t j0, nj;       // F > BT: its whole partitions [j0, j0 + nj)
};

__device__ __forceinline__ BigRun big_run(uint32_t N, uint32_t max_porder)
{
    BigRun r;
    r.N = N;
    const uint32_t tz = N ? (uint32_t)__builtin_ctz(N) : 0u;
    uint32_t P = max_porder < tz ? max_porder : tz;
    P = P > ATG_BIG_MAX_PORDER ? ATG_BIG_MAX_PORDER : P;
    r.P = P;
    r.F = 1u << P;
    r.Sp = N >> P;
    const uint32_t t = threadIdx.x;
    if (r.F <= BT) {
        const uint32_t G = BT / r.F, j = t / G, q = t % G;
        const uint32_t R = (r.Sp + G - 1u) / G;
        uint32_t a = j * r.Sp + q * R, e = a + R;
        e = e < (j + 1u) * r.Sp ? e : (j + 1u) * r.Sp;
        r.ra = a < e ? a : e;
        r.re = e;
        r.j0 = j;
        r.nj = 0;
    } else {
        const uint32_t per = r.F / BT;
        r.j0 = t * per;
        r.nj = per;
        r.ra = r.j0 * r.Sp;
        r.re = r.ra + per * r.Sp;
    }
    return r;
}

struct BigSel {
    uint32_t bits;   // residual section bits (method + order + headers + codes)
    uint32_t porder;
    uint32_t method;
};

struct BigLds {
    uint8_t kb[1u << ATG_BIG_MAX_PORDER]; // Rice parameters of the chosen order
    uint64_t lpart[BT];
    uint64_t ltot[ATG_BIG_MAX_PORDER + 1];
    uint64_t red[NW];
    int cf[ATG_MAX_LPC];
    uint32_t maxk;
};

// Rice parameter of partition j at level lv (flac.c:1437-1505, degenerate
// first partition included: when N >> lv < order it takes every residual)
__device__ __forceinline__ uint32_t big_part_k(uint32_t N, uint32_t lv, uint32_t j,
                                               uint64_t sum_j, uint64_t total, uint32_t order,
                                               uint32_t max_rice, uint64_t *est)
{
    const uint32_t Spl = N >> lv;
    const bool degen = Spl < order;
    const uint32_t plen = j == 0 ? Spl - order : Spl;
    const uint64_t sum = degen ? (j == 0 ? total : 0ull) : sum_j;
    const uint32_t k = rice_param(plen, sum, max_rice);
    if (est)
        *est = part_estimate<uint64_t>(plen, sum, k);
    return k;
}

// One predictor (taps in L.cf, `order`, `shift`): partition-order search
// over every level 0..P and the exact residual bits (flac.c:1326-1505).
// Leaves the chosen level's Rice parameters in L.kb.
__device__ BigSel eval_big(const int32_t *__restrict__ s, uint64_t *__restrict__ pyr,
                           BigLds &L, const BigRun &R, int order, int shift,
                           uint32_t max_rice)
{
    const uint32_t t = threadIdx.x;
    const uint32_t F = R.F, P = R.P, N = R.N;
    // pass A: |r| sums of the finest partitions
    if (F <= BT && t < F)
        L.lpart[t] = 0;
    if (t <= ATG_BIG_MAX_PORDER)
        L.ltot[t] = 0;
    if (t == 0)
        L.maxk = 0;
    __syncthreads();
    if (F <= BT) {
        uint64_t sum = 0;
        for (int i = max((int)R.ra, order); i < (int)R.re; ++i)
            sum += iabs_u(residual_at(s, i, L.cf, order, shift));
        if (sum)
            atomicAdd((unsigned long long *)&L.lpart[R.j0], (unsigned long long)sum);
        __syncthreads();
        if (t < F)
            pyr[F + t] = L.lpart[t];
    } else {
        for (uint32_t j = R.j0; j < R.j0 + R.nj; ++j) {
            uint64_t sum = 0;
            for (int i = max((int)(j * R.Sp), order); i < (int)((j + 1u) * R.Sp); ++i)
                sum += iabs_u(residual_at(s, i, L.cf, order, shift));
            pyr[F + j] = sum;
        }
    }
    __syncthreads();
    // coarser levels: pyr[2^lv + j] = sum of partition j at level lv
    for (int lv = (int)P - 1; lv >= 0; --lv) {
        for (uint32_t j = t; j < (1u << lv); j += BT)
            pyr[(1u << lv) + j] = pyr[(2u << lv) + 2u * j] + pyr[(2u << lv) + 2u * j + 1u];
        __syncthreads();
    }
    const uint64_t total = pyr[1];
    // estimates of every (level, partition), totals per level
    for (uint32_t idx = t + 1u; idx < 2u * F; idx += BT) {
        const uint32_t lv = 31u - (uint32_t)__clz((int)idx);
        const uint32_t j = idx - (1u << lv);
        uint64_t e;
        big_part_k(N, lv, j, pyr[idx], total, (uint32_t)order, max_rice, &e);
        atomicAdd((unsigned long long *)&L.ltot[lv], (unsigned long long)e);
    }
    __syncthreads();
    uint64_t best_tot = ~0ull;
    uint32_t best = 0;
    for (uint32_t lv = 0; lv <= P; ++lv)
        if (L.ltot[lv] < best_tot) {
            best_tot = L.ltot[lv];
            best = lv;
        }
    // Rice parameters of the chosen level
    for (uint32_t j = t; j < (1u << best); j += BT) {
        const uint32_t k = big_part_k(N, best, j, pyr[(1u << best) + j], total, (uint32_t)order,
                                      max_rice, nullptr);
        L.kb[j] = (uint8_t)k;
        atomicMax(&L.maxk, k);
    }
    __syncthreads();
    BigSel sel;
    sel.porder = best;
    sel.method = (max_rice > 14u && L.maxk > 14u) ? 1u : 0u;
    // exact bits of the codes
    const uint32_t Sb = N >> best;
    const bool degen = Sb < (uint32_t)order;
    uint32_t bits = 0;
    for (int i = max((int)R.ra, order); i < (int)R.re; ++i) {
        const uint32_t k = degen ? L.kb[0] : L.kb[(uint32_t)i / Sb];
        bits += (zigzag(residual_at(s, i, L.cf, order, shift)) >> k) + 1u + k;
    }
    bits = wg_sum_u32(bits, L.red);
    sel.bits = 6u + (1u << best) * (sel.method ? 5u : 4u) + bits;
    return sel;
}

__device__ __forceinline__ uint32_t wasted_field_big(uint32_t w) { return w ? w + 1u : 1u; }

} // namespace

// ---------------------------------------------------------------- KB2
template <typename T>
__global__ __launch_bounds__(BT) void k_subframe_search_big(
    FlacParams p, const T *__restrict__ pcm, const FrameInfo *__restrict__ frames,
    const int16_t *__restrict__ coef_tab, const int8_t *__restrict__ shift_tab,
    const uint8_t *__restrict__ est_tab, SubDesc *__restrict__ out,
    uint8_t *__restrict__ rice_big, uint32_t rice_stride, uint8_t *__restrict__ scratch,
    uint64_t slot_bytes, uint64_t row_bytes)
{
    __shared__ BigLds L;
    int32_t *__restrict__ s = (int32_t *)(scratch + (uint64_t)blockIdx.x * slot_bytes);
    uint64_t *__restrict__ pyr =
        (uint64_t *)(scratch + (uint64_t)blockIdx.x * slot_bytes + row_bytes);
    const uint32_t t = threadIdx.x;
    const uint32_t n_sub = p.n_frames * p.n_cand;
    const bool ms = (p.n_cand == 4u) && (p.channels == 2u);

    for (uint32_t sub = blockIdx.x; sub < n_sub; sub += gridDim.x) {
        const uint32_t f = sub / p.n_cand, cand = sub % p.n_cand;
        const FrameInfo fi = frames[f];
        const uint32_t N = fi.n;
        const uint32_t sbps = p.bps + ((ms && cand == 3u) ? 1u : 0u);
        SubDesc *__restrict__ d = out + sub;

        // ---- stage + constant / wasted bits (flac.c:1578-1620)
        const int32_t first = cand_sample(pcm, fi.pcm_start, p.channels, cand, ms);
        uint32_t orv = 0, notsame = 0;
        for (uint32_t i = t; i < N; i += BT) {
            const int32_t v = cand_sample(pcm, fi.pcm_start + i, p.channels, cand, ms);
            s[i] = v;
            orv |= (uint32_t)v;
            notsame |= v != first ? 1u : 0u;
        }
        orv = wg_or_u32(orv, L.red);
        notsame = wg_or_u32(notsame, L.red);
        if (p.try_constant && !notsame) {
            if (t == 0) {
                d->bits = 8u + sbps;
                d->type = SF_CONSTANT;
                d->order = 0;
                d->wasted = 0;
                d->porder = 0;
                d->method = 0;
                d->precision = 0;
                d->shift = 0;
                d->sbps = (uint8_t)sbps;
            }
            __syncthreads();
            continue;
        }
        const uint32_t w = orv ? (uint32_t)__builtin_ctz(orv) : 0u;
        if (w) {
            for (uint32_t i = t; i < N; i += BT)
                s[i] >>= w;
            __syncthreads();
        }
        const BigRun R = big_run(N, p.max_porder);
        const uint32_t wf = wasted_field_big(w);
        const uint32_t rb = sbps - w;

        // ---- FIXED order by |residual| sums over samples [4, N) (flac.c:856-916)
        uint32_t fixed_order = 0;
        if (p.try_fixed) {
            uint64_t s5[5] = {0, 0, 0, 0, 0};
            for (int i = max((int)R.ra, 4); i < (int)R.re; ++i) {
                const uint32_t x0 = (uint32_t)s[i], x1 = (uint32_t)s[i - 1],
                               x2 = (uint32_t)s[i - 2], x3 = (uint32_t)s[i - 3],
                               x4 = (uint32_t)s[i - 4];
                const int32_t d0 = (int32_t)x0;
                const int32_t d1 = (int32_t)(x0 - x1);
                const int32_t d2 = (int32_t)(x0 - 2u * x1 + x2);
                const int32_t d3 = (int32_t)(x0 - 3u * x1 + 3u * x2 - x3);
                const int32_t d4 = (int32_t)(x0 - 4u * x1 + 6u * x2 - 4u * x3 + x4);
                // accumulator += abs(int): abs(INT_MIN) stays negative (flac.c:1628)
                s5[0] += (uint64_t)(int64_t)(int32_t)iabs_u(d0);
                s5[1] += (uint64_t)(int64_t)(int32_t)iabs_u(d1);
                s5[2] += (uint64_t)(int64_t)(int32_t)iabs_u(d2);
                s5[3] += (uint64_t)(int64_t)(int32_t)iabs_u(d3);
                s5[4] += (uint64_t)(int64_t)(int32_t)iabs_u(d4);
            }
            for (int k = 0; k < 5; ++k)
                s5[k] = wg_sum_u64(s5[k], L.red);
            uint64_t best = s5[0];
            if (N > 4)
                for (int k = 1; k < 5; ++k)
                    if (s5[k] < best) {
                        best = s5[k];
                        fixed_order = (uint32_t)k;
                    }
        }

        // ---- LPC candidate orders (flac.c:1034-1126)
        const int16_t *__restrict__ qtab = coef_tab + (size_t)sub * p.coef_stride;
        const int8_t *__restrict__ stab = shift_tab + (size_t)sub * p.max_lpc_order;
        const uint32_t M = p.max_lpc_order;
        const bool dummy = !(N > M + 1u);
        uint32_t lo = 1, hi = 0;
        if (p.try_lpc) {
            if (dummy) {
                lo = hi = 1;
            } else if (p.exhaustive) {
                lo = 1;
                hi = M;
            } else {
                lo = hi = est_tab[sub];
            }
        }

        uint32_t fixed_bits = 0;
        BigSel fixed_sel = {0, 0, 0};
        uint32_t lpc_bits = 0xFFFFFFFFu, lpc_order = 0, lpc_prec = 0;
        int lpc_shift = 0;
        BigSel lpc_sel = {0, 0, 0};
        const uint32_t n_pred = (p.try_fixed ? 1u : 0u) + (p.try_lpc ? hi - lo + 1u : 0u);
        for (uint32_t pi = 0; pi < n_pred; ++pi) {
            const bool is_fixed = p.try_fixed && pi == 0;
            const uint32_t o = is_fixed ? fixed_order : lo + pi - (p.try_fixed ? 1u : 0u);
            int shift = 0;
            uint32_t prec = 0;
            if (!is_fixed && !dummy && o > 0) {
                shift = stab[o - 1u];
                prec = p.qlp_precision;
            } else if (!is_fixed && dummy) {
                prec = 2;
            }
            __syncthreads();
            if (t < o)
                L.cf[t] = is_fixed ? fixed_tap_big(o, t)
                        : dummy    ? 1
                                   : (int)qtab[(size_t)(o - 1u) * p.coef_row + t];
            const BigSel ev = eval_big(s, pyr, L, R, (int)o, shift, p.max_rice);
            if (is_fixed) {
                fixed_bits = 7u + wf + o * rb + ev.bits;
                fixed_sel = ev;
            } else {
                const uint32_t bits = 7u + wf + o * rb + 4u + 5u + o * prec + ev.bits;
                if (bits < lpc_bits) {
                    lpc_bits = bits;
                    lpc_order = o;
                    lpc_shift = shift;
                    lpc_prec = prec;
                    lpc_sel = ev;
                }
            }
        }

        // ---- subframe choice (flac.c:727-809), as K2
        const uint32_t verbatim_cmp = p.try_verbatim ? rb * N : 0x7FFFFFFFu;
        int pick;
        const bool Fx = p.try_fixed, Lp = p.try_lpc, V = p.try_verbatim;
        if (Fx && Lp && V) {
            const uint32_t m = lpc_bits < verbatim_cmp ? lpc_bits : verbatim_cmp;
            pick = fixed_bits < m ? SF_FIXED : (lpc_bits < verbatim_cmp ? SF_LPC : SF_VERBATIM);
        } else if (!Fx && !Lp) {
            pick = SF_VERBATIM;
        } else if (Fx && !Lp && !V) {
            pick = SF_FIXED;
        } else if (!Fx && Lp && !V) {
            pick = SF_LPC;
        } else if (Fx && Lp && !V) {
            pick = fixed_bits < lpc_bits ? SF_FIXED : SF_LPC;
        } else if (Fx && !Lp && V) {
            pick = fixed_bits < verbatim_cmp ? SF_FIXED : SF_VERBATIM;
        } else {
            pick = lpc_bits < verbatim_cmp ? SF_LPC : SF_VERBATIM;
        }

        const BigSel &sel = pick == SF_FIXED ? fixed_sel : lpc_sel;
        if (pick == SF_FIXED || pick == SF_LPC) {
            // re-run the winner for its Rice parameters (deterministic)
            const uint32_t o = pick == SF_FIXED ? fixed_order : lpc_order;
            __syncthreads();
            if (t < o)
                L.cf[t] = pick == SF_FIXED ? fixed_tap_big(o, t)
                        : dummy            ? 1
                                           : (int)qtab[(size_t)(o - 1u) * p.coef_row + t];
            const BigSel again = eval_big(s, pyr, L, R, (int)o,
                                          pick == SF_FIXED ? 0 : lpc_shift, p.max_rice);
            uint8_t *__restrict__ rk = rice_big + (size_t)sub * rice_stride;
            for (uint32_t j = t; j < (1u << again.porder); j += BT)
                rk[j] = L.kb[j];
            if (pick == SF_LPC && t < lpc_order)
                d->coef[t] = (int16_t)(dummy ? 1 : qtab[(size_t)(lpc_order - 1u) * p.coef_row + t]);
        }
        if (t == 0) {
            d->type = (uint8_t)pick;
            d->wasted = (uint8_t)w;
            d->sbps = (uint8_t)sbps;
            d->method = (uint8_t)sel.method;
            d->porder = (uint8_t)sel.porder;
            if (pick == SF_FIXED) {
                d->bits = fixed_bits;
                d->order = (uint8_t)fixed_order;
                d->precision = 0;
                d->shift = 0;
            } else if (pick == SF_LPC) {
                d->bits = lpc_bits;
                d->order = (uint8_t)lpc_order;
                d->precision = (uint8_t)lpc_prec;
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
        __syncthreads(); // the scratch row is reused by the next candidate
    }
}

// ---------------------------------------------------------------- KB5
namespace {

// OR n (1..32) bits of v, MSB-first, at bit `pos` of a big-endian bit image
// whose 32-bit words are stored little-endian in memory (wb = the image's
// word-aligned base)
__device__ __forceinline__ void put_g(uint32_t *wb, uint64_t pos, uint32_t n, uint32_t v)
{
    if (n == 0)
        return;
    const uint64_t val = (uint64_t)(n >= 32u ? v : (v & ((1u << n) - 1u)));
    const uint64_t w = pos >> 5;
    const uint32_t off = (uint32_t)(pos & 31u);
    const uint64_t x = val << (64u - off - n);
    const uint32_t hi = (uint32_t)(x >> 32), lo = (uint32_t)x;
    if (hi)
        atomicOr(&wb[w], __builtin_bswap32(hi));
    if (lo)
        atomicOr(&wb[w + 1u], __builtin_bswap32(lo));
}

__device__ __forceinline__ uint32_t crc16_byte(const uint16_t *tab, uint32_t crc, uint32_t byte)
{
    return ((crc << 8) & 0xFFFFu) ^ tab[((crc >> 8) ^ byte) & 0xFFu];
}

} // namespace

template <typename T>
__global__ __launch_bounds__(BT) void k_frame_pack_big(
    FlacParams p, const T *__restrict__ pcm, const FrameInfo *__restrict__ frames,
    const TrackInfo *__restrict__ tracks, const SubDesc *__restrict__ sub,
    const uint8_t *__restrict__ rice_big, uint32_t rice_stride,
    const FrameDesc *__restrict__ fdesc, uint8_t *__restrict__ out, uint32_t *__restrict__ err,
    uint8_t *__restrict__ scratch, uint64_t slot_bytes)
{
    __shared__ uint16_t crc_tab[256];
    __shared__ uint32_t crc_adv[16];
    __shared__ uint32_t crc_part[BT];
    __shared__ uint32_t scan[NW];
    __shared__ int cf[ATG_MAX_LPC];
    int32_t *__restrict__ s = (int32_t *)(scratch + (uint64_t)blockIdx.x * slot_bytes);
    const uint32_t t = threadIdx.x;
    const bool ms = (p.n_cand == 4u) && (p.channels == 2u);
    {
        // CRC-16 (poly 0x8005, MSB-first, init 0) byte table
        uint32_t c = t << 8;
        for (int b = 0; b < 8; ++b)
            c = (c & 0x8000u) ? ((c << 1) ^ 0x8005u) : (c << 1);
        crc_tab[t] = (uint16_t)(c & 0xFFFFu);
    }
    __syncthreads();

    for (uint32_t f = blockIdx.x; f < p.n_frames; f += gridDim.x) {
        const FrameInfo fi = frames[f];
        const FrameDesc &fd = fdesc[f];
        const TrackInfo ti = tracks[fi.track];
        const uint32_t N = fi.n;
        const uint64_t slot = (uint64_t)p.header_bytes + (uint64_t)ti.n_frames * p.frame_bound;
        if ((uint64_t)p.header_bytes + fd.out_off + fd.bytes > slot) {
            if (t == 0)
                atomicOr(err, 4u);
            continue;
        }
        uint8_t *dst = out + ti.out_base + p.header_bytes + fd.out_off;
        uint32_t *wb = (uint32_t *)((uintptr_t)dst & ~(uintptr_t)3);
        const uint64_t b0 = 8u * (uint64_t)((uintptr_t)dst & 3u); // bit of frame byte 0
        if (t < fd.hdr_len)
            put_g(wb, b0 + 8u * t, 8, fd.hdr[t]);
        uint64_t pos = 8u * (uint64_t)fd.hdr_len;
        const uint32_t R = (N + BT - 1u) / BT;
        const uint32_t ra = min(t * R, N), re = min(ra + R, N);

        for (uint32_t si = 0; si < fd.nsub; ++si) {
            const uint32_t cand = fd.sub[si];
            const size_t sid = (size_t)f * p.n_cand + cand;
            const SubDesc &d = sub[sid];
            const uint32_t type = d.type, order = d.order, w = d.wasted, sbps = d.sbps;
            const uint64_t start = pos;
            __syncthreads(); // previous subframe's readers of s / cf are done
            for (uint32_t i = t; i < N; i += BT)
                s[i] = cand_sample(pcm, fi.pcm_start + i, p.channels, cand, ms) >> w;
            if (t < order)
                cf[t] = type == SF_LPC ? (int)d.coef[t]
                      : order == 1     ? 1
                      : order == 2     ? (t == 0 ? 2 : -1)
                      : order == 3     ? (t == 0 ? 3 : t == 1 ? -3 : 1)
                                       : (t == 0 ? 4 : t == 1 ? -6 : t == 2 ? 4 : -1);
            __syncthreads();
            const uint32_t rb = sbps - w;
            if (type == SF_CONSTANT) {
                // 8 zero header bits, then the raw first sample (flac.c:813-830)
                if (t == 0)
                    put_g(wb, b0 + pos + 8u, sbps, (uint32_t)s[0]);
                pos += 8u + sbps;
            } else {
                const uint32_t code = type == SF_VERBATIM ? 1u
                                    : type == SF_FIXED    ? 8u + order
                                                          : 32u + order - 1u;
                if (t == 0) {
                    put_g(wb, b0 + pos, 7, code);
                    if (w)
                        put_g(wb, b0 + pos + 7u, w + 1u, (1u << w) | 1u);
                }
                const uint64_t hb = 7u + (w ? w + 1u : 1u);
                if (type == SF_VERBATIM) {
                    for (uint32_t i = t; i < N; i += BT)
                        put_g(wb, b0 + pos + hb + (uint64_t)i * rb, rb, (uint32_t)s[i]);
                    pos += hb + (uint64_t)N * rb;
                } else {
                    if (t < order)
                        put_g(wb, b0 + pos + hb + (uint64_t)t * rb, rb, (uint32_t)s[t]);
                    uint64_t q = pos + hb + (uint64_t)order * rb;
                    int shift = 0;
                    if (type == SF_LPC) {
                        shift = d.shift;
                        if (t == 0) {
                            put_g(wb, b0 + q, 4, d.precision - 1u);
                            put_g(wb, b0 + q + 4u, 5, (uint32_t)shift & 31u);
                        }
                        if (t < order)
                            put_g(wb, b0 + q + 9u + (uint64_t)t * d.precision, d.precision,
                                  (uint32_t)cf[t]);
                        q += 9u + (uint64_t)order * d.precision;
                    }
                    if (t == 0) {
                        put_g(wb, b0 + q, 2, d.method);
                        put_g(wb, b0 + q + 2u, 4, d.porder);
                    }
                    const uint64_t rs = q + 6u;
                    const uint32_t po = d.porder;
                    const uint32_t pbits = d.method ? 5u : 4u;
                    const uint32_t Sp = N >> po;
                    const bool degen = Sp < order;
                    const uint8_t *__restrict__ rk = rice_big + sid * rice_stride;
                    // pass 1: bits of this thread's run (codes, plus the
                    // header of every partition j >= 1 starting in it)
                    uint32_t cb = 0;
                    for (uint32_t i = max(ra, order); i < re; ++i) {
                        const uint32_t j = i / Sp;
                        const uint32_t k = degen ? rk[0] : rk[j];
                        const uint32_t u = zigzag(residual_at(s, (int)i, cf, (int)order, shift));
                        cb += (u >> k) + 1u + k;
                        if (!degen && j > 0u && i == j * Sp)
                            cb += pbits;
                    }
                    uint32_t total;
                    const uint32_t excl = wg_excl_scan_u32(cb, scan, total);
                    // pass 2: write
                    uint64_t bp = rs + pbits + excl;
                    for (uint32_t i = max(ra, order); i < re; ++i) {
                        const uint32_t j = i / Sp;
                        const uint32_t k = degen ? rk[0] : rk[j];
                        if (!degen && j > 0u && i == j * Sp) {
                            put_g(wb, b0 + bp, pbits, k);
                            bp += pbits;
                        }
                        const uint32_t u = zigzag(residual_at(s, (int)i, cf, (int)order, shift));
                        const uint32_t z = u >> k;
                        put_g(wb, b0 + bp + z, k + 1u, (1u << k) | (u & ((1u << k) - 1u)));
                        bp += z + 1u + k;
                    }
                    if (t == 0)
                        put_g(wb, b0 + rs, pbits, rk[0]);
                    const uint32_t np = 1u << po;
                    if (degen) // partition 0 holds every residual; the rest are empty
                        for (uint32_t j = 1u + t; j < np; j += BT)
                            put_g(wb, b0 + rs + pbits + total + (uint64_t)(j - 1u) * pbits, pbits,
                                  rk[j]);
                    // `total` already counts the headers of partitions >= 1
                    pos = rs + pbits + total + (degen ? (uint64_t)(np - 1u) * pbits : 0u);
                }
            }
            if (pos - start != d.bits && t == 0)
                atomicOr(err, 2u);
        }

        // CRC-16 of bytes [0, L): 256 chunks of Lc bytes over a virtually
        // zero-prefixed image (leading zeros keep a zero-init CRC at 0),
        // folded on one lane with the "advance by Lc zero bytes" matrix
        __threadfence();
        __syncthreads();
        const uint64_t Lb = fd.bytes - 2u;
        uint64_t Lc = 1;
        while ((uint64_t)BT * Lc < Lb)
            Lc <<= 1;
        const int64_t z = (int64_t)(BT * Lc) - (int64_t)Lb;
        uint32_t crc = 0;
        {
            uint64_t cw = ~0ull;
            uint32_t cv = 0;
            int64_t q = (int64_t)t * (int64_t)Lc - z;
            const int64_t qe = q + (int64_t)Lc;
            q = q < 0 ? (qe < 0 ? qe : 0) : q; // leading virtual zeros leave crc = 0
            for (; q < qe; ++q) {
                const uint64_t ab = (b0 >> 3) + (uint64_t)q; // byte offset from wb
                if ((ab >> 2) != cw) {
                    cw = ab >> 2;
                    cv = __hip_atomic_load(&wb[cw], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                crc = crc16_byte(crc_tab, crc, (cv >> (8u * (uint32_t)(ab & 3u))) & 0xFFu);
            }
        }
        crc_part[t] = crc;
        if (t < 16) {
            uint32_t c = 1u << t;
            for (uint64_t i = 0; i < Lc; ++i)
                c = crc16_byte(crc_tab, c, 0);
            crc_adv[t] = c;
        }
        __syncthreads();
        if (t == 0) {
            uint32_t c = 0;
            for (uint32_t i = 0; i < BT; ++i) {
                uint32_t a = 0;
                for (int b = 0; b < 16; ++b)
                    a ^= ((c >> b) & 1u) ? crc_adv[b] : 0u;
                c = a ^ crc_part[i];
            }
            put_g(wb, b0 + 8u * Lb, 16, c);
        }
        __syncthreads();
    }
}

// ---------------------------------------------------------------- launchers
hipError_t launch_subframe_search_big(const FlacParams &p, const void *pcm, int fmt,
                                      const FrameInfo *frames, const int16_t *coef_tab,
                                      const int8_t *shift_tab, const uint8_t *est_tab,
                                      SubDesc *sub, uint8_t *rice_big, uint32_t rice_stride,
                                      uint8_t *scratch, uint64_t slot_bytes, uint64_t row_bytes,
                                      uint32_t grid, hipStream_t s)
{
    if (p.n_frames == 0 || grid == 0)
        return hipSuccess;
    if (fmt == 0)
        hipLaunchKernelGGL((k_subframe_search_big<int16_t>), dim3(grid), dim3(BT), 0, s, p,
                           (const int16_t *)pcm, frames, coef_tab, shift_tab, est_tab, sub,
                           rice_big, rice_stride, scratch, slot_bytes, row_bytes);
    else
        hipLaunchKernelGGL((k_subframe_search_big<int32_t>), dim3(grid), dim3(BT), 0, s, p,
                           (const int32_t *)pcm, frames, coef_tab, shift_tab, est_tab, sub,
                           rice_big, rice_stride, scratch, slot_bytes, row_bytes);
    return hipGetLastError();
}

hipError_t launch_frame_pack_big(const FlacParams &p, const void *pcm, int fmt,
                                 const FrameInfo *frames, const TrackInfo *tracks,
                                 const SubDesc *sub, const uint8_t *rice_big,
                                 uint32_t rice_stride, const FrameDesc *fd, uint8_t *out,
                                 uint32_t *err, uint8_t *scratch, uint64_t slot_bytes,
                                 uint32_t grid, hipStream_t s)
{
    if (p.n_frames == 0 || grid == 0)
        return hipSuccess;
    if (fmt == 0)
        hipLaunchKernelGGL((k_frame_pack_big<int16_t>), dim3(grid), dim3(BT), 0, s, p,
                           (const int16_t *)pcm, frames, tracks, sub, rice_big, rice_stride, fd,
                           out, err, scratch, slot_bytes);
    else
        hipLaunchKernelGGL((k_frame_pack_big<int32_t>), dim3(grid), dim3(BT), 0, s, p,
                           (const int32_t *)pcm, frames, tracks, sub, rice_big, rice_stride, fd,
                           out, err, scratch, slot_bytes);
    return hipGetLastError();
}
