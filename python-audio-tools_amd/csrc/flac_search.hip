// flac_search.hip — K2: choose the coding of every subframe candidate.
//
// Reference: flacenc_write_subframe and everything it calls,
// src/encoders/flac.c:673-1016, 1326-1505, 1578-1631.  For every candidate
// the reference builds FIXED, LPC (FLAC-8: orders 1..12, each encoded into a
// bit accumulator) and VERBATIM, keeping the smallest with strict `<`.  The
// accumulator only counts bits, so this kernel computes exactly the same
// uint32 counts analytically and serialises nothing (K5 packs the winner).
//
// Mapping: one wave (one 64-thread workgroup) per subframe candidate.  The
// candidate's samples sit in LDS (one pad word per 64 samples: lane runs are
// 64 words apart, so the pad makes per-lane sequential reads conflict-free).
// Lane l owns a contiguous run of <= 64 samples lying inside one finest
// residual partition (for N = 4096 and partition order 6, lane l IS
// partition l).  Per predictor:
//   pass 1  residuals with a register window (v_mad_i32_i24, coefficients in
//           SGPRs), zig-zag codes kept in 64 VGPRs, |r| summed per lane;
//   select  partition sums for orders 6..0 by a butterfly over lanes, Rice
//           parameters by bit-length arithmetic, the reference's size
//           estimate per order, argmin (strict <);
//   pass 2  exact bits sum((u >> k) + 1 + k) from the kept codes.
// Orders > 12 or samples/coefficients too wide for 32-bit accumulation go
// through a generic path with a 64-bit accumulator (v_mad_i64_i32) that
// recomputes residuals in pass 2.
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
constexpr int kK2WavesPerEu = 2;

struct Eval {
    uint32_t bits;    // residual section bits
    PartSel sel;
};

// v_dot2_i32_i16 with a zero accumulator (VOP3 form: no v_mov to clear it)
__device__ __forceinline__ int dot2_first(int a, int b_uniform)
{
    int d;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(d) : "v"(a), "s"(b_uniform));
    return d;
}

// Hot path (N = 4096, samples fit int16, |u| < 2^26): residuals of the
// lane's 64-sample run with TAPS taps (the order rounded up to even),
// v_dot2 on packed sample pairs.  Keeps v = r ^ (r >> 31) = |r| - [r < 0]
// per sample instead of the zig-zag code u = 2v + [r < 0]: |r| = v + [r<0]
// and u >> k = v >> (k - 1) for k >= 1, so the partition search and the
// exact bit count need only v, sum v and #neg.  Sums are 32-bit, two
// samples per v_add3.  Warm-up positions (lane 0, t < order) are masked.
template <int TAPS>
__device__ __forceinline__ uint64_t residuals_full_dot2(const int32_t *__restrict__ sl,
                                                        const RunCtx &c,
                                                        const int (&cfu)[ATG_FAST_ORDER],
                                                        int order, int shift,
                                                        uint32_t (&u)[ATG_RUN], uint32_t &sv,
                                                        uint32_t &nneg)
{
    constexpr int NP = TAPS / 2;
    constexpr int W = ATG_FAST_ORDER;
    int cp[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j)
        cp[j] = uniform_i32((int)(((uint32_t)cfu[2 * j] & 0xFFFFu) |
                                  ((uint32_t)cfu[2 * j + 1] << 16)));
    int base = c.a;
    int h[W + 1]; // s[a-13 .. a-1]
    {
        const int4 *hp = (const int4 *)&sl[saddr(base - W)];
#pragma unroll
        for (int q = 0; q < W / 4; ++q) {
            const int4 v = hp[q];
            h[1 + 4 * q] = v.x;
            h[2 + 4 * q] = v.y;
            h[3 + 4 * q] = v.z;
            h[4 + 4 * q] = v.w;
        }
        h[0] = sl[saddr(base - W - 1)];
    }
    int qw[TAPS]; // qw[k] = Q_{t-1-k} = (s[t-1-k], s[t-2-k])
#pragma unroll
    for (int k = 0; k < TAPS; ++k)
        qw[k] = (int)__builtin_amdgcn_perm((uint32_t)h[W - 1 - k], (uint32_t)h[W - k],
                                           0x05040100u);
    int prev = h[W];
    const int warm = c.a < order ? order - c.a : 0; // lane 0 only
    uint32_t su = 0, sn = 0, pu = 0, pn = 0;
#pragma unroll
    for (int ch = 0; ch < ATG_RUN / 16; ++ch) {
        asm volatile("" : "+v"(base)::"memory");
        int x[16];
        const int4 *p4 = (const int4 *)&sl[saddr(base + 16 * ch)];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int4 v = p4[q];
            x[4 * q] = v.x;
            x[4 * q + 1] = v.y;
            x[4 * q + 2] = v.z;
            x[4 * q + 3] = v.w;
        }
#pragma unroll
        for (int tt = 0; tt < 16; ++tt) {
            const int t = 16 * ch + tt;
            const int s = x[tt];
            int acc = dot2_first(qw[0], cp[0]);
#pragma unroll
            for (int j = 1; j < NP; ++j) {
                short2_t av = __builtin_bit_cast(short2_t, qw[2 * j]);
                short2_t bv = __builtin_bit_cast(short2_t, cp[j]);
                acc = __builtin_amdgcn_sdot2(av, bv, acc, false);
            }
#pragma unroll
            for (int k = TAPS - 1; k > 0; --k)
                qw[k] = qw[k - 1];
            qw[0] = (int)__builtin_amdgcn_perm((uint32_t)prev, (uint32_t)s, 0x05040100u);
            prev = s;
            const int r = (int)((uint32_t)s - (uint32_t)(acc >> shift));
            uint32_t neg = (uint32_t)(r >> 31);
            uint32_t vv = (uint32_t)r ^ neg; // |r| - [r < 0]
            if (t < W) {
                const bool w = t < warm;
                vv = w ? 0u : vv;
                neg = w ? 0u : neg;
            }
            u[t] = vv;
            if (tt & 1) {
                su = su + pu + vv; // v_add3_u32
                sn = sn + pn + neg;
            } else {
                pu = vv;
                pn = neg;
            }
        }
    }
    sv = su;
    nneg = 0u - sn;
    return (uint64_t)su + (uint64_t)nneg;
}

// Other fast cases: 12 taps (residual.h), 64-bit |r| sums, warm-up dropped
// afterwards.
template <bool DOT2, bool FULL>
__device__ __forceinline__ uint64_t residuals_fast(const int32_t *__restrict__ sl,
                                                   const RunCtx &c,
                                                   const int (&cfu)[ATG_FAST_ORDER], int order,
                                                   int shift, uint32_t (&u)[ATG_RUN])
{
    int cf[ATG_FAST_ORDER];
#pragma unroll
    for (int k = 0; k < ATG_FAST_ORDER; ++k)
        cf[k] = uniform_i32(cfu[k]);
    uint64_t sum = lane_residuals<DOT2, FULL>(sl, c.a, c.len, cf, shift, u);
    drop_warmup(c.a, c.len, order, u, sum);
    return sum;
}

// Generic path: any order <= 32, 64-bit accumulator, recompute in pass 2.
__device__ __forceinline__ Eval eval_generic(const int32_t *__restrict__ sl, const RunCtx &c,
                                          const int *__restrict__ cf_lds, int order,
                                          int shift)
{
    uint64_t sum = 0;
    const int start = max(c.a, order);
    const int end = c.a + c.len;
    for (int i = start; i < end; ++i) {
        int64_t acc = 0;
        for (int k = 0; k < order; ++k)
            acc += (int64_t)cf_lds[k] * (int64_t)sl[saddr(i - 1 - k)];
        const int r = (int)((uint32_t)sl[saddr(i)] - (uint32_t)(int32_t)(acc >> shift));
        sum += iabs_u(r);
    }
    Eval ev;
    ev.sel = select_partitions(sum, (uint32_t)order, c);
    const uint32_t k = ev.sel.k_lane;
    uint32_t lb = 0;
    for (int i = start; i < end; ++i) {
        int64_t acc = 0;
        for (int k2 = 0; k2 < order; ++k2)
            acc += (int64_t)cf_lds[k2] * (int64_t)sl[saddr(i - 1 - k2)];
        const int r = (int)((uint32_t)sl[saddr(i)] - (uint32_t)(int32_t)(acc >> shift));
        lb += (zigzag(r) >> k) + 1u + k;
    }
    ev.bits = dpp_wave_sum<uint32_t>(lb) + ev.sel.hdr_bits;
    return ev;
}

// One predictor on the fast paths (order <= 12, exact 32-bit arithmetic):
// residuals with the 64 zig-zag codes of the lane's run kept in VGPRs,
// partition search, exact bits.  cfu[] = wave-uniform taps (0 past order).
__device__ __forceinline__ Eval eval_fast_any(const int32_t *sl, const RunCtx &c,
                                              const int (&cfu)[ATG_FAST_ORDER], int order,
                                              int shift, uint32_t maxabs, uint64_t csum,
                                              int kind)
{
    const bool full = c.N == ATG_MAX_BLOCK;
    // |r| <= max|s| + (sum|c| max|s| >> shift) + 1; 32-bit sums of 64 codes
    // u <= 2|r| + 1 are exact below 2^26 per code
    const uint64_t rbound = (uint64_t)maxabs + ((csum * (uint64_t)maxabs) >> shift) + 1u;
    const bool sum32 = 2u * rbound + 1u < (1ull << 26);
    uint32_t u[ATG_RUN];
    uint64_t sum;
    bool vform = false;      // u[] holds v = |r| - [r<0] instead of zig-zag codes
    uint32_t sv = 0, nneg = 0;
    if (kind == RES_DOT2 && full && sum32) {
        vform = true;
        switch ((order + 1) >> 1) {
        case 0:
        case 1: sum = residuals_full_dot2<2>(sl, c, cfu, order, shift, u, sv, nneg); break;
        case 2: sum = residuals_full_dot2<4>(sl, c, cfu, order, shift, u, sv, nneg); break;
        case 3: sum = residuals_full_dot2<6>(sl, c, cfu, order, shift, u, sv, nneg); break;
        case 4: sum = residuals_full_dot2<8>(sl, c, cfu, order, shift, u, sv, nneg); break;
        case 5: sum = residuals_full_dot2<10>(sl, c, cfu, order, shift, u, sv, nneg); break;
        default: sum = residuals_full_dot2<12>(sl, c, cfu, order, shift, u, sv, nneg); break;
        }
    } else if (kind == RES_DOT2) {
        sum = full ? residuals_fast<true, true>(sl, c, cfu, order, shift, u)
                   : residuals_fast<true, false>(sl, c, cfu, order, shift, u);
    } else {
        sum = full ? residuals_fast<false, true>(sl, c, cfu, order, shift, u)
                   : residuals_fast<false, false>(sl, c, cfu, order, shift, u);
    }
    const int warm = min(max(order - c.a, 0), c.len);
    const int cnt = c.len - warm;
    Eval ev;
    // every lane's sum |r| < 2^25 -> the subframe's < 2^31: 32-bit search
    const bool small = wave_all(sum < (1ull << 25));
    ev.sel = select_partitions(sum, (uint32_t)order, c, small);
    const uint32_t k = ev.sel.k_lane;
    uint32_t lb = (uint32_t)cnt * (1u + k);
    if (vform) {
        // k = 0: sum u = 2 sum v + #neg;  k >= 1: sum (v >> (k - 1))
        const uint32_t kv = k ? k - 1u : 0u;
        uint32_t sh = 0;
#pragma unroll
        for (int t = 0; t < ATG_RUN; t += 2)
            sh = sh + (u[t] >> kv) + (u[t + 1] >> kv); // v_add3_u32
        lb += k ? sh : 2u * sv + nneg;
    } else {
#pragma unroll
        for (int t = 0; t < ATG_RUN; t += 2)
            lb = lb + (u[t] >> k) + (u[t + 1] >> k); // v_add3_u32
    }
    ev.bits = dpp_wave_sum<uint32_t>(lb) + ev.sel.hdr_bits;
    return ev;
}

// FIXED predictor of order o as LPC taps (flac.c:918-1016)
__device__ __forceinline__ int fixed_tap(uint32_t o, int j)
{
    switch (o) {
    case 1: return j == 0 ? 1 : 0;
    case 2: return j == 0 ? 2 : j == 1 ? -1 : 0;
    case 3: return j == 0 ? 3 : j == 1 ? -3 : j == 2 ? 1 : 0;
    case 4: return j == 0 ? 4 : j == 1 ? -6 : j == 2 ? 4 : j == 3 ? -1 : 0;
    default: return 0;
    }
}

__device__ __forceinline__ uint32_t wasted_field(uint32_t w) { return w ? w + 1u : 1u; }

// One subframe candidate (frame f, candidate cand) on one wave; sl/cf_lds
// are the workgroup's LDS.
template <typename T>
__device__ __forceinline__ void search_unit(const FlacParams &p, const T *__restrict__ pcm,
                                            const FrameInfo *__restrict__ frames,
                                            const int16_t *__restrict__ coef_tab,
                                            const int8_t *__restrict__ shift_tab,
                                            const uint8_t *__restrict__ est_tab,
                                            SubDesc *__restrict__ out, uint32_t *__restrict__ err,
                                            uint32_t f, uint32_t cand, int32_t *__restrict__ sl,
                                            int *__restrict__ cf_lds)
{
    const int lane = threadIdx.x;
    const FrameInfo fi = frames[f];
    const uint32_t N = fi.n;
    const bool ms = (p.n_cand == 4u) && (p.channels == 2u);
    const uint32_t sbps = p.bps + ((ms && cand == 3u) ? 1u : 0u);
    const size_t sub = (size_t)f * p.n_cand + cand;
    SubDesc *__restrict__ d = out + sub;

    if (N > ATG_MAX_BLOCK) {
        if (lane == 0)
            atomicOr(err, 1u);
        return;
    }

    // ---- load + constant / wasted-bits detection (flac.c:1578-1620)
    for (int i = lane; i < SL_PRE; i += 64)
        sl[i] = 0;
    const int32_t first = cand_sample(pcm, fi.pcm_start, p.channels, cand, ms);
    uint32_t orv = 0, amax = 0;
    bool same = true;
    stage_candidate_any(pcm, fi.pcm_start, N, p.channels, cand, ms, lane,
                        [&](uint32_t i, int32_t s) {
                            sl[saddr((int)i)] = s;
                            orv |= (uint32_t)s;
                            amax = max(amax, iabs_u(s));
                            same = same && (s == first);
                        });
    orv = dpp_wave_or_u32(orv);
    same = wave_all(same);
    __syncthreads();

    if (p.try_constant && same) {
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
        }
        return;
    }
    const uint32_t w = orv ? (uint32_t)__builtin_ctz(orv) : 0u;
    // every sample is a multiple of 2^w, so max|s >> w| = max|s| >> w
    const uint32_t maxabs = dpp_wave_max_u32(amax) >> w;
    if (w) {
        for (uint32_t i = lane; i < N; i += 64)
            sl[saddr((int)i)] >>= w;
        __syncthreads();
    }

    // ---- lane run inside one finest partition
    RunCtx c;
    c.lane = lane;
    c.N = N;
    c.max_rice = p.max_rice;
    {
        const uint32_t tz = N ? (uint32_t)__builtin_ctz(N) : 0u;
        uint32_t P = p.max_porder < tz ? p.max_porder : tz;
        P = P > ATG_MAX_PORDER ? ATG_MAX_PORDER : P;
        c.P = (int)P;
        const uint32_t G = 64u >> P;
        const uint32_t S = N >> P;
        const uint32_t R = (S + G - 1u) / G;
        const uint32_t j = (uint32_t)lane / G, q = (uint32_t)lane % G;
        uint32_t a = j * S + q * R;
        uint32_t e = a + R;
        const uint32_t pe = (j + 1u) * S;
        e = e < pe ? e : pe;
        a = a < e ? a : e;
        c.a = (int)a;
        c.len = (int)(e - a);
    }
    const uint32_t wf = wasted_field(w);
    const uint32_t rb = sbps - w; // bits per warm-up / verbatim sample

    // ---- FIXED order by |residual| sums over samples [4,N) (flac.c:856-916)
    uint32_t fixed_order = 0;
    if (p.try_fixed) {
        uint64_t s5[5] = {0, 0, 0, 0, 0};
        if (N == ATG_MAX_BLOCK && maxabs < (1u << 21)) {
            // the lane's 64 samples from LDS, differences carried in
            // registers, |d| summed in 32 bits (16 max|s| * 64 < 2^31)
            uint32_t a5[5] = {0, 0, 0, 0, 0};
            const int4 *hp = (const int4 *)&sl[saddr(c.a - 4)];
            const int4 h4 = hp[0];
            int x1 = h4.w, d1p = h4.w - h4.z, d2p = d1p - (h4.z - h4.y);
            int d3p = d2p - ((h4.z - h4.y) - (h4.y - h4.x));
            int base = c.a;
#pragma unroll
            for (int chn = 0; chn < ATG_RUN / 16; ++chn) {
                asm volatile("" : "+v"(base)::"memory");
                const int4 *p4 = (const int4 *)&sl[saddr(base + 16 * chn)];
                int x[16];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int4 v = p4[q];
                    x[4 * q] = v.x;
                    x[4 * q + 1] = v.y;
                    x[4 * q + 2] = v.z;
                    x[4 * q + 3] = v.w;
                }
#pragma unroll
                for (int tt = 0; tt < 16; ++tt) {
                    const int x0 = x[tt];
                    const int d1 = x0 - x1, d2 = d1 - d1p, d3 = d2 - d2p, d4 = d3 - d3p;
                    x1 = x0;
                    d1p = d1;
                    d2p = d2;
                    d3p = d3;
                    // samples 0..3 are outside the sums (lane 0 only)
                    const bool v = chn > 0 || tt >= 4 || c.a > 0;
                    a5[0] += v ? iabs_u(x0) : 0u;
                    a5[1] += v ? iabs_u(d1) : 0u;
                    a5[2] += v ? iabs_u(d2) : 0u;
                    a5[3] += v ? iabs_u(d3) : 0u;
                    a5[4] += v ? iabs_u(d4) : 0u;
                }
            }
#pragma unroll
            for (int k = 0; k < 5; ++k)
                s5[k] = a5[k];
        } else {
            const int st = max(c.a, 4);
            for (int i = st; i < c.a + c.len; ++i) {
                const uint32_t x0 = (uint32_t)sl[saddr(i)], x1 = (uint32_t)sl[saddr(i - 1)],
                               x2 = (uint32_t)sl[saddr(i - 2)], x3 = (uint32_t)sl[saddr(i - 3)],
                               x4 = (uint32_t)sl[saddr(i - 4)];
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
        }
#pragma unroll
        for (int k = 0; k < 5; ++k)
            s5[k] = dpp_wave_sum<uint64_t>(s5[k]);
        uint64_t best = s5[0];
        if (N > 4) {
#pragma unroll
            for (int k = 1; k < 5; ++k)
                if (s5[k] < best) {
                    best = s5[k];
                    fixed_order = (uint32_t)k;
                }
        }
        fixed_order = uniform_u32(fixed_order);
    }

    // ---- LPC candidate orders (flac.c:1034-1126)
    const int16_t *__restrict__ qtab = coef_tab + sub * p.coef_stride;
    const int8_t *__restrict__ stab = shift_tab + sub * (size_t)p.max_lpc_order;
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

    // ---- evaluate every predictor: [FIXED], LPC lo..hi
    uint32_t fixed_bits = 0;
    PartSel fixed_sel = {};
    uint32_t lpc_bits = 0xFFFFFFFFu, lpc_order = 0, lpc_prec = 0;
    int lpc_shift = 0;
    PartSel lpc_sel = {};
    const uint32_t n_pred = (p.try_fixed ? 1u : 0u) + (p.try_lpc ? hi - lo + 1u : 0u);
    for (uint32_t pi = 0; pi < n_pred; ++pi) {
        const bool is_fixed = p.try_fixed && pi == 0;
        const uint32_t o = is_fixed ? fixed_order : lo + pi - (p.try_fixed ? 1u : 0u);
        int shift = 0;
        uint32_t prec = 0;
        // this predictor's taps, wave-uniform (scalar loads of the LPC row)
        const int16_t *__restrict__ row = qtab + (size_t)(o ? o - 1u : 0u) * p.coef_row;
        if (!is_fixed && !dummy) {
            shift = stab[o - 1u];
            prec = p.qlp_precision;
        } else if (dummy) {
            prec = 2;
        }
        int cfu[ATG_FAST_ORDER];
        uint64_t csum = 0;
#pragma unroll
        for (int j = 0; j < ATG_FAST_ORDER; ++j) {
            const int cj = is_fixed ? fixed_tap(o, j)
                         : dummy ? (j == 0 ? 1 : 0)
                         : ((uint32_t)j < o ? (int)row[j] : 0);
            cfu[j] = cj;
            csum += (uint64_t)(cj < 0 ? -cj : cj);
        }
        const int kind = o <= ATG_FAST_ORDER ? residual_kernel(csum, maxabs, (int)o)
                                             : RES_GENERIC;
        Eval ev;
        if (kind == RES_GENERIC) {
            if ((uint32_t)lane < o)
                cf_lds[lane] = is_fixed ? fixed_tap(o, lane) : dummy ? 1 : (int)row[lane];
            __syncthreads();
            ev = eval_generic(sl, c, cf_lds, (int)o, shift);
            __syncthreads();
        } else {
            ev = eval_fast_any(sl, c, cfu, (int)o, shift, maxabs, csum, kind);
        }
        if (is_fixed) {
            fixed_bits = 7u + wf + o * rb + ev.bits;
            fixed_sel = ev.sel;
        } else {
            const uint32_t bits = 7u + wf + o * rb + 4u + 5u + o * prec + ev.bits;
            if (bits < lpc_bits) {
                lpc_bits = bits;
                lpc_order = o;
                lpc_shift = shift;
                lpc_prec = prec;
                lpc_sel = ev.sel;
            }
        }
    }

    // ---- subframe choice (flac.c:727-809)
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

    const PartSel &sel = pick == SF_FIXED ? fixed_sel : lpc_sel;
    if (pick != SF_VERBATIM) {
        // rice parameter of partition j is held by its first lane
        const uint32_t po = sel.porder;
        const uint32_t mask = (64u >> po) - 1u;
        if (((uint32_t)lane & mask) == 0u)
            d->rice[(uint32_t)lane >> (6u - po)] = (uint8_t)sel.k_own;
    }
    if (pick == SF_LPC) {
        if (lane < (int)lpc_order)
            d->coef[lane] = (int16_t)(N > p.max_lpc_order + 1u
                                          ? qtab[(lpc_order - 1u) * p.coef_row + lane]
                                          : 1);
    }
    if (lane == 0) {
        d->type = (uint8_t)pick;
        d->wasted = (uint8_t)w;
        d->sbps = (uint8_t)sbps;
        d->amax = maxabs;
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
}

template <typename T>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kK2WavesPerEu))) void k_subframe_search(
    FlacParams p, const T *__restrict__ pcm, const FrameInfo *__restrict__ frames,
    const int16_t *__restrict__ coef_tab, const int8_t *__restrict__ shift_tab,
    const uint8_t *__restrict__ est_tab, SubDesc *__restrict__ out,
    uint32_t *__restrict__ err)
{
    __shared__ __attribute__((aligned(16))) int32_t sl[SL_WORDS];
    __shared__ int cf_lds[ATG_MAX_LPC];
    uint32_t f, cand;
    xcd_unit_map(blockIdx.x, p.n_cand, &f, &cand);
    if (f >= p.n_frames)
        return;
    search_unit<T>(p, pcm, frames, coef_tab, shift_tab, est_tab, out, err, f, cand, sl, cf_lds);
}

// The candidates the 16-bit search (flac_search16.hip) handed over: a
// grid-stride loop over list[0 .. *count) of frame * n_cand + cand.
template <typename T>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kK2WavesPerEu))) void k_subframe_search_list(
    FlacParams p, const T *__restrict__ pcm, const FrameInfo *__restrict__ frames,
    const int16_t *__restrict__ coef_tab, const int8_t *__restrict__ shift_tab,
    const uint8_t *__restrict__ est_tab, SubDesc *__restrict__ out,
    uint32_t *__restrict__ err, const uint32_t *__restrict__ list,
    const uint32_t *__restrict__ count)
{
    __shared__ __attribute__((aligned(16))) int32_t sl[SL_WORDS];
    __shared__ int cf_lds[ATG_MAX_LPC];
    const uint32_t n = uniform_u32(*count);
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint32_t unit = uniform_u32(list[i]);
        search_unit<T>(p, pcm, frames, coef_tab, shift_tab, est_tab, out, err,
                       unit / p.n_cand, unit % p.n_cand, sl, cf_lds);
        __syncthreads();
    }
}

hipError_t launch_subframe_search(const FlacParams &p, const void *pcm, int fmt,
                                  const FrameInfo *frames, const int16_t *coef_tab,
                                  const int8_t *shift_tab, const uint8_t *est_tab,
                                  SubDesc *sub, uint32_t *err, hipStream_t s)
{
    if (p.n_frames == 0)
        return hipSuccess;
    const uint32_t f8 = (p.n_frames + 7u) / 8u * 8u;
    dim3 grid(f8 * p.n_cand);
    if (fmt == 0)
        hipLaunchKernelGGL((k_subframe_search<int16_t>), grid, dim3(64), 0, s, p,
                           (const int16_t *)pcm, frames, coef_tab, shift_tab, est_tab,
                           sub, err);
    else
        hipLaunchKernelGGL((k_subframe_search<int32_t>), grid, dim3(64), 0, s, p,
                           (const int32_t *)pcm, frames, coef_tab, shift_tab, est_tab,
                           sub, err);
    return hipGetLastError();
}

hipError_t launch_subframe_search_list(const FlacParams &p, const void *pcm, int fmt,
                                       const FrameInfo *frames, const int16_t *coef_tab,
                                       const int8_t *shift_tab, const uint8_t *est_tab,
                                       SubDesc *sub, uint32_t *err, const uint32_t *list,
                                       const uint32_t *count, uint32_t grid, hipStream_t s)
{
    if (p.n_frames == 0 || grid == 0)
        return hipSuccess;
    if (fmt == 0)
        hipLaunchKernelGGL((k_subframe_search_list<int16_t>), dim3(grid), dim3(64), 0, s, p,
                           (const int16_t *)pcm, frames, coef_tab, shift_tab, est_tab, sub, err,
                           list, count);
    else
        hipLaunchKernelGGL((k_subframe_search_list<int32_t>), dim3(grid), dim3(64), 0, s, p,
                           (const int32_t *)pcm, frames, coef_tab, shift_tab, est_tab, sub, err,
                           list, count);
    return hipGetLastError();
}
