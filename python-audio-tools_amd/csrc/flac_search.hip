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
#include "pcm_read.h"
#include "residual.h"
#include "wave.h"

// Rice parameter of one partition: the reference's loop
//   while ((uint64_t)(plength << Rice) < sum) if (Rice < max) Rice++; else break;
// including its 32-bit shift (flac.c:1477-1484).
__device__ __forceinline__ uint32_t rice_param(uint32_t plen, uint64_t sum, uint32_t maxk)
{
    const uint32_t bl = 32u - (uint32_t)__clz((int)plen);
    if (bl + maxk <= 32u) {
        if (sum == 0)
            return 0;
        if (plen == 0)
            return maxk;
        const int a = 64 - __clzll((long long)(sum - 1));
        int k = a - (int)bl;
        k = k < 0 ? 0 : k;
        if (((uint64_t)plen << k) < sum)
            k++;
        return (uint32_t)k < maxk ? (uint32_t)k : maxk;
    }
    uint32_t k = 0;
    while ((uint64_t)(uint32_t)(plen << k) < sum) {
        if (k < maxk)
            k++;
        else
            break;
    }
    return k;
}

struct RunCtx {
    int lane;
    int a;       // first sample of this lane's run
    int len;     // samples in the run
    uint32_t N;
    int P;       // deepest partition order usable (N % 2^P == 0, P <= max)
    uint32_t max_rice;
};

struct PartSel {
    uint32_t porder;
    uint32_t method;
    uint32_t k_lane;  // Rice parameter applied to this lane's residuals
    uint32_t k_own;   // Rice parameter of this lane's partition (for storage)
    uint32_t hdr_bits;
};

// flacenc_encode_residuals' partition-order search (flac.c:1362-1402) from
// per-lane |r| sums.  Level lv partition of lane l is l >> (6 - lv).
__device__ __forceinline__ PartSel select_partitions(uint64_t lane_sum, uint32_t order, const RunCtx &c)
{
    uint64_t S[7];
    S[6] = lane_sum;
#pragma unroll
    for (int b = 0; b < 6; ++b)
        S[5 - b] = S[6 - b] + shfl_xor_u64(S[6 - b], 1 << b);
    const uint64_t total = S[0];

    uint64_t best_tot = ~0ull;
    uint32_t best_p = 0;
    uint32_t kown[7];
#pragma unroll
    for (int lv = 0; lv <= 6; ++lv) {
        kown[lv] = 0;
        if (lv <= c.P) {
            const uint32_t Sp = c.N >> lv;
            const bool degen = Sp < order;
            const uint32_t jp = (uint32_t)c.lane >> (6 - lv);
            const uint32_t plen = jp == 0 ? Sp - order : Sp;
            const uint64_t sum = degen ? (jp == 0 ? total : 0ull) : S[lv];
            const uint32_t k = rice_param(plen, sum, c.max_rice);
            kown[lv] = k;
            uint64_t e;
            if (k > 0)
                e = 4ull + (sum >> (k - 1)) + (uint64_t)(uint32_t)((1u + k) * plen) -
                    (uint64_t)(plen / 2u);
            else
                e = 4ull + (sum << 1) + (uint64_t)plen - (uint64_t)(plen / 2u);
#pragma unroll
            for (int b = 6 - lv; b < 6; ++b)
                e += shfl_xor_u64(e, 1 << b);
            if (e < best_tot) {
                best_tot = e;
                best_p = (uint32_t)lv;
            }
        }
    }
    PartSel r;
    r.porder = best_p;
    uint32_t ko = kown[0];
#pragma unroll
    for (int lv = 1; lv <= 6; ++lv)
        ko = best_p == (uint32_t)lv ? kown[lv] : ko;
    r.k_own = ko;
    const bool degen_best = (c.N >> best_p) < order;
    const uint32_t k0 = (uint32_t)__shfl((int)ko, 0, 64);
    r.k_lane = degen_best ? k0 : ko;
    r.method = 0;
    if (c.max_rice > 14u)
        r.method = wave_max_u32(ko) > 14u ? 1u : 0u;
    r.hdr_bits = 6u + (1u << best_p) * (r.method ? 5u : 4u);
    return r;
}

struct Eval {
    uint32_t bits;    // residual section bits
    PartSel sel;
};

// Fast path: order <= 12 with exact 32-bit accumulation (residual.h); the 64
// zig-zag codes of the lane's run stay in VGPRs for pass 2.
template <bool DOT2, bool FULL>
__device__ __forceinline__ Eval eval_fast(const int32_t *__restrict__ sl, const RunCtx &c,
                                          const int *__restrict__ cf_lds, int order,
                                          int shift)
{
    int cf[ATG_FAST_ORDER];
#pragma unroll
    for (int k = 0; k < ATG_FAST_ORDER; ++k)
        cf[k] = uniform_i32(k < order ? cf_lds[k] : 0);
    uint32_t u[ATG_RUN];
    uint64_t sum = lane_residuals<DOT2, FULL>(sl, c.a, c.len, cf, shift, u);
    const int warm = drop_warmup(c.a, c.len, order, u, sum);
    const int cnt = c.len - warm;
    Eval ev;
    ev.sel = select_partitions(sum, (uint32_t)order, c);
    const uint32_t k = ev.sel.k_lane;
    uint32_t lb = 0;
#pragma unroll
    for (int t = 0; t < ATG_RUN; ++t)
        lb += u[t] >> k;
    lb += (uint32_t)cnt * (1u + k);
    ev.bits = wave_sum_u32(lb) + ev.sel.hdr_bits;
    return ev;
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
    ev.bits = wave_sum_u32(lb) + ev.sel.hdr_bits;
    return ev;
}

__device__ __forceinline__ Eval eval_any(const int32_t *sl, const RunCtx &c,
                                         const int *cf_lds, int order, int shift,
                                         uint32_t maxabs)
{
    uint64_t csum = 0;
    for (int k = 0; k < order; ++k)
        csum += (uint64_t)(cf_lds[k] < 0 ? -(int64_t)cf_lds[k] : cf_lds[k]);
    const int kind = residual_kernel(csum, maxabs, order);
    const bool full = c.N == ATG_MAX_BLOCK;
    if (kind == RES_DOT2)
        return full ? eval_fast<true, true>(sl, c, cf_lds, order, shift)
                    : eval_fast<true, false>(sl, c, cf_lds, order, shift);
    if (kind == RES_MAD24)
        return full ? eval_fast<false, true>(sl, c, cf_lds, order, shift)
                    : eval_fast<false, false>(sl, c, cf_lds, order, shift);
    return eval_generic(sl, c, cf_lds, order, shift);
}

__device__ __forceinline__ uint32_t wasted_field(uint32_t w) { return w ? w + 1u : 1u; }

template <typename T>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3))) void k_subframe_search(
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
    uint32_t orv = 0;
    bool same = true;
    for (uint32_t i = lane; i < N; i += 64) {
        const int32_t s = cand_sample(pcm, fi.pcm_start + i, p.channels, cand, ms);
        sl[saddr((int)i)] = s;
        orv |= (uint32_t)s;
        same = same && (s == first);
    }
    orv = wave_or_u32(orv);
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
    uint32_t maxabs = 0;
    for (uint32_t i = lane; i < N; i += 64) {
        const int32_t s = sl[saddr((int)i)] >> w;
        sl[saddr((int)i)] = s;
        maxabs = max(maxabs, iabs_u(s));
    }
    maxabs = wave_max_u32(maxabs);
    __syncthreads();

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
#pragma unroll
        for (int k = 0; k < 5; ++k)
            s5[k] = wave_sum_u64(s5[k]);
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
        if (is_fixed) {
            // FIXED predictors as integer coefficient sets, shift 0
            const int fc = o == 1 ? (lane == 0 ? 1 : 0)
                         : o == 2 ? (lane == 0 ? 2 : lane == 1 ? -1 : 0)
                         : o == 3 ? (lane == 0 ? 3 : lane == 1 ? -3 : lane == 2 ? 1 : 0)
                         : (lane == 0 ? 4 : lane == 1 ? -6 : lane == 2 ? 4 : lane == 3 ? -1 : 0);
            if (lane < 4)
                cf_lds[lane] = fc;
        } else if (dummy) {
            if (lane == 0)
                cf_lds[0] = 1;
            prec = 2;
        } else {
            if (lane < (int)o)
                cf_lds[lane] = qtab[(o * (o - 1u)) / 2u + (uint32_t)lane];
            shift = stab[o - 1u];
            prec = p.qlp_precision;
        }
        __syncthreads();
        const Eval ev = eval_any(sl, c, cf_lds, (int)o, shift, maxabs);
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
        __syncthreads();
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
                                          ? qtab[(lpc_order * (lpc_order - 1u)) / 2u + lane]
                                          : 1);
    }
    if (lane == 0) {
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
