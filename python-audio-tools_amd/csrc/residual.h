// residual.h — a lane's LPC/FIXED residuals over its run of samples held in
// LDS; shared by the subframe search (K2) and the frame packer (K5) so both
// see the very same integers (reference residual loop: src/encoders/flac.c
// flacenc_encode_lpc_subframe 1060-1126, fixed 918-1016).
//
// LDS sample layout: 4 pad words after every 64 samples, so lane runs (64
// samples apart) start 68 words apart: 16-byte aligned for ds_read_b128 and
// bank-conflict-free across each 16-lane b128 group.  Indices -12..-1
// (history before sample 0) read zeros.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "flac_dev.h"
#include "pcm_read.h"
#include "wave.h"

#define SL_PRE 48
#define SL_WORDS (SL_PRE + ATG_MAX_BLOCK + 4 * (ATG_MAX_BLOCK / 64) + 64 + 8)

__device__ __forceinline__ int saddr(int i) { return SL_PRE + i + 4 * (i >> 6); }

__device__ __forceinline__ uint32_t zigzag(int32_t r)
{
    return ((uint32_t)r << 1) ^ (uint32_t)(r >> 31);
}

__device__ __forceinline__ uint32_t iabs_u(int32_t r)
{
    return r < 0 ? 0u - (uint32_t)r : (uint32_t)r;
}

typedef short short2_t __attribute__((ext_vector_type(2)));

// First v_dot2 of a sum that starts at 0: the VOP3 form with the inline
// constant 0 as the accumulator, so no v_mov seeds it (the compiler's
// v_dot2c form accumulates into its destination and copies a zero in
// first).  b is wave-uniform (an SGPR operand).
__device__ __forceinline__ int dot2_z(uint32_t a, int b_uniform)
{
    int d;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(d) : "v"(a), "s"(b_uniform));
    return d;
}

// Residuals of samples [a, a+len) (len <= 64) with a 12-tap predictor whose
// taps >= order are 0, exact in 32 bits (caller checks sum|c| * max|s| <
// 2^31).  cf[] must be wave-uniform.  Two kernels of arithmetic:
//   DOT2  samples fit int16: v_dot2_i32_i16 takes two taps per instruction
//         on packed pairs Q_m = (s_m, s_{m-1}); pred_t = sum_j C_j . Q_{t-1-2j}
//         -> 1 v_perm + 6 v_dot2 per residual;
//   MAD24 samples fit 24 bits: v_mad_i32_i24, 12 per residual.
// FULL: len == 64 and a % 64 == 0 (N == 4096), samples read 16 at a time
// with ds_read_b128.  Writes the zig-zag codes to u[] (0 past len) and
// returns sum |r| over the run; warm-up positions (< order) are NOT yet
// excluded.
template <bool DOT2, bool FULL>
__device__ __forceinline__ uint64_t lane_residuals(const int32_t *__restrict__ sl, int a, int len,
                                                   const int (&cf)[ATG_FAST_ORDER], int shift,
                                                   uint32_t (&u)[ATG_RUN])
{
    constexpr int W = ATG_FAST_ORDER;
    int cp[W / 2]; // packed coefficient pairs (c_2j, c_2j+1)
#pragma unroll
    for (int j = 0; j < W / 2; ++j)
        cp[j] = uniform_i32((int)(((uint32_t)cf[2 * j] & 0xFFFFu) |
                                  ((uint32_t)cf[2 * j + 1] << 16)));
    uint64_t sum = 0;
    int base = a;
    // history: win[k] = s[i-1-k] (MAD24), qw[k] = Q_{i-1-k} (DOT2)
    int win[W];
    int h[W + 1]; // s[a-13 .. a-1]
    if (FULL) {
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
    } else {
#pragma unroll
        for (int k = 0; k <= W; ++k)
            h[k] = sl[saddr(base - W - 1 + k)];
    }
    int qw[W];
#pragma unroll
    for (int k = 0; k < W; ++k) {
        win[k] = h[W - k];                                     // s[a-1-k]
        qw[k] = (int)__builtin_amdgcn_perm((uint32_t)h[W - 1 - k], (uint32_t)h[W - k],
                                           0x05040100u);       // (s[a-1-k], s[a-2-k])
    }
#pragma unroll
    for (int ch = 0; ch < ATG_RUN / 16; ++ch) {
        // keep each chunk's loads inside the chunk (bounds live registers)
        asm volatile("" : "+v"(base)::"memory");
        int x[16];
        if (FULL) {
            const int4 *p4 = (const int4 *)&sl[saddr(base + 16 * ch)];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int4 v = p4[q];
                x[4 * q] = v.x;
                x[4 * q + 1] = v.y;
                x[4 * q + 2] = v.z;
                x[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int t = 0; t < 16; ++t)
                x[t] = sl[saddr(base + 16 * ch + t)];
        }
#pragma unroll
        for (int tt = 0; tt < 16; ++tt) {
            const int t = 16 * ch + tt;
            const int s = x[tt];
            int acc;
            if (DOT2) {
                acc = 0;
#pragma unroll
                for (int j = 0; j < W / 2; ++j) {
                    short2_t av = __builtin_bit_cast(short2_t, qw[2 * j]);
                    short2_t bv = __builtin_bit_cast(short2_t, cp[j]);
                    acc = __builtin_amdgcn_sdot2(av, bv, acc, false);
                }
                const int prev = win[0];
#pragma unroll
                for (int k = W - 1; k > 0; --k)
                    qw[k] = qw[k - 1];
                qw[0] = (int)__builtin_amdgcn_perm((uint32_t)prev, (uint32_t)s, 0x05040100u);
                win[0] = s;
            } else {
                acc = 0;
#pragma unroll
                for (int k = 0; k < W; ++k)
                    acc = mad24(win[k], cf[k], acc);
#pragma unroll
                for (int k = W - 1; k > 0; --k)
                    win[k] = win[k - 1];
                win[0] = s;
            }
            const int r = (int)((uint32_t)s - (uint32_t)(acc >> shift));
            uint32_t uu = zigzag(r);
            uint32_t ar = iabs_u(r);
            if (!FULL) {
                const bool v = t < len;
                uu = v ? uu : 0u;
                ar = v ? ar : 0u;
            }
            u[t] = uu;
            sum += ar;
        }
    }
    return sum;
}

// Samples too wide for the 32-bit kernels above (24-bit sources): with
// s = hi * 4096 + lo (hi = s >> 12, lo = s & 4095) the predictor is two exact
// v_mad_i32_i24 chains A = sum c hi, B = sum c lo, and the reference's
// 64-bit (sum c s) >> shift (flac.c:999-1008) is
//     BIG (shift >= 12):  (A + (B >> 12)) >> (shift - 12)
//     else:               (A << (12 - shift)) + (B >> shift)
// Exact when sum|c| * (max|s| / 4096 + 1) < 2^31 (caller checks) and
// max|s| < 2^26.  Same outputs as lane_residuals.
template <bool FULL, bool BIG>
__device__ __forceinline__ uint64_t lane_residuals_hl(const int32_t *__restrict__ sl, int a,
                                                      int len, const int (&cf)[ATG_FAST_ORDER],
                                                      int shift, uint32_t (&u)[ATG_RUN])
{
    constexpr int W = ATG_FAST_ORDER;
    const int sa = BIG ? shift - 12 : 12 - shift;
    uint64_t sum = 0;
    int wh[W], wl[W]; // hi / lo of s[i-1-k]
#pragma unroll
    for (int k = 0; k < W; ++k) {
        const int h = sl[saddr(a - 1 - k)];
        wh[k] = h >> 12;
        wl[k] = h & 4095;
    }
#pragma unroll
    for (int ch = 0; ch < ATG_RUN / 16; ++ch) {
        asm volatile("" : "+v"(a)::"memory");
        int x[16];
        if (FULL) {
            const int4 *p4 = (const int4 *)&sl[saddr(a + 16 * ch)];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const int4 v = p4[q];
                x[4 * q] = v.x;
                x[4 * q + 1] = v.y;
                x[4 * q + 2] = v.z;
                x[4 * q + 3] = v.w;
            }
        } else {
#pragma unroll
            for (int t = 0; t < 16; ++t)
                x[t] = sl[saddr(a + 16 * ch + t)];
        }
#pragma unroll
        for (int tt = 0; tt < 16; ++tt) {
            const int t = 16 * ch + tt;
            const int s = x[tt];
            int ah = 0, al = 0;
#pragma unroll
            for (int k = 0; k < W; ++k) {
                ah = mad24(wh[k], cf[k], ah);
                al = mad24(wl[k], cf[k], al);
            }
#pragma unroll
            for (int k = W - 1; k > 0; --k) {
                wh[k] = wh[k - 1];
                wl[k] = wl[k - 1];
            }
            wh[0] = s >> 12;
            wl[0] = s & 4095;
            const int q = BIG ? (ah + (al >> 12)) >> sa : (ah << sa) + (al >> shift);
            const int r = (int)((uint32_t)s - (uint32_t)q);
            uint32_t uu = zigzag(r);
            uint32_t ar = iabs_u(r);
            if (!FULL) {
                const bool v = t < len;
                uu = v ? uu : 0u;
                ar = v ? ar : 0u;
            }
            u[t] = uu;
            sum += ar;
        }
    }
    return sum;
}

// Exclude warm-up positions (< order) from a run's codes and |r| sum.
// |r| = (u + 1) >> 1 for a zig-zag code u.
__device__ __forceinline__ int drop_warmup(int a, int len, int order, uint32_t (&u)[ATG_RUN],
                                           uint64_t &sum)
{
    const int warm = min(max(order - a, 0), len);
    if (warm > 0) {
#pragma unroll
        for (int t = 0; t < ATG_FAST_ORDER; ++t) {
            if (t < warm) {
                sum -= ((uint64_t)u[t] + 1u) >> 1;
                u[t] = 0u;
            }
        }
    }
    return warm;
}

// 32-bit accumulation is exact when every partial sum fits in int32
// (sum |c| * max |s| < 2^31); which arithmetic kernel applies.
enum { RES_GENERIC = 0, RES_DOT2 = 1, RES_MAD24 = 2 };
__device__ __forceinline__ int residual_kernel(uint64_t csum, uint32_t maxabs, int order)
{
    const bool narrow = csum * (uint64_t)maxabs < (1ull << 31);
    if (narrow && order <= ATG_FAST_ORDER) {
        if (maxabs <= 32767u && csum <= 32767u * 12u)
            return RES_DOT2;
        if (maxabs < (1u << 23))
            return RES_MAD24;
    }
    return RES_GENERIC;
}

// Stage candidate `cand` of a frame (samples [0, N)) through registers:
// lane l takes samples l, l + 64, ...; STAGE_U loads per lane are issued
// before any is consumed (one memory latency per STAGE_U x 64 samples
// instead of one per 64).  f(i, s) consumes sample i.
#define STAGE_U 32
template <int MODE, typename T, typename F>
__device__ __forceinline__ void stage_candidate(const T *__restrict__ src, uint32_t N, uint32_t ch,
                                                uint32_t cand, int lane, F &&f)
{
    const uint32_t nlast = N ? N - 1u : 0u;
    for (uint32_t m0 = 0; m0 * 64u < N; m0 += STAGE_U) {
        int32_t v[STAGE_U];
#pragma unroll
        for (int u = 0; u < STAGE_U; ++u) {
            const uint32_t i = (uint32_t)lane + 64u * (m0 + (uint32_t)u);
            v[u] = cand_at<MODE>(src, min(i, nlast), ch, cand);
        }
#pragma unroll
        for (int u = 0; u < STAGE_U; ++u) {
            const uint32_t i = (uint32_t)lane + 64u * (m0 + (uint32_t)u);
            if (i < N)
                f(i, v[u]);
        }
    }
}

template <typename T, typename F>
__device__ __forceinline__ void stage_candidate_any(const T *__restrict__ pcm, uint64_t pcm_start,
                                                    uint32_t N, uint32_t ch, uint32_t cand,
                                                    bool ms, int lane, F &&f)
{
    const T *__restrict__ src = pcm + pcm_start * ch;
    switch (pcm_mode(pcm, ms)) {
    case PCM_MS16: stage_candidate<PCM_MS16>(src, N, ch, cand, lane, f); break;
    case PCM_MS: stage_candidate<PCM_MS>(src, N, ch, cand, lane, f); break;
    default: stage_candidate<PCM_CH>(src, N, ch, cand, lane, f); break;
    }
}

// Register-staged variant of lane_residuals for a full 64-sample run:
// xs(i) = sample (a - 16 + i) (i a compile-time constant after unrolling),
// i.e. xs(16) is the run's first sample and xs(3..15) its predecessors.
// Writes zig-zag codes only.
template <bool DOT2, typename X>
__device__ __forceinline__ void lane_residuals_regs(X &&xs, const int (&cf)[ATG_FAST_ORDER],
                                                    int shift, uint32_t (&u)[ATG_RUN])
{
    constexpr int W = ATG_FAST_ORDER;
    int cp[W / 2];
#pragma unroll
    for (int j = 0; j < W / 2; ++j)
        cp[j] = uniform_i32((int)(((uint32_t)cf[2 * j] & 0xFFFFu) |
                                  ((uint32_t)cf[2 * j + 1] << 16)));
    int win[W], qw[W];
#pragma unroll
    for (int k = 0; k < W; ++k) {
        win[k] = xs(15 - k);                                              // s[a-1-k]
        qw[k] = (int)__builtin_amdgcn_perm((uint32_t)xs(14 - k), (uint32_t)xs(15 - k),
                                           0x05040100u);                  // (s[a-1-k], s[a-2-k])
    }
#pragma unroll
    for (int t = 0; t < ATG_RUN; ++t) {
        const int s = xs(16 + t);
        int acc = 0;
        if (DOT2) {
            acc = dot2_z((uint32_t)qw[0], cp[0]);
#pragma unroll
            for (int j = 1; j < W / 2; ++j) {
                short2_t av = __builtin_bit_cast(short2_t, qw[2 * j]);
                short2_t bv = __builtin_bit_cast(short2_t, cp[j]);
                acc = __builtin_amdgcn_sdot2(av, bv, acc, false);
            }
            const int prev = win[0];
#pragma unroll
            for (int k = W - 1; k > 0; --k)
                qw[k] = qw[k - 1];
            qw[0] = (int)__builtin_amdgcn_perm((uint32_t)prev, (uint32_t)s, 0x05040100u);
            win[0] = s;
        } else {
#pragma unroll
            for (int k = 0; k < W; ++k)
                acc = mad24(win[k], cf[k], acc);
#pragma unroll
            for (int k = W - 1; k > 0; --k)
                win[k] = win[k - 1];
            win[0] = s;
        }
        u[t] = zigzag((int)((uint32_t)s - (uint32_t)(acc >> shift)));
    }
}
