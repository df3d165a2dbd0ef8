// flac_lpc.hip — K1: LPC analysis of every subframe candidate.
//
// Reference: flacenc_best_lpc_coefficients and helpers,
// src/encoders/flac.c:1018-1324.  Byte-exactness hinges on fp64 order:
//   * windowed sample  x[n] = (double)s[n] * window[n]       (flac.c:1164-1166)
//   * autocorrelation  R[L] = sum_{i<N-L} x[i]*x[i+L], ONE accumulator added
//                      left to right, no fused multiply-add (flac.c:1178-1187)
//   * Levinson-Durbin, quantisation with frexp/round        (flac.c:1190-1324)
// This file is compiled with -ffp-contract=off and `#pragma clang fp
// contract(off)`, so every product is rounded before its add.
//
// Mapping: one lane = one subframe candidate of one frame; the candidates of
// a frame sit in adjacent lanes (16 frames per wave for stereo mid/side).  Each lane streams its samples once
// and keeps all LAGS+1 accumulators plus a circular history of the last
// LAGS windowed samples in registers: 13 independent fp64 add chains per
// lane, each bit-identical to the reference's sequential loop.  The
// sequential sum forbids tree/MFMA reductions inside a subframe, so the
// parallelism is across subframes.
//
// The window is applied to the UNSHIFTED candidate samples.  Shifting out
// w wasted bits scales every x[n] by 2^-w exactly, every R[L] by 4^-w
// exactly, and leaves the Levinson coefficients bit-identical (all
// operations are scale-invariant under powers of two in the normal range),
// so K1 does not need to know the wasted bits.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "flac_dev.h"
#include "launch.h"
#include "pcm_read.h"
#include "residual.h"
#include "wave.h"

#pragma clang fp contract(off)

// the VEC4 autocorrelation's PCM loads all issued before the first use
// its window values loaded one sub-group ahead

// (int)x on the reference's x86-64 build is cvttsd2si: NaN and out-of-range
// inputs produce INT_MIN.  v_cvt_i32_f64 saturates instead, so spell it out.
__device__ __forceinline__ int32_t d2i_x86(double x)
{
    if (!(x > -2147483649.0 && x < 2147483648.0))
        return INT32_MIN;
    return (int32_t)x;
}

template <int LAGS>
__device__ __forceinline__ void quantize_store(const double (&lp)[LAGS],
                                               int order, int prec,
                                               int16_t *__restrict__ q, uint32_t row,
                                               int8_t *__restrict__ shift_out)
{
    // flacenc_quantize_coefficients (flac.c:1270-1324)
    double l = 2.2250738585072014e-308; // DBL_MIN
#pragma unroll
    for (int i = 0; i < LAGS; ++i) {
        if (i < order) {
            const double a = fabs(lp[i]);
            l = a > l ? a : l;
        }
    }
    int log2cmax;
    frexp(l, &log2cmax);
    int shift = (prec - 1) - (log2cmax - 1) - 1;
    shift = shift < -16 ? -16 : shift;
    shift = shift > 15 ? 15 : shift;
    const int qmax = (1 << (prec - 1)) - 1;
    const int qmin = -(1 << (prec - 1));
    double err = 0.0;
#pragma unroll
    for (int i = 0; i < LAGS; ++i) {
        if (i < order) {
            if (shift >= 0)
                err += lp[i] * (double)(1 << shift);
            else
                err += lp[i] / (double)(1 << -shift);
            const int32_t ei = d2i_x86(round(err));
            q[i] = (int16_t)(ei < qmin ? qmin : (ei > qmax ? qmax : ei));
            err -= (double)ei;
        }
    }
    // rows are zero past the order: fixed-width readers use them as taps
    for (uint32_t i = (uint32_t)order; i < row; ++i)
        q[i] = 0;
    *shift_out = (int8_t)(shift >= 0 ? shift : 0);
}

// Autocorrelation of one candidate, streamed K samples at a time: all loads
// of a group are issued together (indices clamped, no branches), then the K
// accumulator chains run.  Positions past this lane's N contribute x = 0, which adds +-0.0
// to accumulators that are never -0.0 (exact no-op).
template <int MODE, typename T, int K>
__device__ __forceinline__ void autocorr(const T *__restrict__ src, const double *__restrict__ win,
                                         uint32_t ch, uint32_t cand, uint32_t n_loop,
                                         uint32_t nlast, uint32_t n_max, double (&acc)[K],
                                         double (&hist)[K])
{
    // software pipeline: the loads of group g+1 are in flight while the
    // chains of group g run
    int32_t sv[K];
    double wv[K];
#pragma unroll
    for (int u = 0; u < K; ++u) {
        const uint32_t j = min((uint32_t)u, nlast);
        sv[u] = cand_at<MODE>(src, j, ch, cand);
        wv[u] = win[j];
    }
    for (uint32_t j0 = 0; j0 < n_max; j0 += K) {
        double xv[K];
#pragma unroll
        for (int u = 0; u < K; ++u)
            xv[u] = (j0 + (uint32_t)u < n_loop) ? (double)sv[u] * wv[u] : 0.0;
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const uint32_t j = min(j0 + K + (uint32_t)u, nlast);
            sv[u] = cand_at<MODE>(src, j, ch, cand);
            wv[u] = win[j];
        }
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const double x = xv[u];
            hist[u] = x;
#pragma unroll
            for (int L = 0; L < K; ++L) {
                const double prod = hist[(u - L + K) % K] * x;
                acc[L] = acc[L] + prod;
            }
        }
    }
}

// Hot path: 16-bit stereo pairs, mid/side candidates, every active lane of
// the wave on the same frame length N (one shared window, read with scalar
// loads).  The candidate is one v_dot2 of the (l, r) pair with per-lane
// weights and a shift: L (1,0)>>0, R (0,1)>>0, mid (1,1)>>1, side (1,-1)>>0.
// Full groups of K samples use immediate-offset loads; only the last
// partial group clamps and masks.
template <int K, bool VEC4>
__device__ __forceinline__ void autocorr_ms16(const uint32_t *__restrict__ pairs,
                                              const double *__restrict__ win, uint32_t cand,
                                              uint32_t N, double (&acc)[K], double (&hist)[K])
{
    const uint32_t wts = cand == 0u ? 0x00000001u : cand == 1u ? 0x00010000u
                       : cand == 2u ? 0x00010001u : 0xFFFF0001u;
    const int gsh = cand == 2u ? 1 : 0;
    const uint32_t nfull = N / K * K;
    uint32_t j0 = 0;
    if (VEC4) {
        // groups of 4K samples: K dwordx4 loads (4 pairs each) per lane,
        // all issued before the first is used (left to the compiler, they
        // came two at a time, each pair waited before the next was issued:
        // K/2 memory round trips per group)
        const uint4 *__restrict__ q4 = (const uint4 *)pairs;
        for (; j0 + 4u * K <= N; j0 += 4u * K) {
            uint32_t pv[4 * K];
#pragma unroll
            for (int i = 0; i < K; ++i) {
                const uint4 v = q4[(j0 >> 2) + (uint32_t)i];
                pv[4 * i] = v.x;
                pv[4 * i + 1] = v.y;
                pv[4 * i + 2] = v.z;
                pv[4 * i + 3] = v.w;
            }
#pragma unroll
            for (int i = 0; i < 4 * K; ++i)
                asm volatile("" : "+v"(pv[i]));
#pragma unroll
            for (int sub = 0; sub < 4; ++sub) {
                double xv[K];
#pragma unroll
                for (int u = 0; u < K; ++u) {
                    const int v = __builtin_amdgcn_sdot2(
                        __builtin_bit_cast(short2_t, pv[sub * K + u]),
                        __builtin_bit_cast(short2_t, wts), 0, false);
                    xv[u] = (double)(v >> gsh) * win[j0 + (uint32_t)(sub * K + u)];
                }
#pragma unroll
                for (int u = 0; u < K; ++u) {
                    const double x = xv[u];
                    hist[u] = x;
#pragma unroll
                    for (int L = 0; L < K; ++L) {
                        const double prod = hist[(u - L + K) % K] * x;
                        acc[L] = acc[L] + prod;
                    }
                }
            }
        }
    }
    for (; j0 < nfull; j0 += K) {
        double xv[K];
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const int v = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, pairs[j0 + u]),
                                                 __builtin_bit_cast(short2_t, wts), 0, false);
            xv[u] = (double)(v >> gsh) * win[j0 + u];
        }
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const double x = xv[u];
            hist[u] = x;
#pragma unroll
            for (int L = 0; L < K; ++L) {
                const double prod = hist[(u - L + K) % K] * x;
                acc[L] = acc[L] + prod;
            }
        }
    }
    if (j0 < N) {
        double xv[K];
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const uint32_t j = min(j0 + (uint32_t)u, N - 1u);
            const int v = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2_t, pairs[j]),
                                                 __builtin_bit_cast(short2_t, wts), 0, false);
            xv[u] = j0 + (uint32_t)u < N ? (double)(v >> gsh) * win[j] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < K; ++u) {
            const double x = xv[u];
            hist[u] = x;
#pragma unroll
            for (int L = 0; L < K; ++L) {
                const double prod = hist[(u - L + K) % K] * x;
                acc[L] = acc[L] + prod;
            }
        }
    }
}

template <typename T, int LAGS>
__global__ __launch_bounds__(64) void k_lpc_analyze(
    FlacParams p, const T *__restrict__ pcm,
    const FrameInfo *__restrict__ frames, const double *__restrict__ windows,
    int16_t *__restrict__ coef_tab, int8_t *__restrict__ shift_tab,
    uint8_t *__restrict__ est_tab)
{
    constexpr int K = LAGS + 1;
    // lanes [c*k, c*k + c) = the c candidates of one frame: they read the
    // same interleaved PCM, so a load touches 64 / c frames' lines
    const uint32_t fpw = 64u / p.n_cand;
    const uint32_t fl = threadIdx.x / p.n_cand;
    const uint32_t cand = threadIdx.x - fl * p.n_cand;
    const uint32_t f = blockIdx.x * fpw + fl;
    const bool ms = (p.n_cand == 4u) && (p.channels == 2u);
    const bool active = fl < fpw && f < p.n_frames;
    const FrameInfo fi = frames[active ? f : 0u];
    const int M = (int)p.max_lpc_order;
    const uint32_t N = active ? fi.n : 0u;
    const bool do_lpc = active && N > (uint32_t)M + 1u;
    const uint32_t n_loop = do_lpc ? N : 0u;
    const uint32_t n_max = wave_max_u32(n_loop);
    if (n_max == 0u)
        return;

    double acc[K];
    double hist[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        acc[k] = 0.0;
        hist[k] = 0.0;
    }
    const double *__restrict__ win = windows + fi.win_off;
    const T *__restrict__ src = pcm + fi.pcm_start * p.channels;
    const uint32_t nlast = n_loop ? n_loop - 1u : 0u;
    const int mode = pcm_mode(pcm, ms);
    // uniform frame length over the active lanes -> shared window
    const uint32_t n_first = uniform_u32(do_lpc ? N : 0u);
    const bool uniform_n = wave_all(!active || (do_lpc ? N : 0u) == n_first) && n_first > 0u;
    if (mode == PCM_MS16 && uniform_n) {
        const double *__restrict__ wu =
            windows + uniform_u32(active ? fi.win_off : 0u);
        // 16-byte aligned frame starts in every lane: 4 pairs per load
        const bool al16 = wave_all(((uintptr_t)src & 15u) == 0u);
        if (al16)
            autocorr_ms16<K, true>((const uint32_t *)src, wu, cand, n_first, acc, hist);
        else
            autocorr_ms16<K, false>((const uint32_t *)src, wu, cand, n_first, acc, hist);
    } else switch (mode) {
    case PCM_MS16:
        autocorr<PCM_MS16, T, K>(src, win, p.channels, cand, n_loop, nlast, n_max, acc, hist);
        break;
    case PCM_MS:
        autocorr<PCM_MS, T, K>(src, win, p.channels, cand, n_loop, nlast, n_max, acc, hist);
        break;
    default:
        autocorr<PCM_CH, T, K>(src, win, p.channels, cand, n_loop, nlast, n_max, acc, hist);
    }
    if (!do_lpc)
        return;

    // Levinson-Durbin (flac.c:1190-1231), one row at a time.
    const size_t sub = (size_t)f * p.n_cand + cand;
    int16_t *__restrict__ qout = coef_tab + sub * p.coef_stride;
    int8_t *__restrict__ sout = shift_tab + sub * (size_t)M;
    const int prec = (int)p.qlp_precision;

    double prev[LAGS], cur[LAGS], errv[LAGS];
#pragma unroll
    for (int k = 0; k < LAGS; ++k) {
        prev[k] = 0.0;
        cur[k] = 0.0;
        errv[k] = 0.0;
    }
    double k0 = acc[1] / acc[0];
    cur[0] = k0;
    errv[0] = acc[0] * (1.0 - (k0 * k0));
    quantize_store<LAGS>(cur, 1, prec, qout, p.coef_row, sout);
#pragma unroll
    for (int i = 1; i < LAGS; ++i) {
        if (i < M) {
#pragma unroll
            for (int j = 0; j < LAGS; ++j)
                prev[j] = cur[j];
            double q = acc[i + 1];
#pragma unroll
            for (int j = 0; j < LAGS; ++j)
                if (j < i)
                    q -= (prev[j] * acc[i - j]);
            const double kk = q / errv[i - 1];
#pragma unroll
            for (int j = 0; j < LAGS; ++j)
                if (j < i)
                    cur[j] = prev[j] - (kk * prev[i - j - 1]);
            cur[i] = kk;
            errv[i] = errv[i - 1] * (1.0 - (kk * kk));
            quantize_store<LAGS>(cur, i + 1, prec, qout + i * p.coef_row, p.coef_row,
                                 sout + i);
        }
    }

    if (!p.exhaustive) {
        // flacenc_estimate_best_lpc_order (flac.c:1233-1268)
        const double ln2 = 0.69314718055994530942;
        const double error_scale = (ln2 * ln2) / ((double)N * 2.0);
        int best = 0;
        double best_bits = 1.7976931348623157e308;
        bool done = false;
#pragma unroll
        for (int i = 0; i < LAGS; ++i) {
            if (i < M && !done) {
                const int order = i + 1;
                if (errv[i] > 0.0) {
                    const unsigned header = (unsigned)order * (p.bps + p.qlp_precision);
                    double bpr = log(errv[i] * error_scale) / (ln2 * 2);
                    bpr = bpr > 0.0 ? bpr : 0.0;
                    const double est = (double)header + bpr * (double)(N - (unsigned)order);
                    if (est < best_bits) {
                        best = order;
                        best_bits = est;
                    }
                } else {
                    best = order;
                    done = true;
                }
            }
        }
        est_tab[sub] = (uint8_t)best;
    }
}

template <typename T, int LAGS>
static hipError_t launch_t(const FlacParams &p, const T *pcm, const FrameInfo *frames,
                           const double *windows, int16_t *coef_tab,
                           int8_t *shift_tab, uint8_t *est_tab, hipStream_t s)
{
    const uint32_t fpw = 64u / p.n_cand;
    dim3 grid((p.n_frames + fpw - 1u) / fpw);
    hipLaunchKernelGGL((k_lpc_analyze<T, LAGS>), grid, dim3(64), 0, s, p, pcm,
                       frames, windows, coef_tab, shift_tab, est_tab);
    return hipGetLastError();
}

template <typename T>
static hipError_t launch_lags(const FlacParams &p, const T *pcm,
                              const FrameInfo *frames, const double *windows,
                              int16_t *coef_tab, int8_t *shift_tab,
                              uint8_t *est_tab, hipStream_t s)
{
    const uint32_t M = p.max_lpc_order;
    if (M <= 8)
        return launch_t<T, 8>(p, pcm, frames, windows, coef_tab, shift_tab, est_tab, s);
    if (M <= 12)
        return launch_t<T, 12>(p, pcm, frames, windows, coef_tab, shift_tab, est_tab, s);
    return launch_t<T, ATG_MAX_LPC>(p, pcm, frames, windows, coef_tab, shift_tab,
                                    est_tab, s);
}

hipError_t launch_lpc_analyze(const FlacParams &p, const void *pcm, int fmt,
                              const FrameInfo *frames, const double *windows,
                              int16_t *coef_tab, int8_t *shift_tab,
                              uint8_t *est_tab, hipStream_t s)
{
    if (p.max_lpc_order == 0 || !p.try_lpc || p.n_frames == 0)
        return hipSuccess;
    if (fmt == 0)
        return launch_lags<int16_t>(p, (const int16_t *)pcm, frames, windows,
                                    coef_tab, shift_tab, est_tab, s);
    return launch_lags<int32_t>(p, (const int32_t *)pcm, frames, windows,
                                coef_tab, shift_tab, est_tab, s);
}
