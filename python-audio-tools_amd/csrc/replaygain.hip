// replaygain.hip — ReplayGain title and album analysis (SURVEY §8(a)
// G1–G5) for a batch of tracks: the reference's ReplayGain_title_gain /
// analyze_samples / analyzeResult / get_album_gain (src/replaygain.c
// :186-322, :566-807).
//
//   k_rg_seg     lane per segment of whole 50 ms windows (both channels):
//                the Yule-Walker (10th order) + Butterworth (2nd order) IIR
//                pair in the reference's exact fp64 operation order (no
//                contraction), started a warm-up early from zero state;
//                squared outputs summed with the reference's batch grouping
//                (4096-frame reads, 10-sample prebuffer batch, 50 ms windows;
//                singles for batch % 16, then 16-term groups) into one sum
//                per closed window; peak = max |x|.  Certified against the
//                serial computation (k_rg_seam, k_rg_bin), uncertified tracks
//                analysed again serially.
//   k_rg_bin     thread per window: (int)(1000·log10((l+r)/n/2 + 1e-37))
//                into the track's 12000-bin histogram.
//   k_rg_album   thread per bin: album histogram = sum of its tracks'.
//   k_rg_gain    block per histogram: 95th-percentile bin -> 64.82 - i/100.
//
// Multi-GPU: an album split across ranks all-reduces its uint32 histogram
// (sum, exact) and peak (max) -- the caller does that over RCCL between
// atg_replaygain_device and atg_replaygain_hist_gain (bench.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/atgpu.h"
#include "rg_coeffs.h"

#pragma clang fp contract(off)

namespace {

constexpr int kBins = 12000;

__constant__ double c_yule[20][21];
__constant__ double c_butter[20][5];

thread_local std::string g_rg_err;

atg_status rfail(atg_status s, const std::string &m)
{
    g_rg_err = m;
    return s;
}

#define RHIP(expr)                                                                         \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return rfail(ATG_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

int freq_index(unsigned rate)
{
    static const unsigned rates[20] = {48000, 44100, 32000, 24000, 22050, 16000, 12000,
                                       11025, 8000,  18900, 37800, 56000, 64000, 88200,
                                       96000, 112000, 128000, 144000, 176400, 192000};
    for (int i = 0; i < 20; i++)
        if (rates[i] == rate)
            return i;
    return -1;
}

struct RgTrack {
    uint64_t off;    // first interleaved sample
    uint64_t frames;
    uint32_t ch, bps, fi, window;
    uint64_t chunk_base; // first read() chunk size in the chunk array, ~0: 4096s
    // the certification bound of the track's coefficient set and segment
    // length (rg_bound, k_rg_bin): ginv < 0: no bound, warm segments never
    // certify
    double gmax, gl, gs, ginv;  // G, G_L, max_n ||A^n||_inf, 1 / (1 - ||A^L||)
    double py, pb, qy, qb;      // rounding sums per unit rho into output / state
    double sa, sb, ke, ko, rsf; // coefficient magnitudes; R_s at full scale
};

struct Chan {
    double in[10], yo[10], bo0, bo1; // newest first
};

// filterYule then filterButter for one sample (replaygain.c:566-610), the
// reference's left-to-right sums in its operation order, on a ring history:
// step R of a 10-sample cycle finds the newest input / output at slot
// (10 - R) % 10 and writes the new ones one slot down, so an unrolled cycle
// of 10 samples moves no registers (shifting the history costs ~30
// v_mov_b64 per sample in a loop).  At a cycle boundary the ring is in
// newest-first order.
template <int R>
__device__ __forceinline__ double filt_r(Chan &s, double x, const double *ky, const double *kb,
                                         double &ym, double &bm)
{
    constexpr int h = (10 - R % 10) % 10; // slot of the newest sample
    double y = 1e-10 + x * ky[0];
#pragma unroll
    for (int k = 1; k <= 10; ++k) {
        y = y - s.yo[(h + k - 1) % 10] * ky[2 * k - 1];
        y = y + s.in[(h + k - 1) % 10] * ky[2 * k];
    }
    const double b = y * kb[0] - s.bo0 * kb[1] + s.yo[h] * kb[2] - s.bo1 * kb[3] +
                     s.yo[(h + 1) % 10] * kb[4];
    constexpr int nh = (h + 9) % 10;
    s.in[nh] = x;
    s.yo[nh] = y;
    s.bo1 = s.bo0;
    s.bo0 = b;
    // the magnitudes the certification's rounding bound needs (k_rg_bin)
    ym = fmax(ym, fabs(y));
    bm = fmax(bm, fabs(b));
    return b;
}

// Time-split title analysis.  The Yule + Butterworth pair is a serial
// recurrence per (track, channel), and config 2's 1024 stereo tracks are
// only 2048 chains: a lane per chain leaves 97 % of the GPU idle and the
// step is one chain's latency (65 ms).  Here a track is cut into segments
// of whole 50 ms windows; a lane runs one segment of both channels (two
// independent chains interleaved), starting kRgWarm frames early from zero
// filter state with the exact input history.  The segment's sums and
// windows are then those of the serial computation up to the filter's
// rounding noise: two fp64 trajectories of this ill-conditioned Yule filter
// converge to within ~1e-10 of each other after ~2 k samples and never
// coalesce bit for bit (tools/rg_converge.c, profiles/r04_rg_converge.txt),
// so exactness is certified instead of assumed, with a bound derived from
// the filter (rg_bound, host):
//   * the error state (the 10 Yule and 2 Butterworth outputs; the input
//     history is exact in both) of a warm trajectory against the serial one
//     evolves as D' = A D + r, A the pair's companion matrix, r the two
//     trajectories' rounding differences per sample (|r| <= 2 gamma_k x the
//     magnitudes the sums add, gamma_k = k eps / (1 - k eps), magnitudes
//     from the filters' impulse-response l1 norms x 2^15);
//   * at every seam k_rg_seam measures the warm segment's state against the
//     previous segment's final state (m = the largest over the track).  The
//     previous segment's own error there is A^L D_prev (its start error D_prev
//     after its L counted frames) plus its accumulated rounding sum_k A^k E r;
//     so a counted output n frames into the warm segment errs by at most
//       |C A^n (measured)| + |C A^(n+L) D_prev| + |sum_k C A^(n+k) E r|
//       + its own rounding  <=  G m + G_L D_prev + 1.5 R_b
//     -- the rounding terms count three trajectories, each once: rho (and
//     so R_b = sum_n |C A^n E| rho) is two trajectories' worth, i.e. one
//     trajectory's rounding over ANY set of distinct sample times
//     propagates to the output with at most R_b / 2.  The predecessor's
//     rounding (before the seam) and the warm segment's own (after it)
//     give R_b / 2 each, and the serial trajectory's rounding enters both
//     terms but at disjoint times (before and after the seam), so R_b / 2
//     in all: 1.5 R_b (kRgRbFactor)
//     with G = max_n ||C A^n||_1, G_L = max_{n >= L} ||C A^n||_1, R_b =
//     sum_n |C A^n E| rho (C picks the Butterworth output, E the rounding
//     injection), and D_prev <= (m + R_s) / (1 - ||A^L||_inf) over the track
//     (R_s = sum_n ||A^n E||_inf rho; the first segment is the serial
//     trajectory itself, D = 0);
//   * a window's sum of squares then errs by 2 sqrt(2 n sum) delta +
//     2 n delta^2 + its own summation's rounding; a window of a warm segment
//     whose interval reaches another bin (k_rg_bin) flags the track, and
//     flagged tracks are analysed again as single exact segments from their
//     first frame (the serial computation).
// No constant in the bound is fitted: G, G_L, R_s, R_b, ||A^L|| are computed
// per coefficient set and segment length (rg_bound_compute; 44.1 kHz: G =
// 162, R_b = 1.65e-6, G_L ~ 1e-50).
// Segments that start at frame 0 are exact by construction.
constexpr uint32_t kRgWarm44 = 4096;    // warm-up frames at 44.1 kHz (scaled by rate)
constexpr uint32_t kRgSegWindows = 4;   // windows per segment (rounded to 10-frame cycles)
// Window values within this of a bin edge are binned again on the host with
// the C library's log10 (the reference's): the device log10 is accurate to
// a few ulp, ~1e-12 at values below 12000, not correctly rounded.
constexpr double kRgLogGuard = 1e-9;
// the multiple of R_b in the certification bound (G m + G_L D_prev + 1.5
// R_b above; atg_replaygain_rb_factor reports it)
constexpr double kRgRbFactor = 1.5;

struct RgSeg {
    uint64_t fw, f0, f1; // warm-up start, first counted frame, end (track frames)
    uint64_t ci, c0;     // read holding f0 (chunk index or f0 / 4096) and its first frame
    uint64_t w0;         // first window of the segment (track-relative)
    uint32_t track;
    uint32_t exact;      // fw == 0: the serial trajectory itself
};

__device__ __forceinline__ void save_state(double *d, const Chan &s)
{
#pragma unroll
    for (int k = 0; k < 10; ++k)
        d[k] = s.yo[k];
    d[10] = s.bo0;
    d[11] = s.bo1;
}

// lane per segment; CH = 1 or 2 (a mono track's window sums are used for
// both channels, as the reference duplicates the channel)
template <int CH>
__global__ __launch_bounds__(64) void k_rg_seg(const int32_t *__restrict__ pcm,
                                               const RgTrack *__restrict__ tracks,
                                               const RgSeg *__restrict__ segs, uint32_t nseg,
                                               const uint64_t *__restrict__ win_base,
                                               const uint32_t *__restrict__ chunks,
                                               double *__restrict__ wsum,
                                               uint32_t *__restrict__ amax_out,
                                               unsigned long long *__restrict__ mag_out,
                                               double *__restrict__ seam_in,
                                               double *__restrict__ seam_out)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nseg)
        return;
    const RgSeg S = segs[g];
    const RgTrack T = tracks[S.track];
    const int32_t *__restrict__ src = pcm + T.off;
    double ky[21], kb[5];
    {
        const double *gy = c_yule[T.fi], *gb = c_butter[T.fi];
#pragma unroll
        for (int i = 0; i < 21; ++i) {
            ky[i] = gy[i];
            asm volatile("" : "+v"(ky[i]));
        }
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            kb[i] = gb[i];
            asm volatile("" : "+v"(kb[i]));
        }
    }
    const int xsl = T.bps == 8 ? 8 : 0, xsr = T.bps == 24 ? 8 : 0;
    const uint64_t frames = T.frames;
    // zero filter state, exact input history (newest first: the ring's
    // canonical order at a cycle boundary)
    Chan A = {}, B = {};
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const int64_t f = (int64_t)S.fw - 1 - k;
        if (f >= 0) {
            A.in[k] = (double)((src[f * CH] << xsl) >> xsr);
            if (CH == 2)
                B.in[k] = (double)((src[f * CH + 1] << xsl) >> xsr);
        }
    }
    double *W = wsum + 2 * (win_base[S.track] + S.w0);
    const long window = (long)T.window;
    double sumA = 0, gsA = 0, sumB = 0, gsB = 0;
    uint32_t amax = 0;
    double ymax = 0, bmax = 0;
    // read() / batch / window bookkeeping from f0 on (replaygain.c:210-305):
    // f0 is a window boundary inside read ci, which began at frame c0
    uint64_t ci = S.ci, c0 = S.c0;
    auto read_size = [&](uint64_t c, uint64_t start) -> long {
        if (start >= frames)
            return 0;
        return T.chunk_base != ~0ull ? (long)chunks[T.chunk_base + c]
                                     : (long)(frames - start < 4096 ? frames - start : 4096);
    };
    long n4 = read_size(ci, c0), pos = (long)(S.f0 - c0), batch = n4 - pos, totsamp = 0, nwin = 0;
    int32_t k = 0, cur = 0, singles = 0;
    auto start_batch = [&]() {
        long c = batch > window - totsamp ? window - totsamp : batch;
        if (pos < 10 && c > 10 - pos)
            c = 10 - pos;
        cur = (int32_t)c;
        singles = cur % 16;
        k = 0;
    };
    if (batch > 0)
        start_batch();
    const uint64_t len = S.f1 - S.fw, i0 = S.f0 - S.fw; // i0 % 10 == 0
    for (uint64_t i = 0; i < len; i += 10) {
        if (i == i0) {
            save_state(seam_in + (uint64_t)g * 24, A);
            save_state(seam_in + (uint64_t)g * 24 + 12, B);
        }
        int32_t va[10], vb[10];
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            const uint64_t f = S.fw + i + (uint32_t)r;
            const bool in = f < frames;
            va[r] = in ? src[f * CH] : 0;
            vb[r] = (CH == 2 && in) ? src[f * CH + 1] : 0;
        }
        double oa[10], ob[10];
#define RG_STEP(R)                                                                 \
        oa[R] = filt_r<R>(A, (double)((va[R] << xsl) >> xsr), ky, kb, ymax, bmax); \
        if (CH == 2)                                                               \
            ob[R] = filt_r<R>(B, (double)((vb[R] << xsl) >> xsr), ky, kb, ymax, bmax);
        RG_STEP(0) RG_STEP(1) RG_STEP(2) RG_STEP(3) RG_STEP(4)
        RG_STEP(5) RG_STEP(6) RG_STEP(7) RG_STEP(8) RG_STEP(9)
#undef RG_STEP
        if (i + 10 <= i0)
            continue; // warm-up: filter only
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            const uint64_t ii = i + (uint32_t)r;
            if (ii < i0 || ii >= len || batch <= 0)
                continue;
            const uint32_t ava = (uint32_t)(va[r] < 0 ? -(int64_t)va[r] : va[r]);
            const uint32_t avb = (uint32_t)(vb[r] < 0 ? -(int64_t)vb[r] : vb[r]);
            amax = ava > amax ? ava : amax;
            amax = avb > amax ? avb : amax;
            const double a2 = oa[r] * oa[r];
            const double b2 = CH == 2 ? ob[r] * ob[r] : 0.0;
            if (k < singles) {
                sumA += a2;
                sumB += b2;
            } else {
                const int32_t gi = (k - singles) & 15;
                gsA = gi == 0 ? a2 : gsA + a2;
                gsB = gi == 0 ? b2 : gsB + b2;
                if (gi == 15) {
                    sumA += gsA;
                    sumB += gsB;
                }
            }
            if (++k == cur) { // the batch ends
                batch -= cur;
                pos += cur;
                totsamp += cur;
                if (totsamp == window) {
                    W[2 * nwin] = sumA;
                    W[2 * nwin + 1] = CH == 2 ? sumB : sumA;
                    ++nwin;
                    sumA = 0.;
                    sumB = 0.;
                    totsamp = 0;
                }
                if (batch == 0) { // the next read() result
                    c0 += (uint64_t)n4;
                    ++ci;
                    n4 = read_size(ci, c0);
                    batch = n4;
                    pos = 0;
                }
                if (batch > 0)
                    start_batch();
            }
        }
    }
    if (len % 10 == 0) { // a seam: the state the next segment must start from
        save_state(seam_out + (uint64_t)g * 24, A);
        save_state(seam_out + (uint64_t)g * 24 + 12, B);
    }
    atomicMax(amax_out + S.track, amax);
    // non-negative doubles order as their bit patterns
    atomicMax(mag_out + 2 * S.track, (unsigned long long)__double_as_longlong(ymax));
    atomicMax(mag_out + 2 * S.track + 1, (unsigned long long)__double_as_longlong(bmax));
}

// seam check: segment g (a warm start) against segment g - 1 of the same
// track; the largest state difference of a track's seams, as the positive
// double's bit pattern, into dmax[track]
__global__ __launch_bounds__(256) void k_rg_seam(const RgSeg *__restrict__ segs, uint32_t nseg,
                                                 const double *__restrict__ seam_in,
                                                 const double *__restrict__ seam_out,
                                                 unsigned long long *__restrict__ dmax)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g == 0 || g >= nseg || segs[g].exact || segs[g - 1].track != segs[g].track)
        return;
    double d = 0;
    for (int k = 0; k < 24; ++k) {
        const double e = fabs(seam_in[(uint64_t)g * 24 + k] - seam_out[(uint64_t)(g - 1) * 24 + k]);
        d = (e > d || e != e) ? e : d; // NaN: not converged
    }
    if (d != d)
        d = 1e300;
    atomicMax(dmax + segs[g].track, (unsigned long long)__double_as_longlong(d));
}

// bin every closed window: (int)(1000 log10((lsum + rsum) / n * 0.5 + 1e-37))
// (replaygain.c:713-724), one thread per window; block row y = tlist[y] (or
// y).  Certification (see k_rg_seg): a window from a warm segment (index >=
// warm_win[t]) whose value interval under the track's derived error bound
// reaches another bin flags the track (flag[t] = 1).  A window whose value
// lies within kRgLogGuard of a bin edge is listed in amb (track, window) for
// the host to bin with the reference's log10.  Peaks: max |x| / 2^(bps-1).
__global__ __launch_bounds__(256) void k_rg_bin(const RgTrack *__restrict__ tracks, uint32_t n,
                                                const uint32_t *__restrict__ tlist,
                                                const uint64_t *__restrict__ win_base,
                                                const double *__restrict__ wsum,
                                                const uint32_t *__restrict__ amax,
                                                const unsigned long long *__restrict__ mag,
                                                const uint32_t *__restrict__ warm_win,
                                                const unsigned long long *__restrict__ dmax,
                                                uint32_t *__restrict__ flag,
                                                uint32_t *__restrict__ hist,
                                                double *__restrict__ peaks,
                                                uint32_t *__restrict__ n_amb, uint64_t amb_cap,
                                                uint4 *__restrict__ amb)
{
    if (blockIdx.y >= n)
        return;
    const uint32_t t = tlist ? tlist[blockIdx.y] : blockIdx.y;
    const RgTrack T = tracks[t];
    const uint64_t nw = win_base[t + 1] - win_base[t];
    const double window = (double)T.window;
    const double dm = warm_win ? __longlong_as_double((long long)dmax[t]) : 0.0;
    // the rounding per sample from the track's own magnitudes: inputs |x| <=
    // X (16-bit scale), Yule outputs <= Y, Butterworth outputs <= B, as
    // measured on the warm trajectories plus the most they can differ from
    // the serial one (gs (dm + rsf)); rho_y / rho_b bound two trajectories'
    // rounding difference per sample in the Yule (21 products + 21 sums)
    // and Butterworth (5 + 4) sums
    const double eps = 1.1102230246251565e-16;
    const double g22 = 22.0 * eps / (1.0 - 22.0 * eps), g6 = 6.0 * eps / (1.0 - 6.0 * eps);
    const double am = (double)amax[t];
    const double X = T.bps == 8 ? am * 256.0 : (T.bps == 24 ? am / 256.0 + 1.0 : am);
    const double dmag = T.gs * (dm + 2.0 * T.rsf);
    const double Ym = mag ? __longlong_as_double((long long)mag[2 * t]) : 0.0;
    const double Bm = mag ? __longlong_as_double((long long)mag[2 * t + 1]) : 0.0;
    const double Y = Ym * (1.0 + 1e-12) + dmag, Bv = Bm * (1.0 + 1e-12) + dmag;
    const double rho_y = 2.0 * g22 * (1e-10 + X * T.sb + Y * T.sa);
    const double rho_b = 2.0 * g6 * (T.ke * Y + T.ko * Bv);
    const double Rb = T.py * rho_y + T.pb * rho_b, Rs = T.qy * rho_y + T.qb * rho_b;
    // the bound on a counted output sample's error in the warm segments
    // (the derivation above): measured seam difference, the predecessor's
    // decayed start error, and kRgRbFactor = 1.5 R_b of rounding (three
    // trajectories' worth, see the derivation)
    const double delta = T.gmax * dm + T.gl * (dm + Rs) * T.ginv + kRgRbFactor * Rb;
    const uint32_t ww = warm_win ? warm_win[t] : 0xFFFFFFFFu;
    bool unsure = warm_win && ww != 0xFFFFFFFFu && !(T.ginv > 0.0 && delta < 1e300);
    // rounding of the window's own sum of n squares (both trajectories)
    const double gsum = 2.0 * (window + 1.0) * eps / (1.0 - (window + 1.0) * eps);
    for (uint64_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += gridDim.x * blockDim.x) {
        const double *ws = wsum + 2 * (win_base[t] + w);
        const double sum = ws[0] + ws[1];
        const double arg = sum / window * 0.5 + 1.e-37;
        const double val = 100. * 10. * log10(arg);
        int ival = (int)val;
        ival = ival < 0 ? 0 : (ival >= kBins ? kBins - 1 : ival);
        atomicAdd(&hist[(uint64_t)t * kBins + ival], 1u);
        if (val > kRgLogGuard && val < (double)kBins + 1.0 &&
            (val - floor(val) < kRgLogGuard || ceil(val) - val < kRgLogGuard)) {
            const uint32_t k = atomicAdd(n_amb, 1u);
            if (k < amb_cap)
                amb[k] = make_uint4(t, (uint32_t)w, (uint32_t)(w >> 32), (uint32_t)ival);
        }
        if (w >= ww && !unsure) {
            // |d sum| <= 2 sqrt(2 sum n) delta + 2 n delta^2 over both
            // channels (Cauchy-Schwarz), plus both sums' rounding; the window
            // is certain when both ends of [sum - dsum, sum + dsum] fall in its
            // bin with kRgLogGuard to spare (log10 is monotone: the interval's
            // image is bounded by its ends' values; silence stays in bin 0)
            double dsum = 2.0 * sqrt(2.0 * sum * window) * delta + 2.0 * window * delta * delta;
            dsum += gsum * (sum + dsum);
            const double lo = sum - dsum > 0.0 ? sum - dsum : 0.0;
            const double hi = sum + dsum;
            const double vlo = 100. * 10. * log10(lo / window * 0.5 + 1.e-37) - kRgLogGuard;
            const double vhi = 100. * 10. * log10(hi / window * 0.5 + 1.e-37) + kRgLogGuard;
            int blo = (int)vlo, bhi = (int)vhi;
            blo = blo < 0 ? 0 : (blo >= kBins ? kBins - 1 : blo);
            bhi = bhi < 0 ? 0 : (bhi >= kBins ? kBins - 1 : bhi);
            if (blo != ival || bhi != ival)
                unsure = true;
        }
    }
    if (unsure)
        atomicOr(flag + t, 1u);
    if (blockIdx.x == 0 && threadIdx.x == 0)
        peaks[t] = (double)amax[t] / (double)(1 << (T.bps - 1));
}

// album histogram = sum of its tracks' histograms (tracks [first, first+count))
__global__ __launch_bounds__(256) void k_rg_album(const uint32_t *__restrict__ hist,
                                                  const uint32_t *__restrict__ first,
                                                  const uint32_t *__restrict__ count,
                                                  uint32_t *__restrict__ album)
{
    const uint32_t a = blockIdx.y;
    for (uint32_t b = blockIdx.x * blockDim.x + threadIdx.x; b < kBins; b += gridDim.x * blockDim.x) {
        uint32_t s = 0;
        for (uint32_t t = first[a]; t < first[a] + count[a]; ++t)
            s += hist[(uint64_t)t * kBins + b];
        album[(uint64_t)a * kBins + b] = s;
    }
}

// analyzeResult (replaygain.c:754-776): NaN = not enough samples.  Block
// per histogram: 256 threads own contiguous bin chunks; the answer is the
// largest bin i whose suffix sum reaches upper = ceil(0.05 * total), which
// is exactly where the reference's top-down `upper -= A[i]` loop stops.
__global__ __launch_bounds__(256) void k_rg_gain(const uint32_t *__restrict__ hist, uint32_t n,
                                                 double *__restrict__ gain)
{
    __shared__ uint32_t csum[256];
    __shared__ uint32_t suffix[257];
    const uint32_t h = blockIdx.x, tid = threadIdx.x;
    if (h >= n)
        return;
    const uint32_t *A = hist + (uint64_t)h * kBins;
    const uint32_t per = (kBins + 255) / 256;
    const uint32_t lo = tid * per, hi = lo + per < (uint32_t)kBins ? lo + per : (uint32_t)kBins;
    uint32_t c = 0;
    for (uint32_t i = lo; i < hi; ++i)
        c += A[i];
    csum[tid] = c;
    __syncthreads();
    if (tid == 0) {
        suffix[256] = 0;
        for (int k = 255; k >= 0; --k)
            suffix[k] = suffix[k + 1] + csum[k];
    }
    __syncthreads();
    const uint32_t elems = suffix[0];
    if (elems == 0) {
        if (tid == 0)
            gain[h] = NAN;
        return;
    }
    const int64_t upper = (int32_t)ceil(elems * (1. - 0.95));
    // the chunk where the suffix first reaches upper, scanning downward
    if ((int64_t)suffix[tid] >= upper && (int64_t)suffix[tid + 1] < upper) {
        int64_t run = suffix[tid + 1];
        int i = (int)hi - 1;
        for (; i >= (int)lo; --i) {
            run += A[i];
            if (run >= upper)
                break;
        }
        gain[h] = 64.82 - (double)i / 100.;
    }
}

// a device buffer that grows on demand
struct RBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes)
    {
        if (p && bytes <= cap)
            return hipSuccess;
        (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const size_t want = std::max<size_t>(bytes, 256);
        const hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess)
            cap = want;
        return e;
    }
};

// device buffers of one device (kept across calls; a batch pipeline calls
// this once per album batch)
struct RgCtx {
    std::mutex mu;
    bool coeffs = false;
    RBuf tracks, hist, peaks, gains, alb, meta, wsum, wbase, chunks, segs, seam_in, seam_out,
        amax, dmax, warm, flag, tlist, amb, namb, mag;
};
constexpr int kMaxDevices = 64;
RgCtx g_ctxs[kMaxDevices];

// test hook (atg_replaygain_set_warmup): warm-up frames of every warm
// segment, -1 = the rate-scaled default; 0 starts each segment from zero
// state at its first counted frame, so every seam fails and every track
// takes the exact fallback
int g_rg_warm_override = -1;
// tracks the last call analysed again serially (atg_replaygain_fallback_tracks)
uint32_t g_rg_fallback_tracks = 0;
// windows whose bin the host log10 moved (lifetime count, for tests)
uint64_t g_rg_rebinned = 0;

// ---- the certification bound (see k_rg_seg) -------------------------------
// 12-state error dynamics of the Yule + Butterworth pair for coefficient set
// fi: state (y_n .. y_n-9, b_n, b_n-1); the input history is exact in both
// trajectories, so it drops out of the difference
struct RgBound {
    double gmax, gl, gs, ginv;  // G, G_L, max_n ||A^n||_inf, 1 / (1 - ||A^L||_inf)
    double py, pb, qy, qb;      // sum_n |C A^n E_y|, |C A^n E_b|, ||A^n E_y||, ||A^n E_b||
    double sa, sb, ke, ko;      // Yule feedback / feed-forward and Butterworth magnitudes
    double rsf, rbf;            // R_s and R_b at full scale (documentation, margins)
};

struct Mat12 {
    double m[12][12];
};

Mat12 rg_error_matrix(int fi)
{
    const double *ky = RG_YULE[fi], *kb = RG_BUTTER[fi];
    Mat12 A = {};
    for (int k = 1; k <= 10; ++k)
        A.m[0][k - 1] = -ky[2 * k - 1];
    for (int i = 1; i < 10; ++i)
        A.m[i][i - 1] = 1.0;
    // b_{n+1} = kb0 y_{n+1} + kb2 y_n + kb4 y_{n-1} - kb1 b_n - kb3 b_{n-1}
    for (int j = 0; j < 10; ++j)
        A.m[10][j] = kb[0] * A.m[0][j];
    A.m[10][0] += kb[2];
    A.m[10][1] += kb[4];
    A.m[10][10] = -kb[1];
    A.m[10][11] = -kb[3];
    A.m[11][10] = 1.0;
    return A;
}

Mat12 mul(const Mat12 &a, const Mat12 &b)
{
    Mat12 c = {};
    for (int i = 0; i < 12; ++i)
        for (int k = 0; k < 12; ++k)
            if (a.m[i][k] != 0.0)
                for (int j = 0; j < 12; ++j)
                    c.m[i][j] += a.m[i][k] * b.m[k][j];
    return c;
}

double norm_inf(const Mat12 &a) // max row sum
{
    double r = 0;
    for (int i = 0; i < 12; ++i) {
        double s = 0;
        for (int j = 0; j < 12; ++j)
            s += std::fabs(a.m[i][j]);
        r = std::max(r, s);
    }
    return r;
}

Mat12 mpow(Mat12 a, uint64_t e)
{
    Mat12 r = {};
    for (int i = 0; i < 12; ++i)
        r.m[i][i] = 1.0;
    while (e) {
        if (e & 1)
            r = mul(r, a);
        a = mul(a, a);
        e >>= 1;
    }
    return r;
}

// The certification constants of coefficient set fi and segment length L
// (k_rg_seg's derivation).  Sums over all lags are computed term by term
// until the terms are negligible and the rest is bounded with ||A^M||_inf
// = q < 1: sum_{n >= N} f(n) <= sum_{r < M} f(N + r) / (1 - q) for any f
// with f(n + M) <= q f(n).  ok = false when no such M exists (no bound).
RgBound rg_bound_compute(int fi, uint64_t L)
{
    const double *ky = RG_YULE[fi], *kb = RG_BUTTER[fi];
    const Mat12 A = rg_error_matrix(fi);
    RgBound b = {};
    b.ginv = -1.0;
    // M with q = ||A^M||_inf <= 1/2
    uint64_t M = 1;
    Mat12 P = A;
    while (norm_inf(P) > 0.5 && M < (1ull << 24)) {
        P = mul(P, P);
        M *= 2;
    }
    const double q = norm_inf(P);
    if (!(q < 1.0))
        return b;
    const double tailf = 1.0 / (1.0 - q);
    // sum_k ||A^k||_inf, for the impulse-response tails
    double sA = 0;
    {
        Mat12 Q = {};
        for (int i = 0; i < 12; ++i)
            Q.m[i][i] = 1.0;
        for (uint64_t k = 0; k < M; ++k) {
            sA += norm_inf(Q);
            Q = mul(Q, A);
        }
        sA *= tailf;
    }
    // input magnitudes: |x| <= 2^15 after the reference's conversion to
    // 16-bit scale; |y|, |b| <= the impulse responses' l1 norms x 2^15
    const double X = 32768.0;
    double hy = 0, hb = 0;
    {
        double xh[10] = {0}, yh[10] = {0}, bh[2] = {0};
        const uint64_t N = 40 * M + 64;
        for (uint64_t n = 0; n < N; ++n) {
            const double x = n == 0 ? 1.0 : 0.0;
            double y = ky[0] * x;
            for (int k = 1; k <= 10; ++k)
                y += -ky[2 * k - 1] * yh[k - 1] + ky[2 * k] * xh[k - 1];
            const double bo = kb[0] * y - kb[1] * bh[0] + kb[2] * yh[0] - kb[3] * bh[1] +
                              kb[4] * yh[1];
            for (int k = 9; k > 0; --k) {
                xh[k] = xh[k - 1];
                yh[k] = yh[k - 1];
            }
            xh[0] = x;
            yh[0] = y;
            bh[1] = bh[0];
            bh[0] = bo;
            hy += std::fabs(y);
            hb += std::fabs(bo);
        }
        // the rest: the state (no more input) decays under A
        double st = 0;
        for (int k = 0; k < 10; ++k)
            st = std::max(st, std::fabs(yh[k]));
        st = std::max(st, std::max(std::fabs(bh[0]), std::fabs(bh[1])));
        hy += st * sA;
        hb += st * sA;
    }
    const double Y = 1.01 * (hy * X) + 1e-6, B = 1.01 * (hb * X) + 1e-6;
    const double eps = std::ldexp(1.0, -53);
    auto gam = [&](double k) { return k * eps / (1.0 - k * eps); };
    double sa = 0, sb = std::fabs(ky[0]);
    for (int k = 1; k <= 10; ++k) {
        sa += std::fabs(ky[2 * k - 1]);
        sb += std::fabs(ky[2 * k]);
    }
    // two trajectories' rounding differences per sample at full scale: the
    // Yule sum (21 products + 21 additions) and the Butterworth sum (5 + 4)
    const double ke = std::fabs(kb[0]) + std::fabs(kb[2]) + std::fabs(kb[4]);
    const double ko = std::fabs(kb[1]) + std::fabs(kb[3]);
    const double rho_y = 2.0 * gam(22) * (1e-10 + X * sb + Y * sa);
    const double rho_b = 2.0 * gam(6) * (ke * Y + ko * B);
    // injections: r_y enters y_{n+1} and, through kb0, b_{n+1}; r_b enters b_{n+1}
    double Ey[12] = {0}, Eb[12] = {0};
    Ey[0] = 1.0;
    Ey[10] = kb[0];
    Eb[10] = 1.0;
    // G(n) = ||C A^n||_1 (C picks b_n), p = sum_n |C A^n E|, q = sum_n
    // ||A^n E||_inf, s = max_n ||A^n||_inf (attained below M: ||A^(n+M)|| <=
    // q ||A^n||), G_L = max over n >= L
    double v[12] = {0}, uy[12], ub[12];
    v[10] = 1.0;
    std::copy(Ey, Ey + 12, uy);
    std::copy(Eb, Eb + 12, ub);
    double gmax = 0, gl = 0, py = 0, pb = 0, qy = 0, qb = 0;
    const uint64_t N = 40 * M + 64; // q^40: the terms beyond are ~1e-12 of the first
    double g_tail = 0, qy_tail = 0, qb_tail = 0;
    for (uint64_t n = 0; n < N + M; ++n) {
        double g = 0, cy = 0, cb = 0, my = 0, mb = 0;
        for (int j = 0; j < 12; ++j) {
            g += std::fabs(v[j]);
            cy += v[j] * Ey[j];
            cb += v[j] * Eb[j];
            my = std::max(my, std::fabs(uy[j]));
            mb = std::max(mb, std::fabs(ub[j]));
        }
        if (n < N) {
            gmax = std::max(gmax, g);
            if (n >= L)
                gl = std::max(gl, g);
            py += std::fabs(cy);
            pb += std::fabs(cb);
            qy += my;
            qb += mb;
        } else {
            g_tail += g;
            qy_tail += my;
            qb_tail += mb;
        }
        double nv[12] = {0}, ny[12] = {0}, nb[12] = {0};
        for (int i = 0; i < 12; ++i)
            for (int j = 0; j < 12; ++j) {
                nv[j] += v[i] * A.m[i][j];
                ny[i] += A.m[i][j] * uy[j];
                nb[i] += A.m[i][j] * ub[j];
            }
        std::copy(nv, nv + 12, v);
        std::copy(ny, ny + 12, uy);
        std::copy(nb, nb + 12, ub);
    }
    // beyond N: G(n + M) <= q G(n) and ||A^(n+M) E|| <= q ||A^n E||, so the
    // sums from N on are at most tailf x the M terms after N; |C A^n E| <=
    // G(n) ||E||_inf bounds the output sums' rest
    gmax = std::max(gmax, g_tail);
    gl = std::max(gl, g_tail);
    py += g_tail * tailf * std::max(1.0, std::fabs(kb[0]));
    pb += g_tail * tailf;
    qy += qy_tail * tailf;
    qb += qb_tail * tailf;
    double gs = 0;
    {
        Mat12 Q = {};
        for (int i = 0; i < 12; ++i)
            Q.m[i][i] = 1.0;
        for (uint64_t k = 0; k < M; ++k) {
            gs = std::max(gs, norm_inf(Q));
            Q = mul(Q, A);
        }
    }
    const double al = norm_inf(mpow(A, L));
    if (!(al < 1.0))
        return b;
    // 1 % for the rounding of this computation itself
    b.gmax = 1.01 * gmax;
    b.gl = 1.01 * gl;
    b.gs = 1.01 * gs;
    b.ginv = 1.0 / (1.0 - al);
    b.py = 1.01 * py;
    b.pb = 1.01 * pb;
    b.qy = 1.01 * qy;
    b.qb = 1.01 * qb;
    b.sa = sa;
    b.sb = sb;
    b.ke = ke;
    b.ko = ko;
    b.rsf = b.qy * rho_y + b.qb * rho_b;
    b.rbf = b.py * rho_y + b.pb * rho_b;
    return b;
}

// cached per (coefficient set, segment length)
RgBound rg_bound(int fi, uint64_t L)
{
    static std::mutex mu;
    static std::map<std::pair<int, uint64_t>, RgBound> cache;
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(fi, L);
    auto it = cache.find(key);
    if (it != cache.end())
        return it->second;
    const RgBound b = rg_bound_compute(fi, L);
    cache[key] = b;
    return b;
}

// the counted length of a track's (non-last) segments, as plan_segments cuts
// them: at least `windows` whole windows, a multiple of 10 frames
uint64_t rg_seg_len(uint32_t wsz, uint32_t windows = kRgSegWindows)
{
    uint32_t g10 = 10;
    for (uint32_t x = wsz % 10, y = 10; x;) { // gcd(wsz, 10)
        const uint32_t r = y % x;
        y = x;
        x = r;
        g10 = y;
    }
    uint32_t K = 10 / g10;
    while (K < windows)
        K += 10 / g10;
    return (uint64_t)K * wsz;
}

// Windows per segment for a batch.  A lane filters one segment (its warm-up
// plus its counted frames) as one serial chain, so a batch takes about
// max(segment length, lanes x segment length / P) chain steps, P ~ one wave
// per SIMD (65,536 lanes).  Few long tracks want short segments (more
// lanes), many want long ones (less warm-up): config 2's title analysis
// (1024 x 262,144 frames) measured 8.74 / 5.28 / 5.20 ms at 4 / 2 / 1
// windows, config 4's album scan (1024 x 441,000) 7.37 / 9.78 / 9.73
// (profiles/r05_zz_rg_segments.txt).  Batches of fewer than 8192 lanes at
// the default keep it.
uint32_t rg_seg_windows(const std::vector<RgTrack> &tr, const atg_rg_track *a, uint32_t n)
{
    constexpr double kLanes = 65536.0;
    auto cost = [&](uint32_t K, double &lanes) {
        lanes = 0.0;
        double seg = 0.0;
        for (uint32_t t = 0; t < n; ++t) {
            const uint64_t L = rg_seg_len(tr[t].window, K);
            const uint64_t warm = ((uint64_t)kRgWarm44 * a[t].sample_rate / 44100 + 9) / 10 * 10;
            lanes += (double)((tr[t].frames + L - 1) / L);
            seg = std::max(seg, (double)(L + warm));
        }
        return std::max(seg, lanes * seg / kLanes);
    };
    double lanes4 = 0.0;
    const double c4 = cost(kRgSegWindows, lanes4);
    if (lanes4 < 8192.0 || g_rg_warm_override >= 0)
        return kRgSegWindows;
    uint32_t best = kRgSegWindows;
    double bc = c4, l = 0.0;
    for (uint32_t K : {2u, 1u}) {
        const double c = cost(K, l);
        if (c < bc) {
            bc = c;
            best = K;
        }
    }
    return best;
}

// the segments of track t (appended to `out`): whole windows, a multiple
// of 10 frames long (the filter's ring cycle), warm-up a multiple of 10
void plan_segments(uint32_t t, const RgTrack &T, const atg_rg_track &a, bool exact_only,
                   std::vector<RgSeg> &out, uint32_t &first_warm_window, uint32_t windows)
{
    const uint32_t wsz = T.window;
    const uint64_t L = exact_only ? T.frames + 10 : rg_seg_len(wsz, windows);
    uint64_t warm = (uint64_t)kRgWarm44 * a.sample_rate / 44100;
    warm = (warm + 9) / 10 * 10;
    if (g_rg_warm_override >= 0)
        warm = (uint64_t)g_rg_warm_override / 10 * 10;
    first_warm_window = 0xFFFFFFFFu;
    // read starts for the chunked form (f0 -> read index)
    std::vector<uint64_t> rs;
    if (a.chunk_frames) {
        rs.resize(a.n_chunks + 1, 0);
        for (uint64_t i = 0; i < a.n_chunks; ++i)
            rs[i + 1] = rs[i] + a.chunk_frames[i];
    }
    uint64_t f0 = 0;
    do {
        RgSeg g;
        g.track = t;
        g.f0 = f0;
        g.f1 = std::min<uint64_t>(f0 + L, T.frames);
        g.fw = f0 > warm ? f0 - warm : 0u;
        g.exact = g.fw == 0 && (f0 == 0 || f0 <= warm) ? 1u : 0u;
        if (g_rg_warm_override == 0 && f0)
            g.exact = 0;
        if (a.chunk_frames) {
            const uint64_t ci = (uint64_t)(std::upper_bound(rs.begin(), rs.end(), f0) -
                                           rs.begin()) - 1;
            g.ci = ci;
            g.c0 = rs[ci];
        } else {
            g.ci = f0 / 4096;
            g.c0 = g.ci * 4096u;
        }
        g.w0 = f0 / wsz;
        if (!g.exact && first_warm_window == 0xFFFFFFFFu)
            first_warm_window = g.w0 < 0xFFFFFFFFull ? (uint32_t)g.w0 : 0u;
        out.push_back(g);
        f0 += L;
    } while (f0 < T.frames);
}

// the (track, window, device bin) entries k_rg_bin listed (synchronises s)
atg_status fetch_ambiguous(RgCtx &c, hipStream_t s, uint64_t cap, std::vector<uint4> &out)
{
    uint32_t cnt = 0;
    RHIP(hipMemcpyAsync(&cnt, c.namb.p, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    RHIP(hipStreamSynchronize(s));
    if (cnt > cap)
        return rfail(ATG_ERR_DEVICE, "ambiguous-window list overflow");
    out.resize(cnt);
    if (cnt) {
        RHIP(hipMemcpyAsync(out.data(), c.amb.p, sizeof(uint4) * cnt, hipMemcpyDeviceToHost, s));
        RHIP(hipStreamSynchronize(s));
    }
    return ATG_OK;
}

// bin the listed windows with the host C library's log10 (the reference's,
// replaygain.c:713-724) and move their histogram counts where it says
atg_status rebin_ambiguous(RgCtx &c, hipStream_t s, const std::vector<RgTrack> &tr,
                           const std::vector<uint64_t> &wbase, const std::vector<uint4> &amb)
{
    for (const uint4 &e : amb) {
        const uint32_t t = e.x;
        const uint64_t w = (uint64_t)e.y | ((uint64_t)e.z << 32);
        double ws[2];
        RHIP(hipMemcpyAsync(ws, (const double *)c.wsum.p + 2 * (wbase[t] + w), sizeof(ws),
                            hipMemcpyDeviceToHost, s));
        RHIP(hipStreamSynchronize(s));
        const double sum = ws[0] + ws[1];
        const double val = 100. * 10. * std::log10(sum / (double)tr[t].window * 0.5 + 1.e-37);
        int ival = (int)val;
        ival = ival < 0 ? 0 : (ival >= kBins ? kBins - 1 : ival);
        if ((uint32_t)ival == e.w)
            continue;
        uint32_t *h = (uint32_t *)c.hist.p + (uint64_t)t * kBins;
        uint32_t a = 0, b = 0;
        RHIP(hipMemcpyAsync(&a, h + e.w, 4, hipMemcpyDeviceToHost, s));
        RHIP(hipMemcpyAsync(&b, h + ival, 4, hipMemcpyDeviceToHost, s));
        RHIP(hipStreamSynchronize(s));
        --a;
        ++b;
        RHIP(hipMemcpyAsync(h + e.w, &a, 4, hipMemcpyHostToDevice, s));
        RHIP(hipMemcpyAsync(h + ival, &b, 4, hipMemcpyHostToDevice, s));
        RHIP(hipStreamSynchronize(s));
        ++g_rg_rebinned;
    }
    return ATG_OK;
}

} // namespace

extern "C" {

void atg_replaygain_set_warmup(int frames) { g_rg_warm_override = frames; }

uint32_t atg_replaygain_fallback_tracks(void) { return g_rg_fallback_tracks; }

double atg_replaygain_rb_factor(void) { return kRgRbFactor; }

uint64_t atg_replaygain_rebinned_windows(void) { return g_rg_rebinned; }

atg_status atg_replaygain_bound(uint32_t sample_rate, double *out)
{
    const int fi = freq_index(sample_rate);
    if (fi < 0 || !out)
        return rfail(ATG_ERR_INVALID, "unsupported sample rate");
    const uint64_t L = rg_seg_len((uint32_t)std::ceil(sample_rate * 0.050));
    const RgBound b = rg_bound(fi, L);
    out[0] = b.gmax;
    out[1] = b.rsf;
    out[2] = b.rbf;
    out[3] = b.ginv;
    out[4] = (double)L;
    out[5] = b.gl;
    return ATG_OK;
}


const char *atg_replaygain_last_error(void) { return g_rg_err.c_str(); }

atg_status atg_replaygain_device(const int32_t *d_pcm, const atg_rg_track *tracks, uint32_t n,
                                 uint32_t n_albums, atg_rg_result *results,
                                 uint32_t *d_album_hist, double *album_peaks, void *stream)
{
    if ((!tracks || !results) && n)
        return rfail(ATG_ERR_INVALID, "NULL argument");
    hipStream_t s = (hipStream_t)stream;
    int dev = 0;
    RHIP(hipGetDevice(&dev));
    if (dev < 0 || dev >= kMaxDevices)
        return rfail(ATG_ERR_UNSUPPORTED, "device index too large");
    RgCtx &g_ctx = g_ctxs[dev];
    std::lock_guard<std::mutex> lock(g_ctx.mu);
    if (!g_ctx.coeffs) {
        RHIP(hipMemcpyToSymbol(HIP_SYMBOL(c_yule), RG_YULE, sizeof(RG_YULE)));
        RHIP(hipMemcpyToSymbol(HIP_SYMBOL(c_butter), RG_BUTTER, sizeof(RG_BUTTER)));
        g_ctx.coeffs = true;
    }
    std::vector<RgTrack> tr(n);
    std::vector<uint32_t> chunks;
    std::vector<uint64_t> wbase(n + 1, 0);
    std::vector<uint32_t> first(n_albums, 0), count(n_albums, 0);
    for (uint32_t t = 0; t < n; ++t) {
        const atg_rg_track &a = tracks[t];
        const int fi = freq_index(a.sample_rate);
        if (fi < 0)
            return rfail(ATG_ERR_INVALID, "unsupported sample rate");
        if (a.channels != 1 && a.channels != 2)
            return rfail(ATG_ERR_INVALID, "FrameList must contain only 1 or 2 channels");
        if (a.bits_per_sample != 8 && a.bits_per_sample != 16 && a.bits_per_sample != 24)
            return rfail(ATG_ERR_INVALID, "unsupported bits per sample");
        if (n_albums && a.album >= n_albums)
            return rfail(ATG_ERR_INVALID, "album index out of range");
        if (n_albums && t && a.album < tracks[t - 1].album)
            return rfail(ATG_ERR_INVALID, "tracks must be grouped by album");
        uint64_t cbase = ~0ull;
        if (a.chunk_frames) {
            uint64_t tot = 0;
            for (uint64_t i = 0; i < a.n_chunks; ++i) {
                if (!a.chunk_frames[i])
                    return rfail(ATG_ERR_INVALID, "read() chunk sizes must be positive");
                tot += a.chunk_frames[i];
            }
            if (tot != a.pcm_frames)
                return rfail(ATG_ERR_INVALID, "read() chunk sizes must add up to pcm_frames");
            cbase = chunks.size();
            chunks.insert(chunks.end(), a.chunk_frames, a.chunk_frames + a.n_chunks);
        }
        const uint32_t wsz = (uint32_t)std::ceil(a.sample_rate * 0.050);
        tr[t] = RgTrack{a.pcm_offset * a.channels, a.pcm_frames, a.channels, a.bits_per_sample,
                        (uint32_t)fi, wsz, cbase, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
        wbase[t + 1] = wbase[t] + a.pcm_frames / tr[t].window;
        if (n_albums) {
            if (!count[a.album])
                first[a.album] = t;
            ++count[a.album];
        }
    }
    // the batch's segment length, then each track's certification bound for it
    const uint32_t seg_windows = rg_seg_windows(tr, tracks, n);
    for (uint32_t t = 0; t < n; ++t) {
        const RgBound bd = rg_bound((int)tr[t].fi, rg_seg_len(tr[t].window, seg_windows));
        RgTrack &T = tr[t];
        T.gmax = bd.gmax;
        T.gl = bd.gl;
        T.gs = bd.gs;
        T.ginv = bd.ginv;
        T.py = bd.py;
        T.pb = bd.pb;
        T.qy = bd.qy;
        T.qb = bd.qb;
        T.sa = bd.sa;
        T.sb = bd.sb;
        T.ke = bd.ke;
        T.ko = bd.ko;
        T.rsf = bd.rsf;
    }
    RHIP(g_ctx.tracks.ensure(sizeof(RgTrack) * std::max<uint32_t>(n, 1)));
    RHIP(g_ctx.hist.ensure(sizeof(uint32_t) * kBins * (size_t)std::max<uint32_t>(n, 1)));
    RHIP(g_ctx.peaks.ensure(sizeof(double) * std::max<uint32_t>(n, 1)));
    RHIP(g_ctx.gains.ensure(sizeof(double) * ((size_t)n + n_albums + 1)));
    RHIP(g_ctx.alb.ensure(sizeof(uint32_t) * kBins * (size_t)std::max<uint32_t>(n_albums, 1)));
    RHIP(g_ctx.meta.ensure(sizeof(uint32_t) * 2 * (size_t)std::max<uint32_t>(n_albums, 1)));
    if (!n) { // empty albums: peak 0.0 (replaygain.c:180), empty histograms
        if (album_peaks)
            for (uint32_t a = 0; a < n_albums; ++a)
                album_peaks[a] = 0.0;
        if (n_albums) {
            uint32_t *album = d_album_hist ? d_album_hist : (uint32_t *)g_ctx.alb.p;
            RHIP(hipMemsetAsync(album, 0, sizeof(uint32_t) * kBins * (size_t)n_albums, s));
            RHIP(hipStreamSynchronize(s));
        }
        return ATG_OK;
    }
    // segments: mono tracks' first, then stereo (one launch per channel count)
    std::vector<RgSeg> segs, segs2;
    std::vector<uint32_t> warm_win(n);
    for (uint32_t t = 0; t < n; ++t)
        plan_segments(t, tr[t], tracks[t], false, tr[t].ch == 1 ? segs : segs2, warm_win[t],
                      seg_windows);
    const uint32_t nseg1 = (uint32_t)segs.size();
    segs.insert(segs.end(), segs2.begin(), segs2.end());
    const uint32_t nseg = (uint32_t)segs.size();
    RHIP(g_ctx.chunks.ensure(sizeof(uint32_t) * std::max<size_t>(chunks.size(), 1)));
    if (!chunks.empty())
        RHIP(hipMemcpyAsync(g_ctx.chunks.p, chunks.data(), sizeof(uint32_t) * chunks.size(),
                            hipMemcpyHostToDevice, s));
    RHIP(g_ctx.wsum.ensure(sizeof(double) * 2 * (wbase[n] + 1)));
    RHIP(g_ctx.wbase.ensure(sizeof(uint64_t) * (n + 1)));
    RHIP(g_ctx.segs.ensure(sizeof(RgSeg) * nseg));
    RHIP(g_ctx.seam_in.ensure(sizeof(double) * 24 * (size_t)nseg));
    RHIP(g_ctx.seam_out.ensure(sizeof(double) * 24 * (size_t)nseg));
    RHIP(g_ctx.amax.ensure(sizeof(uint32_t) * n));
    RHIP(g_ctx.mag.ensure(sizeof(unsigned long long) * 2 * n));
    RHIP(g_ctx.dmax.ensure(sizeof(unsigned long long) * n));
    RHIP(g_ctx.warm.ensure(sizeof(uint32_t) * n));
    RHIP(g_ctx.flag.ensure(sizeof(uint32_t) * n));
    RHIP(g_ctx.tlist.ensure(sizeof(uint32_t) * n));
    const uint64_t amb_cap = wbase[n] + 1;
    RHIP(g_ctx.amb.ensure(sizeof(uint4) * amb_cap));
    RHIP(g_ctx.namb.ensure(sizeof(uint32_t)));
    RHIP(hipMemcpyAsync(g_ctx.tracks.p, tr.data(), sizeof(RgTrack) * n, hipMemcpyHostToDevice, s));
    RHIP(hipMemcpyAsync(g_ctx.wbase.p, wbase.data(), sizeof(uint64_t) * (n + 1),
                        hipMemcpyHostToDevice, s));
    RHIP(hipMemcpyAsync(g_ctx.segs.p, segs.data(), sizeof(RgSeg) * nseg, hipMemcpyHostToDevice, s));
    RHIP(hipMemcpyAsync(g_ctx.warm.p, warm_win.data(), sizeof(uint32_t) * n,
                        hipMemcpyHostToDevice, s));
    RHIP(hipMemsetAsync(g_ctx.hist.p, 0, sizeof(uint32_t) * kBins * (size_t)n, s));
    RHIP(hipMemsetAsync(g_ctx.amax.p, 0, sizeof(uint32_t) * n, s));
    RHIP(hipMemsetAsync(g_ctx.mag.p, 0, sizeof(unsigned long long) * 2 * n, s));
    RHIP(hipMemsetAsync(g_ctx.dmax.p, 0, sizeof(unsigned long long) * n, s));
    RHIP(hipMemsetAsync(g_ctx.flag.p, 0, sizeof(uint32_t) * n, s));
    RHIP(hipMemsetAsync(g_ctx.namb.p, 0, sizeof(uint32_t), s));
    const RgTrack *dtr = (const RgTrack *)g_ctx.tracks.p;
    const uint64_t *dwb = (const uint64_t *)g_ctx.wbase.p;
    const uint32_t *dch = (const uint32_t *)g_ctx.chunks.p;
    double *dws = (double *)g_ctx.wsum.p;
    auto run_segments = [&](const RgSeg *dseg, uint32_t n1, uint32_t ntot, double *sin,
                            double *sout) -> atg_status {
        if (n1)
            hipLaunchKernelGGL(k_rg_seg<1>, dim3((n1 + 63) / 64), dim3(64), 0, s, d_pcm, dtr,
                               dseg, n1, dwb, dch, dws, (uint32_t *)g_ctx.amax.p,
                               (unsigned long long *)g_ctx.mag.p, sin, sout);
        if (ntot > n1)
            hipLaunchKernelGGL(k_rg_seg<2>, dim3((ntot - n1 + 63) / 64), dim3(64), 0, s, d_pcm,
                               dtr, dseg + n1, ntot - n1, dwb, dch, dws, (uint32_t *)g_ctx.amax.p,
                               (unsigned long long *)g_ctx.mag.p,
                               sin + 24 * (size_t)n1, sout + 24 * (size_t)n1);
        RHIP(hipGetLastError());
        return ATG_OK;
    };
    atg_status st = run_segments((const RgSeg *)g_ctx.segs.p, nseg1, nseg,
                                 (double *)g_ctx.seam_in.p, (double *)g_ctx.seam_out.p);
    if (st != ATG_OK)
        return st;
    hipLaunchKernelGGL(k_rg_seam, dim3((nseg + 255) / 256), dim3(256), 0, s,
                       (const RgSeg *)g_ctx.segs.p, nseg, (const double *)g_ctx.seam_in.p,
                       (const double *)g_ctx.seam_out.p, (unsigned long long *)g_ctx.dmax.p);
    RHIP(hipGetLastError());
    hipLaunchKernelGGL(k_rg_bin, dim3(4, n), dim3(256), 0, s, dtr, n, (const uint32_t *)nullptr,
                       dwb, (const double *)dws, (const uint32_t *)g_ctx.amax.p,
                       (const unsigned long long *)g_ctx.mag.p,
                       (const uint32_t *)g_ctx.warm.p, (const unsigned long long *)g_ctx.dmax.p,
                       (uint32_t *)g_ctx.flag.p, (uint32_t *)g_ctx.hist.p,
                       (double *)g_ctx.peaks.p, (uint32_t *)g_ctx.namb.p, amb_cap,
                       (uint4 *)g_ctx.amb.p);
    RHIP(hipGetLastError());
    // the tracks certification could not vouch for: analysed again as one
    // exact segment each (the serial computation), then binned again
    std::vector<uint32_t> flags(n);
    RHIP(hipMemcpyAsync(flags.data(), g_ctx.flag.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost,
                        s));
    std::vector<uint4> amb;
    st = fetch_ambiguous(g_ctx, s, amb_cap, amb);
    if (st != ATG_OK)
        return st;
    std::vector<uint32_t> redo;
    for (uint32_t t = 0; t < n; ++t)
        if (flags[t])
            redo.push_back(t);
    // a redone track is binned again below: its first-pass entries go
    amb.erase(std::remove_if(amb.begin(), amb.end(), [&](const uint4 &e) { return flags[e.x] != 0; }),
              amb.end());
    g_rg_fallback_tracks = (uint32_t)redo.size();
    if (!redo.empty()) {
        std::vector<RgSeg> e1, e2;
        uint32_t unused = 0;
        for (uint32_t t : redo)
            plan_segments(t, tr[t], tracks[t], true, tr[t].ch == 1 ? e1 : e2, unused,
                          seg_windows);
        const uint32_t m1 = (uint32_t)e1.size();
        e1.insert(e1.end(), e2.begin(), e2.end());
        const uint32_t m = (uint32_t)e1.size();
        RHIP(hipMemcpyAsync(g_ctx.segs.p, e1.data(), sizeof(RgSeg) * m, hipMemcpyHostToDevice, s));
        RHIP(hipMemcpyAsync(g_ctx.tlist.p, redo.data(), sizeof(uint32_t) * redo.size(),
                            hipMemcpyHostToDevice, s));
        RHIP(hipMemsetAsync(g_ctx.namb.p, 0, sizeof(uint32_t), s));
        for (uint32_t t : redo)
            RHIP(hipMemsetAsync((uint32_t *)g_ctx.hist.p + (size_t)t * kBins, 0,
                                sizeof(uint32_t) * kBins, s));
        st = run_segments((const RgSeg *)g_ctx.segs.p, m1, m, (double *)g_ctx.seam_in.p,
                          (double *)g_ctx.seam_out.p);
        if (st != ATG_OK)
            return st;
        hipLaunchKernelGGL(k_rg_bin, dim3(4, (uint32_t)redo.size()), dim3(256), 0, s, dtr,
                           (uint32_t)redo.size(), (const uint32_t *)g_ctx.tlist.p, dwb,
                           (const double *)dws, (const uint32_t *)g_ctx.amax.p,
                           (const unsigned long long *)nullptr,
                           (const uint32_t *)nullptr, (const unsigned long long *)nullptr,
                           (uint32_t *)nullptr, (uint32_t *)g_ctx.hist.p,
                           (double *)g_ctx.peaks.p, (uint32_t *)g_ctx.namb.p, amb_cap,
                           (uint4 *)g_ctx.amb.p);
        RHIP(hipGetLastError());
        std::vector<uint4> amb2;
        st = fetch_ambiguous(g_ctx, s, amb_cap, amb2);
        if (st != ATG_OK)
            return st;
        amb.insert(amb.end(), amb2.begin(), amb2.end());
    }
    // windows next to a bin edge: binned with the reference's log10
    st = rebin_ambiguous(g_ctx, s, tr, wbase, amb);
    if (st != ATG_OK)
        return st;
    hipLaunchKernelGGL(k_rg_gain, dim3(n), dim3(256), 0, s, (const uint32_t *)g_ctx.hist.p, n,
                       (double *)g_ctx.gains.p);
    RHIP(hipGetLastError());
    uint32_t *album = d_album_hist ? d_album_hist : (uint32_t *)g_ctx.alb.p;
    if (n_albums) {
        RHIP(hipMemcpyAsync(g_ctx.meta.p, first.data(), sizeof(uint32_t) * n_albums,
                            hipMemcpyHostToDevice, s));
        RHIP(hipMemcpyAsync((uint32_t *)g_ctx.meta.p + n_albums, count.data(),
                            sizeof(uint32_t) * n_albums, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_rg_album, dim3((kBins + 255) / 256, n_albums), dim3(256), 0, s,
                           (const uint32_t *)g_ctx.hist.p, (const uint32_t *)g_ctx.meta.p,
                           (const uint32_t *)g_ctx.meta.p + n_albums, album);
        RHIP(hipGetLastError());
    }
    std::vector<double> gains(n), peaks(n);
    RHIP(hipMemcpyAsync(gains.data(), g_ctx.gains.p, sizeof(double) * n, hipMemcpyDeviceToHost,
                        s));
    RHIP(hipMemcpyAsync(peaks.data(), g_ctx.peaks.p, sizeof(double) * n, hipMemcpyDeviceToHost,
                        s));
    RHIP(hipStreamSynchronize(s));
    if (album_peaks)
        for (uint32_t a = 0; a < n_albums; ++a)
            album_peaks[a] = 0.0; // album_peak starts at 0.0 (replaygain.c:180)
    for (uint32_t t = 0; t < n; ++t) {
        // title_gain returns 0.0 when no window completed (replaygain.c:311-318)
        results[t].status = std::isnan(gains[t]) ? 1 : 0;
        results[t].title_gain = std::isnan(gains[t]) ? 0.0 : gains[t];
        results[t].title_peak = peaks[t];
        if (album_peaks && n_albums)
            album_peaks[tracks[t].album] = std::max(album_peaks[tracks[t].album], peaks[t]);
    }
    return ATG_OK;
}

atg_status atg_replaygain_hist_gain(const uint32_t *d_hist, uint32_t n, double *gains,
                                    void *stream)
{
    if (!n)
        return ATG_OK;
    hipStream_t s = (hipStream_t)stream;
    double *d_g = nullptr;
    RHIP(hipMalloc(&d_g, sizeof(double) * n));
    hipLaunchKernelGGL(k_rg_gain, dim3(n), dim3(256), 0, s, d_hist, n, d_g);
    hipError_t e = hipGetLastError();
    if (e == hipSuccess)
        e = hipMemcpyAsync(gains, d_g, sizeof(double) * n, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess)
        e = hipStreamSynchronize(s);
    (void)hipFree(d_g);
    if (e != hipSuccess)
        return rfail(ATG_ERR_DEVICE, hipGetErrorString(e));
    return ATG_OK;
}

} // extern "C"
