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
#include <mutex>
#include <string>
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
__device__ __forceinline__ double filt_r(Chan &s, double x, const double *ky, const double *kb)
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
// so exactness is certified instead of assumed:
//   * at every seam the warm segment's starting state is compared with the
//     previous segment's final state (k_rg_seam); a difference above
//     kRgConverge means the warm-up did not converge;
//   * a window of a warm segment whose bin value lies within the error that
//     difference allows of a bin edge (k_rg_bin) could bin differently;
// either flags the track, and flagged tracks are analysed again as single
// exact segments from their first frame (the serial computation).  Segments
// that start at frame 0 are exact by construction.
constexpr uint32_t kRgWarm44 = 4096;    // warm-up frames at 44.1 kHz (scaled by rate)
constexpr uint32_t kRgSegWindows = 4;   // windows per segment (rounded to 10-frame cycles)
constexpr double kRgConverge = 1e-4;    // largest seam state difference accepted

struct RgSeg {
    uint32_t track;
    uint32_t fw, f0, f1; // warm-up start, first counted frame, end (track frames)
    uint32_t ci, c0;     // read holding f0 (chunk index or f0 / 4096) and its first frame
    uint32_t w0;         // first window of the segment (track-relative)
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
    const uint32_t len = S.f1 - S.fw, i0 = S.f0 - S.fw; // i0 % 10 == 0
    for (uint32_t i = 0; i < len; i += 10) {
        if (i == i0) {
            save_state(seam_in + (uint64_t)g * 24, A);
            save_state(seam_in + (uint64_t)g * 24 + 12, B);
        }
        int32_t va[10], vb[10];
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            const uint64_t f = (uint64_t)S.fw + i + (uint32_t)r;
            const bool in = f < frames;
            va[r] = in ? src[f * CH] : 0;
            vb[r] = (CH == 2 && in) ? src[f * CH + 1] : 0;
        }
        double oa[10], ob[10];
#define RG_STEP(R)                                                                 \
        oa[R] = filt_r<R>(A, (double)((va[R] << xsl) >> xsr), ky, kb);            \
        if (CH == 2)                                                               \
            ob[R] = filt_r<R>(B, (double)((vb[R] << xsl) >> xsr), ky, kb);
        RG_STEP(0) RG_STEP(1) RG_STEP(2) RG_STEP(3) RG_STEP(4)
        RG_STEP(5) RG_STEP(6) RG_STEP(7) RG_STEP(8) RG_STEP(9)
#undef RG_STEP
        if (i + 10 <= i0)
            continue; // warm-up: filter only
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            const uint32_t ii = i + (uint32_t)r;
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
// warm_win[t]) whose value lies within the error the track's seam
// difference allows of a bin edge flags the track (flag[t] = 1), as does a
// seam difference above kRgConverge.  Peaks: max |x| / 2^(bps-1).
__global__ __launch_bounds__(256) void k_rg_bin(const RgTrack *__restrict__ tracks, uint32_t n,
                                                const uint32_t *__restrict__ tlist,
                                                const uint64_t *__restrict__ win_base,
                                                const double *__restrict__ wsum,
                                                const uint32_t *__restrict__ amax,
                                                const uint32_t *__restrict__ warm_win,
                                                const unsigned long long *__restrict__ dmax,
                                                uint32_t *__restrict__ flag,
                                                uint32_t *__restrict__ hist,
                                                double *__restrict__ peaks)
{
    if (blockIdx.y >= n)
        return;
    const uint32_t t = tlist ? tlist[blockIdx.y] : blockIdx.y;
    const uint64_t nw = win_base[t + 1] - win_base[t];
    const double window = (double)tracks[t].window;
    const double dm = warm_win ? __longlong_as_double((long long)dmax[t]) : 0.0;
    // per-sample output error allowed for the warm trajectory: 16x the seam
    // difference plus a floor well above the filter's rounding noise
    const double delta = 16.0 * dm + 1e-9;
    const uint32_t ww = warm_win ? warm_win[t] : 0xFFFFFFFFu;
    bool unsure = warm_win && dm > kRgConverge;
    for (uint64_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += gridDim.x * blockDim.x) {
        const double *ws = wsum + 2 * (win_base[t] + w);
        const double sum = ws[0] + ws[1];
        const double arg = sum / window * 0.5 + 1.e-37;
        const double val = 100. * 10. * log10(arg);
        int ival = (int)val;
        ival = ival < 0 ? 0 : (ival >= kBins ? kBins - 1 : ival);
        atomicAdd(&hist[(uint64_t)t * kBins + ival], 1u);
        if (w >= ww) {
            // |d sum| <= 2 sqrt(2 sum n) delta + 2 n delta^2 over both channels;
            // the window is certain when both ends of [sum - dsum, sum + dsum]
            // fall in its bin (log10 is monotone, so the interval's image is
            // bounded by its ends' values; silence stays in bin 0)
            const double dsum = 2.0 * sqrt(2.0 * sum * window) * delta + 2.0 * window * delta * delta;
            const double lo = sum - dsum > 0.0 ? sum - dsum : 0.0;
            const double hi = sum + dsum;
            const double vlo = 100. * 10. * log10(lo / window * 0.5 + 1.e-37);
            const double vhi = 100. * 10. * log10(hi / window * 0.5 + 1.e-37);
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
        peaks[t] = (double)amax[t] / (double)(1 << (tracks[t].bps - 1));
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
        amax, dmax, warm, flag, tlist;
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

// the segments of track t (appended to `out`): whole windows, a multiple
// of 10 frames long (the filter's ring cycle), warm-up a multiple of 10
void plan_segments(uint32_t t, const RgTrack &T, const atg_rg_track &a, bool exact_only,
                   std::vector<RgSeg> &out, uint32_t &first_warm_window)
{
    const uint32_t wsz = T.window;
    uint32_t g10 = 10;
    for (uint32_t x = wsz % 10, y = 10; x;) { // gcd(wsz, 10)
        const uint32_t r = y % x;
        y = x;
        x = r;
        g10 = y;
    }
    uint32_t K = 10 / g10;
    while (K < kRgSegWindows)
        K += 10 / g10;
    const uint64_t L = exact_only ? T.frames + 10 : (uint64_t)K * wsz;
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
        g.f0 = (uint32_t)f0;
        g.f1 = (uint32_t)std::min<uint64_t>(f0 + L, T.frames);
        g.fw = f0 > warm ? (uint32_t)(f0 - warm) : 0u;
        g.exact = g.fw == 0 && (f0 == 0 || f0 <= warm) ? 1u : 0u;
        if (g_rg_warm_override == 0 && f0)
            g.exact = 0;
        if (a.chunk_frames) {
            const uint64_t ci = (uint64_t)(std::upper_bound(rs.begin(), rs.end(), f0) -
                                           rs.begin()) - 1;
            g.ci = (uint32_t)ci;
            g.c0 = (uint32_t)rs[ci];
        } else {
            g.ci = (uint32_t)(f0 / 4096);
            g.c0 = g.ci * 4096u;
        }
        g.w0 = (uint32_t)(f0 / wsz);
        if (!g.exact && first_warm_window == 0xFFFFFFFFu)
            first_warm_window = g.w0;
        out.push_back(g);
        f0 += L;
    } while (f0 < T.frames);
}

} // namespace

extern "C" {

void atg_replaygain_set_warmup(int frames) { g_rg_warm_override = frames; }

uint32_t atg_replaygain_fallback_tracks(void) { return g_rg_fallback_tracks; }


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
        tr[t] = RgTrack{a.pcm_offset * a.channels, a.pcm_frames, a.channels, a.bits_per_sample,
                        (uint32_t)fi, (uint32_t)std::ceil(a.sample_rate * 0.050), cbase};
        wbase[t + 1] = wbase[t] + a.pcm_frames / tr[t].window;
        if (n_albums) {
            if (!count[a.album])
                first[a.album] = t;
            ++count[a.album];
        }
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
        plan_segments(t, tr[t], tracks[t], false, tr[t].ch == 1 ? segs : segs2, warm_win[t]);
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
    RHIP(g_ctx.dmax.ensure(sizeof(unsigned long long) * n));
    RHIP(g_ctx.warm.ensure(sizeof(uint32_t) * n));
    RHIP(g_ctx.flag.ensure(sizeof(uint32_t) * n));
    RHIP(g_ctx.tlist.ensure(sizeof(uint32_t) * n));
    RHIP(hipMemcpyAsync(g_ctx.tracks.p, tr.data(), sizeof(RgTrack) * n, hipMemcpyHostToDevice, s));
    RHIP(hipMemcpyAsync(g_ctx.wbase.p, wbase.data(), sizeof(uint64_t) * (n + 1),
                        hipMemcpyHostToDevice, s));
    RHIP(hipMemcpyAsync(g_ctx.segs.p, segs.data(), sizeof(RgSeg) * nseg, hipMemcpyHostToDevice, s));
    RHIP(hipMemcpyAsync(g_ctx.warm.p, warm_win.data(), sizeof(uint32_t) * n,
                        hipMemcpyHostToDevice, s));
    RHIP(hipMemsetAsync(g_ctx.hist.p, 0, sizeof(uint32_t) * kBins * (size_t)n, s));
    RHIP(hipMemsetAsync(g_ctx.amax.p, 0, sizeof(uint32_t) * n, s));
    RHIP(hipMemsetAsync(g_ctx.dmax.p, 0, sizeof(unsigned long long) * n, s));
    RHIP(hipMemsetAsync(g_ctx.flag.p, 0, sizeof(uint32_t) * n, s));
    const RgTrack *dtr = (const RgTrack *)g_ctx.tracks.p;
    const uint64_t *dwb = (const uint64_t *)g_ctx.wbase.p;
    const uint32_t *dch = (const uint32_t *)g_ctx.chunks.p;
    double *dws = (double *)g_ctx.wsum.p;
    auto run_segments = [&](const RgSeg *dseg, uint32_t n1, uint32_t ntot, double *sin,
                            double *sout) -> atg_status {
        if (n1)
            hipLaunchKernelGGL(k_rg_seg<1>, dim3((n1 + 63) / 64), dim3(64), 0, s, d_pcm, dtr,
                               dseg, n1, dwb, dch, dws, (uint32_t *)g_ctx.amax.p, sin, sout);
        if (ntot > n1)
            hipLaunchKernelGGL(k_rg_seg<2>, dim3((ntot - n1 + 63) / 64), dim3(64), 0, s, d_pcm,
                               dtr, dseg + n1, ntot - n1, dwb, dch, dws, (uint32_t *)g_ctx.amax.p,
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
                       (const uint32_t *)g_ctx.warm.p, (const unsigned long long *)g_ctx.dmax.p,
                       (uint32_t *)g_ctx.flag.p, (uint32_t *)g_ctx.hist.p,
                       (double *)g_ctx.peaks.p);
    RHIP(hipGetLastError());
    // the tracks certification could not vouch for: analysed again as one
    // exact segment each (the serial computation), then binned again
    std::vector<uint32_t> flags(n);
    RHIP(hipMemcpyAsync(flags.data(), g_ctx.flag.p, sizeof(uint32_t) * n, hipMemcpyDeviceToHost,
                        s));
    RHIP(hipStreamSynchronize(s));
    std::vector<uint32_t> redo;
    for (uint32_t t = 0; t < n; ++t)
        if (flags[t])
            redo.push_back(t);
    g_rg_fallback_tracks = (uint32_t)redo.size();
    if (!redo.empty()) {
        std::vector<RgSeg> e1, e2;
        uint32_t unused = 0;
        for (uint32_t t : redo)
            plan_segments(t, tr[t], tracks[t], true, tr[t].ch == 1 ? e1 : e2, unused);
        const uint32_t m1 = (uint32_t)e1.size();
        e1.insert(e1.end(), e2.begin(), e2.end());
        const uint32_t m = (uint32_t)e1.size();
        RHIP(hipMemcpyAsync(g_ctx.segs.p, e1.data(), sizeof(RgSeg) * m, hipMemcpyHostToDevice, s));
        RHIP(hipMemcpyAsync(g_ctx.tlist.p, redo.data(), sizeof(uint32_t) * redo.size(),
                            hipMemcpyHostToDevice, s));
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
                           (const uint32_t *)nullptr, (const unsigned long long *)nullptr,
                           (uint32_t *)nullptr, (uint32_t *)g_ctx.hist.p,
                           (double *)g_ctx.peaks.p);
        RHIP(hipGetLastError());
    }
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
