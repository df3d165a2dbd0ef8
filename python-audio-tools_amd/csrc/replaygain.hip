// replaygain.hip — ReplayGain title and album analysis (SURVEY §8(a)
// G1–G5) for a batch of tracks: the reference's ReplayGain_title_gain /
// analyze_samples / analyzeResult / get_album_gain (src/replaygain.c
// :186-322, :566-807).
//
//   k_rg_title   lane per (track, channel): the Yule-Walker (10th order) +
//                Butterworth (2nd order) IIR pair is a serial recurrence, so
//                each lane runs it over its whole channel from zero state, in
//                the reference's exact fp64 operation order (no contraction),
//                summing squared outputs with the reference's batch grouping
//                (4096-frame reads, 10-sample prebuffer batch, 50 ms windows;
//                singles for batch % 16, then 16-term groups) into one sum
//                per closed window; title peak = max |x| / 2^(bps-1).
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

// filt on a ring history: step R of a 10-sample cycle finds the newest
// input / output at slot (10 - R) % 10 and writes the new ones one slot
// down, so an unrolled cycle of 10 samples moves no registers (the shift
// of filt costs ~30 v_mov_b64 per sample in a loop).  Same operations in
// the same order as filt.
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

// filterYule then filterButter for one sample (replaygain.c:566-610):
// left-to-right sums exactly as the reference's expressions
__device__ __forceinline__ double filt(Chan &s, double x, const double *ky, const double *kb)
{
    double y = 1e-10 + x * ky[0];
#pragma unroll
    for (int k = 1; k <= 10; ++k) {
        y = y - s.yo[k - 1] * ky[2 * k - 1];
        y = y + s.in[k - 1] * ky[2 * k];
    }
    const double b = y * kb[0] - s.bo0 * kb[1] + s.yo[0] * kb[2] - s.bo1 * kb[3] + s.yo[1] * kb[4];
#pragma unroll
    for (int k = 9; k > 0; --k) {
        s.in[k] = s.in[k - 1];
        s.yo[k] = s.yo[k - 1];
    }
    s.in[0] = x;
    s.yo[0] = y;
    s.bo1 = s.bo0;
    s.bo0 = b;
    return b;
}

// lane per (track, channel): the reference keeps separate accumulators for
// the two channels (lsum, rsum) and only adds them when a window closes, so
// each lane filters one channel and writes its per-window sums; k_rg_bin
// bins (lsum + rsum) / window / 2 per window.  Mono tracks filter once and
// use the same sums for both channels (the reference duplicates the channel).
//
// The filter is a serial recurrence whose every step depends on the last
// output from its second operation on (the reference's operation order), so
// a lane's time is (samples) x (the latency of ~26 dependent fp64 adds):
// nothing else may stall it.  The wave's 32 tracks are staged through LDS
// in chunks of 64 frames, double-buffered: at each chunk boundary the lanes
// store the chunk loaded one boundary earlier and issue the next chunk's
// loads, which then have 64 samples of filtering to arrive; the sample loop
// reads the lane's channel from LDS.  Every lane handles sample f at step f
// (the read()/batch/window bookkeeping only groups the running sums), so the
// chunk schedule is wave-uniform; the bookkeeping is a per-lane state
// machine.
constexpr uint32_t kRgChunk = 80; // a multiple of filt_r's 10-sample cycle
constexpr uint32_t kRgStride = 2 * kRgChunk + 2; // ints per track per buffer (conflict-free reads)

__global__ __launch_bounds__(64) void k_rg_title(const int32_t *__restrict__ pcm,
                                                 const RgTrack *__restrict__ tracks, uint32_t n,
                                                 const uint64_t *__restrict__ win_base,
                                                 const uint32_t *__restrict__ chunks,
                                                 double *__restrict__ wsum,
                                                 double *__restrict__ peaks)
{
    __shared__ int32_t buf[2][32 * kRgStride];
    const uint32_t lane = threadIdx.x, j = lane >> 1, chan = lane & 1;
    const uint32_t g = blockIdx.x * 64 + lane, t = g >> 1;
    const bool have = t < n;
    RgTrack T = {};
    if (have)
        T = tracks[t];
    // lanes of a track past the batch or the second channel of a mono track
    // only help with the loads
    const bool run = have && !(chan == 1 && T.ch == 1);
    const uint64_t frames = have ? T.frames : 0;
    uint64_t fmax = frames;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1)
        fmax = max(fmax, (uint64_t)__shfl_xor((unsigned long long)fmax, o));
    const uint32_t ch = have ? T.ch : 1u;
    const int32_t *__restrict__ src = pcm + (have ? T.off : 0);
    // chunk loads: the lane pair of track j fetches its 64 frames x ch ints,
    // lane h the ints [64 h, 64 h + 64) of them
    int32_t ld[kRgChunk];
    auto load_chunk = [&](uint64_t F) {
        const uint64_t lim = frames * ch; // ints of the track
#pragma unroll
        for (uint32_t i = 0; i < kRgChunk; ++i) {
            const uint64_t q = F * ch + chan * kRgChunk + i;
            ld[i] = (have && q < lim && chan * kRgChunk + i < kRgChunk * ch) ? src[q] : 0;
        }
    };
    auto store_chunk = [&](int b) {
#pragma unroll
        for (uint32_t i = 0; i < kRgChunk; ++i)
            buf[b][j * kRgStride + chan * kRgChunk + i] = ld[i];
    };
    // the lane's coefficients in registers, opaque to the compiler (it
    // otherwise re-loads them from the constant table inside the unrolled
    // sample cycle to save registers; a lone wave per SIMD has 512)
    double ky[21], kb[5];
    {
        const double *gy = c_yule[have ? T.fi : 0], *gb = c_butter[have ? T.fi : 0];
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
    double *W = wsum + 2 * (have ? win_base[t] : 0) + chan;
    const long window = have ? (long)T.window : 1;
    Chan S = {};
    double sum = 0, gs = 0;
    uint32_t amax = 0;
    // read() / batch / window bookkeeping (replaygain.c:210-305)
    uint64_t ci = have ? T.chunk_base : 0, c0 = 0;
    auto next_read = [&]() -> long {
        if (c0 >= frames)
            return 0;
        return T.chunk_base != ~0ull ? (long)chunks[ci++]
                                     : (long)(frames - c0 < 4096 ? frames - c0 : 4096);
    };
    long n4 = run ? next_read() : 0, pos = 0, batch = n4, totsamp = 0, nwin = 0;
    // per-sample state in 32 bits: a batch is at most one window (< 2^31)
    int32_t k = 0, cur = 0, singles = 0;
    auto start_batch = [&]() {
        long c = batch > window - totsamp ? window - totsamp : batch;
        if (pos < 10 && c > 10 - pos)
            c = 10 - pos;
        cur = (int32_t)c;
        singles = cur % 16;
        k = 0;
    };
    start_batch();
    load_chunk(0);
    for (uint64_t F = 0; F < fmax; F += kRgChunk) {
        const int b = (int)((F / kRgChunk) & 1);
        store_chunk(b);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (F + kRgChunk < fmax)
            load_chunk(F + kRgChunk);
        const int32_t *xb = &buf[b][j * kRgStride + chan];
        const uint64_t nk = run && frames > F ? min((uint64_t)kRgChunk, frames - F) : 0;
        // samples in cycles of 10 (filt_r's ring; a chunk is 8 cycles).  A
        // cycle's 10 filter steps are one straight-line block, so one
        // sample's Butterworth stage and the next one's Yule products fill
        // the gaps of the dependent Yule chain; the bookkeeping follows.
        // Past nk (the lane's track ends inside this chunk) the row's stale
        // words are filtered and never used.
        for (uint32_t k10 = 0; k10 < nk; k10 += 10) {
            int32_t iv[10];
#pragma unroll
            for (int r = 0; r < 10; ++r)
                iv[r] = xb[(k10 + (uint32_t)r) * ch];
            // 8-bit: x << 8, 16-bit: x, 24-bit: x >> 8 (as shift amounts: no
            // per-sample branches on the lane's format)
            double ov[10];
            ov[0] = filt_r<0>(S, (double)((iv[0] << xsl) >> xsr), ky, kb);
            ov[1] = filt_r<1>(S, (double)((iv[1] << xsl) >> xsr), ky, kb);
            ov[2] = filt_r<2>(S, (double)((iv[2] << xsl) >> xsr), ky, kb);
            ov[3] = filt_r<3>(S, (double)((iv[3] << xsl) >> xsr), ky, kb);
            ov[4] = filt_r<4>(S, (double)((iv[4] << xsl) >> xsr), ky, kb);
            ov[5] = filt_r<5>(S, (double)((iv[5] << xsl) >> xsr), ky, kb);
            ov[6] = filt_r<6>(S, (double)((iv[6] << xsl) >> xsr), ky, kb);
            ov[7] = filt_r<7>(S, (double)((iv[7] << xsl) >> xsr), ky, kb);
            ov[8] = filt_r<8>(S, (double)((iv[8] << xsl) >> xsr), ky, kb);
            ov[9] = filt_r<9>(S, (double)((iv[9] << xsl) >> xsr), ky, kb);
#pragma unroll
        for (int r = 0; r < 10; ++r) {
            const uint32_t kk = k10 + (uint32_t)r;
            if (kk < nk) {
            const uint32_t av = (uint32_t)(iv[r] < 0 ? -(int64_t)iv[r] : iv[r]);
            amax = av > amax ? av : amax;
            const double o = ov[r];
            const double o2 = o * o;
            if (k < singles) {
                sum += o2;
            } else {
                const int32_t gi = (k - singles) & 15;
                gs = gi == 0 ? o2 : gs + o2;
                if (gi == 15)
                    sum += gs;
            }
            if (++k == cur) { // the batch ends
                batch -= cur;
                pos += cur;
                totsamp += cur;
                if (totsamp == window) {
                    W[2 * nwin] = sum;
                    if (T.ch == 1)
                        W[2 * nwin + 1] = sum;
                    ++nwin;
                    sum = 0.;
                    totsamp = 0;
                }
                if (batch == 0) { // the next read() result
                    c0 += (uint64_t)n4;
                    n4 = next_read();
                    batch = n4;
                    pos = 0;
                }
                if (batch > 0)
                    start_batch();
            }
        }
        }
        }
        // the buffer is rewritten two boundaries later: every lane's reads
        // of it are done before its next store (in-order LDS per wave)
        __builtin_amdgcn_wave_barrier();
    }
    if (!run)
        return;
    const double peak = (double)amax / (double)(1 << (T.bps - 1));
    peaks[2 * t + chan] = peak;
    if (T.ch == 1)
        peaks[2 * t + 1] = peak;
}

// bin every closed window: (int)(1000 log10((lsum + rsum) / n * 0.5 + 1e-37))
// (replaygain.c:713-724), one thread per window
__global__ __launch_bounds__(256) void k_rg_bin(const RgTrack *__restrict__ tracks, uint32_t n,
                                                const uint64_t *__restrict__ win_base,
                                                const double *__restrict__ wsum,
                                                const double *__restrict__ peak2,
                                                uint32_t *__restrict__ hist,
                                                double *__restrict__ peaks)
{
    const uint32_t t = blockIdx.y;
    if (t >= n)
        return;
    const uint64_t nw = win_base[t + 1] - win_base[t];
    const double window = (double)tracks[t].window;
    for (uint64_t w = blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += gridDim.x * blockDim.x) {
        const double *ws = wsum + 2 * (win_base[t] + w);
        const double val = 100. * 10. * log10((ws[0] + ws[1]) / window * 0.5 + 1.e-37);
        int ival = (int)val;
        ival = ival < 0 ? 0 : (ival >= kBins ? kBins - 1 : ival);
        atomicAdd(&hist[(uint64_t)t * kBins + ival], 1u);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        peaks[t] = fmax(peak2[2 * t], peak2[2 * t + 1]);
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

// device buffers of one device (kept across calls; a batch pipeline calls
// this once per album batch)
struct RgCtx {
    std::mutex mu;
    bool coeffs = false;
    void *tracks = nullptr, *hist = nullptr, *peaks = nullptr, *gains = nullptr, *alb = nullptr,
         *meta = nullptr, *wsum = nullptr, *wbase = nullptr, *peak2 = nullptr, *chunks = nullptr;
    size_t cap_tracks = 0, cap_albums = 0, cap_win = 0, cap_wbase = 0, cap_peak2 = 0,
           cap_chunks = 0;
};
constexpr int kMaxDevices = 64;
RgCtx g_ctxs[kMaxDevices];

} // namespace

extern "C" {

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
    if (n > g_ctx.cap_tracks) {
        for (void *p : {g_ctx.tracks, g_ctx.hist, g_ctx.peaks, g_ctx.gains})
            (void)hipFree(p);
        RHIP(hipMalloc(&g_ctx.tracks, sizeof(RgTrack) * n));
        RHIP(hipMalloc(&g_ctx.hist, sizeof(uint32_t) * kBins * (size_t)n));
        RHIP(hipMalloc(&g_ctx.peaks, sizeof(double) * n));
        RHIP(hipMalloc(&g_ctx.gains,
                       sizeof(double) * (n + std::max<size_t>(n_albums, g_ctx.cap_albums) + 1)));
        g_ctx.cap_tracks = n;
    }
    if (n_albums > g_ctx.cap_albums) {
        (void)hipFree(g_ctx.alb);
        (void)hipFree(g_ctx.meta);
        RHIP(hipMalloc(&g_ctx.alb, sizeof(uint32_t) * kBins * (size_t)n_albums));
        RHIP(hipMalloc(&g_ctx.meta, sizeof(uint32_t) * 2 * n_albums));
        (void)hipFree(g_ctx.gains);
        RHIP(hipMalloc(&g_ctx.gains, sizeof(double) * (g_ctx.cap_tracks + n_albums + 1)));
        g_ctx.cap_albums = n_albums;
    }
    if (!n) { // empty albums: peak 0.0 (replaygain.c:180), empty histograms
        if (album_peaks)
            for (uint32_t a = 0; a < n_albums; ++a)
                album_peaks[a] = 0.0;
        if (n_albums) {
            uint32_t *album = d_album_hist ? d_album_hist : (uint32_t *)g_ctx.alb;
            RHIP(hipMemsetAsync(album, 0, sizeof(uint32_t) * kBins * (size_t)n_albums, s));
            RHIP(hipStreamSynchronize(s));
        }
        return ATG_OK;
    }
    if (chunks.size() > g_ctx.cap_chunks || !g_ctx.chunks) {
        (void)hipFree(g_ctx.chunks);
        g_ctx.chunks = nullptr;
        const size_t want = std::max<size_t>(chunks.size(), 1);
        RHIP(hipMalloc(&g_ctx.chunks, sizeof(uint32_t) * want));
        g_ctx.cap_chunks = want;
    }
    if (!chunks.empty())
        RHIP(hipMemcpyAsync(g_ctx.chunks, chunks.data(), sizeof(uint32_t) * chunks.size(),
                            hipMemcpyHostToDevice, s));
    if (wbase[n] + 1 > g_ctx.cap_win) {
        (void)hipFree(g_ctx.wsum);
        (void)hipFree(g_ctx.wbase);
        RHIP(hipMalloc(&g_ctx.wsum, sizeof(double) * 2 * (wbase[n] + 1)));
        RHIP(hipMalloc(&g_ctx.wbase, sizeof(uint64_t) * (n + 1)));
        g_ctx.cap_win = wbase[n] + 1;
        g_ctx.cap_wbase = n + 1;
    }
    if (n + 1 > g_ctx.cap_wbase) {
        (void)hipFree(g_ctx.wbase);
        RHIP(hipMalloc(&g_ctx.wbase, sizeof(uint64_t) * (n + 1)));
        g_ctx.cap_wbase = n + 1;
    }
    if (!g_ctx.peak2 || n > g_ctx.cap_peak2) {
        (void)hipFree(g_ctx.peak2);
        RHIP(hipMalloc(&g_ctx.peak2, sizeof(double) * 2 * n));
        g_ctx.cap_peak2 = n;
    }
    RHIP(hipMemcpyAsync(g_ctx.tracks, tr.data(), sizeof(RgTrack) * n, hipMemcpyHostToDevice, s));
    RHIP(hipMemcpyAsync(g_ctx.wbase, wbase.data(), sizeof(uint64_t) * (n + 1),
                        hipMemcpyHostToDevice, s));
    RHIP(hipMemsetAsync(g_ctx.hist, 0, sizeof(uint32_t) * kBins * (size_t)n, s));
    hipLaunchKernelGGL(k_rg_title, dim3((2 * n + 63) / 64), dim3(64), 0, s, d_pcm,
                       (const RgTrack *)g_ctx.tracks, n, (const uint64_t *)g_ctx.wbase,
                       (const uint32_t *)g_ctx.chunks, (double *)g_ctx.wsum,
                       (double *)g_ctx.peak2);
    RHIP(hipGetLastError());
    hipLaunchKernelGGL(k_rg_bin, dim3(4, n), dim3(256), 0, s, (const RgTrack *)g_ctx.tracks, n,
                       (const uint64_t *)g_ctx.wbase, (const double *)g_ctx.wsum,
                       (const double *)g_ctx.peak2, (uint32_t *)g_ctx.hist,
                       (double *)g_ctx.peaks);
    RHIP(hipGetLastError());
    hipLaunchKernelGGL(k_rg_gain, dim3(n), dim3(256), 0, s, (const uint32_t *)g_ctx.hist, n,
                       (double *)g_ctx.gains);
    RHIP(hipGetLastError());
    uint32_t *album = d_album_hist ? d_album_hist : (uint32_t *)g_ctx.alb;
    if (n_albums) {
        RHIP(hipMemcpyAsync(g_ctx.meta, first.data(), sizeof(uint32_t) * n_albums,
                            hipMemcpyHostToDevice, s));
        RHIP(hipMemcpyAsync((uint32_t *)g_ctx.meta + n_albums, count.data(),
                            sizeof(uint32_t) * n_albums, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_rg_album, dim3((kBins + 255) / 256, n_albums), dim3(256), 0, s,
                           (const uint32_t *)g_ctx.hist, (const uint32_t *)g_ctx.meta,
                           (const uint32_t *)g_ctx.meta + n_albums, album);
        RHIP(hipGetLastError());
    }
    std::vector<double> gains(n), peaks(n);
    RHIP(hipMemcpyAsync(gains.data(), g_ctx.gains, sizeof(double) * n, hipMemcpyDeviceToHost, s));
    RHIP(hipMemcpyAsync(peaks.data(), g_ctx.peaks, sizeof(double) * n, hipMemcpyDeviceToHost, s));
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
