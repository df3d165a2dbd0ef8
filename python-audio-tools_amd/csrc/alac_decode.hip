// alac_decode.hip — MI355X batch ALAC decoder: the
// reference's ALACDecoder (src/decoders/alac.c: parse_decoding_parameters
// :439-672, read() :183-254, read_frame :818-951, read_residuals
// :1017-1085, decode_subframe :1147-1235, decorrelate_channels :1237-1259,
// alac_order_to_wave_order :709-816) for a batch of M4A images, status for
// status.
//
// Framesets are variable-length and only the parse of one finds the next,
// so the serial read() loop becomes passes that are each parallel (the
// FLAC decoder's plan, flac_decode.hip):
//
//   K1 k_adec_parse    lane per predicted frameset: the stsz atom gives
//                      every frameset's size, so each lane parses the
//                      frameset at its predicted offset -- frame headers,
//                      subframe headers, and the adaptive-Golomb residual
//                      blocks (counting, no prediction) -- and records where
//                      each channel's data lies, the frameset length and
//                      status.
//   K2 k_adec_chain    wave per track, twice: the read() walk from the
//                      start position with remaining_frames (64 chained
//                      predictions a step, then serially); a frameset
//                      whose position the prediction missed (a damaged or
//                      absent stsz) is parsed inline, so the walk is always
//                      the reference's.  Pass 1 counts, a host prefix places
//                      the output, pass 2 writes the frameset list.
//   K3 k_adec_channel  lane per (frameset, channel): residuals + the
//                      sign-LMS adaptive restore (or verbatim samples) into
//                      a planar scratch.
//   K4 k_adec_interleave block per frameset: stereo decorrelation,
//                      uncompressed LSBs, ALAC -> wave channel order,
//                      interleaved int32 (the FrameList layout).
#include "handle_lock.h"
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/atgpu.h"
#include "alac_common.h"

// Active lanes per 64-thread block of the walk kernels.  The read() chain
// walk runs one track per wave (it was one track per lane: 3.6 -> 1.5 ms,
// then a wave's lanes check 64 chained predictions at once).  The
// frameset parse and the channel restore stay at 64: 16 and 32 lanes a
// wave were slower (17.6 -> 23.4 ms, 12.6 -> 17.1 ms; 8 and 16 slower
// still), their waves already cover the SIMDs' latency
constexpr uint32_t kAdecParseLpw = 64, kAdecChannelLpw = 64;
// device bytes the parse may fill with a batch's residuals (config 5: 30 k
// framesets x 6 channels x 4096 x 4 B = 2.9 GB)
constexpr uint64_t kResidMax = 12ull << 30;

namespace {

enum {
    AD_OK = 0, AD_IO_ERROR = 1, AD_UNUSED_BITS = 2, AD_INVALID_ALAC_ATOM = 3,
    AD_INVALID_MDHD_ATOM = 4, AD_MDIA_NOT_FOUND = 5, AD_STSD_NOT_FOUND = 6,
    AD_MDHD_NOT_FOUND = 7, AD_INVALID_SEEKTABLE = 8, AD_NO_MDAT = 9, AD_CHANNEL_MISMATCH = 10
};

struct ADTrack {
    uint64_t img;        // absolute byte of the image start
    uint64_t end;        // absolute byte end of the image
    uint64_t start;      // absolute byte of the first frameset to read
    uint64_t remaining;  // remaining_frames
    uint32_t maxn, bps, hm, ih, mk, channels;
    uint32_t pred_first, pred_n; // predicted framesets (K1 records)
    uint64_t fs_base;    // pass 2: first dense frameset slot
    uint64_t pcm_base;   // pass 2: first interleaved output sample of the track
    uint64_t job_base;   // pass 2: first channel job
};

struct AElem {
    uint32_t N;          // sample_count of the frame header
    uint8_t cc, uncompressed, lsbs, shift;
    uint8_t lw, pad0, pad1, pad2;
    uint32_t data_bit;   // verbatim samples (relative to the frameset's first bit)
    uint32_t lsb_bit;    // uncompressed LSB block
    uint32_t sub_bit[2]; // subframe headers
    uint32_t res_bit[2]; // residual blocks
    uint32_t nres[2];    // samples each channel produced
};

struct AFs {
    uint64_t res_base;   // residuals stored by the parse: channel k at
                         // res + res_base + k * stride (~0: not stored)
    uint64_t start;      // absolute byte
    uint32_t bytes;      // frameset length (byte aligned)
    int32_t status;
    uint32_t nelem, nch, n0, track;
    uint64_t pcm_start;  // pass 2: first interleaved output sample
    uint64_t job0;       // pass 2: the frameset's first channel job (its planar slots)
    AElem e[8];
};

struct ACount {
    uint64_t pcm_frames;
    uint32_t n_fs;
    int32_t status;
    uint32_t max_n0; // the track's longest frameset (the planar slot stride)
    uint32_t pad;
};

// one frameset at absolute byte `start` (read_frame x elements, alac.c:204-233)
// a lane's values to its own 16-byte aligned region, four per store (the
// lanes of a wave write different regions: four values fill a quarter
// line per store instead of one word)
struct Out4 {
    int32_t *p;
    int4 b;
    __device__ __forceinline__ void put(uint32_t i, int32_t v)
    {
        const uint32_t q = i & 3u;
        b.x = q == 0u ? v : b.x;
        b.y = q == 1u ? v : b.y;
        b.z = q == 2u ? v : b.z;
        b.w = q == 3u ? v : b.w;
        if (q == 3u)
            *(int4 *)(p + i - 3u) = b;
    }
    // the samples of the last, partial group (i = samples written)
    __device__ __forceinline__ void flush(uint32_t i)
    {
        const uint32_t q = i & 3u, a = i - q;
        if (q > 0u)
            p[a] = b.x;
        if (q > 1u)
            p[a + 1u] = b.y;
        if (q > 2u)
            p[a + 2u] = b.z;
    }
};

// res: where this frameset's residuals go (channel k at res + k * stride,
// at most stride values each), or null
__device__ void parse_fs(const uint32_t *w, const ADTrack &T, uint64_t start, AFs &F,
                         int32_t *res = nullptr, uint32_t stride = 0)
{
    ABitRC r;
    const uint64_t b0 = start * 8;
    r.init(w, b0, T.end * 8);
    F.res_base = ~0ull;
    F.start = start;
    F.bytes = 0;
    F.status = AD_OK;
    F.nelem = 0;
    F.nch = 0;
    F.n0 = 0;
    uint32_t cc = r.get(3) + 1u;
    while (!r.eof && cc != 8u) {
        if (r.get(16) != 0u) {
            F.status = r.eof ? AD_IO_ERROR : AD_UNUSED_BITS;
            return;
        }
        const uint32_t has_size = r.get(1), lsbs = r.get(2), nc = r.get(1);
        const uint32_t N = has_size ? r.get(32) : T.maxn;
        if (r.eof)
            break;
        if (F.nch + cc > 8u || N > (1u << 24)) { // beyond any encoder's output
            F.status = AD_IO_ERROR;
            return;
        }
        AElem &E = F.e[F.nelem];
        E.N = N;
        E.cc = (uint8_t)cc;
        E.uncompressed = (uint8_t)nc;
        E.lsbs = (uint8_t)lsbs;
        E.shift = 0;
        E.lw = 0;
        E.pad0 = E.pad1 = E.pad2 = 0;
        E.lsb_bit = 0;
        E.sub_bit[0] = E.sub_bit[1] = 0;
        E.res_bit[0] = E.res_bit[1] = 0;
        E.nres[0] = E.nres[1] = 0;
        if (nc) { // verbatim samples (alac.c:841-865)
            E.data_bit = (uint32_t)(r.pos - b0);
            const uint64_t need = (uint64_t)N * cc * T.bps;
            if (r.pos + need > r.end) {
                r.eof = true;
                break;
            }
            r.pos += need;
            E.nres[0] = E.nres[1] = N;
        } else {
            E.shift = (uint8_t)r.get(8);
            E.lw = (uint8_t)r.get(8);
            for (uint32_t c = 0; c < cc; ++c) {
                E.sub_bit[c] = (uint32_t)(r.pos - b0);
                r.get(4);
                r.get(4);
                r.get(3);
                const uint32_t order = r.get(5);
                if (r.pos + 16ull * order > r.end) {
                    r.eof = true;
                    break;
                }
                r.pos += 16ull * order;
            }
            if (r.eof)
                break;
            E.lsb_bit = (uint32_t)(r.pos - b0);
            if (lsbs) {
                const uint64_t need = (uint64_t)cc * N * lsbs * 8u;
                if (r.pos + need > r.end) {
                    r.eof = true;
                    break;
                }
                r.pos += need;
            }
            const uint32_t ss = T.bps - lsbs * 8u + (cc - 1u);
            for (uint32_t c = 0; c < cc && !r.eof; ++c) {
                E.res_bit[c] = (uint32_t)(r.pos - b0);
                AResidualReader g;
                g.init(N, ss, T.ih, T.hm, T.mk);
                uint32_t n = 0;
                int32_t v;
                // the walk on the windowed reader while 128 bits remain
                // before the end, then on the exact one from the same
                // position (field widths the window cannot take go to the
                // exact reader at once); two loops, so the hot one holds
                // only the windowed step
                const bool fast = ss <= 32u && T.mk <= 32u;
                auto walk = [&](auto &&use) {
                    bool done = false;
                    if (fast) {
                        AFastBits fb;
                        fb.init(w, r.pos, r.end);
                        const uint64_t p0 = r.pos;
                        while (!fb.careful()) {
                            if (!alac_next_fast(g, fb, v)) {
                                done = true;
                                break;
                            }
                            use(v);
                        }
                        r.pos = p0 + fb.used;
                    }
                    if (!done)
                        while (g.next(r, v))
                            use(v);
                };
                if (res) {
                    // the values too, for the channel restore (k_adec_channel
                    // then runs the adaptive filter without decoding again)
                    Out4 q;
                    q.p = res + (uint64_t)(F.nch + c) * stride;
                    q.b = make_int4(0, 0, 0, 0);
                    walk([&](int32_t x) {
                        if (n < stride)
                            q.put(n, x);
                        ++n;
                    });
                    q.flush(n < stride ? n : stride);
                    if (n > stride)
                        res = nullptr; // a channel longer than the slot: not stored
                } else {
                    walk([&](int32_t) { ++n; });
                }
                E.nres[c] = n;
            }
        }
        F.nch += cc;
        F.nelem += 1;
        if (r.eof)
            break;
        cc = r.get(3) + 1u;
    }
    if (r.eof) {
        F.status = AD_IO_ERROR;
        return;
    }
    const uint64_t endb = (r.pos + 7) >> 3;
    F.bytes = (uint32_t)(endb - start);
    F.n0 = F.nelem ? F.e[0].nres[0] : 0;
    // the frameset's channels must agree (aa_int_to_FrameList, pcmconv.c:75-85)
    bool mismatch = F.nch != T.channels;
    for (uint32_t k = 0; k < F.nelem; ++k)
        for (uint32_t c = 0; c < F.e[k].cc; ++c)
            mismatch = mismatch || F.e[k].nres[c] != F.n0;
    if (mismatch)
        F.status = AD_CHANNEL_MISMATCH;
}

// K1: every predicted frameset
__global__ __launch_bounds__(64) void k_adec_parse(const uint32_t *__restrict__ w,
                                                   const ADTrack *__restrict__ tr,
                                                   const uint32_t *__restrict__ pred_track,
                                                   const uint64_t *__restrict__ pred_start,
                                                   uint64_t npred, AFs *__restrict__ recs,
                                                   int32_t *__restrict__ resid, uint64_t res_fs,
                                                   uint32_t res_stride)
{
    if (threadIdx.x >= kAdecParseLpw)
        return;
    const uint64_t i = (uint64_t)blockIdx.x * kAdecParseLpw + threadIdx.x;
    if (i >= npred)
        return;
    const ADTrack T = tr[pred_track[i]];
    AFs F;
    int32_t *res = resid ? resid + i * res_fs : nullptr;
    parse_fs(w, T, pred_start[i], F, res, res_stride);
    // every channel's residuals stored (parse_fs drops res on a channel
    // longer than the slot; a failed parse is never restored)
    if (res && F.status == AD_OK) {
        bool fit = F.nch * (uint64_t)res_stride <= res_fs;
        for (uint32_t k = 0; k < F.nelem; ++k)
            for (uint32_t c = 0; c < F.e[k].cc; ++c)
                fit = fit && F.e[k].nres[c] <= res_stride;
        if (fit)
            F.res_base = i * res_fs;
    }
    F.track = pred_track[i];
    F.pcm_start = 0;
    F.job0 = 0;
    recs[i] = F;
}

// exclusive prefix sum over the wave
template <typename V>
__device__ __forceinline__ V wave_excl_sum(V v, int lane)
{
    V x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const V y = __shfl_up(x, d, 64);
        x += lane >= d ? y : (V)0;
    }
    return x - v;
}

// K2: the read() walk per track (alac.c:183-254, remaining_frames), a wave
// per track.  While the predictions chain -- each starts where the one
// before it ends and parsed without error -- the wave takes 64 framesets a
// step: a lane per frameset checks its link and its share of
// remaining_frames, prefix sums place the counts (and in pass 2 the dense
// records and channel jobs), and the walk advances past the first lane
// that does not qualify.  From there lane 0 walks on serially, as before
// (a missed prediction is parsed inline, a status stops the track).  The
// serial walk alone was a chain of dependent loads per frameset (its
// position comes from the record before), ~1.7 ms per pass for config 5.
__global__ __launch_bounds__(64) void k_adec_chain(const uint32_t *__restrict__ w,
                                                   const ADTrack *__restrict__ tr, uint32_t nt,
                                                   const uint64_t *__restrict__ pred_start,
                                                   const AFs *__restrict__ recs,
                                                   ACount *__restrict__ counts, int pass,
                                                   AFs *__restrict__ dense,
                                                   uint2 *__restrict__ jobs)
{
    const uint32_t t = blockIdx.x;
    const int lane = (int)threadIdx.x;
    if (t >= nt)
        return;
    const ADTrack T = tr[t];
    uint64_t pos = T.start, remaining = T.remaining, pcm = 0;
    uint32_t nfs = 0, k = 0, njob = 0, max_n0 = 0;
    int32_t status = AD_OK;
    while (remaining && k < T.pred_n) {
        const uint32_t idx = k + (uint32_t)lane;
        const bool valid = idx < T.pred_n;
        uint64_t ps = ~0ull, fend = 0;
        uint32_t n0 = 0, nch = 0;
        int32_t st = AD_IO_ERROR;
        if (valid) {
            const AFs &R = recs[T.pred_first + idx];
            ps = pred_start[T.pred_first + idx];
            st = R.status;
            n0 = R.n0;
            nch = R.nch;
            fend = R.start + R.bytes;
        }
        uint64_t at = __shfl_up(fend, 1, 64);
        at = lane == 0 ? pos : at;
        const uint64_t before = wave_excl_sum<uint64_t>((uint64_t)n0, lane);
        const uint32_t jbefore = wave_excl_sum<uint32_t>(nch, lane);
        const bool take = valid && ps == at && st == AD_OK && before < remaining;
        const uint64_t bad = __ballot(!take);
        const uint32_t m = bad ? (uint32_t)__ffsll((long long)bad) - 1u : 64u;
        if (pass == 2 && (uint32_t)lane < m) {
            AFs F = recs[T.pred_first + idx];
            F.track = t;
            F.pcm_start = T.pcm_base + (pcm + before) * T.channels;
            F.job0 = T.job_base + njob + jbefore;
            dense[T.fs_base + nfs + (uint32_t)lane] = F;
            for (uint32_t c = 0; c < F.nch; ++c)
                jobs[T.job_base + njob + jbefore + c] =
                    make_uint2((uint32_t)(T.fs_base + nfs + (uint32_t)lane), c);
        }
        if (m == 0u)
            break;
        // the state after lanes [0, m), from lane m - 1
        const uint64_t s_n0 = __shfl(before + n0, (int)m - 1, 64);
        const uint32_t s_nch = __shfl(jbefore + nch, (int)m - 1, 64);
        const uint64_t end_m = __shfl(fend, (int)m - 1, 64);
        uint32_t mx = (uint32_t)lane < m ? n0 : 0u;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1)
            mx = max(mx, (uint32_t)__shfl_xor((int)mx, d, 64));
        max_n0 = max(max_n0, mx);
        remaining = remaining > s_n0 ? remaining - s_n0 : 0u;
        pcm += s_n0;
        njob += s_nch;
        nfs += m;
        pos = end_m;
        k += m;
        if (m < 64u)
            break;
    }
    if (lane != 0)
        return;
    while (remaining) {
        // the prediction for this position, if any (predictions ascend)
        while (k < T.pred_n && pred_start[T.pred_first + k] < pos)
            ++k;
        AFs F;
        if (k < T.pred_n && pred_start[T.pred_first + k] == pos) {
            F = recs[T.pred_first + k];
            ++k;
        } else {
            parse_fs(w, T, pos, F);
        }
        if (F.status == AD_OK || F.status == AD_CHANNEL_MISMATCH)
            remaining -= remaining < F.n0 ? remaining : F.n0;
        if (F.status != AD_OK) {
            status = F.status;
            break;
        }
        if (pass == 2) {
            F.track = t;
            F.pcm_start = T.pcm_base + pcm * T.channels;
            F.job0 = T.job_base + njob;
            dense[T.fs_base + nfs] = F;
            for (uint32_t c = 0; c < F.nch; ++c)
                jobs[T.job_base + njob + c] = make_uint2((uint32_t)(T.fs_base + nfs), c);
        }
        njob += F.nch;
        ++nfs;
        pcm += F.n0;
        max_n0 = F.n0 > max_n0 ? F.n0 : max_n0;
        pos = F.start + F.bytes;
    }
    if (pass == 1) {
        ACount c;
        c.pcm_frames = pcm;
        c.n_fs = nfs;
        c.status = status;
        c.max_n0 = max_n0;
        c.pad = 0;
        counts[t] = c;
    }
}

// decode_subframe (alac.c:1147-1235) for one channel, ORDER coefficients in
// registers; out[i] for i < n (16-byte aligned)
template <int ORDER, class R, class G>
__device__ __forceinline__ void restore_fixed(R &r, G &g, const int32_t *coef_in,
                              uint32_t qshift, uint32_t ss, uint32_t n, int32_t *out)
{
    int32_t c[ORDER], h[ORDER + 1]; // h[0] newest
#pragma unroll
    for (int j = 0; j < ORDER; ++j)
        c[j] = coef_in[j];
#pragma unroll
    for (int j = 0; j <= ORDER; ++j)
        h[j] = 0;
    Out4 ob;
    ob.p = out;
    ob.b = make_int4(0, 0, 0, 0);
    for (uint32_t i = 0; i < n; ++i) {
        int32_t res;
        if (!g.next(r, res)) {
            ob.flush(i);
            return;
        }
        int32_t s;
        if (i == 0) {
            s = res;
        } else if (i < ORDER + 1u) {
            s = alac_trunc(res + h[0], ss);
        } else {
            const int32_t base = h[ORDER];
            int64_t sum = (int64_t)1 << (qshift - 1);
#pragma unroll
            for (int j = 0; j < ORDER; ++j)
                sum += (int64_t)c[j] * (int64_t)(h[j] - base);
            sum >>= qshift;
            sum += base;
            s = alac_trunc((int32_t)(res + sum), ss);
            // adaptive update (branch-free over the early exits): step j
            // touches c[ORDER-1-j] with diff = base - s[i-ORDER+j]
            int32_t e = res;
            const bool pos = res > 0;
            bool live = res != 0;
#pragma unroll
            for (int j = 0; j < ORDER; ++j) {
                const int32_t diff = base - h[ORDER - 1 - j];
                const int32_t sg = alac_sgn(diff);
                const int32_t step = pos ? sg : -sg;
                c[ORDER - 1 - j] -= live ? step : 0;
                e -= live ? ((diff * step) >> qshift) * (j + 1) : 0;
                live = live && (pos ? e > 0 : e < 0);
            }
        }
        ob.put(i, s);
#pragma unroll
        for (int j = ORDER; j > 0; --j)
            h[j] = h[j - 1];
        h[0] = s;
    }
    ob.flush(n);
}

// any other order (the encoder writes only 4 and 8): history in the output
template <class R, class G>
__device__ __forceinline__ void restore_generic(R &r, G &g, int32_t *c, uint32_t order,
                                uint32_t qshift, uint32_t ss, uint32_t n, int32_t *out)
{
    if (order >= 31) { // the reference's verbatim branch advances i twice
        uint32_t i = 0;    // (alac.c:1228-1233): samples 1, 3, 5, ... from
        int32_t res, last = 0; // their predecessor slot, the others stay 0
        for (uint32_t k = 0; k < n; ++k) {
            if (!g.next(r, res))
                return;
            int32_t v = 0;
            if (k == i) {
                v = i == 0 ? res : alac_trunc(res + last, ss);
                i += i == 0 ? 1u : 2u;
            }
            out[k] = v;
            last = v;
        }
        return;
    }
    // 1 << (qshift - 1) as the reference build computes it: an int shift
    // whose count the x86 shifter masks to 5 bits (qshift 0 -> INT_MIN)
    const int64_t init = (int64_t)(int32_t)(1u << ((qshift - 1u) & 31u));
    for (uint32_t i = 0; i < n; ++i) {
        int32_t res;
        if (!g.next(r, res))
            return;
        if (i == 0) {
            out[i] = res;
        } else if (i < order + 1u) {
            out[i] = alac_trunc(res + out[i - 1], ss);
        } else {
            const int32_t base = out[i - (order + 1)];
            int64_t sum = init;
            for (uint32_t j = 0; j < order; ++j)
                sum += (int64_t)c[j] * (int64_t)(out[i - j - 1] - base);
            sum >>= qshift;
            sum += base;
            out[i] = alac_trunc((int32_t)(res + sum), ss);
            int32_t e = res;
            if (e > 0) {
                for (uint32_t j = 0; j < order; ++j) {
                    const int32_t diff = base - out[i - order + j];
                    const int32_t sg = alac_sgn(diff);
                    c[order - j - 1] -= sg;
                    e -= ((diff * sg) >> qshift) * (int32_t)(j + 1);
                    if (e <= 0)
                        break;
                }
            } else if (e < 0) {
                for (uint32_t j = 0; j < order; ++j) {
                    const int32_t diff = base - out[i - order + j];
                    const int32_t sg = alac_sgn(diff);
                    c[order - j - 1] += sg;
                    e -= ((diff * -sg) >> qshift) * (int32_t)(j + 1);
                    if (e >= 0)
                        break;
                }
            }
        }
    }
}

// The residuals the parse stored, as AResidualReader hands them out: four
// per 16-byte load, the next four loaded while these are used
struct StoredRes {
    const int32_t *p;
    uint32_t i, n;
    int4 cur, nxt;
    __device__ __forceinline__ void init(const int32_t *base, uint32_t count)
    {
        p = base;
        i = 0;
        n = count;
        cur = n ? *(const int4 *)p : make_int4(0, 0, 0, 0);
        nxt = n > 4u ? *(const int4 *)(p + 4) : make_int4(0, 0, 0, 0);
    }
    template <class R>
    __device__ __forceinline__ bool next(R &, int32_t &out)
    {
        if (i >= n)
            return false;
        const uint32_t q = i & 3u;
        out = q == 0u ? cur.x : q == 1u ? cur.y : q == 2u ? cur.z : cur.w;
        ++i;
        if (q == 3u) {
            cur = nxt;
            if (i + 4u < n)
                nxt = *(const int4 *)(p + i + 4u);
        }
        return true;
    }
};

// decode_subframe for one channel from a residual source G (the bitstream
// reader or the parse's stored values)
template <class R, class G>
__device__ __forceinline__ void restore_channel(R &r, G &g, int32_t *coef, uint32_t order,
                                                uint32_t qshift, uint32_t ss, uint32_t n,
                                                int32_t *out)
{
    if (order == 4 && qshift >= 1) {
        int32_t c4[4] = {coef[0], coef[1], coef[2], coef[3]};
        restore_fixed<4>(r, g, c4, qshift, ss, n, out);
    } else if (order == 8 && qshift >= 1) {
        int32_t c8[8];
#pragma unroll
        for (int k = 0; k < 8; ++k)
            c8[k] = coef[k];
        restore_fixed<8>(r, g, c8, qshift, ss, n, out);
    } else {
        restore_generic(r, g, coef, order, qshift, ss, n, out);
    }
}

// K3: one channel of one frameset -> its planar slot, planar[job * pstride + i]
__global__ __launch_bounds__(64) void k_adec_channel(const uint32_t *__restrict__ w,
                                                     const ADTrack *__restrict__ tr,
                                                     const AFs *__restrict__ dense,
                                                     const uint2 *__restrict__ jobs,
                                                     uint64_t njobs, int32_t *__restrict__ planar,
                                                     uint32_t pstride,
                                                     const int32_t *__restrict__ resid,
                                                     uint32_t res_stride)
{
    if (threadIdx.x >= kAdecChannelLpw)
        return;
    const uint64_t j = (uint64_t)blockIdx.x * kAdecChannelLpw + threadIdx.x;
    if (j >= njobs)
        return;
    const uint2 jb = jobs[j];
    const AFs &F = dense[jb.x];
    const ADTrack T = tr[F.track];
    // channel jb.y -> element and position within it
    uint32_t e = 0, c = jb.y;
    while (e + 1 < F.nelem && c >= F.e[e].cc) {
        c -= F.e[e].cc;
        ++e;
    }
    const AElem E = F.e[e];
    const uint64_t b0 = F.start * 8;
    int32_t *out = planar + j * pstride; // the job's slot (= (F.job0 + jb.y) * pstride)
    ABitR r;
    if (E.uncompressed) {
        const uint64_t stride = (uint64_t)E.cc * T.bps;
        for (uint32_t i = 0; i < E.N; ++i) {
            r.init(w, b0 + E.data_bit + i * stride + (uint64_t)c * T.bps, T.end * 8);
            out[i] = r.get_signed(T.bps);
        }
        return;
    }
    r.init(w, b0 + E.sub_bit[c], T.end * 8);
    r.get(4);
    const uint32_t qshift = r.get(4);
    r.get(3);
    const uint32_t order = r.get(5);
    int32_t coef[32];
    for (uint32_t k = 0; k < order; ++k)
        coef[k] = r.get_signed(16);
    const uint32_t ss = T.bps - E.lsbs * 8u + (E.cc - 1u);
    const uint32_t n = E.nres[c];
    if (F.res_base != ~0ull) { // the parse stored this channel's residuals
        ABitRC none;
        StoredRes g;
        g.init(resid + F.res_base + (uint64_t)jb.y * res_stride, n);
        restore_channel(none, g, coef, order, qshift, ss, n, out);
        return;
    }
    ABitRC rc;
    rc.init(w, b0 + E.res_bit[c], T.end * 8);
    AResidualReader g;
    g.init(E.N, ss, T.ih, T.hm, T.mk);
    restore_channel(rc, g, coef, order, qshift, ss, n, out);
}

// K4: decorrelate (alac.c:1237-1259), prepend LSBs (:930-941), wave order
// (:709-816), interleave.  Per 1024 samples of the frameset: a thread takes
// four consecutive samples of every channel (16-byte loads from the planar
// slots), writes them in output order into an LDS tile, and the block
// copies the tile out as one contiguous run of the interleaved PCM
// (consecutive threads, consecutive words), whatever the frameset's
// alignment.
constexpr uint32_t kIlvTile = 1024; // samples per tile (x 8 channels x 4 bytes = 32 KB)

__global__ __launch_bounds__(256) void k_adec_interleave(const uint32_t *__restrict__ w,
                                                         const ADTrack *__restrict__ tr,
                                                         const AFs *__restrict__ dense,
                                                         const int32_t *__restrict__ planar,
                                                         uint32_t pstride,
                                                         int32_t *__restrict__ pcm)
{
    __shared__ int32_t tile[kIlvTile * 8];
    __shared__ uint8_t inv[16]; // ALAC channel -> output position
    const AFs &F = dense[blockIdx.x];
    const ADTrack T = tr[F.track];
    const uint32_t nch = F.nch, n0 = F.n0, tid = threadIdx.x;
    static const uint8_t M[9][8] = {{0}, {0}, {0, 1}, {1, 2, 0}, {1, 2, 0, 3}, {1, 2, 0, 3, 4},
                                    {1, 2, 0, 5, 3, 4}, {1, 2, 0, 6, 3, 4, 5},
                                    {3, 4, 0, 7, 5, 6, 1, 2}};
    if (tid < 16)
        inv[tid] = (uint8_t)tid;
    __syncthreads();
    if (nch <= 8 && tid < nch)
        inv[M[nch][tid]] = (uint8_t)tid;
    __syncthreads();
    const int32_t *src = planar + F.job0 * pstride; // channel k at src + k * pstride
    int32_t *dst = pcm + F.pcm_start;
    const uint64_t b0 = F.start * 8;
    for (uint32_t base = 0; base < n0; base += kIlvTile) {
        const uint32_t cnt = min(kIlvTile, n0 - base);
        const uint32_t i0 = base + 4u * tid; // this thread's samples i0 .. i0 + 3
        if (4u * tid < cnt) {
            uint32_t ch = 0;
            for (uint32_t e = 0; e < F.nelem; ++e) {
                const AElem E = F.e[e];
                // a slot holds pstride (a multiple of 4, >= n0) values: the
                // 16-byte loads stay inside it past n0
                const int4 A = *(const int4 *)(src + (uint64_t)ch * pstride + i0);
                const int4 Bv = E.cc == 2 ? *(const int4 *)(src + (uint64_t)(ch + 1) * pstride + i0)
                                          : make_int4(0, 0, 0, 0);
                int32_t a[4] = {A.x, A.y, A.z, A.w}, b[4] = {Bv.x, Bv.y, Bv.z, Bv.w};
                const uint32_t oa = inv[ch], ob = inv[ch + 1u];
#pragma unroll
                for (uint32_t q = 0; q < 4; ++q) {
                    const uint32_t i = i0 + q;
                    if (!E.uncompressed) {
                        if (E.cc == 2 && E.lw > 0) {
                            int64_t t = (int64_t)(b[q] * (int32_t)E.lw);
                            t >>= (E.shift & 63u); // x86 sar count masking (the reference build)
                            const int32_t rs = a[q] - (int32_t)t;
                            a[q] = b[q] + rs;
                            b[q] = rs;
                        }
                        if (E.lsbs && i < E.N) {
                            const uint32_t lb = E.lsbs * 8u;
                            ABitR r;
                            r.init(w, b0 + E.lsb_bit + ((uint64_t)i * E.cc) * lb, T.end * 8);
                            const int32_t la = (int32_t)r.get(lb);
                            a[q] = (int32_t)((uint32_t)a[q] << lb) | la;
                            if (E.cc == 2) {
                                const int32_t lb2 = (int32_t)r.get(lb);
                                b[q] = (int32_t)((uint32_t)b[q] << lb) | lb2;
                            }
                        }
                    }
                    const uint32_t row = (4u * tid + q) * nch;
                    tile[row + oa] = a[q];
                    if (E.cc == 2)
                        tile[row + ob] = b[q];
                }
                ch += E.cc;
            }
        }
        __syncthreads();
        int32_t *__restrict__ out = dst + (uint64_t)base * nch;
        for (uint32_t q = tid; q < cnt * nch; q += blockDim.x)
            out[q] = tile[q];
        __syncthreads();
    }
}

// ------------------------------------------------------------------ host
thread_local std::string g_adec_err;

atg_status adfail(atg_status s, const std::string &m)
{
    g_adec_err = m;
    return s;
}

#define ADHIP(expr)                                                                         \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess)                                                               \
            return adfail(ATG_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

struct DBufA {
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

const int kADTimed = 5;
const char *kADNames[kADTimed] = {"adec_parse", "adec_chain", "adec_channel", "adec_interleave",
                                  "adec_total"};

uint32_t be32(const uint8_t *p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

// find_atom (alac.c:1261-1285) within [off, end)
bool find_atom(const uint8_t *d, uint64_t off, uint64_t end, const char *name, uint64_t &b0,
               uint64_t &b1)
{
    for (;;) {
        if (off + 8 > end)
            return false;
        const uint32_t size = be32(d + off);
        if (!std::memcmp(d + off + 4, name, 4)) {
            if (size < 8 || off + size > end)
                return false;
            b0 = off + 8;
            b1 = off + size;
            return true;
        }
        off = off + 8 + (uint32_t)(size - 8u); // skip_bytes(size - 8), unsigned
    }
}

bool find_path(const uint8_t *d, uint64_t off, uint64_t end, std::initializer_list<const char *> p,
               uint64_t &b0, uint64_t &b1)
{
    for (const char *n : p) {
        if (!find_atom(d, off, end, n, b0, b1))
            return false;
        off = b0;
        end = b1;
    }
    return true;
}

} // namespace

struct atg_alac_decoder {
    std::recursive_mutex mu; // held by every public entry point (handle_lock.h)
    int device = 0;
    hipStream_t s = nullptr;
    hipEvent_t ev[kADTimed] = {};
    float times[kADTimed] = {};
    bool have_times = false;
    DBufA data, tracks, ptrack, pstart, recs, counts, dense, jobs, planar, pcm;
    DBufA resid; // the parse's stored residuals (k_adec_channel reads them)
    std::vector<ADTrack> tr;
    std::vector<ACount> cnt;
    uint64_t total_samples = 0, total_fs = 0;
};

extern "C" {

const char *atg_alac_decoder_last_error(void) { return g_adec_err.c_str(); }

int atg_alac_read_info(const uint8_t *d, uint64_t len, atg_alac_info *info,
                       atg_alac_seekpoint *sp, uint32_t sp_cap, uint32_t *frame_sizes,
                       uint32_t fs_cap, uint32_t *n_frame_sizes)
{
    if (!d || !info)
        return AD_IO_ERROR;
    std::memset(info, 0, sizeof(*info));
    if (n_frame_sizes)
        *n_frame_sizes = 0;
    uint64_t m0, m1, a0, a1;
    if (!find_path(d, 0, len, {"moov", "trak", "mdia"}, m0, m1))
        return AD_MDIA_NOT_FOUND;
    if (!find_path(d, m0, m1, {"minf", "stbl", "stsd"}, a0, a1))
        return AD_STSD_NOT_FOUND;
    // read_alac_atom (alac.c:1354-1395): 80 bytes of fixed fields
    if (a1 - a0 < 80)
        return AD_IO_ERROR;
    const uint8_t *p = d + a0 + 8;
    const uint8_t *alac1 = p + 4, *alac2 = p + 36 + 4;
    p += 48;
    info->max_samples_per_frame = be32(p);
    info->bits_per_sample = p[5];
    info->history_multiplier = p[6];
    info->initial_history = p[7];
    info->maximum_k = p[8];
    info->channels = p[9];
    info->sample_rate = be32(p + 20);
    if (std::memcmp(alac1, "alac", 4) || std::memcmp(alac2, "alac", 4))
        return AD_INVALID_ALAC_ATOM;
    if (!find_path(d, m0, m1, {"mdhd"}, a0, a1))
        return AD_MDHD_NOT_FOUND;
    if (a1 - a0 < 4)
        return AD_IO_ERROR;
    if (d[a0] != 0)
        return AD_INVALID_MDHD_ATOM;
    if (a1 - a0 < 24)
        return AD_IO_ERROR;
    info->total_frames = be32(d + a0 + 16);
    // seektable from stts / stsc / stco (alac.c:500-672)
    uint64_t t0, t1, c0, c1, o0, o1;
    bool have = find_path(d, m0, m1, {"minf", "stbl", "stts"}, t0, t1) &&
                find_path(d, m0, m1, {"minf", "stbl", "stsc"}, c0, c1) &&
                find_path(d, m0, m1, {"minf", "stbl", "stco"}, o0, o1);
    uint32_t nt = 0, nc = 0, no = 0;
    if (have) {
        nt = t1 - t0 >= 8 ? be32(d + t0 + 4) : 0;
        nc = c1 - c0 >= 8 ? be32(d + c0 + 4) : 0;
        no = o1 - o0 >= 8 ? be32(d + o0 + 4) : 0;
        have = t1 - t0 >= 8 && (t1 - t0 - 8) / 8 >= nt && c1 - c0 >= 8 &&
               (c1 - c0 - 8) / 12 >= nc && o1 - o0 >= 8 && (o1 - o0 - 8) / 4 >= no;
    }
    if (have) {
        uint32_t sum = 0;
        uint64_t nframes = 0;
        for (uint32_t i = 0; i < nt; ++i) {
            sum += be32(d + t0 + 8 + 8 * i) * be32(d + t0 + 12 + 8 * i);
            nframes += be32(d + t0 + 8 + 8 * i);
        }
        if (sum != info->total_frames || nframes == 0 || nc == 0)
            return AD_INVALID_SEEKTABLE;
        uint32_t ti = 0, tleft = be32(d + t0 + 8);
        uint64_t left = nframes, pcm = 0, nchunks = 0;
        for (uint32_t i = 0; i < nc; ++i) {
            const uint32_t first = be32(d + c0 + 8 + 12 * i), per = be32(d + c0 + 12 + 12 * i);
            if (per == 0)
                return AD_INVALID_SEEKTABLE;
            const bool last = i + 1 >= nc;
            const uint32_t next_first = last ? 0 : be32(d + c0 + 8 + 12 * (i + 1));
            for (uint32_t j = first; last ? left > 0 : j < next_first; ++j) {
                if (left < per)
                    return AD_INVALID_SEEKTABLE;
                uint64_t chunk = 0;
                for (uint32_t k = 0; k < per; ++k) {
                    while (tleft == 0) {
                        ++ti;
                        tleft = be32(d + t0 + 8 + 8 * ti);
                    }
                    chunk += be32(d + t0 + 12 + 8 * ti);
                    --tleft;
                }
                left -= per;
                if (nchunks < no && sp && nchunks < sp_cap) {
                    sp[nchunks].pcm_frames_offset = (uint32_t)pcm;
                    sp[nchunks].file_offset = be32(d + o0 + 8 + 4 * nchunks);
                }
                pcm += (uint32_t)chunk;
                ++nchunks;
            }
        }
        if (nchunks != no)
            return AD_INVALID_SEEKTABLE;
        info->n_seekpoints = (uint32_t)nchunks;
    }
    // the stsz frameset sizes (a decoding hint; the reference never reads them)
    uint64_t z0, z1;
    if (find_path(d, m0, m1, {"minf", "stbl", "stsz"}, z0, z1) && z1 - z0 >= 12) {
        const uint32_t fixed = be32(d + z0 + 4), n = be32(d + z0 + 8);
        if (fixed == 0 && (z1 - z0 - 12) / 4 >= n) {
            if (n_frame_sizes)
                *n_frame_sizes = n;
            for (uint32_t i = 0; frame_sizes && i < n && i < fs_cap; ++i)
                frame_sizes[i] = be32(d + z0 + 12 + 4 * i);
        }
    }
    // seek_mdat (alac.c:953-971)
    uint64_t off = 0;
    for (;;) {
        if (off + 8 > len)
            return AD_NO_MDAT;
        const uint32_t size = be32(d + off);
        if (!std::memcmp(d + off + 4, "mdat", 4))
            break;
        off = off + 8 + (uint32_t)(size - 8u);
    }
    info->mdat_offset = off + 8;
    return AD_OK;
}

atg_status atg_alac_decoder_create(int device, atg_alac_decoder **out)
{
    if (!out)
        return adfail(ATG_ERR_INVALID, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return adfail(ATG_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= n)
        return adfail(ATG_ERR_INVALID, "device index out of range");
    ADHIP(hipSetDevice(device));
    atg_alac_decoder *d = new atg_alac_decoder();
    d->device = device;
    ADHIP(hipStreamCreateWithFlags(&d->s, hipStreamNonBlocking));
    for (auto &e : d->ev)
        ADHIP(hipEventCreate(&e));
    *out = d;
    return ATG_OK;
}

void atg_alac_decoder_destroy(atg_alac_decoder *d)
{
    if (!d)
        return;
    (void)hipSetDevice(d->device);
    (void)hipStreamSynchronize(d->s);
    for (DBufA *b : {&d->data, &d->tracks, &d->ptrack, &d->pstart, &d->recs, &d->counts,
                     &d->dense, &d->jobs, &d->planar, &d->pcm, &d->resid})
        b->release();
    for (auto &e : d->ev)
        (void)hipEventDestroy(e);
    (void)hipStreamDestroy(d->s);
    delete d;
}

} // extern "C"

static atg_status run_adecode(atg_alac_decoder *d, const uint8_t *d_data, uint64_t len,
                              const atg_alac_dec_track *tracks, uint32_t n,
                              atg_alac_dec_result *res)
{
    hipStream_t s = d->s;
    d->tr.assign(n, ADTrack());
    std::vector<uint32_t> ptrack;
    std::vector<uint64_t> pstart;
    for (uint32_t t = 0; t < n; ++t) {
        const atg_alac_dec_track &a = tracks[t];
        ADTrack &b = d->tr[t];
        if (a.data_offset > len || a.data_bytes > len - a.data_offset || a.start > a.data_bytes)
            return adfail(ATG_ERR_INVALID, "track data range outside the buffer");
        if (a.data_offset & 3)
            return adfail(ATG_ERR_INVALID, "track images must start 4-byte aligned");
        if (a.channels < 1 || a.channels > 8)
            return adfail(ATG_ERR_UNSUPPORTED, "channels must be 1..8");
        if (a.bits_per_sample < 1 || a.bits_per_sample > 32)
            return adfail(ATG_ERR_UNSUPPORTED, "bits per sample must be 1..32");
        b.img = a.data_offset;
        b.end = a.data_offset + a.data_bytes;
        b.start = a.data_offset + a.start;
        b.remaining = a.remaining;
        b.maxn = a.max_samples_per_frame;
        b.bps = a.bits_per_sample;
        b.hm = a.history_multiplier;
        b.ih = a.initial_history;
        b.mk = a.maximum_k;
        b.channels = a.channels;
        b.pred_first = (uint32_t)pstart.size();
        uint64_t pos = b.start;
        for (uint64_t k = 0; a.frameset_bytes && k < a.n_frameset_bytes; ++k) {
            if (pos >= b.end)
                break;
            ptrack.push_back(t);
            pstart.push_back(pos);
            pos += a.frameset_bytes[k];
        }
        b.pred_n = (uint32_t)pstart.size() - b.pred_first;
    }
    const uint64_t np = pstart.size();
    // a slot per predicted frameset for its residuals: channels x the
    // largest frame (rounded to 16 bytes per channel), when the whole batch
    // fits kResidMax; otherwise the restore decodes the residuals again
    uint32_t res_stride = 0, res_ch = 0;
    for (const ADTrack &b : d->tr) {
        res_stride = std::max(res_stride, b.maxn);
        res_ch = std::max(res_ch, b.channels);
    }
    res_stride = (res_stride + 3u) & ~3u;
    uint64_t res_fs = (uint64_t)res_ch * res_stride;
    const bool store_res = np && res_stride && np * res_fs * 4u <= kResidMax;
    if (store_res)
        ADHIP(d->resid.ensure(sizeof(int32_t) * np * res_fs));
    ADHIP(d->tracks.ensure(sizeof(ADTrack) * std::max<uint32_t>(n, 1)));
    ADHIP(d->ptrack.ensure(sizeof(uint32_t) * std::max<uint64_t>(np, 1)));
    ADHIP(d->pstart.ensure(sizeof(uint64_t) * std::max<uint64_t>(np, 1)));
    ADHIP(d->recs.ensure(sizeof(AFs) * std::max<uint64_t>(np, 1)));
    ADHIP(d->counts.ensure(sizeof(ACount) * std::max<uint32_t>(n, 1)));
    if (n)
        ADHIP(hipMemcpyAsync(d->tracks.p, d->tr.data(), sizeof(ADTrack) * n,
                             hipMemcpyHostToDevice, s));
    if (np) {
        ADHIP(hipMemcpyAsync(d->ptrack.p, ptrack.data(), sizeof(uint32_t) * np,
                             hipMemcpyHostToDevice, s));
        ADHIP(hipMemcpyAsync(d->pstart.p, pstart.data(), sizeof(uint64_t) * np,
                             hipMemcpyHostToDevice, s));
    }
    const uint32_t *w = (const uint32_t *)d_data;
    const ADTrack *dtr = (const ADTrack *)d->tracks.p;
    ADHIP(hipEventRecord(d->ev[0], s));
    if (np)
        hipLaunchKernelGGL(k_adec_parse,
                           dim3((unsigned)((np + kAdecParseLpw - 1) / kAdecParseLpw)),
                           dim3(64), 0, s, w, dtr,
                           (const uint32_t *)d->ptrack.p, (const uint64_t *)d->pstart.p, np,
                           (AFs *)d->recs.p, store_res ? (int32_t *)d->resid.p : nullptr,
                           res_fs, res_stride);
    ADHIP(hipGetLastError());
    ADHIP(hipEventRecord(d->ev[1], s));
    const dim3 tg(n); // a wave per track
    if (n)
        hipLaunchKernelGGL(k_adec_chain, tg, dim3(64), 0, s, w, dtr, n,
                           (const uint64_t *)d->pstart.p, (const AFs *)d->recs.p,
                           (ACount *)d->counts.p, 1, (AFs *)nullptr, (uint2 *)nullptr);
    ADHIP(hipGetLastError());
    d->cnt.assign(n, ACount());
    if (n)
        ADHIP(hipMemcpyAsync(d->cnt.data(), d->counts.p, sizeof(ACount) * n,
                             hipMemcpyDeviceToHost, s));
    ADHIP(hipStreamSynchronize(s));
    // every frameset of a track has the track's channel count (else the
    // walk stopped with AD_CHANNEL_MISMATCH): tracks' interleaved samples
    // back to back, pcm_base = the track's first sample
    uint64_t fb = 0, samples = 0, jb = 0;
    uint32_t pstride = 0; // planar slot per channel job: the longest frameset, 16-byte rounded
    for (uint32_t t = 0; t < n; ++t)
        pstride = std::max(pstride, d->cnt[t].max_n0);
    pstride = (pstride + 3u) & ~3u;
    for (uint32_t t = 0; t < n; ++t) {
        ADTrack &b = d->tr[t];
        b.fs_base = fb;
        b.pcm_base = samples;
        b.job_base = jb;
        fb += d->cnt[t].n_fs;
        samples += d->cnt[t].pcm_frames * b.channels;
        jb += (uint64_t)d->cnt[t].n_fs * b.channels;
    }
    d->total_samples = samples;
    d->total_fs = fb;
    ADHIP(d->dense.ensure(sizeof(AFs) * std::max<uint64_t>(fb, 1)));
    ADHIP(d->jobs.ensure(sizeof(uint2) * std::max<uint64_t>(jb, 1)));
    ADHIP(d->planar.ensure(sizeof(int32_t) * std::max<uint64_t>(jb * pstride, 1)));
    ADHIP(d->pcm.ensure(sizeof(int32_t) * std::max<uint64_t>(samples, 1)));
    if (n)
        ADHIP(hipMemcpyAsync(d->tracks.p, d->tr.data(), sizeof(ADTrack) * n,
                             hipMemcpyHostToDevice, s));
    if (n)
        hipLaunchKernelGGL(k_adec_chain, tg, dim3(64), 0, s, w, dtr, n,
                           (const uint64_t *)d->pstart.p, (const AFs *)d->recs.p,
                           (ACount *)d->counts.p, 2, (AFs *)d->dense.p, (uint2 *)d->jobs.p);
    ADHIP(hipGetLastError());
    ADHIP(hipEventRecord(d->ev[2], s));
    if (jb)
        hipLaunchKernelGGL(k_adec_channel,
                           dim3((unsigned)((jb + kAdecChannelLpw - 1) / kAdecChannelLpw)),
                           dim3(64), 0, s, w,
                           dtr, (const AFs *)d->dense.p, (const uint2 *)d->jobs.p, jb,
                           (int32_t *)d->planar.p, pstride, (const int32_t *)d->resid.p,
                           res_stride);
    ADHIP(hipGetLastError());
    ADHIP(hipEventRecord(d->ev[3], s));
    if (fb)
        hipLaunchKernelGGL(k_adec_interleave, dim3((unsigned)fb), dim3(256), 0, s, w, dtr,
                           (const AFs *)d->dense.p, (const int32_t *)d->planar.p, pstride,
                           (int32_t *)d->pcm.p);
    ADHIP(hipGetLastError());
    ADHIP(hipEventRecord(d->ev[4], s));
    ADHIP(hipStreamSynchronize(s));
    for (int k = 0; k < kADTimed - 1; ++k)
        (void)hipEventElapsedTime(&d->times[k], d->ev[k], d->ev[k + 1]);
    (void)hipEventElapsedTime(&d->times[kADTimed - 1], d->ev[0], d->ev[kADTimed - 1]);
    d->have_times = true;
    uint64_t fbase = 0;
    for (uint32_t t = 0; t < n; ++t) {
        atg_alac_dec_result &r = res[t];
        r.sample_offset = d->tr[t].pcm_base;
        r.pcm_frames = d->cnt[t].pcm_frames;
        r.first_frameset = (uint32_t)fbase;
        r.n_framesets = d->cnt[t].n_fs;
        r.status = d->cnt[t].status;
        r.channels = d->tr[t].channels;
        fbase += d->cnt[t].n_fs;
    }
    return ATG_OK;
}

extern "C" {

atg_status atg_alac_decode_device(atg_alac_decoder *d, const void *d_data, uint64_t len,
                                  const atg_alac_dec_track *tracks, uint32_t n,
                                  atg_alac_dec_result *results, const int32_t **d_pcm,
                                  uint64_t *total_samples)
{
    ATG_HANDLE_LOCK(d);
    if (!d || (!tracks && n) || (!results && n) || (!d_data && len))
        return adfail(ATG_ERR_INVALID, "NULL argument");
    if (((uintptr_t)d_data) & 3)
        return adfail(ATG_ERR_INVALID, "d_data must be 4-byte aligned");
    ADHIP(hipSetDevice(d->device));
    atg_status st = run_adecode(d, (const uint8_t *)d_data, len, tracks, n, results);
    if (st != ATG_OK)
        return st;
    if (d_pcm)
        *d_pcm = (const int32_t *)d->pcm.p;
    if (total_samples)
        *total_samples = d->total_samples;
    return ATG_OK;
}

atg_status atg_alac_decode_host(atg_alac_decoder *d, const uint8_t *data, uint64_t len,
                                const atg_alac_dec_track *tracks, uint32_t n,
                                atg_alac_dec_result *results, uint64_t *total_samples,
                                uint64_t *total_framesets)
{
    ATG_HANDLE_LOCK(d);
    if (!d || (!tracks && n) || (!results && n) || (!data && len))
        return adfail(ATG_ERR_INVALID, "NULL argument");
    ADHIP(hipSetDevice(d->device));
    ADHIP(d->data.ensure(len + 64));
    ADHIP(hipMemsetAsync((uint8_t *)d->data.p + (len & ~3ull), 0, 64, d->s));
    if (len)
        ADHIP(hipMemcpyAsync(d->data.p, data, len, hipMemcpyHostToDevice, d->s));
    atg_status st = run_adecode(d, (const uint8_t *)d->data.p, len, tracks, n, results);
    if (st != ATG_OK)
        return st;
    if (total_samples)
        *total_samples = d->total_samples;
    if (total_framesets)
        *total_framesets = d->total_fs;
    return ATG_OK;
}

atg_status atg_alac_decode_fetch(atg_alac_decoder *d, int32_t *pcm, uint64_t pcm_cap,
                                 uint32_t *frameset_frames, uint64_t *frameset_offsets,
                                 uint64_t fs_cap)
{
    ATG_HANDLE_LOCK(d);
    if (!d)
        return adfail(ATG_ERR_INVALID, "NULL decoder");
    if ((pcm && pcm_cap < d->total_samples) ||
        ((frameset_frames || frameset_offsets) && fs_cap < d->total_fs))
        return adfail(ATG_ERR_CAPACITY, "output buffer too small for the decoded batch");
    ADHIP(hipSetDevice(d->device));
    if (pcm && d->total_samples)
        ADHIP(hipMemcpyAsync(pcm, d->pcm.p, sizeof(int32_t) * d->total_samples,
                             hipMemcpyDeviceToHost, d->s));
    std::vector<AFs> fs;
    if ((frameset_frames || frameset_offsets) && d->total_fs) {
        fs.resize(d->total_fs);
        ADHIP(hipMemcpyAsync(fs.data(), d->dense.p, sizeof(AFs) * d->total_fs,
                             hipMemcpyDeviceToHost, d->s));
    }
    ADHIP(hipStreamSynchronize(d->s));
    for (uint64_t i = 0; i < fs.size(); ++i) {
        if (frameset_frames)
            frameset_frames[i] = fs[i].n0;
        if (frameset_offsets)
            frameset_offsets[i] = fs[i].start - d->tr[fs[i].track].img;
    }
    return ATG_OK;
}

int atg_alac_decoder_kernel_times(atg_alac_decoder *d, const char **names, float *ms, int cap)
{
    ATG_HANDLE_LOCK(d);
    if (!d || !d->have_times)
        return 0;
    const int k = cap < kADTimed ? cap : kADTimed;
    for (int i = 0; i < k; ++i) {
        if (names)
            names[i] = kADNames[i];
        if (ms)
            ms[i] = d->times[i];
    }
    return k;
}

} // extern "C"
