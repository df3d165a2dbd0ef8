// engine.hip — host side of libatgpu: the C ABI in include/atgpu.h.
//
// One engine per process and device (the reference runs one encoder per
// process, ExecProgressQueue; src/encoders/flac.c keeps no global state).
// The engine owns two HIP streams: the encoder chain runs on `main`, the
// per-track MD5 chain (a serial hash per track) runs concurrently on `aux`
// and joins before the stream headers are written.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/atgpu.h"
#include "flac_dev.h"
#include "launch.h"

// timing experiments only (tools/gpu_exp.sh); 0 in every product build
#ifndef ATG_EXP
#define ATG_EXP 0
#endif

namespace {

thread_local std::string g_err;

atg_status fail(atg_status s, const std::string &msg)
{
    g_err = msg;
    return s;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t e_ = (expr);                                                         \
        if (e_ != hipSuccess)                                                           \
            return fail(ATG_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

struct DevBuf {
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
        size_t want = std::max<size_t>(bytes, 256);
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

const int kNumTimed = 8;
const char *kTimedNames[kNumTimed] = {"lpc_analyze", "subframe_search", "frame_decide",
                                      "track_scan",  "frame_pack",      "track_md5",
                                      "stream_header", "total"};

// CRC-16 (0x8005) slicing tables t16[k][b] = CRC of byte b followed by k
// zero bytes, the CRC-8 table, and "advance by 2^m zero bytes" matrices
void build_crc_tables(uint32_t t16[4][256], uint32_t *t8, uint16_t adv[24][16])
{
    for (uint32_t b = 0; b < 256; ++b) {
        uint32_t c = b << 8, c8 = b;
        for (int i = 0; i < 8; ++i) {
            c = (c & 0x8000u) ? ((c << 1) ^ 0x8005u) : (c << 1);
            c8 = (c8 & 0x80u) ? ((c8 << 1) ^ 0x07u) : (c8 << 1);
        }
        t16[0][b] = c & 0xFFFFu;
        t8[b] = c8 & 0xFFu;
    }
    for (int k = 1; k < 4; ++k)
        for (uint32_t b = 0; b < 256; ++b) {
            const uint32_t c = t16[k - 1][b];
            t16[k][b] = ((c << 8) ^ t16[0][(c >> 8) & 0xFFu]) & 0xFFFFu;
        }
    // m = 0: one zero byte
    for (int i = 0; i < 16; ++i) {
        uint32_t s = 1u << i;
        s = ((s << 8) ^ t16[0][(s >> 8) & 0xFFu]) & 0xFFFFu;
        adv[0][i] = (uint16_t)s;
    }
    for (int m = 1; m < 24; ++m) {
        for (int i = 0; i < 16; ++i) {
            // apply adv[m-1] twice to basis vector i
            uint32_t v = adv[m - 1][i], r = 0;
            for (int j = 0; j < 16; ++j)
                if ((v >> j) & 1u)
                    r ^= adv[m - 1][j];
            adv[m][i] = (uint16_t)r;
        }
    }
}

} // namespace

struct atg_engine {
    int device = 0;
    hipStream_t s_main = nullptr, s_aux = nullptr;
    hipEvent_t ev[2 * kNumTimed] = {};
    hipEvent_t ev_tables = nullptr, ev_md5 = nullptr;
    DevBuf frames, tracks, order, windows, coef, shift, est, sub, fdesc, tout, err;
    DevBuf h_pcm, h_out; // staging for the host-memory API
    std::map<uint32_t, uint32_t> win_off;
    std::vector<double> win_host;
    size_t win_uploaded = 0;
    float times[kNumTimed] = {};
    bool have_times = false;
    // plan cache: a batch with the same geometry as the previous call reuses
    // the plan and the frame/track tables already on the device
    std::vector<uint8_t> plan_key, plan_key_pending;
    void *plan_cached = nullptr; // Plan*
};

namespace {

struct Plan {
    FlacParams p;
    std::vector<FrameInfo> frames;
    std::vector<TrackInfo> tracks;
    std::vector<uint32_t> track_frame_pos; // first position in track order
    std::vector<uint32_t> order;           // track-order position -> frame id
    uint64_t frame_bound = 0;               // worst-case frame bytes
    uint64_t out_bytes = 0;
    uint32_t n_reg_prefix = 0; // leading frame ids of 4096 samples at 4-frame-aligned starts
};

uint32_t qlp_precision_for(uint32_t n)
{
    return n <= 192 ? 7 : n <= 384 ? 8 : n <= 576 ? 9 : n <= 1152 ? 10 : n <= 2304 ? 11
         : n <= 4608 ? 12 : 13;
}

atg_status make_plan(const atg_flac_options *o, const atg_track *tracks, uint32_t n_tracks,
                     uint32_t channels, uint32_t bps, uint32_t rate, Plan &pl)
{
    if (!o)
        return fail(ATG_ERR_INVALID, "options is NULL");
    if (channels < 1 || channels > 8)
        return fail(ATG_ERR_INVALID, "channels must be 1..8");
    if (bps < 4 || bps > 24)
        return fail(ATG_ERR_UNSUPPORTED, "bits_per_sample must be 4..24 on the GPU path");
    if (o->block_size == 0)
        return fail(ATG_ERR_INVALID, "block_size must be > 0");
    if (o->block_size > ATG_MAX_BLOCK)
        return fail(ATG_ERR_UNSUPPORTED, "block_size > 4096 not supported on the GPU path");
    if (o->max_lpc_order > ATG_MAX_LPC)
        return fail(ATG_ERR_INVALID, "max_lpc_order must be <= 32");
    if (o->max_residual_partition_order > ATG_MAX_PORDER)
        return fail(ATG_ERR_UNSUPPORTED, "max_residual_partition_order > 6 not supported");
    if (o->padding_size > 0xFFFFFFu)
        return fail(ATG_ERR_INVALID, "padding_size must fit in 24 bits");
    if (rate == 0)
        return fail(ATG_ERR_INVALID, "sample_rate must be > 0");
    FlacParams &p = pl.p;
    std::memset(&p, 0, sizeof(p));
    p.block_size = o->block_size;
    p.max_lpc_order = o->max_lpc_order;
    p.max_porder = o->max_residual_partition_order;
    p.qlp_precision = qlp_precision_for(o->block_size);
    p.max_rice = bps <= 16 ? 14 : 30;
    p.mid_side = o->mid_side != 0;
    p.adaptive_mid_side = o->adaptive_mid_side != 0;
    p.exhaustive = o->exhaustive_model_search != 0;
    p.try_verbatim = !o->disable_verbatim_subframes;
    p.try_constant = !o->disable_constant_subframes;
    p.try_fixed = !o->disable_fixed_subframes;
    p.try_lpc = !(o->disable_lpc_subframes || o->max_lpc_order == 0);
    p.channels = channels;
    p.bps = bps;
    p.sample_rate = rate;
    p.n_cand = (channels == 2 && (p.mid_side || p.adaptive_mid_side)) ? 4 : channels;
    p.n_tracks = n_tracks;
    const uint32_t M = p.max_lpc_order;
    p.coef_row = std::max<uint32_t>(2, (M + 1u) & ~1u);
    p.coef_stride = std::max<uint32_t>(1, M) * p.coef_row;
    p.padding_size = o->padding_size;
    p.header_bytes = 4 + 4 + 34 + 4 + 4 + 29 + 4 + 4 + o->padding_size;

    // worst-case frame: verbatim subframes (+1 bit side channel) + headers;
    // without VERBATIM a predictor may exceed that, so bound by LDS instead
    const uint64_t B = o->block_size;
    const uint64_t nsub = channels;
    uint64_t fb = 16 + nsub * ((8 + 32 + B * (bps + 1) + 7) / 8) + 2;
    if (!p.try_verbatim)
        fb = std::max<uint64_t>(fb, 120 * 1024);
    pl.frame_bound = fb;
    p.frame_lds_words = (uint32_t)((fb + 3) / 4 + 2);
    if (p.frame_lds_words * 4ull > 128 * 1024)
        return fail(ATG_ERR_UNSUPPORTED, "frame image exceeds the pack kernel's LDS budget");

    // frame table: every frame's length, in track order
    pl.tracks.resize(n_tracks);
    std::vector<uint32_t> lens;
    std::vector<uint32_t> owner;
    for (uint32_t t = 0; t < n_tracks; ++t) {
        const atg_track &tr = tracks[t];
        TrackInfo &ti = pl.tracks[t];
        ti.pcm_start = tr.pcm_offset;
        ti.pcm_frames = tr.pcm_frames;
        ti.first_pos = (uint32_t)lens.size();
        if (tr.frame_sizes) {
            uint64_t sum = 0;
            for (uint64_t k = 0; k < tr.n_frame_sizes; ++k) {
                const uint32_t n = tr.frame_sizes[k];
                if (n == 0 || n > ATG_MAX_BLOCK)
                    return fail(n ? ATG_ERR_UNSUPPORTED : ATG_ERR_INVALID,
                                "explicit frame sizes must be 1..4096");
                sum += n;
                lens.push_back(n);
                owner.push_back(t);
            }
            if (sum != tr.pcm_frames)
                return fail(ATG_ERR_INVALID, "frame sizes do not sum to pcm_frames");
        } else {
            for (uint64_t done = 0; done < tr.pcm_frames; done += B) {
                lens.push_back((uint32_t)std::min<uint64_t>(B, tr.pcm_frames - done));
                owner.push_back(t);
            }
        }
        ti.n_frames = (uint32_t)(lens.size() - ti.first_pos);
        if (lens.size() > 0x7FFFFFFFull)
            return fail(ATG_ERR_INVALID, "too many frames in one batch");
    }
    // frame ids: block_size-long frames first, the rest after, so LPC waves
    // over 64 frames share one window (uniform loads)
    const size_t nfr = lens.size();
    pl.order.resize(nfr);
    pl.frames.resize(nfr);
    pl.track_frame_pos.resize(n_tracks);
    size_t n_full = 0;
    for (size_t i = 0; i < nfr; ++i)
        n_full += lens[i] == B ? 1 : 0;
    size_t id_full = 0, id_other = n_full;
    std::vector<uint64_t> start(n_tracks, 0);
    std::vector<uint32_t> idx(n_tracks, 0);
    for (size_t i = 0; i < nfr; ++i) {
        const uint32_t t = owner[i];
        const size_t id = lens[i] == B ? id_full++ : id_other++;
        pl.order[i] = (uint32_t)id;
        FrameInfo &f = pl.frames[id];
        f.pcm_start = pl.tracks[t].pcm_start + start[t];
        f.n = lens[i];
        f.track = t;
        f.index = idx[t]++;
        f.win_off = 0;
        start[t] += lens[i];
    }
    // frames longer than block_size (explicit sizes) widen the bound
    uint32_t maxn = 0;
    for (size_t i = 0; i < nfr; ++i)
        maxn = std::max(maxn, lens[i]);
    if (maxn > B) {
        fb = 16 + nsub * ((8 + 32 + (uint64_t)maxn * (bps + 1) + 7) / 8) + 2;
        if (!p.try_verbatim)
            fb = std::max<uint64_t>(fb, 120 * 1024);
        pl.frame_bound = fb;
        p.frame_lds_words = (uint32_t)((fb + 3) / 4 + 2);
        if (p.frame_lds_words * 4ull > 128 * 1024)
            return fail(ATG_ERR_UNSUPPORTED, "frame image exceeds the pack kernel's LDS budget");
    }
    uint64_t out = 0;
    for (uint32_t t = 0; t < n_tracks; ++t) {
        TrackInfo &ti = pl.tracks[t];
        pl.track_frame_pos[t] = ti.first_pos;
        ti.out_base = out;
        out += p.header_bytes + (uint64_t)ti.n_frames * fb;
        out = (out + 15) & ~15ull;
    }
    p.n_frames = (uint32_t)pl.frames.size();
    pl.out_bytes = out;
    // register-staged packer (K5): 16-bit stereo mid/side, 4096-sample
    // frames whose first pair is 16-byte aligned (with an aligned base)
    pl.n_reg_prefix = 0;
    if (channels == 2 && p.n_cand == 4 && bps <= 16 && B == ATG_MAX_BLOCK)
        while (pl.n_reg_prefix < p.n_frames && pl.frames[pl.n_reg_prefix].n == ATG_MAX_BLOCK &&
               (pl.frames[pl.n_reg_prefix].pcm_start & 3u) == 0)
            pl.n_reg_prefix++;
    return ATG_OK;
}

// Tukey(0.5) window exactly as flacenc_window_signal (flac.c:1139-1161),
// computed with the host libm cos so the bits match the reference build.
void tukey(uint32_t N, double *w)
{
    const double alpha = 0.5;
    const unsigned window1 = (unsigned)(alpha * (N - 1)) / 2;
    const unsigned window2 = (unsigned)((N - 1) * (1.0 - (alpha / 2.0)));
    for (unsigned n = 0; n < N; n++) {
        if (n <= window1)
            w[n] = 0.5 * (1.0 + std::cos(M_PI * (((2 * n) / (alpha * (N - 1))) - 1.0)));
        else if (n <= window2)
            w[n] = 1.0;
        else
            w[n] = 0.5 * (1.0 + std::cos(M_PI * (((2.0 * n) / (alpha * (N - 1))) -
                                                 (2.0 / alpha) + 1.0)));
    }
}

atg_status prepare_windows(atg_engine *e, Plan &pl)
{
    if (!pl.p.try_lpc)
        return ATG_OK;
    const uint32_t M = pl.p.max_lpc_order;
    for (FrameInfo &f : pl.frames) {
        if (f.n <= M + 1)
            continue;
        auto it = e->win_off.find(f.n);
        if (it == e->win_off.end()) {
            const uint32_t off = (uint32_t)e->win_host.size();
            e->win_host.resize(off + f.n);
            tukey(f.n, e->win_host.data() + off);
            it = e->win_off.emplace(f.n, off).first;
        }
        f.win_off = it->second;
    }
    if (e->win_host.size() != e->win_uploaded) {
        HIP_TRY(e->windows.ensure(e->win_host.size() * sizeof(double) + 64));
        HIP_TRY(hipMemcpyAsync(e->windows.p, e->win_host.data(),
                               e->win_host.size() * sizeof(double), hipMemcpyHostToDevice,
                               e->s_main));
        e->win_uploaded = e->win_host.size();
    }
    return ATG_OK;
}

atg_status run_batch(atg_engine *e, Plan &pl, bool upload, const void *d_pcm, int fmt,
                     uint8_t *d_out, uint64_t out_cap, std::vector<TrackOut> &tout_h,
                     std::vector<FrameDesc> *fdesc_h)
{
    FlacParams &p = pl.p;
    if (pl.out_bytes > out_cap)
        return fail(ATG_ERR_CAPACITY, "output buffer too small for this batch");
    p.n_reg_frames = (fmt == ATG_PCM_S16 && ((uintptr_t)d_pcm & 15u) == 0) ? pl.n_reg_prefix : 0u;
    HIP_TRY(hipSetDevice(e->device));
    atg_status st = prepare_windows(e, pl);
    if (st != ATG_OK)
        return st;
    const size_t nf = pl.frames.size(), nt = pl.tracks.size();
    {
        void *f0 = e->frames.p, *t0 = e->tracks.p, *o0 = e->order.p;
        HIP_TRY(e->frames.ensure(nf * sizeof(FrameInfo)));
        HIP_TRY(e->tracks.ensure(nt * sizeof(TrackInfo)));
        HIP_TRY(e->order.ensure(nf * sizeof(uint32_t)));
        if (f0 != e->frames.p || t0 != e->tracks.p || o0 != e->order.p)
            upload = true;
    }
    HIP_TRY(e->coef.ensure(nf * p.n_cand * p.coef_stride * sizeof(int16_t)));
    HIP_TRY(e->shift.ensure(nf * p.n_cand * std::max<uint32_t>(1, p.max_lpc_order)));
    HIP_TRY(e->est.ensure(nf * p.n_cand));
    HIP_TRY(e->sub.ensure(nf * p.n_cand * sizeof(SubDesc)));
    HIP_TRY(e->fdesc.ensure(nf * sizeof(FrameDesc)));
    HIP_TRY(e->tout.ensure(nt * sizeof(TrackOut)));
    HIP_TRY(e->err.ensure(sizeof(uint32_t)));
    if (upload && nf)
        HIP_TRY(hipMemcpyAsync(e->frames.p, pl.frames.data(), nf * sizeof(FrameInfo),
                               hipMemcpyHostToDevice, e->s_main));
    if (upload && nt)
        HIP_TRY(hipMemcpyAsync(e->tracks.p, pl.tracks.data(), nt * sizeof(TrackInfo),
                               hipMemcpyHostToDevice, e->s_main));
    if (upload && nf)
        HIP_TRY(hipMemcpyAsync(e->order.p, pl.order.data(), nf * sizeof(uint32_t),
                               hipMemcpyHostToDevice, e->s_main));
    HIP_TRY(hipMemsetAsync(e->err.p, 0, sizeof(uint32_t), e->s_main));
    HIP_TRY(hipEventRecord(e->ev_tables, e->s_main));

    const FrameInfo *dfr = (const FrameInfo *)e->frames.p;
    const TrackInfo *dtr = (const TrackInfo *)e->tracks.p;
    TrackOut *dto = (TrackOut *)e->tout.p;
    uint32_t *derr = (uint32_t *)e->err.p;

    HIP_TRY(hipEventRecord(e->ev[14], e->s_main));
    HIP_TRY(hipEventRecord(e->ev[0], e->s_main));
    HIP_TRY(launch_lpc_analyze(p, d_pcm, fmt, dfr, (const double *)e->windows.p,
                               (int16_t *)e->coef.p, (int8_t *)e->shift.p,
                               (uint8_t *)e->est.p, e->s_main));
    HIP_TRY(hipEventRecord(e->ev[1], e->s_main));
    // MD5 chains on the aux stream, concurrent with the search and pack
    // kernels.  They start after the LPC kernel: its grid is only ~1.3
    // waves per SIMD deep, so a SIMD shared with a (high-priority) chain
    // would leave straggler waves; the search/pack grids are >60 deep and
    // absorb it.
#if ATG_EXP == 10
    hipStream_t s_md5 = e->s_main; // timing experiment: MD5 alone, serialized
#else
    hipStream_t s_md5 = e->s_aux;
#endif
    HIP_TRY(hipStreamWaitEvent(s_md5, e->ev[1], 0));
    HIP_TRY(hipEventRecord(e->ev[2 * 5], s_md5));
    HIP_TRY(launch_track_md5(p, d_pcm, fmt, dtr, dto, s_md5));
    HIP_TRY(hipEventRecord(e->ev[2 * 5 + 1], s_md5));
    HIP_TRY(hipEventRecord(e->ev_md5, s_md5));
    HIP_TRY(hipEventRecord(e->ev[2], e->s_main));
    HIP_TRY(launch_subframe_search(p, d_pcm, fmt, dfr, (const int16_t *)e->coef.p,
                                   (const int8_t *)e->shift.p, (const uint8_t *)e->est.p,
                                   (SubDesc *)e->sub.p, derr, e->s_main));
    HIP_TRY(hipEventRecord(e->ev[3], e->s_main));
    HIP_TRY(hipEventRecord(e->ev[4], e->s_main));
    HIP_TRY(launch_frame_decide(p, dfr, (const SubDesc *)e->sub.p, (FrameDesc *)e->fdesc.p,
                                e->s_main));
    HIP_TRY(hipEventRecord(e->ev[5], e->s_main));
    HIP_TRY(hipEventRecord(e->ev[6], e->s_main));
    HIP_TRY(launch_track_scan(p, dtr, (const uint32_t *)e->order.p, (FrameDesc *)e->fdesc.p,
                              dto, e->s_main));
    HIP_TRY(hipEventRecord(e->ev[7], e->s_main));
    HIP_TRY(hipEventRecord(e->ev[8], e->s_main));
    HIP_TRY(launch_frame_pack(p, d_pcm, fmt, dfr, dtr, (const SubDesc *)e->sub.p,
                              (const FrameDesc *)e->fdesc.p, d_out, derr, e->s_main));
    HIP_TRY(hipEventRecord(e->ev[9], e->s_main));
    HIP_TRY(hipStreamWaitEvent(e->s_main, e->ev_md5, 0));
    HIP_TRY(hipEventRecord(e->ev[12], e->s_main));
    HIP_TRY(launch_stream_header(p, dtr, dto, d_out, e->s_main));
    HIP_TRY(hipEventRecord(e->ev[13], e->s_main));
    HIP_TRY(hipEventRecord(e->ev[15], e->s_main));

    tout_h.resize(nt);
    uint32_t err_h = 0;
    if (nt)
        HIP_TRY(hipMemcpyAsync(tout_h.data(), dto, nt * sizeof(TrackOut), hipMemcpyDeviceToHost,
                               e->s_main));
    if (fdesc_h) {
        fdesc_h->resize(nf);
        if (nf)
            HIP_TRY(hipMemcpyAsync(fdesc_h->data(), e->fdesc.p, nf * sizeof(FrameDesc),
                                   hipMemcpyDeviceToHost, e->s_main));
    }
    HIP_TRY(hipMemcpyAsync(&err_h, derr, sizeof(uint32_t), hipMemcpyDeviceToHost, e->s_main));
    HIP_TRY(hipStreamSynchronize(e->s_main));
    for (int k = 0; k < kNumTimed; ++k) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, e->ev[2 * k], e->ev[2 * k + 1]) != hipSuccess)
            ms = 0.f;
        e->times[k] = ms;
    }
    e->have_times = true;
    if (err_h & 1u)
        return fail(ATG_ERR_UNSUPPORTED, "frame longer than the GPU block limit");
#if ATG_EXP != 0
    err_h = 0; // timing experiments do not produce valid streams
#endif
    if (err_h)
        return fail(ATG_ERR_DEVICE, "GPU consistency check failed (code " +
                                        std::to_string(err_h) + ")");
    return ATG_OK;
}

void fill_results(const Plan &pl, const std::vector<TrackOut> &to, atg_track_result *res,
                  const std::vector<FrameDesc> *fd, uint64_t *frame_offsets,
                  uint32_t *frame_pcm)
{
    for (size_t t = 0; t < pl.tracks.size(); ++t) {
        const TrackInfo &ti = pl.tracks[t];
        atg_track_result &r = res[t];
        r.out_offset = ti.out_base;
        r.bytes = to[t].bytes;
        r.first_frame = pl.track_frame_pos[t];
        r.n_frames = ti.n_frames;
        r.min_frame_bytes = to[t].min_fs;
        r.max_frame_bytes = to[t].max_fs;
        std::memcpy(r.md5, to[t].md5, 16);
        r.status = 0;
        r.reserved = 0;
        if (fd) {
            for (uint32_t i = 0; i < ti.n_frames; ++i) {
                const uint32_t f = pl.order[ti.first_pos + i];
                if (frame_offsets)
                    frame_offsets[r.first_frame + i] = (*fd)[f].out_off;
                if (frame_pcm)
                    frame_pcm[r.first_frame + i] = pl.frames[f].n;
            }
        }
    }
}

std::vector<uint8_t> plan_key(const atg_flac_options *o, const atg_track *tracks,
                              uint32_t n_tracks, uint32_t channels, uint32_t bps, uint32_t rate)
{
    std::vector<uint8_t> k;
    auto put = [&k](const void *p, size_t n) {
        const uint8_t *b = (const uint8_t *)p;
        k.insert(k.end(), b, b + n);
    };
    put(o, sizeof(*o));
    put(&n_tracks, 4);
    put(&channels, 4);
    put(&bps, 4);
    put(&rate, 4);
    for (uint32_t t = 0; t < n_tracks; ++t) {
        put(&tracks[t].pcm_offset, 8);
        put(&tracks[t].pcm_frames, 8);
        put(&tracks[t].n_frame_sizes, 8);
        if (tracks[t].frame_sizes)
            put(tracks[t].frame_sizes, tracks[t].n_frame_sizes * 4);
    }
    return k;
}

// plan for this call: the cached one when the geometry repeats (fresh=false:
// device tables are current), else a new plan that replaces the cache
atg_status get_plan(atg_engine *e, const atg_flac_options *o, const atg_track *tracks,
                    uint32_t n_tracks, uint32_t channels, uint32_t bps, uint32_t rate,
                    Plan *&pl, bool &fresh)
{
    std::vector<uint8_t> key = plan_key(o, tracks, n_tracks, channels, bps, rate);
    if (e->plan_cached && key == e->plan_key) {
        pl = (Plan *)e->plan_cached;
        fresh = false;
        return ATG_OK;
    }
    Plan *np = new Plan();
    atg_status st = make_plan(o, tracks, n_tracks, channels, bps, rate, *np);
    if (st != ATG_OK) {
        delete np;
        return st;
    }
    delete (Plan *)e->plan_cached;
    e->plan_cached = np;
    e->plan_key.clear();            // valid only once its tables are uploaded
    e->plan_key_pending.swap(key);  // committed by commit_plan()
    pl = np;
    fresh = true;
    return ATG_OK;
}

void commit_plan(atg_engine *e, bool fresh)
{
    if (fresh)
        e->plan_key.swap(e->plan_key_pending);
}

} // namespace

extern "C" {

int atg_abi_version(void) { return ATG_ABI_VERSION; }

const char *atg_last_error(void) { return g_err.c_str(); }

atg_status atg_engine_create(int device, atg_engine **out)
{
    if (!out)
        return fail(ATG_ERR_INVALID, "out is NULL");
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return fail(ATG_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= n)
        return fail(ATG_ERR_INVALID, "device index out of range");
    HIP_TRY(hipSetDevice(device));
    atg_engine *e = new atg_engine();
    e->device = device;
    HIP_TRY(hipStreamCreateWithFlags(&e->s_main, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&e->s_aux, hipStreamNonBlocking));
    for (auto &ev : e->ev)
        HIP_TRY(hipEventCreate(&ev));
    HIP_TRY(hipEventCreateWithFlags(&e->ev_tables, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&e->ev_md5, hipEventDisableTiming));
    static uint32_t t16[4][256], t8[256];
    static uint16_t adv[24][16];
    build_crc_tables(t16, t8, adv);
    HIP_TRY(upload_crc_tables(&adv[0][0], &t16[0][0], t8));
    *out = e;
    return ATG_OK;
}

void atg_engine_destroy(atg_engine *e)
{
    if (!e)
        return;
    (void)hipSetDevice(e->device);
    (void)hipStreamSynchronize(e->s_main);
    (void)hipStreamSynchronize(e->s_aux);
    for (DevBuf *b : {&e->frames, &e->tracks, &e->order, &e->windows, &e->coef, &e->shift, &e->est,
                      &e->sub, &e->fdesc, &e->tout, &e->err, &e->h_pcm, &e->h_out})
        b->release();
    for (auto &ev : e->ev)
        (void)hipEventDestroy(ev);
    (void)hipEventDestroy(e->ev_tables);
    (void)hipEventDestroy(e->ev_md5);
    delete (Plan *)e->plan_cached;
    (void)hipStreamDestroy(e->s_main);
    (void)hipStreamDestroy(e->s_aux);
    delete e;
}

atg_status atg_flac_batch_bounds(const atg_flac_options *opts, const atg_track *tracks,
                                 uint32_t n_tracks, uint32_t channels, uint32_t bps,
                                 uint64_t *total_frames, uint64_t *out_bytes)
{
    Plan pl;
    atg_status st = make_plan(opts, tracks, n_tracks, channels, bps, 44100, pl);
    if (st != ATG_OK)
        return st;
    if (total_frames)
        *total_frames = pl.frames.size();
    if (out_bytes)
        *out_bytes = pl.out_bytes;
    return ATG_OK;
}

atg_status atg_flac_encode_device(atg_engine *e, const atg_flac_options *opts,
                                  const void *d_pcm, atg_pcm_format format,
                                  const atg_track *tracks, uint32_t n_tracks,
                                  uint32_t channels, uint32_t bps, uint32_t rate, void *d_out,
                                  uint64_t out_cap, atg_track_result *results)
{
    if (!e || (!tracks && n_tracks) || (!results && n_tracks))
        return fail(ATG_ERR_INVALID, "NULL argument");
    if (format == ATG_PCM_S16 && bps > 16)
        return fail(ATG_ERR_INVALID, "S16 container with bits_per_sample > 16");
    Plan *pl = nullptr;
    bool fresh = true;
    atg_status st = get_plan(e, opts, tracks, n_tracks, channels, bps, rate, pl, fresh);
    if (st != ATG_OK)
        return st;
    std::vector<TrackOut> to;
    st = run_batch(e, *pl, fresh, d_pcm, (int)format, (uint8_t *)d_out, out_cap, to, nullptr);
    if (st != ATG_OK) {
        e->plan_key.clear(); // tables may not be on the device
        return st;
    }
    commit_plan(e, fresh);
    fill_results(*pl, to, results, nullptr, nullptr, nullptr);
    return ATG_OK;
}

atg_status atg_flac_encode_host(atg_engine *e, const atg_flac_options *opts, const void *pcm,
                                atg_pcm_format format, const atg_track *tracks,
                                uint32_t n_tracks, uint32_t channels, uint32_t bps,
                                uint32_t rate, uint8_t *out, uint64_t out_cap,
                                atg_track_result *results, uint64_t *frame_offsets,
                                uint32_t *frame_pcm_frames)
{
    if (!e || (!tracks && n_tracks) || (!results && n_tracks))
        return fail(ATG_ERR_INVALID, "NULL argument");
    if (format == ATG_PCM_S16 && bps > 16)
        return fail(ATG_ERR_INVALID, "S16 container with bits_per_sample > 16");
    Plan *plp = nullptr;
    bool fresh = true;
    atg_status st = get_plan(e, opts, tracks, n_tracks, channels, bps, rate, plp, fresh);
    if (st != ATG_OK)
        return st;
    Plan &pl = *plp;
    if (pl.out_bytes > out_cap) {
        e->plan_key.clear();
        return fail(ATG_ERR_CAPACITY, "output buffer too small for this batch");
    }
    uint64_t samples = 0;
    for (uint32_t t = 0; t < n_tracks; ++t)
        samples = std::max<uint64_t>(samples, (tracks[t].pcm_offset + tracks[t].pcm_frames) *
                                                  channels);
    const size_t elem = format == ATG_PCM_S16 ? 2 : 4;
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(e->h_pcm.ensure(samples * elem + 16));
    HIP_TRY(e->h_out.ensure(pl.out_bytes + 16));
    if (samples)
        HIP_TRY(hipMemcpyAsync(e->h_pcm.p, pcm, samples * elem, hipMemcpyHostToDevice,
                               e->s_main));
    std::vector<TrackOut> to;
    std::vector<FrameDesc> fd;
    st = run_batch(e, pl, fresh, e->h_pcm.p, (int)format, (uint8_t *)e->h_out.p, e->h_out.cap,
                   to, &fd);
    if (st != ATG_OK) {
        e->plan_key.clear(); // tables may not be on the device
        return st;
    }
    for (size_t t = 0; t < pl.tracks.size(); ++t)
        if (to[t].bytes)
            HIP_TRY(hipMemcpyAsync(out + pl.tracks[t].out_base,
                                   (uint8_t *)e->h_out.p + pl.tracks[t].out_base, to[t].bytes,
                                   hipMemcpyDeviceToHost, e->s_main));
    HIP_TRY(hipStreamSynchronize(e->s_main));
    commit_plan(e, fresh);
    fill_results(pl, to, results, &fd, frame_offsets, frame_pcm_frames);
    return ATG_OK;
}

int atg_engine_kernel_times(atg_engine *e, const char **names, float *ms, int cap)
{
    if (!e || !e->have_times)
        return 0;
    const int n = cap < kNumTimed ? cap : kNumTimed;
    for (int k = 0; k < n; ++k) {
        if (names)
            names[k] = kTimedNames[k];
        if (ms)
            ms[k] = e->times[k];
    }
    return n;
}

atg_status atg_device_alloc(atg_engine *e, uint64_t bytes, void **d_ptr)
{
    if (!e || !d_ptr)
        return fail(ATG_ERR_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipMalloc(d_ptr, bytes ? bytes : 1));
    return ATG_OK;
}

atg_status atg_device_free(atg_engine *e, void *d_ptr)
{
    if (!e)
        return fail(ATG_ERR_INVALID, "NULL engine");
    HIP_TRY(hipSetDevice(e->device));
    if (d_ptr)
        HIP_TRY(hipFree(d_ptr));
    return ATG_OK;
}

atg_status atg_copy_to_device(atg_engine *e, void *d_dst, const void *src, uint64_t bytes)
{
    if (!e)
        return fail(ATG_ERR_INVALID, "NULL engine");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipMemcpy(d_dst, src, bytes, hipMemcpyHostToDevice));
    return ATG_OK;
}

atg_status atg_copy_to_host(atg_engine *e, void *dst, const void *d_src, uint64_t bytes)
{
    if (!e)
        return fail(ATG_ERR_INVALID, "NULL engine");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipMemcpy(dst, d_src, bytes, hipMemcpyDeviceToHost));
    return ATG_OK;
}

} // extern "C"
