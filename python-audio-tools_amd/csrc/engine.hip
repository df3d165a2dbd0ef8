// engine.hip — host side of libatgpu: the C ABI in include/atgpu.h.
//
// One engine per process and device (the reference runs one encoder per
// process, ExecProgressQueue; src/encoders/flac.c keeps no global state).
// The engine owns two HIP streams: the encoder chain runs on `main`, the
// per-track MD5 chain (a serial hash per track) runs concurrently on `aux`
// and joins before the stream headers are written.
#include "handle_lock.h"
#include <hip/hip_runtime.h>

#include <sched.h>

#include <algorithm>
#include <array>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/atgpu.h"
#include "flac_dev.h"
#include "launch.h"
#include "md5_cpu.h"

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
void build_crc_tables(uint32_t t16[4][256], uint32_t *t8, uint16_t adv[24][16],
                      uint16_t advq[kCrcQ][6][16])
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
    // advq[q - 1][s]: 4 q 2^s zero bytes = (4 bytes)^q, squared s times
    auto apply = [](const uint16_t *a, uint32_t v) {
        uint32_t r = 0;
        for (int j = 0; j < 16; ++j)
            if ((v >> j) & 1u)
                r ^= a[j];
        return (uint16_t)r;
    };
    for (int i = 0; i < 16; ++i)
        advq[0][0][i] = adv[2][i];
    for (int q = 1; q < kCrcQ; ++q)
        for (int i = 0; i < 16; ++i)
            advq[q][0][i] = apply(adv[2], advq[q - 1][0][i]);
    for (int q = 0; q < kCrcQ; ++q)
        for (int s = 1; s < 6; ++s)
            for (int i = 0; i < 16; ++i)
                advq[q][s][i] = apply(advq[q][s - 1], advq[q][s - 1][i]);
}

} // namespace

namespace {
struct Plan;
struct HostJob;
}

// One batch in flight: its device workspace, its MD5/header stream and the
// pinned host copies of its results.  Two slots let batch k's MD5 chains and
// stream headers (on the slot's aux stream) run under batch k+1's search.
struct EncSlot {
    DevBuf frames, tracks, order, coef, shift, est, sub, fdesc, tout, err;
    DevBuf rice_big, scratch; // large-frame path (flac_big.hip)
    DevBuf slow;              // [count, pad x3][list]: candidates the 16-bit search hands over
    hipStream_t s_aux = nullptr;
    hipEvent_t ev[2 * kNumTimed] = {};
    hipEvent_t ev_tables = nullptr, ev_pack = nullptr, ev_done = nullptr;
    std::shared_ptr<Plan> plan;      // the batch's plan (kept alive while in flight)
    const Plan *uploaded = nullptr;  // plan whose tables this slot's device holds
    // the host pipeline packs a collected chunk's images on the copy stream
    // from this slot's track tables after the slot is free: the next batch
    // in the slot writes its tables only after that pack (ev_reuse)
    hipEvent_t ev_reuse = nullptr;
    bool reuse_pending = false;
    TrackOut *tout_h = nullptr;      // pinned
    size_t tout_cap = 0;
    FrameDesc *fdesc_h = nullptr;    // pinned
    size_t fdesc_cap = 0;
    uint32_t *err_h = nullptr;       // pinned
    size_t err_cap = 0;
    bool want_fdesc = false;
    // the batch's second MD5 part, stream headers and result copies are
    // enqueued one batch later (after the next batch's LPC kernel), or when
    // the batch is waited: batch_end()
    bool end_pending = false;
    const void *pend_pcm = nullptr;
    int pend_fmt = 0;
    uint8_t *pend_out = nullptr;
    bool pend_split = false;         // part 1 of a split MD5 chain still to run
    atg_status end_status = ATG_OK;  // the batch end failed to queue: its wait reports this
    std::string end_error;
    // host-MD5 mode (want_host_md5): the PCM goes to pinned host memory and
    // the pool's threads hash it; the digests go back before the headers
    bool md5_host = false;
    uint8_t *hpcm = nullptr;         // pinned: the tracks' MD5 byte streams
    size_t hpcm_cap = 0;
    DevBuf dpack;                    // the same streams packed on the device
    uint8_t *hmd5 = nullptr;         // pinned: 16 bytes per track
    size_t hmd5_cap = 0;
    DevBuf md5in;                    // the digests on the device
    hipEvent_t ev_hpcm = nullptr;    // the PCM copies are done
    std::vector<std::future<void>> hash_jobs;
    // rolled mode (e->depth >= kRollMinDepth, pipelined device
    // batches): the chain runs as roll_parts slices on the engine's MD5
    // stream, one per later enqueue; the tail follows the last slice there
    bool rolled = false;
    uint32_t roll_parts = 0, roll_done = 0;
    bool busy = false;               // enqueued, not yet waited
    bool done = false;               // waited: results below are valid
    bool host = false;               // a chunk of a host-memory job
    uint64_t ticket = 0;
    atg_status status = ATG_OK;
    std::string error;
    float times[kNumTimed] = {};
};

// the slots' aux streams (MD5 chains, stream headers, result copies) at
// high stream priority.  With GPU_MAX_HW_QUEUES = 4 (HIP's default) the
// engine's six streams otherwise share hardware queues, and a host job's
// chunks queue their MD5 chains behind one another on a shared queue: the
// host-to-host leg runs 1.09 M frames/s at normal priority, 1.83 M at high
// (profiles/r03_d_*); the device-resident step is the same either way.
// 0 only for experiments (tools/build_exp.sh)
// K1 (and the batch's table uploads) on the slot's stream rather than the
// main one: the LPC kernels of the batches behind run beside this batch's
// search and pack (tools/gpu_r4p.sh: 9.22 -> 8.87 ms per config-2 step)
// K3-K5 of pipelined device batches on an engine-wide pack stream (section
// 4a''' of DESIGN.md); 0 keeps them on the main stream


// batches in flight on an engine (each its own device workspace): the MD5
// chains of a batch run ~12 ms (one serial hash per 1 MiB track, whatever
// the batch width), longer than a wide batch's search chain, so a third slot
// keeps them off the critical path.  A narrow batch (a rank's share of a
// strong-scaling job: 128 tracks need ~1.2 ms of kernels) needs more
// batches in flight to hide the same chain: atg_engine_set_inflight raises
// the slot rotation up to kMaxSlots (default kEncSlots)
constexpr uint64_t kEncSlots = 3;
constexpr uint64_t kMaxSlots = 32;
static_assert(kMaxSlots <= kRollMax, "one rolled launch covers every slot");
// rolled MD5 from this depth on (atg_engine_set_inflight); below it every
// slot keeps its own aux stream and the two-part split
constexpr uint64_t kRollMinDepth = 4;

// host pipeline stages (device PCM / image buffers): one more than the
// batches in flight, so chunk c + 3's upload is queued on the copy engine
// before the host waits for chunk c's batch (its MD5 chains, ~15-18 ms for
// a 512 MiB chunk, longer than the next two uploads)
constexpr uint64_t kHostStages = kEncSlots + 1;

// bytes per device-to-host copy of a batch's track results (section 3)
constexpr size_t kResultCopy = 8192;

// one stage of the host pipeline (chunk c uses stage c % kHostStages)
struct HostStage {
    DevBuf d_pcm, d_img, d_pack, d_off;
    uint8_t *p_in = nullptr, *p_out = nullptr; // pinned staging (pageable callers)
    size_t p_in_cap = 0, p_out_cap = 0;
    uint64_t *p_off = nullptr;                 // pinned: packed offsets to upload
    size_t p_off_cap = 0;
    hipEvent_t ev_h2d = nullptr;    // chunk PCM on the device
    hipEvent_t ev_packed = nullptr; // images moved out of d_img
    hipEvent_t ev_d2h = nullptr;    // packed images in host memory
};

// host threads for the host-MD5 mode: a fixed pool, one task per track
struct HashPool {
    std::vector<std::thread> th;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::packaged_task<void()>> q;
    bool stop = false;
    explicit HashPool(unsigned n)
    {
        for (unsigned i = 0; i < n; ++i)
            th.emplace_back([this] {
                for (;;) {
                    std::packaged_task<void()> job;
                    {
                        std::unique_lock<std::mutex> lk(mu);
                        cv.wait(lk, [this] { return stop || !q.empty(); });
                        if (q.empty())
                            return;
                        job = std::move(q.front());
                        q.pop_front();
                    }
                    job();
                }
            });
    }
    std::future<void> submit(std::function<void()> f)
    {
        std::packaged_task<void()> job(std::move(f));
        std::future<void> fut = job.get_future();
        {
            std::lock_guard<std::mutex> lk(mu);
            q.push_back(std::move(job));
        }
        cv.notify_one();
        return fut;
    }
    ~HashPool()
    {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
        }
        cv.notify_all();
        for (std::thread &t : th)
            t.join();
    }
};

struct atg_engine {
    std::recursive_mutex mu; // held by every public entry point (handle_lock.h)
    int device = 0;
    uint32_t flags = 0;      // atg_engine_create_ex flags
    std::unique_ptr<HashPool> pool; // host-MD5 threads, created on first use
    bool sync_call = false; // inside atg_flac_encode_device (enqueue + wait)
    hipStream_t s_main = nullptr;
    // pipelined device batches (atg_flac_encode_device_async): K3-K5 of
    // batch k on their own stream, so batch k+1's search starts beside
    // batch k's pack (null: everything on s_main)
    hipStream_t s_pack = nullptr;
    EncSlot slot[kMaxSlots];
    uint64_t depth = kEncSlots; // slots in rotation (atg_engine_set_inflight)
    // the caller fixed the depth (atg_engine_set_inflight n >= 3); otherwise
    // a pipelined device batch that starts a pipeline sets it (auto_depth)
    bool depth_user = false;
    // rolled mode: every batch's MD5 slices, tails, stream headers and
    // result copies on s_md5 (high priority: one stream whatever the depth,
    // instead of one aux stream per slot); the tables + LPC kernels on the
    // default slots' aux streams in turn (a stream created after s_md5 for
    // them landed on s_md5's hardware queue and serialised with the slices,
    // profiles/r05_e_narrow_trace.txt); roll_q = rolled batches with
    // slices to run, oldest first
    hipStream_t s_md5 = nullptr;
    std::deque<EncSlot *> roll_q;
    DevBuf windows;
    // host-memory API (atg_flac_encode_host): per pipeline stage, device
    // PCM / image / packed-image buffers and pinned host staging (used only
    // for pageable caller buffers), plus copy streams, so chunk c+1's upload,
    // chunk c's encode and chunk c-1's download overlap
    HostStage hs[kHostStages];
    hipStream_t s_h2d = nullptr, s_d2h = nullptr;
    // a collected chunk's offsets upload and pack kernel: not behind the
    // previous chunk's download, since the slot's next batch waits for the
    // pack (EncSlot::ev_reuse)
    hipStream_t s_hpack = nullptr;
    // PCM bytes per chunk.  A chunk's MD5 chains take ~15 ms per MiB of
    // track whatever its track count, so fewer, larger chunks keep fewer
    // chains in flight: config 2, queued jobs, 256 MB 28.8 ms per batch,
    // 512 MB 27.0 ms, 768 MB 40.3 ms; one synchronous call 41.1 / 37.9 /
    // 48.2 ms (profiles/r03_h_host_chunks.txt)
    uint64_t chunk_bytes = 512ull << 20;
    // host jobs (atg_flac_encode_host_async), oldest first; their chunks
    // flow through the stages in submission order, kEncSlots in flight
    std::deque<std::unique_ptr<HostJob>> hjobs;
    std::deque<std::pair<HostJob *, size_t>> hflight; // (job, chunk): enqueued, not collected
    HostJob *hcopy_job = nullptr;                     // staged chunk whose host copy is pending
    size_t hcopy_chunk = 0;
    uint64_t hseq = 0; // chunks enqueued so far (stage = seq % kHostStages)
    uint64_t next_hjob = 1;
    std::map<uint32_t, uint32_t> win_off;
    std::vector<double> win_host;
    size_t win_uploaded = 0;
    // recorded after the last window upload (on the uploading batch's slot
    // stream): every later batch's LPC kernel, on whichever slot stream,
    // waits for it
    hipEvent_t ev_win = nullptr;
    float times[kNumTimed] = {};
    bool have_times = false;
    uint64_t next_ticket = 1;
    // plan cache: a batch with the same geometry as the previous call reuses
    // the plan (and a slot's frame/track tables when it last ran that plan)
    std::vector<uint8_t> plan_key;
    std::shared_ptr<Plan> plan_cached;
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
    // large-frame path (flac_big.hip): a frame longer than 4096 samples or a
    // partition order above 6 anywhere in the batch
    bool big = false;
    uint32_t big_nmax = 0;       // longest frame
    uint32_t big_porder = 0;     // deepest usable partition order
    // streaming segment (atg_flac_encode_frames): frames only, numbered from
    // a base, no stream header and no MD5 (the caller hashes the PCM)
    bool frames_only = false;
};

// persistent grid of the large-frame kernels and their per-workgroup
// scratch: the candidate's samples, then the partition-sum pyramid
const uint32_t kBigGrid = 1024;

uint64_t big_row_bytes(const Plan &pl) { return ((uint64_t)pl.big_nmax * 4u + 255u) & ~255ull; }

uint64_t big_slot_bytes(const Plan &pl)
{
    return big_row_bytes(pl) + (16ull << pl.big_porder);
}

uint32_t qlp_precision_for(uint32_t n)
{
    return n <= 192 ? 7 : n <= 384 ? 8 : n <= 576 ? 9 : n <= 1152 ? 10 : n <= 2304 ? 11
         : n <= 4608 ? 12 : 13;
}

atg_status make_plan(const atg_flac_options *o, const atg_track *tracks, uint32_t n_tracks,
                     uint32_t channels, uint32_t bps, uint32_t rate, Plan &pl,
                     bool frames_only = false, uint32_t index_base = 0,
                     const uint32_t *index_bases = nullptr)
{
    if (!o)
        return fail(ATG_ERR_INVALID, "options is NULL");
    if (channels < 1 || channels > 8)
        return fail(ATG_ERR_INVALID, "channels must be 1..8");
    if (bps < 4 || bps > 24)
        return fail(ATG_ERR_UNSUPPORTED, "bits_per_sample must be 4..24 on the GPU path");
    if (o->block_size == 0)
        return fail(ATG_ERR_INVALID, "block_size must be > 0");
    if (o->block_size > ATG_BIG_MAX_BLOCK)
        return fail(ATG_ERR_UNSUPPORTED, "block_size > 65535 cannot be framed");
    if (o->max_lpc_order > ATG_MAX_LPC)
        return fail(ATG_ERR_INVALID, "max_lpc_order must be <= 32");
    if (o->max_residual_partition_order > ATG_BIG_MAX_PORDER)
        return fail(ATG_ERR_INVALID, "max_residual_partition_order must be <= 15");
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
    p.header_bytes = frames_only ? 0u : 4 + 4 + 34 + 4 + 4 + 29 + 4 + 4 + o->padding_size;
    pl.frames_only = frames_only;

    const uint64_t B = o->block_size;
    const uint64_t nsub = channels;

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
                if (n == 0 || n > ATG_BIG_MAX_BLOCK)
                    return fail(n ? ATG_ERR_UNSUPPORTED : ATG_ERR_INVALID,
                                "explicit frame sizes must be 1..65535");
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
        f.index = (index_bases ? index_bases[t] : index_base) + idx[t]++;
        f.win_off = 0;
        start[t] += lens[i];
    }
    // worst-case frame: verbatim subframes (+1 bit side channel) + headers.
    // Without VERBATIM a predictor may exceed that: the 4096-sample packer is
    // bounded by its LDS image, the large-frame packer checks the track's
    // slot on the device (error bit 4)
    uint32_t maxn = 0;
    for (size_t i = 0; i < nfr; ++i)
        maxn = std::max(maxn, lens[i]);
    const uint64_t nb = std::max<uint64_t>(B, maxn);
    uint64_t fb = 16 + nsub * ((8 + 32 + nb * (bps + 1) + 7) / 8) + 2;
    pl.big = nb > ATG_MAX_BLOCK || p.max_porder > ATG_MAX_PORDER;
    if (!p.try_verbatim)
        fb = pl.big ? 2 * fb + 120 * 1024 : std::max<uint64_t>(fb, 120 * 1024);
    pl.frame_bound = fb;
    p.frame_bound = (uint32_t)fb;
    p.frame_lds_words = (uint32_t)((fb + 3) / 4 + 2);
    if (!pl.big && p.frame_lds_words * 4ull > 128 * 1024)
        return fail(ATG_ERR_UNSUPPORTED, "frame image exceeds the pack kernel's LDS budget");
    if (pl.big) {
        pl.big_nmax = maxn;
        pl.big_porder = 0;
        for (size_t i = 0; i < nfr; ++i) {
            const uint32_t tz = (uint32_t)__builtin_ctz(lens[i]);
            pl.big_porder = std::max(pl.big_porder, std::min<uint32_t>(p.max_porder, tz));
        }
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
    if (channels == 2 && p.n_cand == 4 && bps <= 16 && B == ATG_MAX_BLOCK && !pl.big)
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

// (uploaded on stream s, the one the batch's LPC kernel runs on)
atg_status prepare_windows(atg_engine *e, Plan &pl, hipStream_t s)
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
        const size_t need = e->win_host.size() * sizeof(double) + 64;
        // a larger table replaces the buffer: earlier batches' LPC kernels
        // (other slot streams) may still read the old one
        if (need > e->windows.cap && e->windows.p)
            HIP_TRY(hipDeviceSynchronize());
        HIP_TRY(e->windows.ensure(need));
        HIP_TRY(hipMemcpyAsync(e->windows.p, e->win_host.data(),
                               e->win_host.size() * sizeof(double), hipMemcpyHostToDevice,
                               s));
        e->win_uploaded = e->win_host.size();
        if (!e->ev_win)
            HIP_TRY(hipEventCreateWithFlags(&e->ev_win, hipEventDisableTiming));
        HIP_TRY(hipEventRecord(e->ev_win, s));
    } else if (e->ev_win) {
        HIP_TRY(hipStreamWaitEvent(s, e->ev_win, 0));
    }
    return ATG_OK;
}

// memcpy split over host threads (pageable <-> pinned staging of large
// chunks runs at several times one core's copy bandwidth)
void par_memcpy(void *dst, const void *src, size_t n, unsigned nt)
{
    const size_t kMin = 8u << 20;
    if (n < kMin || nt < 2) {
        std::memcpy(dst, src, n);
        return;
    }
    nt = (unsigned)std::min<size_t>(nt, n / (kMin / 4));
    std::vector<std::thread> th;
    const size_t part = (n / nt + 4095) & ~(size_t)4095;
    for (unsigned i = 0; i < nt; ++i) {
        const size_t a = (size_t)i * part;
        if (a >= n)
            break;
        const size_t len = std::min(part, n - a);
        th.emplace_back([=] { std::memcpy((uint8_t *)dst + a, (const uint8_t *)src + a, len); });
    }
    for (auto &t : th)
        t.join();
}

// page-locked host memory (hipHostMalloc / hipHostRegister): DMA-able as is
bool is_pinned(const void *p)
{
    if (!p)
        return false;
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError(); // pageable memory: not an error for the caller
        return false;
    }
    return a.type == hipMemoryTypeHost;
}

template <class T>
hipError_t ensure_pinned(T *&p, size_t &cap, size_t n)
{
    if (p && n <= cap)
        return hipSuccess;
    if (p)
        (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    const size_t want = std::max<size_t>(n, 16);
    hipError_t e = hipHostMalloc((void **)&p, want * sizeof(T), hipHostMallocDefault);
    if (e == hipSuccess)
        cap = want;
    return e;
}

// The tail of a batch on its slot's stream: MD5 part 1 (+ the lane-per-
// track finishing kernel), then, once the pack is done, the stream headers
// and the results to pinned host memory.  `after`: an event the MD5 part
// waits for (the next batch's LPC kernel), or none.
atg_status batch_end_queue(atg_engine *e, EncSlot &sl, hipEvent_t after);

// batch_end_queue, and if any of its HIP calls fails the slot's batch is
// marked failed (its ev_done was never recorded, so a wait must not trust it)
atg_status batch_end(atg_engine *e, EncSlot &sl, hipEvent_t after)
{
    sl.end_pending = false;
    const atg_status st = batch_end_queue(e, sl, after);
    if (st != ATG_OK) {
        sl.end_status = st;
        sl.end_error = g_err;
    }
    return st;
}

atg_status batch_end_queue(atg_engine *e, EncSlot &sl, hipEvent_t after)
{
    const Plan &pl = *sl.plan;
    const FlacParams &p = pl.p;
    const size_t nf = pl.frames.size(), nt = pl.tracks.size();
    const TrackInfo *dtr = (const TrackInfo *)sl.tracks.p;
    TrackOut *dto = (TrackOut *)sl.tout.p;
    uint32_t *derr = (uint32_t *)sl.err.p;
    hipEvent_t *ev = sl.ev;
    // a rolled batch's tail runs on the engine's MD5 stream right after its
    // last slice; the others on the slot's aux stream
    hipStream_t q = sl.rolled ? e->s_md5 : sl.s_aux;
    if (sl.rolled) {
        if (!pl.frames_only)
            HIP_TRY(launch_track_md5_finish(p, sl.pend_pcm, sl.pend_fmt, dtr, dto, q));
    } else if (sl.pend_split && !pl.frames_only) {
        if (after)
            HIP_TRY(hipStreamWaitEvent(q, after, 0));
        HIP_TRY(launch_track_md5(p, sl.pend_pcm, sl.pend_fmt, dtr, dto, 1, q));
    }
    HIP_TRY(hipEventRecord(ev[2 * 5 + 1], q));
    // headers once both the pack and the MD5 chains are done
    HIP_TRY(hipStreamWaitEvent(q, sl.ev_pack, 0));
    HIP_TRY(hipEventRecord(ev[12], q));
    if (!pl.frames_only)
        HIP_TRY(launch_stream_header(p, dtr, dto, sl.pend_out, q));
    HIP_TRY(hipEventRecord(ev[13], q));
    HIP_TRY(hipEventRecord(ev[15], q));
    // the track results in 8 KiB copies: one 32 KiB copy per 1024-track
    // batch measured 8.10-8.12 ms per step, 8 KiB pieces 8.01-8.04
    // (profiles/r05_zz_dec_spec.txt; past 16 KiB a copy takes another path)
    for (size_t o = 0, nb = nt * sizeof(TrackOut); o < nb; o += kResultCopy)
        HIP_TRY(hipMemcpyAsync((uint8_t *)sl.tout_h + o, (const uint8_t *)dto + o,
                               std::min<size_t>(kResultCopy, nb - o), hipMemcpyDeviceToHost, q));
    if (sl.want_fdesc && nf)
        HIP_TRY(hipMemcpyAsync(sl.fdesc_h, sl.fdesc.p, nf * sizeof(FrameDesc),
                               hipMemcpyDeviceToHost, q));
    HIP_TRY(hipMemcpyAsync(sl.err_h, derr, sizeof(uint32_t), hipMemcpyDeviceToHost, q));
    HIP_TRY(hipEventRecord(sl.ev_done, q));
    return ATG_OK;
}

atg_status ensure_aux_stream(EncSlot &sl);

// ---- rolled mode -------------------------------------------------------------
atg_status ensure_roll_streams(atg_engine *e)
{
    if (e->s_md5)
        return ATG_OK;
    int prio_lo = 0, prio_hi = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    HIP_TRY(hipStreamCreateWithPriority(&e->s_md5, hipStreamNonBlocking, prio_hi));
    return ATG_OK;
}

// One rolled launch on s_md5 after `after`: every batch in roll_q advances by
// its next slice (or, with `only`, that batch alone by all its remaining
// slices -- a wait that cannot count on later enqueues); batches whose last
// slice ran get their tail queued behind it and leave roll_q.
atg_status roll_step(atg_engine *e, hipEvent_t after, EncSlot *only)
{
    MdRollArgs a;
    std::memset(&a, 0, sizeof(a));
    std::vector<EncSlot *> starting, finished;
    uint32_t wg = 0;
    for (EncSlot *sl : e->roll_q) {
        if (only && sl != only)
            continue;
        const FlacParams &p = sl->plan->p;
        MdRollBatch &b = a.b[a.n++];
        b.pcm = sl->pend_pcm;
        b.tracks = (const TrackInfo *)sl->tracks.p;
        b.tout = (TrackOut *)sl->tout.p;
        b.n_tracks = p.n_tracks;
        b.channels = p.channels;
        b.bps = p.bps;
        b.fmt = (uint32_t)sl->pend_fmt;
        b.wg0 = wg;
        b.parts = sl->roll_parts;
        b.part = sl->roll_done;
        b.part_end = only ? sl->roll_parts : sl->roll_done + 1u;
        wg += (p.n_tracks + 63u) / 64u;
        if (b.part == 0)
            starting.push_back(sl);
        sl->roll_done = b.part_end;
        if (sl->roll_done == sl->roll_parts)
            finished.push_back(sl);
    }
    if (!a.n)
        return ATG_OK;
    if (after)
        HIP_TRY(hipStreamWaitEvent(e->s_md5, after, 0));
    for (EncSlot *sl : starting)
        HIP_TRY(hipEventRecord(sl->ev[2 * 5], e->s_md5));
    HIP_TRY(launch_track_md5_roll(a, e->s_md5));
    for (EncSlot *sl : finished) {
        e->roll_q.erase(std::find(e->roll_q.begin(), e->roll_q.end(), sl));
        const atg_status st = batch_end(e, *sl, nullptr);
        if (st != ATG_OK)
            return st;
    }
    return ATG_OK;
}

// every stream a slot's batch may have work on
void drain_slot(atg_engine *e, EncSlot &sl)
{
    (void)hipStreamSynchronize(e->s_main);
    for (hipStream_t q : {e->s_pack, e->s_md5, sl.s_aux})
        if (q)
            (void)hipStreamSynchronize(q);
}

// ---- host-MD5 mode ---------------------------------------------------------
// Host threads available to this process: the affinity mask, bounded by a
// cgroup CPU quota (a GPU box shares its host: os.cpu_count() sees every
// core, cpu.max the share this job may use), at most 32.
unsigned host_hash_threads()
{
    unsigned n = std::max(1u, std::thread::hardware_concurrency());
    cpu_set_t cs;
    if (sched_getaffinity(0, sizeof(cs), &cs) == 0)
        n = std::max(1, CPU_COUNT(&cs));
    if (FILE *f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        unsigned long per = 0;
        if (std::fscanf(f, "%31s %lu", q, &per) == 2 && std::strcmp(q, "max") != 0 && per)
            n = std::min<unsigned>(n, std::max(1ul, std::strtoul(q, nullptr, 10) / per));
        std::fclose(f);
    }
    return std::min(n, 32u);
}

// Host or GPU for this batch's MD5.  A GPU chain hashes one 64-byte block
// per ~0.8 us (one wave per track, md5.hip), so the batch's MD5 ends when
// its longest track's chain does; on the host a core hashes 16 tracks at
// once at ~6 GB/s with AVX-512 (md5_cpu.h hash_bytes_multi; ~0.45 GB/s per
// thread without), after the packed streams' download (~40 GB/s pinned).
// The host side wins only for few, long tracks whose chains would outlast
// the GPU work they overlap (config 5: 8.6 MB tracks, ~110 ms chains); the
// GPU otherwise (config 2: 1 MiB tracks, ~13 ms chains under the next
// batches' search kernels).
constexpr size_t kHashGroup = md5cpu::kMultiLanes; // tracks per host hash task

bool want_host_md5(atg_engine *e, const Plan &pl, int fmt, bool md5_early)
{
    const FlacParams &p = pl.p;
    if (pl.frames_only || md5_early || p.bps < 8 || p.bps % 8 || pl.tracks.empty())
        return false;
    if (e->flags & ATG_ENGINE_MD5_GPU)
        return false;
    if (e->flags & ATG_ENGINE_MD5_HOST)
        return true;
    const uint64_t bb = p.bps / 8, cs = fmt == ATG_PCM_S16 ? 2 : 4;
    uint64_t maxb = 0, tot = 0;
    for (const TrackInfo &t : pl.tracks) {
        const uint64_t b = t.pcm_frames * p.channels * bb;
        maxb = std::max(maxb, b);
        tot += b;
    }
    (void)cs;
    const double gpu_ms = (double)maxb / 64.0 * 0.8e-3;
    const unsigned th = host_hash_threads();
    const uint64_t groups = (pl.tracks.size() + kHashGroup - 1) / kHashGroup;
    const double hash_ms = md5cpu::multi_simd()
                               ? (double)tot / (double)std::min<uint64_t>(th, groups) / 6e6
                               : (double)tot / (th * 450e3);
    const double host_ms = hash_ms + (double)tot / 40e6;
    return gpu_ms > 40.0 && host_ms < gpu_ms;
}

// The tracks' PCM to pinned host memory on the slot's stream (copy engine),
// then one pool task per track: wait for the copies, hash the containers'
// little-endian bytes (md5_cpu.h) into sl.hmd5.  finish_batch joins them.
atg_status start_host_md5(atg_engine *e, EncSlot &sl, const Plan &pl, const void *d_pcm, int fmt)
{
    const FlacParams &p = pl.p;
    const size_t nt = pl.tracks.size();
    const uint64_t cs = fmt == ATG_PCM_S16 ? 2 : 4;
    const uint32_t bb = p.bps / 8;
    for (std::future<void> &f : sl.hash_jobs) // a failed earlier batch's tasks
        f.wait();
    sl.hash_jobs.clear();
    // each track's byte stream at a 16-byte aligned offset
    std::vector<uint64_t> off(nt), len(nt);
    uint64_t total = 0;
    for (size_t t = 0; t < nt; ++t) {
        len[t] = pl.tracks[t].pcm_frames * p.channels * bb;
        off[t] = total;
        total += (len[t] + 15u) & ~15ull;
    }
    HIP_TRY(ensure_pinned(sl.hpcm, sl.hpcm_cap, (size_t)std::max<uint64_t>(total, 1)));
    HIP_TRY(ensure_pinned(sl.hmd5, sl.hmd5_cap, 16 * nt));
    HIP_TRY(sl.md5in.ensure(16 * nt));
    HIP_TRY(sl.dpack.ensure((size_t)std::max<uint64_t>(total, 1)));
    if (!sl.ev_hpcm)
        HIP_TRY(hipEventCreateWithFlags(&sl.ev_hpcm, hipEventDisableTiming));
    for (size_t t = 0; t < nt; ++t) {
        const TrackInfo &ti = pl.tracks[t];
        HIP_TRY(launch_md5_pack((const uint8_t *)d_pcm + ti.pcm_start * p.channels * cs,
                                fmt == ATG_PCM_S16, ti.pcm_frames * p.channels, bb,
                                (uint8_t *)sl.dpack.p + off[t], sl.s_aux));
    }
    if (total)
        HIP_TRY(hipMemcpyAsync(sl.hpcm, sl.dpack.p, total, hipMemcpyDeviceToHost, sl.s_aux));
    HIP_TRY(hipEventRecord(sl.ev_hpcm, sl.s_aux));
    if (!e->pool)
        e->pool.reset(new HashPool(host_hash_threads()));
    const hipEvent_t ev = sl.ev_hpcm;
    // one pool task per group of kHashGroup tracks: their chains side by
    // side in one core's vector registers
    for (size_t g0 = 0; g0 < nt; g0 += kHashGroup) {
        const int n = (int)std::min<size_t>(kHashGroup, nt - g0);
        std::array<const uint8_t *, kHashGroup> src{};
        std::array<uint64_t, kHashGroup> bytes{};
        for (int i = 0; i < n; ++i) {
            src[i] = sl.hpcm + off[g0 + i];
            bytes[i] = len[g0 + i];
        }
        uint8_t(*dst)[16] = (uint8_t(*)[16])(sl.hmd5 + 16 * g0);
        sl.hash_jobs.push_back(e->pool->submit([=] {
            (void)hipEventSynchronize(ev);
            md5cpu::hash_bytes_multi(src.data(), bytes.data(), n, dst);
        }));
    }
    return ATG_OK;
}

// the host digests into TrackOut on the slot's stream (before the headers)
atg_status finish_host_md5(EncSlot &sl)
{
    for (std::future<void> &f : sl.hash_jobs)
        f.wait();
    sl.hash_jobs.clear();
    const size_t nt = sl.plan->tracks.size();
    if (nt) {
        HIP_TRY(hipMemcpyAsync(sl.md5in.p, sl.hmd5, 16 * nt, hipMemcpyHostToDevice, sl.s_aux));
        HIP_TRY(launch_put_md5((TrackOut *)sl.tout.p, (const uint8_t *)sl.md5in.p, (uint32_t)nt,
                               sl.s_aux));
    }
    return ATG_OK;
}

// Enqueue one batch on slot `sl`: the search chain on the engine's main
// stream, the MD5 chains from the start of the batch and the stream headers
// on the slot's aux stream, then the results back to pinned host memory.
// Returns without waiting.
atg_status enqueue_batch(atg_engine *e, EncSlot &sl, const std::shared_ptr<Plan> &plp,
                         const void *d_pcm, int fmt, uint8_t *d_out, uint64_t out_cap,
                         bool want_fdesc, hipEvent_t wait_before = nullptr, bool pipelined = false,
                         bool md5_early = false)
{
    Plan &pl = *plp;
    FlacParams &p = pl.p;
    if (pl.out_bytes > out_cap)
        return fail(ATG_ERR_CAPACITY, "output buffer too small for this batch");
    p.n_reg_frames = (fmt == ATG_PCM_S16 && ((uintptr_t)d_pcm & 15u) == 0) ? pl.n_reg_prefix : 0u;
    HIP_TRY(hipSetDevice(e->device));
    sl.md5_host = want_host_md5(e, pl, fmt, md5_early);
    // rolled mode: many narrow batches in flight (atg_engine_set_inflight)
    sl.rolled = pipelined && !md5_early && !sl.md5_host && !pl.frames_only &&
                e->depth >= kRollMinDepth && track_md5_paired(p, fmt);
    // a rolled batch's tables and LPC kernel go on one of the default slots'
    // aux streams in turn (high priority, a hardware queue each, created
    // before s_md5), so batch k+1's LPC kernel runs beside batch k's search
    EncSlot &pre = sl.rolled ? e->slot[sl.ticket % kEncSlots] : sl;
    {
        atg_status st0 = sl.rolled ? ensure_aux_stream(pre) : ensure_aux_stream(sl);
        if (st0 == ATG_OK && sl.rolled)
            st0 = ensure_roll_streams(e);
        if (st0 != ATG_OK)
            return st0;
    }
    // the tables, the LPC kernel and the MD5 chains on the slot's stream:
    // the next batches' LPC kernels run beside this batch's search and pack.
    // Whatever the LPC kernel reads is written on this stream (or waited
    // for through wait_before): nothing the caller queued on the main
    // stream is ordered before it
    hipStream_t s_pre = pre.s_aux;
    if (wait_before)
        HIP_TRY(hipStreamWaitEvent(s_pre, wait_before, 0));
    if (sl.reuse_pending) {
        HIP_TRY(hipStreamWaitEvent(s_pre, sl.ev_reuse, 0));
        sl.reuse_pending = false;
    }
    atg_status st = prepare_windows(e, pl, s_pre);
    if (st != ATG_OK)
        return st;
    const size_t nf = pl.frames.size(), nt = pl.tracks.size();
    bool upload = sl.uploaded != &pl;
    {
        void *f0 = sl.frames.p, *t0 = sl.tracks.p, *o0 = sl.order.p;
        HIP_TRY(sl.frames.ensure(nf * sizeof(FrameInfo)));
        HIP_TRY(sl.tracks.ensure(nt * sizeof(TrackInfo)));
        HIP_TRY(sl.order.ensure(nf * sizeof(uint32_t)));
        if (f0 != sl.frames.p || t0 != sl.tracks.p || o0 != sl.order.p)
            upload = true;
    }
    HIP_TRY(sl.coef.ensure(nf * p.n_cand * p.coef_stride * sizeof(int16_t)));
    HIP_TRY(sl.shift.ensure(nf * p.n_cand * std::max<uint32_t>(1, p.max_lpc_order)));
    HIP_TRY(sl.est.ensure(nf * p.n_cand));
    HIP_TRY(sl.sub.ensure(nf * p.n_cand * sizeof(SubDesc)));
    HIP_TRY(sl.fdesc.ensure(nf * sizeof(FrameDesc)));
    HIP_TRY(sl.tout.ensure(nt * sizeof(TrackOut)));
    HIP_TRY(sl.err.ensure(sizeof(uint32_t)));
    // 16-bit search (flac_search16.hip) for full 4096-sample frames; what it
    // cannot take goes through the general kernel as a list
    const bool fast16 = !pl.big && p.block_size == ATG_MAX_BLOCK &&
                        p.max_lpc_order <= ATG_FAST_ORDER && p.bps <= 16u;
    // wider sources (24-bit): the hi/lo split search, same hand-over list
    const bool fast_hl = !pl.big && p.block_size == ATG_MAX_BLOCK &&
                         p.max_lpc_order <= ATG_FAST_ORDER && p.bps > 16u;
    if (fast16 || fast_hl)
        HIP_TRY(sl.slow.ensure((4 + nf * p.n_cand) * sizeof(uint32_t)));
    const uint32_t big_grid =
        pl.big ? (uint32_t)std::min<uint64_t>(kBigGrid, std::max<uint64_t>(nf, 1) * p.n_cand) : 0u;
    const uint32_t rice_stride = 1u << pl.big_porder;
    if (pl.big) {
        HIP_TRY(sl.rice_big.ensure(nf * p.n_cand * (size_t)rice_stride));
        HIP_TRY(sl.scratch.ensure(big_grid * big_slot_bytes(pl)));
    }
    HIP_TRY(ensure_pinned(sl.tout_h, sl.tout_cap, nt));
    HIP_TRY(ensure_pinned(sl.err_h, sl.err_cap, 1));
    if (want_fdesc)
        HIP_TRY(ensure_pinned(sl.fdesc_h, sl.fdesc_cap, nf));
    sl.uploaded = nullptr;
    if (upload && nf)
        HIP_TRY(hipMemcpyAsync(sl.frames.p, pl.frames.data(), nf * sizeof(FrameInfo),
                               hipMemcpyHostToDevice, s_pre));
    if (upload && nt)
        HIP_TRY(hipMemcpyAsync(sl.tracks.p, pl.tracks.data(), nt * sizeof(TrackInfo),
                               hipMemcpyHostToDevice, s_pre));
    if (upload && nf)
        HIP_TRY(hipMemcpyAsync(sl.order.p, pl.order.data(), nf * sizeof(uint32_t),
                               hipMemcpyHostToDevice, s_pre));
    HIP_TRY(hipMemsetAsync(sl.err.p, 0, sizeof(uint32_t), s_pre));
    HIP_TRY(hipEventRecord(sl.ev_tables, s_pre));

    const FrameInfo *dfr = (const FrameInfo *)sl.frames.p;
    const TrackInfo *dtr = (const TrackInfo *)sl.tracks.p;
    TrackOut *dto = (TrackOut *)sl.tout.p;
    uint32_t *derr = (uint32_t *)sl.err.p;
    hipEvent_t *ev = sl.ev;

    HIP_TRY(hipEventRecord(ev[14], s_pre));
    HIP_TRY(hipEventRecord(ev[0], s_pre));
    HIP_TRY(launch_lpc_analyze(p, d_pcm, fmt, dfr, (const double *)e->windows.p,
                               (int16_t *)sl.coef.p, (int8_t *)sl.shift.p, (uint8_t *)sl.est.p,
                               s_pre));
    HIP_TRY(hipEventRecord(ev[1], s_pre));
    HIP_TRY(hipStreamWaitEvent(e->s_main, ev[1], 0));
    // MD5 chains (a serial hash per track, high-priority waves) on the slot's
    // stream once the LPC kernel is done.  Split
    // (pipelined device batches of 16-bit PCM): part 0 = 60 % of every
    // track's blocks now, part 1 after the next batch's LPC kernel
    // (batch_end), so no chain runs beside an LPC grid; otherwise the whole
    // chain now (a caller waiting on each batch gains nothing from a split)
    // md5_early (host pipeline chunks): the whole chain as soon as the
    // chunk's PCM is uploaded -- a host caller waits for its last chunk's
    // chains, so they start as early as possible
    // host-MD5 mode (few long tracks, want_host_md5): the PCM copies start
    // with the batch, the hashes run on host threads, nothing on the GPU
    const bool split_md5 = !sl.rolled && pipelined && !md5_early && !sl.md5_host &&
                           ((fmt == ATG_PCM_S16 && p.bps == 16u) ||
                            (fmt == ATG_PCM_S32 && p.bps % 8u == 0u));
    // (md5_early: after the chunk's upload and this batch's track tables --
    // ev_tables is recorded behind both).  Rolled batches: below.
    if (!sl.rolled) {
        HIP_TRY(hipStreamWaitEvent(sl.s_aux, (md5_early || sl.md5_host) ? sl.ev_tables : ev[1],
                                   0));
        HIP_TRY(hipEventRecord(ev[2 * 5], sl.s_aux));
    }
    if (!pl.frames_only && !sl.rolled) {
        if (sl.md5_host) {
            sl.plan = plp; // the pool's tasks read the plan's tracks through the slot
            st = start_host_md5(e, sl, pl, d_pcm, fmt);
            if (st != ATG_OK)
                return st;
        } else {
            HIP_TRY(launch_track_md5(p, d_pcm, fmt, dtr, dto, split_md5 ? 0 : 2, sl.s_aux));
        }
    }
    HIP_TRY(hipEventRecord(ev[2], e->s_main));
    if (pl.big)
        HIP_TRY(launch_subframe_search_big(p, d_pcm, fmt, dfr, (const int16_t *)sl.coef.p,
                                           (const int8_t *)sl.shift.p, (const uint8_t *)sl.est.p,
                                           (SubDesc *)sl.sub.p, (uint8_t *)sl.rice_big.p,
                                           rice_stride, (uint8_t *)sl.scratch.p,
                                           big_slot_bytes(pl), big_row_bytes(pl), big_grid,
                                           e->s_main));
    else if (fast16 || fast_hl) {
        uint32_t *cnt = (uint32_t *)sl.slow.p, *list = cnt + 4;
        HIP_TRY(hipMemsetAsync(cnt, 0, sizeof(uint32_t), e->s_main));
        if (fast16)
            HIP_TRY(launch_subframe_search16(p, d_pcm, fmt, dfr, (const int16_t *)sl.coef.p,
                                             (const int8_t *)sl.shift.p,
                                             (const uint8_t *)sl.est.p, (SubDesc *)sl.sub.p,
                                             list, cnt, e->s_main));
        else
            HIP_TRY(launch_subframe_search_hl(p, d_pcm, fmt, dfr, (const int16_t *)sl.coef.p,
                                              (const int8_t *)sl.shift.p,
                                              (const uint8_t *)sl.est.p, (SubDesc *)sl.sub.p,
                                              list, cnt, e->s_main));
        const uint32_t units = (uint32_t)(nf * p.n_cand);
        HIP_TRY(launch_subframe_search_list(p, d_pcm, fmt, dfr, (const int16_t *)sl.coef.p,
                                            (const int8_t *)sl.shift.p,
                                            (const uint8_t *)sl.est.p, (SubDesc *)sl.sub.p,
                                            derr, list, cnt, std::min<uint32_t>(units, 4096u),
                                            e->s_main));
    } else
        HIP_TRY(launch_subframe_search(p, d_pcm, fmt, dfr, (const int16_t *)sl.coef.p,
                                       (const int8_t *)sl.shift.p, (const uint8_t *)sl.est.p,
                                       (SubDesc *)sl.sub.p, derr, e->s_main));
    HIP_TRY(hipEventRecord(ev[3], e->s_main));
    // K3-K5: on the pack stream for pipelined device batches (each reads
    // only its own slot's tables and writes its own output), else in order
    // on the main stream.  Everything after them waits for ev_pack.
    hipStream_t s_k5 = (e->s_pack && pipelined && !md5_early) ? e->s_pack : e->s_main;
    if (s_k5 != e->s_main)
        HIP_TRY(hipStreamWaitEvent(s_k5, ev[3], 0));
    HIP_TRY(hipEventRecord(ev[4], s_k5));
    HIP_TRY(launch_frame_decide(p, dfr, (const SubDesc *)sl.sub.p, (FrameDesc *)sl.fdesc.p,
                                s_k5));
    HIP_TRY(hipEventRecord(ev[5], s_k5));
    HIP_TRY(hipEventRecord(ev[6], s_k5));
    HIP_TRY(launch_track_scan(p, dtr, (const uint32_t *)sl.order.p, (FrameDesc *)sl.fdesc.p, dto,
                              s_k5));
    HIP_TRY(hipEventRecord(ev[7], s_k5));
    HIP_TRY(hipEventRecord(ev[8], s_k5));
    if (pl.big) {
        // the large-frame packer ORs bits into a zeroed image
        HIP_TRY(hipMemsetAsync(d_out, 0, pl.out_bytes, s_k5));
        HIP_TRY(launch_frame_pack_big(p, d_pcm, fmt, dfr, dtr, (const SubDesc *)sl.sub.p,
                                      (const uint8_t *)sl.rice_big.p, rice_stride,
                                      (const FrameDesc *)sl.fdesc.p, d_out, derr,
                                      (uint8_t *)sl.scratch.p, big_slot_bytes(pl),
                                      (uint32_t)std::min<uint64_t>(kBigGrid, nf), s_k5));
    } else {
        HIP_TRY(launch_frame_pack(p, d_pcm, fmt, dfr, dtr, (const SubDesc *)sl.sub.p,
                                  (const FrameDesc *)sl.fdesc.p, d_out, derr, s_k5));
    }
    HIP_TRY(hipEventRecord(ev[9], s_k5));
    HIP_TRY(hipEventRecord(sl.ev_pack, s_k5));
    sl.uploaded = &pl;
    sl.plan = plp;
    sl.end_status = ATG_OK;
    sl.end_error.clear();
    sl.want_fdesc = want_fdesc;
    sl.end_pending = !sl.rolled;
    sl.pend_pcm = d_pcm;
    sl.pend_fmt = fmt;
    sl.pend_out = d_out;
    sl.pend_split = split_md5;
    if (sl.rolled) {
        // the chain in depth - 2 slices: one per enqueue from this one on,
        // all batches' slices in one launch, so the tail of batch k is queued
        // with batch k + depth - 3's enqueue, two launches before a caller
        // that keeps `depth` batches in flight waits for it: the MD5 stream
        // always holds the next launch while the host waits.  The launch
        // needs only this batch's track table (ev_tables), not its LPC
        // kernel: at these widths the chains are the step
        sl.roll_parts = (uint32_t)e->depth - 2u;
        sl.roll_done = 0;
        e->roll_q.push_back(&sl);
        atg_status st2 = roll_step(e, sl.ev_tables, nullptr);
        if (st2 != ATG_OK)
            return st2;
    } else if (!split_md5 && !sl.md5_host) {
        atg_status st2 = batch_end(e, sl, nullptr);
        if (st2 != ATG_OK)
            return st2;
    }
    // the previous batches' second MD5 parts start now that this batch's
    // LPC kernel is done (a host-MD5 batch ends when it is waited)
    for (EncSlot &o : e->slot)
        if (&o != &sl && o.end_pending && !o.md5_host) {
            atg_status st2 = batch_end(e, o, ev[1]);
            if (st2 != ATG_OK)
                return st2;
        }
    return ATG_OK;
}

// wait for the slot's batch; records its kernel times and error status
atg_status finish_batch(atg_engine *e, EncSlot &sl)
{
    HIP_TRY(hipSetDevice(e->device));
    // a rolled batch with slices left (no later enqueue ran them): advance
    // every rolled batch together until this one is through -- the batches
    // behind it then drain concurrently rather than one after another
    while (sl.rolled && sl.roll_done < sl.roll_parts) {
        atg_status st = roll_step(e, nullptr, nullptr);
        if (st != ATG_OK) {
            drain_slot(e, sl);
            return st;
        }
    }
    if (sl.end_pending && sl.md5_host) {
        atg_status st = finish_host_md5(sl);
        if (st != ATG_OK) {
            sl.end_pending = false;
            (void)hipStreamSynchronize(e->s_main);
            if (e->s_pack)
                (void)hipStreamSynchronize(e->s_pack);
            (void)hipStreamSynchronize(sl.s_aux);
            return st;
        }
    }
    if (sl.end_pending) {
        atg_status st = batch_end(e, sl, nullptr);
        if (st != ATG_OK)
            return st;
    }
    if (sl.end_status != ATG_OK) {
        // ev_done was never recorded: drain the slot's streams, report the error
        drain_slot(e, sl);
        return fail(sl.end_status, sl.end_error);
    }
    HIP_TRY(hipEventSynchronize(sl.ev_done));
    for (int k = 0; k < kNumTimed; ++k) {
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, sl.ev[2 * k], sl.ev[2 * k + 1]) != hipSuccess)
            ms = 0.f;
        sl.times[k] = ms;
        e->times[k] = ms;
    }
    e->have_times = true;
    uint32_t err_h = *sl.err_h;
    if (err_h & 1u)
        return fail(ATG_ERR_UNSUPPORTED, "frame longer than the GPU block limit");
    if (err_h & 4u)
        return fail(ATG_ERR_CAPACITY, "a frame exceeds its track's output slot");
    if (err_h)
        return fail(ATG_ERR_DEVICE, "GPU consistency check failed (code " +
                                        std::to_string(err_h) + ")");
    return ATG_OK;
}

void fill_results(const Plan &pl, const TrackOut *to, atg_track_result *res,
                  const FrameDesc *fd, uint64_t *frame_offsets, uint32_t *frame_pcm)
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
                    frame_offsets[r.first_frame + i] = fd[f].out_off;
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

// plan for this call: the cached one when the geometry repeats, else a new
// plan that replaces the cache (slots that ran the old one keep it alive)
atg_status get_plan(atg_engine *e, const atg_flac_options *o, const atg_track *tracks,
                    uint32_t n_tracks, uint32_t channels, uint32_t bps, uint32_t rate,
                    std::shared_ptr<Plan> &pl)
{
    std::vector<uint8_t> key = plan_key(o, tracks, n_tracks, channels, bps, rate);
    if (e->plan_cached && key == e->plan_key) {
        pl = e->plan_cached;
        return ATG_OK;
    }
    auto np = std::make_shared<Plan>();
    atg_status st = make_plan(o, tracks, n_tracks, channels, bps, rate, *np);
    if (st != ATG_OK)
        return st;
    e->plan_cached = np;
    e->plan_key.swap(key);
    pl = np;
    return ATG_OK;
}

// A streaming engine (ATG_ENGINE_STREAMING) creates streams on first use: a process
// that only streams segments (atg_flac_encode_frames, one slot) holds
// s_main and one aux stream, not six -- under track2track many such
// processes share one GPU, and with every process at GPU_MAX_HW_QUEUES
// hardware queues the device's queue slots are oversubscribed and
// time-sliced.
atg_status ensure_aux_stream(EncSlot &sl)
{
    if (sl.s_aux)
        return ATG_OK;
    // the MD5 / header streams at the highest stream priority
    int prio_lo = 0, prio_hi = 0;
    HIP_TRY(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
    HIP_TRY(hipStreamCreateWithPriority(&sl.s_aux, hipStreamNonBlocking, prio_hi));
    return ATG_OK;
}

atg_status ensure_host_streams(atg_engine *e)
{
    if (!e->s_h2d)
        HIP_TRY(hipStreamCreateWithFlags(&e->s_h2d, hipStreamNonBlocking));
    if (!e->s_d2h)
        HIP_TRY(hipStreamCreateWithFlags(&e->s_d2h, hipStreamNonBlocking));
    return ATG_OK;
}

// the host pipeline's pack stream, created on the first host job: created
// with the engine it would take the hardware queue s_pack gets (created
// last for that reason) and serialise the device path's K3-K5 with K2
atg_status ensure_host_pack_stream(atg_engine *e)
{
    if (!e->s_hpack)
        HIP_TRY(hipStreamCreateWithFlags(&e->s_hpack, hipStreamNonBlocking));
    return ATG_OK;
}

// the slot for a new batch: the one after the last ticket's.  A slot still
// holding an unwaited batch is never reused (its results would be lost):
// the caller must wait the oldest ticket first, as with the decoder
atg_status take_slot(atg_engine *e, EncSlot *&out, uint64_t &ticket)
{
    EncSlot &sl = e->slot[e->next_ticket % e->depth];
    if (sl.busy)
        return fail(ATG_ERR_INVALID, "as many encode batches in flight as the engine has slots "
                                     "(atg_engine_set_inflight): wait for the oldest");
    ticket = e->next_ticket++;
    sl.ticket = ticket;
    sl.done = false;
    out = &sl;
    return ATG_OK;
}

// results of ticket t (waits if still running)
atg_status wait_ticket(atg_engine *e, uint64_t t, EncSlot *&out)
{
    EncSlot &sl = e->slot[t % e->depth];
    if (sl.ticket != t || (!sl.busy && !sl.done))
        return fail(ATG_ERR_INVALID, "unknown or expired encode ticket");
    if (sl.busy) {
        sl.status = finish_batch(e, sl);
        sl.error = g_err;
        sl.busy = false;
        sl.done = true;
    }
    out = &sl;
    if (sl.status != ATG_OK)
        return fail(sl.status, sl.error);
    return ATG_OK;
}


// ---- host-memory jobs (atg_flac_encode_host[_async]) ----------------------
// A job is cut into chunks of consecutive tracks (~chunk_bytes of PCM); the
// chunks of all jobs flow through the kEncSlots pipeline stages in
// submission order: chunk c+1's upload, chunk c's encode (its MD5 chains
// from the moment its PCM is on the device) and chunk c-1's download
// overlap, across job boundaries too, so back-to-back jobs keep the PCIe
// link busy.
struct HostChunk {
    uint32_t t0 = 0, t1 = 0;          // tracks [t0, t1) of the job
    uint64_t pcm0 = 0, samples = 0;   // first sample and samples of the chunk's PCM span
    std::vector<atg_track> tr;
    std::shared_ptr<Plan> plan;
    uint64_t ticket = 0;
    size_t stage = 0;
    uint64_t out0 = 0, out_bytes = 0; // packed span in the job's `out`
    bool staged_out = false;          // D2H went to pinned staging
};

struct HostJob {
    uint64_t id = 0;
    const uint8_t *pcm = nullptr;
    size_t elem = 2;
    int fmt = ATG_PCM_S16;
    uint8_t *out = nullptr;
    atg_track_result *results = nullptr;
    uint64_t *frame_offsets = nullptr;
    uint32_t *frame_pcm_frames = nullptr;
    bool pin_in = false, pin_out = false;
    Plan whole;
    std::vector<HostChunk> chunks;
    size_t collected = 0;             // chunks whose results are filled
    uint64_t out_pos = 0;
    atg_status status = ATG_OK;
    std::string error;
};

unsigned host_threads()
{
    return std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
}

// the staged chunk's bytes to the caller's buffer once its D2H is done
atg_status host_finish_copy(atg_engine *e)
{
    if (!e->hcopy_job)
        return ATG_OK;
    HostJob &j = *e->hcopy_job;
    HostChunk &c = j.chunks[e->hcopy_chunk];
    e->hcopy_job = nullptr;
    HostStage &h = e->hs[c.stage];
    HIP_TRY(hipEventSynchronize(h.ev_d2h));
    if (c.staged_out && c.out_bytes)
        par_memcpy(j.out + c.out0, h.p_out, c.out_bytes, host_threads());
    return ATG_OK;
}

// the oldest chunk in flight: wait for its batch, pack its images on the
// device, queue their copy to host memory, fill its results
atg_status host_collect(atg_engine *e)
{
    HostJob &j = *e->hflight.front().first;
    const size_t ci = e->hflight.front().second;
    e->hflight.pop_front();
    HostChunk &c = j.chunks[ci];
    HostStage &h = e->hs[c.stage];
    EncSlot *sl = nullptr;
    atg_status s2 = wait_ticket(e, c.ticket, sl);
    if (s2 != ATG_OK)
        return s2;
    sl->host = false;
    const Plan &cp = *c.plan;
    const size_t nt = cp.tracks.size();
    // the stage's previous offsets upload (before its pack, same stream)
    // has read p_off
    HIP_TRY(hipEventSynchronize(h.ev_packed));
    HIP_TRY(ensure_pinned(h.p_off, h.p_off_cap, std::max<size_t>(nt, 1)));
    uint64_t pos = 0;
    for (size_t k = 0; k < nt; ++k) {
        h.p_off[k] = pos;
        pos += (sl->tout_h[k].bytes + 15u) & ~15ull;
    }
    c.out0 = j.out_pos;
    c.out_bytes = pos;
    j.out_pos += pos;
    // growth frees the stage's buffers: the previous occupant's offsets
    // upload, pack and download must be done
    if (std::max<size_t>(nt, 1) * sizeof(uint64_t) > h.d_off.cap ||
        std::max<uint64_t>(pos, 16) > h.d_pack.cap) {
        HIP_TRY(hipStreamSynchronize(e->s_hpack));
        HIP_TRY(hipStreamSynchronize(e->s_d2h));
    }
    HIP_TRY(h.d_off.ensure(std::max<size_t>(nt, 1) * sizeof(uint64_t)));
    HIP_TRY(h.d_pack.ensure(std::max<uint64_t>(pos, 16)));
    // the pack overwrites d_pack: the previous occupant's download is done
    HIP_TRY(hipStreamWaitEvent(e->s_hpack, h.ev_d2h, 0));
    if (nt)
        HIP_TRY(hipMemcpyAsync(h.d_off.p, h.p_off, nt * sizeof(uint64_t), hipMemcpyHostToDevice,
                               e->s_hpack));
    HIP_TRY(launch_pack_images((const uint8_t *)h.d_img.p, (const TrackInfo *)sl->tracks.p,
                               (const TrackOut *)sl->tout.p, (const uint64_t *)h.d_off.p,
                               (uint32_t)nt, (uint8_t *)h.d_pack.p, e->s_hpack));
    HIP_TRY(hipEventRecord(h.ev_packed, e->s_hpack));
    HIP_TRY(hipEventRecord(sl->ev_reuse, e->s_hpack));
    sl->reuse_pending = true;
    HIP_TRY(hipStreamWaitEvent(e->s_d2h, h.ev_packed, 0));
    c.staged_out = !j.pin_out;
    uint8_t *dst = j.out + c.out0;
    if (c.staged_out) {
        HIP_TRY(ensure_pinned(h.p_out, h.p_out_cap, std::max<uint64_t>(pos, 16)));
        dst = h.p_out;
    }
    if (pos)
        HIP_TRY(hipMemcpyAsync(dst, h.d_pack.p, pos, hipMemcpyDeviceToHost, e->s_d2h));
    HIP_TRY(hipEventRecord(h.ev_d2h, e->s_d2h));
    for (size_t k = 0; k < nt; ++k) {
        const uint32_t t = c.t0 + (uint32_t)k;
        const TrackOut &to = sl->tout_h[k];
        atg_track_result &r = j.results[t];
        r.out_offset = c.out0 + h.p_off[k];
        r.bytes = to.bytes;
        r.first_frame = j.whole.track_frame_pos[t];
        r.n_frames = j.whole.tracks[t].n_frames;
        r.min_frame_bytes = to.min_fs;
        r.max_frame_bytes = to.max_fs;
        std::memcpy(r.md5, to.md5, 16);
        r.status = 0;
        r.reserved = 0;
        const TrackInfo &ti = cp.tracks[k];
        for (uint32_t i = 0; i < ti.n_frames; ++i) {
            const uint32_t f = cp.order[ti.first_pos + i];
            if (j.frame_offsets)
                j.frame_offsets[r.first_frame + i] = sl->fdesc_h[f].out_off;
            if (j.frame_pcm_frames)
                j.frame_pcm_frames[r.first_frame + i] = cp.frames[f].n;
        }
    }
    // the previous staged chunk's bytes are in host memory by now
    s2 = host_finish_copy(e);
    if (s2 != ATG_OK)
        return s2;
    e->hcopy_job = &j;
    e->hcopy_chunk = ci;
    ++j.collected;
    return ATG_OK;
}

// a failure inside the pipeline: drain the device, fail every job in
// flight (their device state is gone) and free the slots
atg_status host_drain(atg_engine *e, atg_status err)
{
    const std::string msg = g_err;
    const bool device_ok = hipDeviceSynchronize() == hipSuccess;
    // a fully collected job may still have its last chunk's images in pinned
    // staging: its D2H is complete now, so finish the copy (or fail the job
    // if the device itself failed) rather than drop it
    if (e->hcopy_job) {
        HostJob &j = *e->hcopy_job;
        const HostChunk &c = j.chunks[e->hcopy_chunk];
        if (device_ok && c.staged_out && c.out_bytes)
            par_memcpy(j.out + c.out0, e->hs[c.stage].p_out, c.out_bytes, host_threads());
        else if (!device_ok && j.status == ATG_OK) {
            j.status = err;
            j.error = msg;
        }
        e->hcopy_job = nullptr;
    }
    for (EncSlot &s2 : e->slot)
        if (s2.busy && s2.host) {
            s2.busy = false;
            s2.done = false;
            s2.host = false;
            s2.ticket = 0;
            s2.end_pending = false;
        }
    for (auto &jp : e->hjobs)
        if (jp->collected < jp->chunks.size() && jp->status == ATG_OK) {
            jp->status = err;
            jp->error = msg;
        }
    e->hflight.clear();
    g_err = msg;
    return err;
}

// upload chunk ci of job j and enqueue its encode.  The upload is queued
// first; then, when every slot is busy, the oldest chunk is collected (its
// batch waited) before this chunk's encode is enqueued -- so the copy
// engine already holds this upload while the host waits
atg_status host_enqueue(atg_engine *e, HostJob &j, size_t ci, const atg_flac_options *opts)
{
    (void)opts;
    {
        atg_status st = ensure_host_streams(e);
        if (st == ATG_OK)
            st = ensure_host_pack_stream(e);
        if (st != ATG_OK)
            return st;
    }
    // the stage's previous occupant (kHostStages chunks back) must be
    // collected: with kEncSlots chunks in flight it is, except when a
    // caller's pipeline is shallower than the stages
    while (e->hflight.size() >= kHostStages) {
        atg_status st = host_collect(e);
        if (st != ATG_OK)
            return st;
    }
    HostChunk &c = j.chunks[ci];
    c.stage = (size_t)(e->hseq % kHostStages);
    HostStage &h = e->hs[c.stage];
    const uint64_t in_bytes = c.samples * j.elem;
    // stage c.stage last held the chunk kHostStages enqueues back, collected
    // (waited, packed) by now; its device buffers are reused in stream order.
    // A buffer that must grow is freed only once the copy stream is idle:
    // the previous occupant's pack kernel and download may still read it
    if (in_bytes + 16 > h.d_pcm.cap || c.plan->out_bytes + 16 > h.d_img.cap)
        HIP_TRY(hipStreamSynchronize(e->s_hpack));
    HIP_TRY(h.d_pcm.ensure(in_bytes + 16));
    HIP_TRY(h.d_img.ensure(c.plan->out_bytes + 16));
    const uint8_t *src = j.pcm + c.pcm0 * j.elem;
    if (in_bytes && !j.pin_in) {
        HIP_TRY(hipEventSynchronize(h.ev_h2d)); // its previous upload has finished
        HIP_TRY(ensure_pinned(h.p_in, h.p_in_cap, in_bytes + 16));
        par_memcpy(h.p_in, src, in_bytes, host_threads());
        src = h.p_in;
    }
    // the encode overwrites d_img: the previous occupant's images must have
    // been packed first
    HIP_TRY(hipStreamWaitEvent(e->s_h2d, h.ev_packed, 0));
    if (in_bytes)
        HIP_TRY(hipMemcpyAsync(h.d_pcm.p, src, in_bytes, hipMemcpyHostToDevice, e->s_h2d));
    HIP_TRY(hipEventRecord(h.ev_h2d, e->s_h2d));
    if (e->hflight.size() >= kEncSlots) {
        atg_status st = host_collect(e);
        if (st != ATG_OK)
            return st;
    }
    EncSlot *sl = nullptr;
    uint64_t ticket = 0;
    atg_status st = take_slot(e, sl, ticket);
    if (st == ATG_OK)
        st = enqueue_batch(e, *sl, c.plan, h.d_pcm.p, j.fmt, (uint8_t *)h.d_img.p, h.d_img.cap,
                           true, h.ev_h2d, true, true);
    if (st != ATG_OK) {
        if (sl) {
            sl->uploaded = nullptr;
            sl->ticket = 0;
            sl->end_pending = false;
        }
        return st;
    }
    sl->busy = true;
    sl->host = true;
    c.ticket = ticket;
    ++e->hseq;
    e->hflight.emplace_back(&j, ci);
    return ATG_OK;
}

// no batch or host job in flight
bool engine_idle(const atg_engine *e)
{
    for (const EncSlot &sl : e->slot)
        if (sl.busy)
            return false;
    return e->hjobs.empty() && e->hflight.empty();
}

// a new slot rotation of n slots (the engine idle): tickets map to slots by
// ticket % depth, so the rotation starts clean; slots past the new depth
// give their device workspaces back (a 1024-track config-2 slot holds ~130
// MB of tables)
void set_depth(atg_engine *e, uint64_t n)
{
    for (EncSlot &sl : e->slot) {
        sl.ticket = 0;
        sl.done = false;
    }
    for (uint64_t k = n; k < kMaxSlots; ++k) {
        EncSlot &sl = e->slot[k];
        for (DevBuf *b : {&sl.frames, &sl.tracks, &sl.order, &sl.coef, &sl.shift, &sl.est,
                          &sl.sub, &sl.fdesc, &sl.tout, &sl.err, &sl.rice_big, &sl.scratch,
                          &sl.slow, &sl.md5in, &sl.dpack})
            b->release();
        sl.uploaded = nullptr;
        sl.plan.reset();
    }
    e->depth = n;
}

// Batches in flight for a pipelined device batch when the caller has not
// set the depth.  A batch's MD5 chains take ~0.8 us per 64-byte block of its
// longest track whatever the batch width (md5.hip), its kernels ~8 ms per
// 65,536 frames of 4096 samples (config 2); with chain / kernels = r the
// rolled MD5 hides the chains at: 12 in flight for r <= 2 (config 2, 1024
// tracks: 7.99 ms per step against 8.30 at 3), 24 for r <= 4 (512 tracks:
// 8.12-8.15 M frames/s against 7.95-8.05 at 16), 32 above (256 and 128
// tracks: 5.91-5.94 M at 128 tracks against 5.76-5.83 at 24) -- the
// narrow-leg measurements of round 5 (profiles/r05_zz_final_bench.json,
// r05_zm_narrow_depth.json).  Bounded so the slots' tables (~2 KB per
// frame) stay under 16 GB; 3 (the split-chain rotation) when the chains
// are short next to the kernels or not on the GPU at all.
uint64_t auto_depth(atg_engine *e, const Plan &pl, int fmt)
{
    const FlacParams &p = pl.p;
    if (pl.frames_only || pl.tracks.empty() || want_host_md5(e, pl, fmt, false) ||
        !track_md5_paired(p, fmt))
        return kEncSlots;
    uint64_t maxb = 0, samples = 0;
    for (const TrackInfo &t : pl.tracks) {
        maxb = std::max<uint64_t>(maxb, t.pcm_frames * p.channels * ((p.bps + 7) / 8));
        samples += t.pcm_frames;
    }
    const double chain_ms = (double)maxb / 64.0 * 0.8e-3;
    // (a batch's seven launches and copies take ~0.5 ms however small it is)
    const double kernel_ms = std::max(0.5, (double)samples / 4096.0 * (8.0 / 65536.0) *
                                               (double)p.channels / 2.0);
    const double r = chain_ms / kernel_ms;
    uint64_t d = r < 0.25 ? kEncSlots : r <= 2.0 ? 12 : r <= 4.0 ? 24 : kMaxSlots;
    const uint64_t cap = (16ull << 30) / std::max<uint64_t>(1, pl.frames.size() * 2048ull);
    return std::max<uint64_t>(kEncSlots, std::min(d, cap));
}

} // namespace

extern "C" {

int atg_abi_version(void) { return ATG_ABI_VERSION; }

const char *atg_last_error(void) { return g_err.c_str(); }

atg_status atg_engine_create(int device, atg_engine **out)
{
    return atg_engine_create_ex(device, 0, out);
}

atg_status atg_engine_create_ex(int device, uint32_t flags, atg_engine **out)
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
    e->flags = flags;
    HIP_TRY(hipStreamCreateWithFlags(&e->s_main, hipStreamNonBlocking));
    // every stream now, in this order, unless the caller streams one track
    // at a time (ATG_ENGINE_STREAMING): the order fixes the streams'
    // hardware queues, and the device-resident step is 9.4 ms with it
    // against 10.3 ms with streams created on first use
    // (profiles/r03_l_streams_ab.txt).  A streaming engine (encode_flac, one
    // process per track under track2track) holds two streams, and 8 such
    // processes run 49.8 k frames/s against 17.6 k
    if (!(flags & ATG_ENGINE_STREAMING)) {
        // the default rotation's aux streams; more slots (set_inflight) run
        // rolled, on two engine streams created on first use
        for (uint64_t k = 0; k < kEncSlots; ++k)
            if (ensure_aux_stream(e->slot[k]) != ATG_OK)
                return ATG_ERR_DEVICE;
        if (ensure_host_streams(e) != ATG_OK)
            return ATG_ERR_DEVICE;
        // created last: the streams above keep their hardware queues
        HIP_TRY(hipStreamCreateWithFlags(&e->s_pack, hipStreamNonBlocking));
    }
    for (EncSlot &sl : e->slot) {
        for (auto &ev : sl.ev)
            HIP_TRY(hipEventCreate(&ev));
        HIP_TRY(hipEventCreateWithFlags(&sl.ev_tables, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&sl.ev_pack, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&sl.ev_reuse, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&sl.ev_done, hipEventDisableTiming));
    }
    for (HostStage &h : e->hs) {
        HIP_TRY(hipEventCreateWithFlags(&h.ev_h2d, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&h.ev_packed, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&h.ev_d2h, hipEventDisableTiming));
    }
    static uint32_t t16[4][256], t8[256];
    static uint16_t adv[24][16], advq[kCrcQ][6][16];
    build_crc_tables(t16, t8, adv, advq);
    HIP_TRY(upload_crc_tables(&adv[0][0], &t16[0][0], t8, &advq[0][0][0]));
    *out = e;
    return ATG_OK;
}

void atg_engine_destroy(atg_engine *e)
{
    if (!e)
        return;
    (void)hipSetDevice(e->device);
    (void)hipStreamSynchronize(e->s_main);
    for (hipStream_t q : {e->s_pack, e->s_md5})
        if (q)
            (void)hipStreamSynchronize(q);
    for (EncSlot &sl : e->slot) {
        for (std::future<void> &f : sl.hash_jobs) // a batch never waited
            f.wait();
        sl.hash_jobs.clear();
        if (sl.s_aux)
            (void)hipStreamSynchronize(sl.s_aux);
        for (DevBuf *b : {&sl.frames, &sl.tracks, &sl.order, &sl.coef, &sl.shift, &sl.est,
                          &sl.sub, &sl.fdesc, &sl.tout, &sl.err, &sl.rice_big, &sl.scratch,
                          &sl.md5in, &sl.dpack})
            b->release();
        for (void *q : {(void *)sl.hpcm, (void *)sl.hmd5})
            if (q)
                (void)hipHostFree(q);
        if (sl.ev_hpcm)
            (void)hipEventDestroy(sl.ev_hpcm);
        for (auto &ev : sl.ev)
            (void)hipEventDestroy(ev);
        (void)hipEventDestroy(sl.ev_tables);
        (void)hipEventDestroy(sl.ev_pack);
        if (sl.ev_reuse)
            (void)hipEventDestroy(sl.ev_reuse);
        (void)hipEventDestroy(sl.ev_done);
        if (sl.tout_h)
            (void)hipHostFree(sl.tout_h);
        if (sl.fdesc_h)
            (void)hipHostFree(sl.fdesc_h);
        if (sl.err_h)
            (void)hipHostFree(sl.err_h);
        if (sl.s_aux)
            (void)hipStreamDestroy(sl.s_aux);
    }
    for (hipStream_t q : {e->s_h2d, e->s_hpack, e->s_d2h})
        if (q)
            (void)hipStreamSynchronize(q);
    for (HostStage &h : e->hs) {
        for (DevBuf *b : {&h.d_pcm, &h.d_img, &h.d_pack, &h.d_off})
            b->release();
        for (void *q : {(void *)h.p_in, (void *)h.p_out, (void *)h.p_off})
            if (q)
                (void)hipHostFree(q);
        (void)hipEventDestroy(h.ev_h2d);
        (void)hipEventDestroy(h.ev_packed);
        (void)hipEventDestroy(h.ev_d2h);
    }
    for (hipStream_t q : {e->s_h2d, e->s_hpack, e->s_d2h})
        if (q)
            (void)hipStreamDestroy(q);
    e->windows.release();
    if (e->ev_win)
        (void)hipEventDestroy(e->ev_win);
    for (hipStream_t q : {e->s_pack, e->s_md5})
        if (q)
            (void)hipStreamDestroy(q);
    (void)hipStreamDestroy(e->s_main);
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

atg_status atg_flac_encode_device_async(atg_engine *e, const atg_flac_options *opts,
                                        const void *d_pcm, atg_pcm_format format,
                                        const atg_track *tracks, uint32_t n_tracks,
                                        uint32_t channels, uint32_t bps, uint32_t rate,
                                        void *d_out, uint64_t out_cap, uint64_t *ticket)
{
    ATG_HANDLE_LOCK(e);
    if (!e || (!tracks && n_tracks) || !ticket)
        return fail(ATG_ERR_INVALID, "NULL argument");
    if (format == ATG_PCM_S16 && bps > 16)
        return fail(ATG_ERR_INVALID, "S16 container with bits_per_sample > 16");
    if (!e->hflight.empty())
        return fail(ATG_ERR_INVALID, "a host encode job is in flight: wait for it first");
    std::shared_ptr<Plan> pl;
    atg_status st = get_plan(e, opts, tracks, n_tracks, channels, bps, rate, pl);
    if (st != ATG_OK)
        return st;
    // the first batch of a pipeline picks the depth unless the caller set it
    if (!e->depth_user && !e->sync_call && engine_idle(e)) {
        const uint64_t d = auto_depth(e, *pl, (int)format);
        if (d != e->depth)
            set_depth(e, d);
    }
    EncSlot *sl = nullptr;
    uint64_t t = 0;
    st = take_slot(e, sl, t);
    if (st != ATG_OK)
        return st;
    st = enqueue_batch(e, *sl, pl, d_pcm, (int)format, (uint8_t *)d_out, out_cap, false, nullptr,
                       !e->sync_call);
    if (st != ATG_OK) {
        // nothing of this batch may be relied on: drain what was queued
        drain_slot(e, *sl);
        auto it = std::find(e->roll_q.begin(), e->roll_q.end(), sl);
        if (it != e->roll_q.end())
            e->roll_q.erase(it);
        sl->uploaded = nullptr;
        sl->ticket = 0;
        sl->end_pending = false;
        return st;
    }
    sl->busy = true;
    *ticket = t;
    return ATG_OK;
}

atg_status atg_flac_encode_wait(atg_engine *e, uint64_t ticket, atg_track_result *results)
{
    ATG_HANDLE_LOCK(e);
    if (!e)
        return fail(ATG_ERR_INVALID, "NULL engine");
    EncSlot *sl = nullptr;
    atg_status st = wait_ticket(e, ticket, sl);
    if (st != ATG_OK)
        return st;
    if (results)
        fill_results(*sl->plan, sl->tout_h, results, nullptr, nullptr, nullptr);
    return ATG_OK;
}

atg_status atg_flac_encode_device(atg_engine *e, const atg_flac_options *opts,
                                  const void *d_pcm, atg_pcm_format format,
                                  const atg_track *tracks, uint32_t n_tracks,
                                  uint32_t channels, uint32_t bps, uint32_t rate, void *d_out,
                                  uint64_t out_cap, atg_track_result *results)
{
    ATG_HANDLE_LOCK(e);
    if (!e || (!tracks && n_tracks) || (!results && n_tracks))
        return fail(ATG_ERR_INVALID, "NULL argument");
    uint64_t t = 0;
    e->sync_call = true; // waited at once: no split MD5 chain
    atg_status st = atg_flac_encode_device_async(e, opts, d_pcm, format, tracks, n_tracks,
                                                 channels, bps, rate, d_out, out_cap, &t);
    e->sync_call = false;
    if (st != ATG_OK)
        return st;
    return atg_flac_encode_wait(e, t, results);
}

atg_status atg_flac_encode_host_async(atg_engine *e, const atg_flac_options *opts,
                                      const void *pcm, atg_pcm_format format,
                                      const atg_track *tracks, uint32_t n_tracks,
                                      uint32_t channels, uint32_t bps, uint32_t rate,
                                      uint8_t *out, uint64_t out_cap, atg_track_result *results,
                                      uint64_t *frame_offsets, uint32_t *frame_pcm_frames,
                                      uint64_t *ticket)
{
    ATG_HANDLE_LOCK(e);
    if (!e || (!tracks && n_tracks) || (!results && n_tracks) || !ticket)
        return fail(ATG_ERR_INVALID, "NULL argument");
    if (format == ATG_PCM_S16 && bps > 16)
        return fail(ATG_ERR_INVALID, "S16 container with bits_per_sample > 16");
    auto jp = std::make_unique<HostJob>();
    HostJob &j = *jp;
    // the whole job's layout (what atg_flac_batch_bounds sized)
    atg_status st = make_plan(opts, tracks, n_tracks, channels, bps, rate, j.whole);
    if (st != ATG_OK)
        return st;
    if (j.whole.out_bytes > out_cap)
        return fail(ATG_ERR_CAPACITY, "output buffer too small for this batch");
    HIP_TRY(hipSetDevice(e->device));
    // the slots' device state is shared: an unwaited device batch would
    // lose its results
    for (EncSlot &s2 : e->slot)
        if (s2.busy && !s2.host)
            return fail(ATG_ERR_INVALID, "an async encode batch is in flight: wait for it first");
    // the host pipeline runs kEncSlots chunks on the default rotation (the
    // slots with aux streams from creation); an automatic deeper rotation a
    // device pipeline left behind is undone
    if (!e->depth_user && e->depth != kEncSlots && engine_idle(e))
        set_depth(e, kEncSlots);
    j.elem = format == ATG_PCM_S16 ? 2 : 4;
    j.fmt = (int)format;
    j.pcm = (const uint8_t *)pcm;
    j.out = out;
    j.results = results;
    j.frame_offsets = frame_offsets;
    j.frame_pcm_frames = frame_pcm_frames;
    // page-locked caller buffers are copied by DMA directly; pageable ones
    // go through pinned staging (copied on host threads)
    j.pin_in = is_pinned(pcm);
    j.pin_out = is_pinned(out);
    {
        uint32_t t = 0;
        while (t < n_tracks) {
            HostChunk c;
            c.t0 = t;
            uint64_t lo = UINT64_MAX, hi = 0;
            do {
                lo = std::min<uint64_t>(lo, tracks[t].pcm_offset * channels);
                hi = std::max<uint64_t>(hi, (tracks[t].pcm_offset + tracks[t].pcm_frames) *
                                                channels);
                ++t;
            } while (t < n_tracks && (hi - std::min<uint64_t>(lo, tracks[t].pcm_offset * channels) +
                                      tracks[t].pcm_frames * channels) * j.elem <= e->chunk_bytes);
            c.t1 = t;
            c.pcm0 = lo == UINT64_MAX ? 0 : lo;
            c.samples = hi > c.pcm0 ? hi - c.pcm0 : 0;
            for (uint32_t k = c.t0; k < c.t1; ++k) {
                atg_track a = tracks[k];
                a.pcm_offset -= c.pcm0 / channels;
                c.tr.push_back(a);
            }
            c.plan = std::make_shared<Plan>();
            st = make_plan(opts, c.tr.data(), (uint32_t)c.tr.size(), channels, bps, rate, *c.plan);
            if (st != ATG_OK)
                return st;
            j.chunks.push_back(std::move(c));
        }
    }
    j.id = e->next_hjob++;
    e->hjobs.push_back(std::move(jp));
    for (size_t ci = 0; ci < j.chunks.size(); ++ci) {
        st = host_enqueue(e, j, ci, opts);
        if (st != ATG_OK) {
            host_drain(e, st);
            break;
        }
    }
    *ticket = j.id;
    return ATG_OK; // a failure above is reported by the job's wait
}

atg_status atg_flac_encode_host_wait(atg_engine *e, uint64_t ticket)
{
    ATG_HANDLE_LOCK(e);
    if (!e)
        return fail(ATG_ERR_INVALID, "NULL engine");
    size_t k = 0;
    while (k < e->hjobs.size() && e->hjobs[k]->id != ticket)
        ++k;
    if (k == e->hjobs.size())
        return fail(ATG_ERR_INVALID, "unknown or expired host job ticket");
    HostJob *j = e->hjobs[k].get();
    HIP_TRY(hipSetDevice(e->device));
    // chunks are collected in submission order: everything up to this job's
    // last chunk, then its last staged copy
    while (j->status == ATG_OK && j->collected < j->chunks.size()) {
        if (e->hflight.empty())
            break;
        atg_status st = host_collect(e);
        if (st != ATG_OK)
            host_drain(e, st);
    }
    if (j->status == ATG_OK && e->hcopy_job == j) {
        atg_status st = host_finish_copy(e);
        if (st != ATG_OK)
            host_drain(e, st);
    }
    const atg_status st = j->status;
    const std::string msg = j->error;
    e->hjobs.erase(e->hjobs.begin() + (std::ptrdiff_t)k);
    if (st != ATG_OK)
        return fail(st, msg);
    return ATG_OK;
}

atg_status atg_flac_encode_host(atg_engine *e, const atg_flac_options *opts, const void *pcm,
                                atg_pcm_format format, const atg_track *tracks,
                                uint32_t n_tracks, uint32_t channels, uint32_t bps,
                                uint32_t rate, uint8_t *out, uint64_t out_cap,
                                atg_track_result *results, uint64_t *frame_offsets,
                                uint32_t *frame_pcm_frames)
{
    ATG_HANDLE_LOCK(e);
    uint64_t t = 0;
    atg_status st = atg_flac_encode_host_async(e, opts, pcm, format, tracks, n_tracks, channels,
                                               bps, rate, out, out_cap, results, frame_offsets,
                                               frame_pcm_frames, &t);
    if (st != ATG_OK)
        return st;
    return atg_flac_encode_host_wait(e, t);
}

uint64_t atg_flac_stream_header(const atg_flac_options *o, uint32_t channels, uint32_t bps,
                                uint32_t rate, uint64_t total_samples, uint32_t min_frame_bytes,
                                uint32_t max_frame_bytes, const uint8_t *md5, uint8_t *out,
                                uint64_t cap)
{
    // fLaC + STREAMINFO (flacenc_write_streaminfo, flac.c:376-409, fields
    // clamped) + VORBIS_COMMENT with the vendor string + PADDING
    // (flac.c:208-238): the bytes k_stream_header writes on the device
    static const char vendor[] = "Python Audio Tools 2.22alpha1";
    const uint32_t vlen = (uint32_t)sizeof(vendor) - 1u;
    if (!o || !md5 || channels < 1 || bps < 1 || o->padding_size > 0xFFFFFFu)
        return 0;
    const uint64_t need = 4 + 4 + 34 + 4 + 4 + vlen + 4 + 4 + (uint64_t)o->padding_size;
    if (!out || cap < need)
        return 0;
    uint64_t n = 0;
    auto put = [&](uint8_t b) { out[n++] = b; };
    put('f'); put('L'); put('a'); put('C');
    put(0x00); put(0); put(0); put(34);
    // 34 STREAMINFO bytes, MSB first
    uint8_t si[34] = {0};
    uint32_t bitpos = 0;
    auto bits = [&](uint32_t count, uint64_t v) {
        for (uint32_t i = count; i-- > 0; ++bitpos)
            if ((v >> i) & 1u)
                si[bitpos >> 3] |= (uint8_t)(0x80u >> (bitpos & 7u));
    };
    const uint32_t bs = o->block_size > 0xFFFFu ? 0xFFFFu : o->block_size;
    bits(16, bs);
    bits(16, bs);
    bits(24, min_frame_bytes > 0xFFFFFFu ? 0xFFFFFFu : min_frame_bytes);
    bits(24, max_frame_bytes > 0xFFFFFFu ? 0xFFFFFFu : max_frame_bytes);
    bits(20, rate > 0xFFFFFu ? 0xFFFFFu : rate);
    bits(3, channels - 1u > 7u ? 7u : channels - 1u);
    bits(5, bps - 1u > 31u ? 31u : bps - 1u);
    bits(36, total_samples & 0xFFFFFFFFFull);
    for (int i = 0; i < 16; ++i)
        bits(8, md5[i]);
    for (int i = 0; i < 34; ++i)
        put(si[i]);
    const uint32_t vc = 4u + vlen + 4u;
    put(0x04); put((uint8_t)(vc >> 16)); put((uint8_t)(vc >> 8)); put((uint8_t)vc);
    put((uint8_t)vlen); put(0); put(0); put(0);
    for (uint32_t i = 0; i < vlen; ++i)
        put((uint8_t)vendor[i]);
    put(0); put(0); put(0); put(0);
    put(0x81); put((uint8_t)(o->padding_size >> 16)); put((uint8_t)(o->padding_size >> 8));
    put((uint8_t)o->padding_size);
    std::memset(out + n, 0, o->padding_size);
    return need;
}

atg_status atg_flac_encode_frames_batch(atg_engine *e, const atg_flac_options *opts,
                                        const void *pcm, atg_pcm_format format,
                                        const atg_segment *segs, uint32_t n, uint32_t channels,
                                        uint32_t bps, uint32_t rate, uint8_t *out,
                                        uint64_t out_cap, uint64_t *seg_offsets,
                                        uint64_t *seg_bytes, uint32_t *frame_bytes)
{
    ATG_HANDLE_LOCK(e);
    if (!e || (!segs && n) || (!seg_offsets && n) || (!seg_bytes && n))
        return fail(ATG_ERR_INVALID, "NULL argument");
    if (format == ATG_PCM_S16 && bps > 16)
        return fail(ATG_ERR_INVALID, "S16 container with bits_per_sample > 16");
    for (EncSlot &s2 : e->slot)
        if (s2.busy)
            return fail(ATG_ERR_INVALID, "an async encode batch is in flight: wait for it first");
    std::vector<atg_track> tr(n);
    std::vector<uint32_t> bases(n);
    uint64_t pcm_end = 0;
    for (uint32_t k = 0; k < n; ++k) {
        const atg_segment &g = segs[k];
        const uint64_t nfr = g.frame_sizes ? g.n_frame_sizes
                                           : (opts && opts->block_size
                                                  ? (g.pcm_frames + opts->block_size - 1) /
                                                        opts->block_size
                                                  : 0);
        // the frame header's UTF-8 number holds 31 bits (flac.c:1531-1566)
        if (g.first_frame_number + nfr > 0x7FFFFFFFull)
            return fail(ATG_ERR_INVALID, "frame numbers beyond 2^31 - 1");
        tr[k].pcm_offset = g.pcm_offset;
        tr[k].pcm_frames = g.pcm_frames;
        tr[k].frame_sizes = g.frame_sizes;
        tr[k].n_frame_sizes = g.n_frame_sizes;
        bases[k] = (uint32_t)g.first_frame_number;
        pcm_end = std::max<uint64_t>(pcm_end, g.pcm_offset + g.pcm_frames);
    }
    if (!pcm && pcm_end)
        return fail(ATG_ERR_INVALID, "NULL pcm");
    auto pl = std::make_shared<Plan>();
    atg_status st = make_plan(opts, tr.data(), n, channels, bps, rate, *pl, true, 0,
                              bases.data());
    if (st != ATG_OK)
        return st;
    HIP_TRY(hipSetDevice(e->device));
    HostStage &h = e->hs[0];
    const size_t elem = format == ATG_PCM_S16 ? 2 : 4;
    const uint64_t in_bytes = pcm_end * channels * elem;
    HIP_TRY(h.d_pcm.ensure(in_bytes + 16));
    HIP_TRY(h.d_img.ensure(pl->out_bytes + 16));
    // the previous host-pipeline batch is finished (no slot busy); its
    // packing kernel may still read d_img
    HIP_TRY(hipStreamWaitEvent(e->s_main, h.ev_packed, 0));
    if (in_bytes)
        HIP_TRY(hipMemcpyAsync(h.d_pcm.p, pcm, in_bytes, hipMemcpyHostToDevice, e->s_main));
    HIP_TRY(hipEventRecord(h.ev_h2d, e->s_main)); // the batch's LPC kernel waits for it
    // a synchronous call (no slot busy, checked above) always takes slot 0:
    // one aux stream for a streaming process's whole life.  The slot's
    // earlier results are gone with it (atgpu.h)
    e->next_ticket += (e->depth - e->next_ticket % e->depth) % e->depth;
    EncSlot *sl = nullptr;
    uint64_t ticket = 0;
    st = take_slot(e, sl, ticket);
    if (st == ATG_OK)
        st = enqueue_batch(e, *sl, pl, h.d_pcm.p, (int)format, (uint8_t *)h.d_img.p,
                           h.d_img.cap, true, h.ev_h2d, false);
    if (st != ATG_OK) {
        (void)hipDeviceSynchronize();
        if (sl) {
            sl->uploaded = nullptr;
            sl->ticket = 0;
            sl->end_pending = false;
        }
        return st;
    }
    sl->busy = true;
    st = wait_ticket(e, ticket, sl);
    if (st != ATG_OK)
        return st;
    // the segments' frames packed back to back, 16-byte aligned
    uint64_t pos = 0;
    HIP_TRY(ensure_pinned(h.p_off, h.p_off_cap, std::max<size_t>(n, 1)));
    for (uint32_t k = 0; k < n; ++k) {
        seg_offsets[k] = pos;
        seg_bytes[k] = sl->tout_h[k].bytes;
        h.p_off[k] = pos;
        pos += (sl->tout_h[k].bytes + 15u) & ~15ull;
    }
    if (pos > out_cap)
        return fail(ATG_ERR_CAPACITY, "output buffer too small for the segments' frames");
    if (pos) {
        HIP_TRY(h.d_off.ensure(std::max<size_t>(n, 1) * sizeof(uint64_t)));
        HIP_TRY(h.d_pack.ensure(pos));
        HIP_TRY(hipMemcpyAsync(h.d_off.p, h.p_off, n * sizeof(uint64_t), hipMemcpyHostToDevice,
                               e->s_main));
        HIP_TRY(launch_pack_images((const uint8_t *)h.d_img.p, (const TrackInfo *)sl->tracks.p,
                                   (const TrackOut *)sl->tout.p, (const uint64_t *)h.d_off.p, n,
                                   (uint8_t *)h.d_pack.p, e->s_main));
        HIP_TRY(hipEventRecord(h.ev_packed, e->s_main));
        HIP_TRY(hipMemcpyAsync(out, h.d_pack.p, pos, hipMemcpyDeviceToHost, e->s_main));
        HIP_TRY(hipStreamSynchronize(e->s_main));
    }
    if (frame_bytes) {
        uint64_t q = 0;
        for (uint32_t k = 0; k < n; ++k) {
            const TrackInfo &ti = pl->tracks[k];
            for (uint32_t i = 0; i < ti.n_frames; ++i)
                frame_bytes[q++] = sl->fdesc_h[pl->order[ti.first_pos + i]].bytes;
        }
    }
    return ATG_OK;
}

atg_status atg_flac_encode_frames(atg_engine *e, const atg_flac_options *opts, const void *pcm,
                                  atg_pcm_format format, uint64_t pcm_frames,
                                  const uint32_t *frame_sizes, uint64_t n_frame_sizes,
                                  uint32_t channels, uint32_t bps, uint32_t rate,
                                  uint64_t first_frame_number, uint8_t *out, uint64_t out_cap,
                                  uint64_t *out_bytes, uint32_t *frame_bytes)
{
    if (!e || (!pcm && pcm_frames) || !out_bytes)
        return fail(ATG_ERR_INVALID, "NULL argument");
    atg_segment g;
    g.pcm_offset = 0;
    g.pcm_frames = pcm_frames;
    g.frame_sizes = frame_sizes;
    g.n_frame_sizes = n_frame_sizes;
    g.first_frame_number = first_frame_number;
    uint64_t off = 0;
    // the packed segment is 16-byte padded: room for it, then the true size
    const uint64_t need = atg_flac_max_frames_bytes(opts, pcm_frames, frame_sizes,
                                                    n_frame_sizes, channels, bps);
    if (need && out_cap < ((need + 15u) & ~15ull)) {
        std::vector<uint8_t> tmp((need + 15u) & ~15ull);
        const atg_status st = atg_flac_encode_frames_batch(
            e, opts, pcm, format, &g, 1, channels, bps, rate, tmp.data(), tmp.size(), &off,
            out_bytes, frame_bytes);
        if (st != ATG_OK)
            return st;
        if (*out_bytes > out_cap)
            return fail(ATG_ERR_CAPACITY, "output buffer too small for the segment's frames");
        std::memcpy(out, tmp.data(), *out_bytes);
        return ATG_OK;
    }
    return atg_flac_encode_frames_batch(e, opts, pcm, format, &g, 1, channels, bps, rate, out,
                                        out_cap, &off, out_bytes, frame_bytes);
}

uint64_t atg_flac_max_frames_bytes(const atg_flac_options *opts, uint64_t pcm_frames,
                                   const uint32_t *frame_sizes, uint64_t n_frame_sizes,
                                   uint32_t channels, uint32_t bps)
{
    atg_track tr;
    tr.pcm_offset = 0;
    tr.pcm_frames = pcm_frames;
    tr.frame_sizes = frame_sizes;
    tr.n_frame_sizes = n_frame_sizes;
    Plan pl;
    if (make_plan(opts, &tr, 1, channels, bps, 44100, pl, true, 0) != ATG_OK)
        return 0;
    return pl.out_bytes;
}

atg_status atg_engine_set_inflight(atg_engine *e, uint32_t n)
{
    ATG_HANDLE_LOCK(e);
    if (!e || (n != 0 && (n < kEncSlots || n > kMaxSlots)))
        return fail(ATG_ERR_INVALID, "in-flight batches must be 3..32 (or 0: automatic)");
    if (!engine_idle(e))
        return fail(ATG_ERR_INVALID, "an encode batch or host job is in flight: wait for it first");
    e->depth_user = n != 0;
    if (n)
        set_depth(e, n);
    return ATG_OK;
}

uint32_t atg_engine_inflight(atg_engine *e)
{
    ATG_HANDLE_LOCK(e);
    return e ? (uint32_t)e->depth : 0u;
}

atg_status atg_engine_set_host_chunk_bytes(atg_engine *e, uint64_t bytes)
{
    ATG_HANDLE_LOCK(e);
    if (!e || !bytes)
        return fail(ATG_ERR_INVALID, "NULL engine or zero chunk size");
    e->chunk_bytes = bytes;
    return ATG_OK;
}

int atg_engine_kernel_times(atg_engine *e, const char **names, float *ms, int cap)
{
    ATG_HANDLE_LOCK(e);
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
    ATG_HANDLE_LOCK(e);
    if (!e || !d_ptr)
        return fail(ATG_ERR_INVALID, "NULL argument");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipMalloc(d_ptr, bytes ? bytes : 1));
    return ATG_OK;
}

atg_status atg_device_free(atg_engine *e, void *d_ptr)
{
    ATG_HANDLE_LOCK(e);
    if (!e)
        return fail(ATG_ERR_INVALID, "NULL engine");
    HIP_TRY(hipSetDevice(e->device));
    if (d_ptr)
        HIP_TRY(hipFree(d_ptr));
    return ATG_OK;
}

atg_status atg_host_alloc(uint64_t bytes, void **ptr)
{
    if (!ptr)
        return fail(ATG_ERR_INVALID, "NULL argument");
    *ptr = nullptr;
    if (hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
        *ptr = nullptr;
        return fail(ATG_ERR_NOMEM, "hipHostMalloc failed");
    }
    return ATG_OK;
}

void atg_host_free(void *ptr)
{
    if (ptr)
        (void)hipHostFree(ptr);
}

atg_status atg_copy_to_device(atg_engine *e, void *d_dst, const void *src, uint64_t bytes)
{
    ATG_HANDLE_LOCK(e);
    if (!e)
        return fail(ATG_ERR_INVALID, "NULL engine");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipMemcpy(d_dst, src, bytes, hipMemcpyHostToDevice));
    return ATG_OK;
}

atg_status atg_copy_device(atg_engine *e, void *d_dst, const void *d_src, uint64_t bytes)
{
    ATG_HANDLE_LOCK(e);
    if (!e)
        return fail(ATG_ERR_INVALID, "NULL engine");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipMemcpy(d_dst, d_src, bytes, hipMemcpyDeviceToDevice));
    return ATG_OK;
}

atg_status atg_host_gather(void *dst, const void *const *srcs, const uint64_t *bytes,
                           uint64_t n, uint32_t threads)
{
    if ((!dst || !srcs || !bytes) && n)
        return fail(ATG_ERR_INVALID, "NULL argument");
    std::vector<uint64_t> off(n + 1, 0);
    for (uint64_t i = 0; i < n; ++i)
        off[i + 1] = off[i] + bytes[i];
    const uint64_t total = off[n];
    const unsigned nt = (unsigned)std::max<uint64_t>(
        1, std::min<uint64_t>({threads ? threads : host_threads(), n, total / (4u << 20) + 1}));
    auto run = [&](unsigned k) {
        // parts whose first byte falls in thread k's share of the bytes
        const uint64_t lo = total * k / nt, hi = total * (k + 1) / nt;
        uint64_t i = (uint64_t)(std::upper_bound(off.begin(), off.end(), lo) - off.begin()) - 1;
        if (k == 0)
            i = 0;
        else if (off[i] < lo)
            ++i;
        for (; i < n && off[i] < hi; ++i)
            std::memcpy((uint8_t *)dst + off[i], srcs[i], bytes[i]);
    };
    if (nt == 1) {
        run(0);
        return ATG_OK;
    }
    std::vector<std::thread> th;
    for (unsigned k = 1; k < nt; ++k)
        th.emplace_back(run, k);
    run(0);
    for (auto &t : th)
        t.join();
    return ATG_OK;
}

atg_status atg_copy_to_host(atg_engine *e, void *dst, const void *d_src, uint64_t bytes)
{
    ATG_HANDLE_LOCK(e);
    if (!e)
        return fail(ATG_ERR_INVALID, "NULL engine");
    HIP_TRY(hipSetDevice(e->device));
    HIP_TRY(hipMemcpy(dst, d_src, bytes, hipMemcpyDeviceToHost));
    return ATG_OK;
}

} // extern "C"
