// Teardown probe: the bench's call sequence through the C ABI, in one
// process, for a host-instrumented (AddressSanitizer on host code only)
// build of libatgpu's objects (csrc/Makefile `asan`).  It replays what the
// round-5 bench did before its two exit-time crashes:
// pipelined device batches at depth 12 (rolled MD5), set_inflight(3), host
// jobs from pinned and from pageable buffers, a decoder at depth 8 over the
// images, then exits -- with every handle destroyed (`destroy`) or none
// (`leak`, the path an interpreter's finalisation takes when it never closes
// them).  ASan reports any host write through a freed or out-of-bounds
// pointer (engine threads, par_memcpy, result fills) with its stack.
//
//   teardown_probe [destroy|leak] [tracks] [frames]
#include "../include/atgpu.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        atg_status s_ = (x);                                                          \
        if (s_ != ATG_OK) {                                                           \
            std::fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, s_,  \
                         atg_last_error());                                           \
            std::exit(2);                                                             \
        }                                                                             \
    } while (0)

int main(int argc, char **argv)
{
    const bool leak = argc > 1 && std::strcmp(argv[1], "leak") == 0;
    const uint32_t n_tracks = argc > 2 ? (uint32_t)std::atoi(argv[2]) : 256u;
    const uint64_t frames = argc > 3 ? (uint64_t)std::atoi(argv[3]) : 16u;
    const uint64_t ns = frames * 4096u;
    const uint64_t total = (uint64_t)n_tracks * ns * 2u;

    // seeded sine + noise, as bench.py synth_batch (shape only)
    std::vector<int16_t> pcm(total);
    uint64_t rng = 0x5EED;
    for (uint32_t t = 0; t < n_tracks; ++t) {
        const double f1 = 100.0 + 19.0 * (t % 97), f2 = 2000.0 + 97.0 * (t % 89);
        for (uint64_t i = 0; i < ns; ++i)
            for (int c = 0; c < 2; ++c) {
                rng = rng * 6364136223846793005ull + 1442695040888963407ull;
                const double ph = 2.0 * M_PI * (double)i / 44100.0 * (c ? 1.3 : 1.0);
                double x = (0.4 * std::sin(ph * f1) + 0.2 * std::sin(ph * f2)) * 32767.0 +
                           (double)((int64_t)(rng >> 40) % 128 - 64);
                x = x > 32767 ? 32767 : x < -32768 ? -32768 : x;
                pcm[((uint64_t)t * ns + i) * 2 + c] = (int16_t)std::lrint(x);
            }
    }
    std::vector<atg_track> tr(n_tracks);
    for (uint32_t t = 0; t < n_tracks; ++t)
        tr[t] = {(uint64_t)t * ns, ns, nullptr, 0};
    atg_flac_options o = {4096, 12, 0, 6, 1, 0, 1, 0, 0, 0, 0, 4096};

    atg_engine *e = nullptr;
    CK(atg_engine_create(0, &e));
    uint64_t nf = 0, cap = 0;
    CK(atg_flac_batch_bounds(&o, tr.data(), n_tracks, 2, 16, &nf, &cap));
    void *d_pcm = nullptr;
    CK(atg_device_alloc(e, total * 2, &d_pcm));
    CK(atg_copy_to_device(e, d_pcm, pcm.data(), total * 2));

    // 1. pipelined device batches, 12 in flight (rolled MD5)
    const uint32_t depth = 12;
    CK(atg_engine_set_inflight(e, depth));
    std::vector<void *> d_out(depth);
    for (auto &p : d_out)
        CK(atg_device_alloc(e, cap, &p));
    std::vector<atg_track_result> res(n_tracks);
    std::deque<uint64_t> pend;
    for (uint32_t k = 0; k < 3 * depth; ++k) {
        uint64_t t = 0;
        CK(atg_flac_encode_device_async(e, &o, d_pcm, ATG_PCM_S16, tr.data(), n_tracks, 2, 16,
                                        44100, (uint8_t *)d_out[k % depth], cap, &t));
        pend.push_back(t);
        if (pend.size() >= depth) {
            CK(atg_flac_encode_wait(e, pend.front(), res.data()));
            pend.pop_front();
        }
    }
    uint64_t last_slot = 0;
    for (uint64_t k = 3 * depth - pend.size(); !pend.empty(); ++k) {
        CK(atg_flac_encode_wait(e, pend.front(), res.data()));
        pend.pop_front();
        last_slot = k % depth;
    }
    std::vector<uint8_t> images(cap);
    CK(atg_copy_to_host(e, images.data(), d_out[last_slot], cap));
    const std::vector<atg_track_result> dev_res = res; // the images' layout

    // 2. the host pipeline: queued pinned jobs, a synchronous pinned call,
    // a pageable call
    CK(atg_engine_set_inflight(e, 3));
    void *pin_in = nullptr, *pin_out[3] = {};
    CK(atg_host_alloc(total * 2, &pin_in));
    std::memcpy(pin_in, pcm.data(), total * 2);
    for (auto &p : pin_out)
        CK(atg_host_alloc(cap, &p));
    std::vector<uint64_t> offs(nf);
    std::vector<uint32_t> fpcm(nf);
    std::vector<std::vector<atg_track_result>> hres(3, std::vector<atg_track_result>(n_tracks));
    std::vector<std::vector<uint64_t>> hoffs(3, std::vector<uint64_t>(nf));
    std::vector<std::vector<uint32_t>> hfp(3, std::vector<uint32_t>(nf));
    std::deque<uint64_t> hp;
    for (uint32_t k = 0; k < 8; ++k) {
        uint64_t t = 0;
        CK(atg_flac_encode_host_async(e, &o, pin_in, ATG_PCM_S16, tr.data(), n_tracks, 2, 16,
                                      44100, (uint8_t *)pin_out[k % 3], cap,
                                      hres[k % 3].data(), hoffs[k % 3].data(), hfp[k % 3].data(),
                                      &t));
        hp.push_back(t);
        if (hp.size() > 2) {
            CK(atg_flac_encode_host_wait(e, hp.front()));
            hp.pop_front();
        }
    }
    while (!hp.empty()) {
        CK(atg_flac_encode_host_wait(e, hp.front()));
        hp.pop_front();
    }
    CK(atg_flac_encode_host(e, &o, pin_in, ATG_PCM_S16, tr.data(), n_tracks, 2, 16, 44100,
                            (uint8_t *)pin_out[0], cap, res.data(), offs.data(), fpcm.data()));
    std::vector<uint8_t> page_out(cap);
    CK(atg_flac_encode_host(e, &o, pcm.data(), ATG_PCM_S16, tr.data(), n_tracks, 2, 16, 44100,
                            page_out.data(), cap, res.data(), offs.data(), fpcm.data()));
    int bad = 0;
    for (uint32_t t = 0; t < n_tracks; ++t) {
        const atg_track_result &r = res[t];
        if (std::memcmp(page_out.data() + r.out_offset, (const uint8_t *)pin_out[0] + r.out_offset,
                        r.bytes) != 0)
            ++bad;
    }

    // 3. the decoder over the device images, 8 in flight (rolled MD5)
    atg_decoder *d = nullptr;
    CK(atg_decoder_create(0, &d));
    CK(atg_decoder_set_inflight(d, 8));
    std::vector<atg_flac_dec_track> dt(n_tracks);
    for (uint32_t t = 0; t < n_tracks; ++t) {
        atg_flac_streaminfo si;
        const atg_track_result &r = dev_res[t];
        if (atg_flac_read_metadata(images.data() + r.out_offset, r.bytes, &si, nullptr, 0) != 0) {
            std::fprintf(stderr, "metadata of track %u\n", t);
            return 2;
        }
        dt[t].data_offset = r.out_offset + si.frames_offset;
        dt[t].data_bytes = r.bytes - si.frames_offset;
        dt[t].total_samples = si.total_samples;
        dt[t].sample_rate = si.sample_rate;
        dt[t].channels = si.channels;
        dt[t].bits_per_sample = si.bits_per_sample;
        dt[t].max_block_size = si.max_block_size;
        std::memcpy(dt[t].md5, si.md5, 16);
    }
    std::vector<atg_flac_dec_result> dres(n_tracks);
    std::deque<uint64_t> dp;
    int dec_bad = 0;
    for (uint32_t k = 0; k < 20; ++k) {
        uint64_t t = 0;
        if (atg_flac_decode_device_async(d, d_out[last_slot], cap, dt.data(), n_tracks, &t) !=
            ATG_OK) {
            std::fprintf(stderr, "decode enqueue: %s\n", atg_decoder_last_error());
            return 2;
        }
        dp.push_back(t);
        if (dp.size() >= 8 || k == 19) {
            while (!dp.empty() && (dp.size() >= 8 || k == 19)) {
                const int32_t *pp = nullptr;
                uint64_t ts = 0;
                if (atg_flac_decode_wait(d, dp.front(), dres.data(), &pp, &ts) != ATG_OK) {
                    std::fprintf(stderr, "decode wait: %s\n", atg_decoder_last_error());
                    return 2;
                }
                for (const auto &r : dres)
                    dec_bad += r.status != 0;
                dp.pop_front();
            }
        }
    }
    // the streaming path (encode_flac's segments)
    std::vector<uint8_t> seg(atg_flac_max_frames_bytes(&o, ns, nullptr, 0, 2, 16) + 64);
    std::vector<uint32_t> fb(frames);
    uint64_t seg_bytes = 0;
    for (int k = 0; k < 4; ++k)
        CK(atg_flac_encode_frames(e, &o, pcm.data() + (uint64_t)k * ns * 2, ATG_PCM_S16, ns,
                                  nullptr, 0, 2, 16, 44100, 0, seg.data(), seg.size(), &seg_bytes,
                                  fb.data()));
    // a job left unwaited (the interpreter-exit case when `leak`)
    uint64_t dangling = 0;
    if (leak)
        CK(atg_flac_encode_host_async(e, &o, pcm.data(), ATG_PCM_S16, tr.data(), n_tracks, 2, 16,
                                      44100, page_out.data(), cap, res.data(), offs.data(),
                                      fpcm.data(), &dangling));
    std::printf("{\"mode\": \"%s\", \"tracks\": %u, \"frames\": %llu, \"host_pageable_vs_pinned_"
                "mismatches\": %d, \"decode_bad_status\": %d}\n",
                leak ? "leak" : "destroy", n_tracks, (unsigned long long)frames, bad, dec_bad);
    std::fflush(stdout);
    if (leak)
        return bad || dec_bad ? 1 : 0; // everything still open, a host job in flight
    atg_decoder_destroy(d);
    for (auto &p : d_out)
        CK(atg_device_free(e, p));
    CK(atg_device_free(e, d_pcm));
    atg_host_free(pin_in);
    for (auto &p : pin_out)
        atg_host_free(p);
    atg_engine_destroy(e);
    return bad || dec_bad ? 1 : 0;
}
