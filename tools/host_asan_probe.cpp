// Host-code probe, CPU only, under AddressSanitizer (csrc/Makefile
// `host-asan`: the library's objects with the host side instrumented).  No
// HIP call is made; it exercises the host code that parses untrusted bytes
// or writes caller memory:
//   * atg_flac_read_metadata / atg_alac_read_info on real images, every
//     truncation of them and byte-mutated copies (the metadata and atom
//     walkers must stay inside `len`);
//   * atg_flac_batch_bounds / atg_flac_max_frames_bytes / the stream
//     header on edge geometries;
//   * md5_cpu.h (the engine's host-hash mode) against the extension's
//     byte-wise MD5 for every container width;
//   * atg_host_gather against memcpy;
//   * the encoder service client against fake services on an abstract
//     socket: a good reply, a reply whose frame count or sizes disagree
//     with the request, an oversized byte count or error text, and a
//     service that never answers -- refused, nothing written past the
//     caller's buffers (guard words).
// Prints one JSON line; exit status 0 when every check passed.
#include "../include/atgpu.h"
#include "../python-audio-tools_amd/csrc/md5_cpu.h"
#include "../python-audio-tools_amd/csrc/service.h"
extern "C" {
#include "../python-audio-tools_amd/csrc/ext/md5_host.h"
}

#include <sys/socket.h>
#include <sys/un.h>
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

static int g_fail = 0;
#define CHECK(c)                                                                       \
    do {                                                                               \
        if (!(c)) {                                                                    \
            std::fprintf(stderr, "%s:%d check failed: %s\n", __FILE__, __LINE__, #c);  \
            ++g_fail;                                                                  \
        }                                                                              \
    } while (0)

static std::vector<uint8_t> slurp(const char *path)
{
    std::vector<uint8_t> v;
    if (FILE *f = std::fopen(path, "rb")) {
        uint8_t buf[65536];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0)
            v.insert(v.end(), buf, buf + n);
        std::fclose(f);
    }
    return v;
}

static int metadata_fuzz(const std::vector<uint8_t> &img, bool alac, std::mt19937_64 &rng)
{
    int calls = 0;
    atg_flac_streaminfo si;
    atg_flac_seekpoint sp[64];
    atg_alac_info ai;
    atg_alac_seekpoint asp[64];
    uint32_t fs[256], nfs = 0;
    auto one = [&](const std::vector<uint8_t> &b, size_t len) {
        // a heap copy of exactly len bytes: ASan sees any read past it
        std::vector<uint8_t> c(b.begin(), b.begin() + (long)len);
        const uint8_t *p = len ? c.data() : nullptr;
        if (alac)
            (void)atg_alac_read_info(p, len, &ai, asp, 64, fs, 256, &nfs);
        else
            (void)atg_flac_read_metadata(p, len, &si, sp, 64);
        ++calls;
    };
    const size_t n = img.size();
    for (size_t len = 0; len <= n; len += (len < 4096 ? 1 : 997))
        one(img, len);
    for (int k = 0; k < 400; ++k) {
        std::vector<uint8_t> m(img);
        const int flips = 1 + (int)(rng() % 8);
        for (int f = 0; f < flips; ++f)
            m[rng() % std::min<size_t>(n, 8192)] = (uint8_t)rng();
        one(m, n);
        one(m, (size_t)(rng() % (n + 1)));
    }
    return calls;
}

static void md5_ref(const uint8_t *p, size_t n, uint8_t out[16])
{
    md5_ctx m;
    md5_init(&m);
    md5_update(&m, p, n);
    md5_final(&m, out);
}

static int md5_check(std::mt19937_64 &rng)
{
    int cases = 0;
    for (uint32_t bps : {8u, 16u, 24u, 32u})
        for (uint64_t n : {0ull, 1ull, 15ull, 16ull, 17ull, 63ull, 64ull, 1000ull, 4096ull * 3 + 5}) {
            const uint32_t bb = bps / 8;
            std::vector<int32_t> s32(n);
            std::vector<int16_t> s16(n);
            std::vector<uint8_t> bytes(n * bb);
            for (uint64_t i = 0; i < n; ++i) {
                const int32_t v = (int32_t)(rng() >> 32) >> (32 - bps);
                s32[i] = v;
                s16[i] = (int16_t)v;
                for (uint32_t b = 0; b < bb; ++b)
                    bytes[i * bb + b] = (uint8_t)((uint32_t)v >> (8 * b));
            }
            uint8_t want[16], got[16];
            md5_ref(bytes.data(), bytes.size(), want);
            md5cpu::hash_s32(s32.data(), n, bb, got);
            CHECK(std::memcmp(want, got, 16) == 0);
            if (bps <= 16) {
                std::vector<uint8_t> b16(n * bb);
                for (uint64_t i = 0; i < n; ++i)
                    for (uint32_t b = 0; b < bb; ++b)
                        b16[i * bb + b] = (uint8_t)((uint32_t)(int32_t)s16[i] >> (8 * b));
                md5_ref(b16.data(), b16.size(), want);
                md5cpu::hash_s16(s16.data(), n, bb, got);
                CHECK(std::memcmp(want, got, 16) == 0);
            }
            ++cases;
        }
    // the multi-stream hash (16 chains side by side) on streams of unequal
    // lengths, exact-size heap buffers so a read past a stream is reported
    for (int t = 0; t < 40; ++t) {
        const int n = 1 + (int)(rng() % 16);
        std::vector<std::vector<uint8_t>> st(n);
        const uint8_t *p[16];
        uint64_t len[16];
        for (int i = 0; i < n; ++i) {
            st[i].resize(t % 2 ? (size_t)(rng() % 3000) : (size_t)(64 * (rng() % 40)));
            for (uint8_t &b : st[i])
                b = (uint8_t)rng();
            p[i] = st[i].empty() ? nullptr : st[i].data();
            len[i] = st[i].size();
        }
        uint8_t got[16][16], want[16];
        md5cpu::hash_bytes_multi(p, len, n, got);
        for (int i = 0; i < n; ++i) {
            md5_ref(p[i], (size_t)len[i], want);
            CHECK(std::memcmp(want, got[i], 16) == 0);
        }
        ++cases;
    }
    return cases;
}

static int gather_check(std::mt19937_64 &rng)
{
    int cases = 0;
    for (int t = 0; t < 20; ++t) {
        const size_t parts = 1 + rng() % 3000;
        std::vector<std::vector<uint8_t>> src(parts);
        std::vector<const void *> ptr(parts);
        std::vector<uint64_t> len(parts);
        size_t total = 0;
        for (size_t i = 0; i < parts; ++i) {
            src[i].resize(rng() % (t & 1 ? 70000 : 300));
            for (auto &b : src[i])
                b = (uint8_t)rng();
            ptr[i] = src[i].data();
            len[i] = src[i].size();
            total += len[i];
        }
        std::vector<uint8_t> dst(total), want;
        for (auto &s : src)
            want.insert(want.end(), s.begin(), s.end());
        CHECK(atg_host_gather(dst.data(), ptr.data(), len.data(), parts, (uint32_t)(t % 5)) ==
              ATG_OK);
        CHECK(dst == want);
        ++cases;
    }
    return cases;
}

static int bounds_check()
{
    atg_flac_options o = {4096, 12, 0, 6, 1, 0, 1, 0, 0, 0, 0, 4096};
    int cases = 0;
    for (uint64_t frames : {0ull, 1ull, 4095ull, 4096ull, 4097ull, 1ull << 20}) {
        atg_track tr = {0, frames, nullptr, 0};
        uint64_t nf = 0, nb = 0;
        CHECK(atg_flac_batch_bounds(&o, &tr, 1, 2, 16, &nf, &nb) == ATG_OK);
        CHECK(atg_flac_max_frames_bytes(&o, frames, nullptr, 0, 2, 16) > 0 || frames == 0);
        ++cases;
    }
    std::vector<uint32_t> sizes = {1, 65535, 16, 4096, 7};
    uint64_t sum = 0;
    for (uint32_t s : sizes)
        sum += s;
    atg_track tr = {0, sum, sizes.data(), sizes.size()};
    uint64_t nf = 0, nb = 0;
    CHECK(atg_flac_batch_bounds(&o, &tr, 1, 8, 24, &nf, &nb) == ATG_OK && nf == sizes.size());
    tr.pcm_frames = sum + 1; // sizes that do not add up: refused
    CHECK(atg_flac_batch_bounds(&o, &tr, 1, 8, 24, &nf, &nb) != ATG_OK);
    std::vector<uint8_t> hdr(4096 + o.padding_size);
    uint8_t md5[16] = {0};
    CHECK(atg_flac_stream_header(&o, 2, 16, 44100, 123456, 10, 9000, md5, hdr.data(), hdr.size()) >
          0);
    CHECK(atg_flac_stream_header(&o, 2, 16, 44100, 123456, 10, 9000, md5, hdr.data(), 10) == 0);
    return cases + 3;
}

// ---- the service client against fake services
static void fake_service(const std::string &name, std::vector<uint8_t> reply, bool answer)
{
    const int fd = socket(AF_UNIX, SOCK_STREAM, 0);
    sockaddr_un a;
    std::memset(&a, 0, sizeof(a));
    a.sun_family = AF_UNIX;
    std::memcpy(a.sun_path + 1, name.data(), name.size());
    const socklen_t al = (socklen_t)(offsetof(sockaddr_un, sun_path) + 1 + name.size());
    if (bind(fd, (sockaddr *)&a, al) != 0 || listen(fd, 2) != 0) {
        close(fd);
        return;
    }
    const int c = accept(fd, nullptr, nullptr);
    if (c >= 0) {
        atg_svc_request q;
        size_t got = 0;
        while (got < sizeof(q)) {
            const ssize_t r = recv(c, (uint8_t *)&q + got, sizeof(q) - got, 0);
            if (r <= 0)
                break;
            got += (size_t)r;
        }
        uint64_t rest = q.n_frame_sizes * 4 + q.pcm_bytes;
        std::vector<uint8_t> sink(65536);
        while (rest) {
            const ssize_t r = recv(c, sink.data(), std::min<uint64_t>(rest, sink.size()), 0);
            if (r <= 0)
                break;
            rest -= (uint64_t)r;
        }
        if (answer && !reply.empty())
            (void)send(c, reply.data(), reply.size(), MSG_NOSIGNAL);
        usleep(answer ? 200000 : 1500000);
        close(c);
    }
    close(fd);
}

static std::vector<uint8_t> response(int32_t status, const std::string &msg, uint64_t n_frames,
                                     const std::vector<uint32_t> &sizes, uint64_t out_bytes,
                                     size_t body)
{
    atg_svc_response r;
    r.status = status;
    r.msg_len = (uint32_t)msg.size();
    r.out_bytes = out_bytes;
    r.n_frames = n_frames;
    std::vector<uint8_t> v((const uint8_t *)&r, (const uint8_t *)&r + sizeof(r));
    v.insert(v.end(), msg.begin(), msg.end());
    v.insert(v.end(), (const uint8_t *)sizes.data(), (const uint8_t *)(sizes.data() + sizes.size()));
    v.resize(v.size() + body, 0x5A);
    return v;
}

static int service_case(const char *tag, std::vector<uint8_t> reply, bool answer, bool want_ok)
{
    const std::string name = std::string("atg-asan-fake-") + std::to_string(getpid()) + "-" + tag;
    std::thread t(fake_service, name, reply, answer);
    usleep(50000);
    setenv("ATG_ENCODER_SOCKET", name.c_str(), 1);
    setenv("ATG_SERVICE_TIMEOUT_MS", "300", 1);
    atg_service *svc = nullptr;
    int ok = 0;
    if (atg_service_connect(0, 0, &svc) == ATG_OK) {
        atg_flac_options o = {4096, 12, 0, 6, 1, 0, 1, 0, 0, 0, 0, 4096};
        const uint64_t frames = 4096 * 3;
        std::vector<int16_t> pcm(frames * 2, 0);
        const size_t cap = 64, guard = 64;
        std::vector<uint32_t> fb(cap + guard, 0xA5A5A5A5u);
        std::vector<uint8_t> out(1 << 20);
        uint64_t nb = 0;
        const atg_status st = atg_service_encode_frames(svc, &o, pcm.data(), ATG_PCM_S16, frames,
                                                         nullptr, 0, 2, 16, 44100, 0, out.data(),
                                                         out.size(), &nb, fb.data());
        for (size_t i = cap; i < cap + guard; ++i)
            CHECK(fb[i] == 0xA5A5A5A5u);
        ok = (st == ATG_OK) == want_ok;
        atg_service_close(svc);
    }
    unsetenv("ATG_ENCODER_SOCKET");
    unsetenv("ATG_SERVICE_TIMEOUT_MS");
    t.join();
    CHECK(ok);
    return 1;
}

static int service_check()
{
    int n = 0;
    const std::vector<uint32_t> three = {100, 200, 300};
    n += service_case("good", response(ATG_OK, "", 3, three, 600, 600), true, true);
    n += service_case("count", response(ATG_OK, "", 300, std::vector<uint32_t>(300, 2), 600, 600),
                      true, false);
    n += service_case("sizes", response(ATG_OK, "", 3, {100, 200, 301}, 600, 600), true, false);
    n += service_case("bytes", response(ATG_OK, "", 3, three, 1ull << 40, 600), true, false);
    n += service_case("msg", response(ATG_ERR_DEVICE, std::string(1 << 20, 'x'), 0, {}, 0, 0), true,
                      false);
    n += service_case("mute", {}, false, false);
    return n;
}

int main(int argc, char **argv)
{
    const std::string root = argc > 1 ? argv[1] : ".";
    std::mt19937_64 rng(20261018);
    int flac_calls = 0, alac_calls = 0;
    for (const char *f : {"flac-seektable.flac", "flac-allframes.flac", "flac-id3.flac",
                          "flac-nomask1.flac", "tone1.flac"}) {
        const auto img = slurp((root + "/tests/golden/fixtures/" + f).c_str());
        CHECK(!img.empty());
        if (!img.empty())
            flac_calls += metadata_fuzz(img, false, rng);
    }
    const auto m4a = slurp((root + "/tests/golden/fixtures/alac-allframes.m4a").c_str());
    CHECK(!m4a.empty());
    if (!m4a.empty())
        alac_calls = metadata_fuzz(m4a, true, rng);
    const int md5 = md5_check(rng), gather = gather_check(rng), bounds = bounds_check(),
              svc = service_check();
    std::printf("{\"flac_metadata_calls\": %d, \"alac_info_calls\": %d, \"md5_cases\": %d, "
                "\"gather_cases\": %d, \"bounds_cases\": %d, \"service_cases\": %d, "
                "\"failures\": %d}\n",
                flac_calls, alac_calls, md5, gather, bounds, svc, g_fail);
    return g_fail ? 1 : 0;
}
