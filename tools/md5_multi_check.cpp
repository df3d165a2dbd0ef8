// md5_multi_check.cpp -- CPU check of md5_cpu.h's multi-stream MD5
// (hash_bytes_multi, 16 chains in AVX-512 lanes) against its scalar path
// on random stream counts and lengths, RFC 1321's "abc" vector, and the
// throughput of 16 config-5 sized tracks both ways (tests/test_md5_multi.py).
#include "../python-audio-tools_amd/csrc/md5_cpu.h"
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <chrono>
int main() {
    srand(7);
    int bad = 0, cases = 0;
    for (int trial = 0; trial < 300; ++trial) {
        int n = 1 + rand() % 16;
        std::vector<std::vector<uint8_t>> bufs(n);
        const uint8_t *p[16]; uint64_t len[16];
        uint64_t base = (uint64_t)(rand() % 3000);
        for (int i = 0; i < n; ++i) {
            uint64_t L = (trial % 3 == 0) ? base : (uint64_t)(rand() % 5000);
            bufs[i].resize(L + 1);
            for (auto &b : bufs[i]) b = (uint8_t)rand();
            p[i] = bufs[i].data(); len[i] = L;
        }
        uint8_t a[16][16], b[16][16];
        md5cpu::hash_bytes_multi(p, len, n, a, true);
        md5cpu::hash_bytes_multi(p, len, n, b, false);
        for (int i = 0; i < n; ++i) { cases++; if (memcmp(a[i], b[i], 16)) bad++; }
    }
    // known answer: MD5("abc")
    const uint8_t *q[2] = {(const uint8_t *)"abc", (const uint8_t *)"abc"}; uint64_t l2[2] = {3, 3};
    uint8_t o[2][16]; md5cpu::hash_bytes_multi(q, l2, 2, o, true);
    printf("cases %d bad %d abc %02x%02x%02x%02x\n", cases, bad, o[0][0], o[0][1], o[0][2], o[0][3]);
    // speed: 16 x 8.6 MB
    std::vector<std::vector<uint8_t>> big(16, std::vector<uint8_t>(8640000, 1));
    const uint8_t *bp[16]; uint64_t bl[16];
    for (int i = 0; i < 16; ++i) { bp[i] = big[i].data(); bl[i] = big[i].size(); }
    uint8_t d[16][16];
    for (int simd = 1; simd >= 0; --simd) {
        auto t0 = std::chrono::steady_clock::now();
        md5cpu::hash_bytes_multi(bp, bl, 16, d, simd);
        auto t1 = std::chrono::steady_clock::now();
        double ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        printf("simd=%d: 16 x 8.64 MB in %.1f ms = %.2f GB/s\n", simd, ms, 16 * 8.64e6 / ms / 1e6);
    }
    return bad != 0;
}
