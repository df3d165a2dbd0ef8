// md5_cpu.h — RFC 1321 MD5 on host cores for the engine's host-hash mode
// (engine.hip, `md5_host`): the STREAMINFO MD5 of a track's little-endian
// PCM bytes (reference: src/encoders/flac.c:187-188, 1570-1576) computed
// from the int16 / int32 sample containers directly -- the packing of a
// group of samples into the byte stream is fused with the hash, so a host
// thread reads each container once and writes nothing.
//
// Few long tracks (config 5: 64 tracks of 8.6 MB of 24-bit 5.1 PCM) give the
// GPU one serial MD5 chain per track, ~0.8 us per 64-byte block on one wave
// (md5.hip), i.e. ~110 ms per batch whatever the GPU's width; host cores
// hash the same bytes at ~0.6 GB/s each, all tracks at once.
#pragma once
#include <stdint.h>
#include <string.h>

namespace md5cpu {

static inline uint32_t rotl(uint32_t x, int s) { return (x << s) | (x >> (32 - s)); }

#define M5_F1(x, y, z) ((z) ^ ((x) & ((y) ^ (z))))
#define M5_F2(x, y, z) ((y) ^ ((z) & ((x) ^ (y))))
#define M5_F3(x, y, z) ((x) ^ (y) ^ (z))
#define M5_F4(x, y, z) ((y) ^ ((x) | ~(z)))
#define M5_STEP(f, a, b, c, d, x, t, s) a = b + rotl(a + f(b, c, d) + (x) + (t), s)

// one 64-byte block, message words X[0..15] (little-endian already)
static inline void compress(uint32_t h[4], const uint32_t X[16])
{
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    M5_STEP(M5_F1, a, b, c, d, X[0], 0xd76aa478, 7);
    M5_STEP(M5_F1, d, a, b, c, X[1], 0xe8c7b756, 12);
    M5_STEP(M5_F1, c, d, a, b, X[2], 0x242070db, 17);
    M5_STEP(M5_F1, b, c, d, a, X[3], 0xc1bdceee, 22);
    M5_STEP(M5_F1, a, b, c, d, X[4], 0xf57c0faf, 7);
    M5_STEP(M5_F1, d, a, b, c, X[5], 0x4787c62a, 12);
    M5_STEP(M5_F1, c, d, a, b, X[6], 0xa8304613, 17);
    M5_STEP(M5_F1, b, c, d, a, X[7], 0xfd469501, 22);
    M5_STEP(M5_F1, a, b, c, d, X[8], 0x698098d8, 7);
    M5_STEP(M5_F1, d, a, b, c, X[9], 0x8b44f7af, 12);
    M5_STEP(M5_F1, c, d, a, b, X[10], 0xffff5bb1, 17);
    M5_STEP(M5_F1, b, c, d, a, X[11], 0x895cd7be, 22);
    M5_STEP(M5_F1, a, b, c, d, X[12], 0x6b901122, 7);
    M5_STEP(M5_F1, d, a, b, c, X[13], 0xfd987193, 12);
    M5_STEP(M5_F1, c, d, a, b, X[14], 0xa679438e, 17);
    M5_STEP(M5_F1, b, c, d, a, X[15], 0x49b40821, 22);
    M5_STEP(M5_F2, a, b, c, d, X[1], 0xf61e2562, 5);
    M5_STEP(M5_F2, d, a, b, c, X[6], 0xc040b340, 9);
    M5_STEP(M5_F2, c, d, a, b, X[11], 0x265e5a51, 14);
    M5_STEP(M5_F2, b, c, d, a, X[0], 0xe9b6c7aa, 20);
    M5_STEP(M5_F2, a, b, c, d, X[5], 0xd62f105d, 5);
    M5_STEP(M5_F2, d, a, b, c, X[10], 0x02441453, 9);
    M5_STEP(M5_F2, c, d, a, b, X[15], 0xd8a1e681, 14);
    M5_STEP(M5_F2, b, c, d, a, X[4], 0xe7d3fbc8, 20);
    M5_STEP(M5_F2, a, b, c, d, X[9], 0x21e1cde6, 5);
    M5_STEP(M5_F2, d, a, b, c, X[14], 0xc33707d6, 9);
    M5_STEP(M5_F2, c, d, a, b, X[3], 0xf4d50d87, 14);
    M5_STEP(M5_F2, b, c, d, a, X[8], 0x455a14ed, 20);
    M5_STEP(M5_F2, a, b, c, d, X[13], 0xa9e3e905, 5);
    M5_STEP(M5_F2, d, a, b, c, X[2], 0xfcefa3f8, 9);
    M5_STEP(M5_F2, c, d, a, b, X[7], 0x676f02d9, 14);
    M5_STEP(M5_F2, b, c, d, a, X[12], 0x8d2a4c8a, 20);
    M5_STEP(M5_F3, a, b, c, d, X[5], 0xfffa3942, 4);
    M5_STEP(M5_F3, d, a, b, c, X[8], 0x8771f681, 11);
    M5_STEP(M5_F3, c, d, a, b, X[11], 0x6d9d6122, 16);
    M5_STEP(M5_F3, b, c, d, a, X[14], 0xfde5380c, 23);
    M5_STEP(M5_F3, a, b, c, d, X[1], 0xa4beea44, 4);
    M5_STEP(M5_F3, d, a, b, c, X[4], 0x4bdecfa9, 11);
    M5_STEP(M5_F3, c, d, a, b, X[7], 0xf6bb4b60, 16);
    M5_STEP(M5_F3, b, c, d, a, X[10], 0xbebfbc70, 23);
    M5_STEP(M5_F3, a, b, c, d, X[13], 0x289b7ec6, 4);
    M5_STEP(M5_F3, d, a, b, c, X[0], 0xeaa127fa, 11);
    M5_STEP(M5_F3, c, d, a, b, X[3], 0xd4ef3085, 16);
    M5_STEP(M5_F3, b, c, d, a, X[6], 0x04881d05, 23);
    M5_STEP(M5_F3, a, b, c, d, X[9], 0xd9d4d039, 4);
    M5_STEP(M5_F3, d, a, b, c, X[12], 0xe6db99e5, 11);
    M5_STEP(M5_F3, c, d, a, b, X[15], 0x1fa27cf8, 16);
    M5_STEP(M5_F3, b, c, d, a, X[2], 0xc4ac5665, 23);
    M5_STEP(M5_F4, a, b, c, d, X[0], 0xf4292244, 6);
    M5_STEP(M5_F4, d, a, b, c, X[7], 0x432aff97, 10);
    M5_STEP(M5_F4, c, d, a, b, X[14], 0xab9423a7, 15);
    M5_STEP(M5_F4, b, c, d, a, X[5], 0xfc93a039, 21);
    M5_STEP(M5_F4, a, b, c, d, X[12], 0x655b59c3, 6);
    M5_STEP(M5_F4, d, a, b, c, X[3], 0x8f0ccc92, 10);
    M5_STEP(M5_F4, c, d, a, b, X[10], 0xffeff47d, 15);
    M5_STEP(M5_F4, b, c, d, a, X[1], 0x85845dd1, 21);
    M5_STEP(M5_F4, a, b, c, d, X[8], 0x6fa87e4f, 6);
    M5_STEP(M5_F4, d, a, b, c, X[15], 0xfe2ce6e0, 10);
    M5_STEP(M5_F4, c, d, a, b, X[6], 0xa3014314, 15);
    M5_STEP(M5_F4, b, c, d, a, X[13], 0x4e0811a1, 21);
    M5_STEP(M5_F4, a, b, c, d, X[4], 0xf7537e82, 6);
    M5_STEP(M5_F4, d, a, b, c, X[11], 0xbd3af235, 10);
    M5_STEP(M5_F4, c, d, a, b, X[2], 0x2ad7d2bb, 15);
    M5_STEP(M5_F4, b, c, d, a, X[9], 0xeb86d391, 21);
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

#undef M5_F1
#undef M5_F2
#undef M5_F3
#undef M5_F4
#undef M5_STEP

// streaming state over an arbitrary byte sequence
struct Ctx {
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    uint64_t len = 0;
    uint8_t buf[64];

    void update(const uint8_t *p, size_t n)
    {
        size_t have = (size_t)(len & 63u);
        len += n;
        if (have) {
            const size_t take = 64 - have < n ? 64 - have : n;
            memcpy(buf + have, p, take);
            p += take;
            n -= take;
            if (have + take < 64)
                return;
            block(buf);
        }
        for (; n >= 64; p += 64, n -= 64)
            block(p);
        memcpy(buf, p, n);
    }
    void block(const uint8_t *p)
    {
        uint32_t X[16];
        memcpy(X, p, 64); // little-endian host
        compress(h, X);
    }
    void final(uint8_t out[16])
    {
        const uint64_t bits = len * 8u;
        static const uint8_t pad[64] = {0x80};
        const size_t have = (size_t)(len & 63u);
        update(pad, have < 56 ? 56 - have : 120 - have);
        uint8_t lb[8];
        for (int i = 0; i < 8; ++i)
            lb[i] = (uint8_t)(bits >> (8 * i));
        update(lb, 8);
        for (int i = 0; i < 4; ++i)
            for (int k = 0; k < 4; ++k)
                out[4 * i + k] = (uint8_t)(h[i] >> (8 * k));
    }
};

// MD5 of n samples held in int32 containers, as the little-endian byte
// stream of their low `bb` bytes (1..4): samples are packed a few hundred at
// a time into a stack buffer and hashed from there
static inline void hash_s32(const int32_t *s, uint64_t n, uint32_t bb, uint8_t out[16])
{
    Ctx c;
    uint8_t tmp[4096]; // 1024 samples of up to 4 bytes
    const uint64_t chunk = 1024;
    for (uint64_t i = 0; i < n; i += chunk) {
        const uint64_t m = n - i < chunk ? n - i : chunk;
        uint8_t *q = tmp;
        const int32_t *p = s + i;
        if (bb == 3) {
            uint64_t k = 0;
            for (; k + 4 <= m; k += 4, q += 12) { // 4 samples = 3 words
                const uint32_t a = (uint32_t)p[k], b = (uint32_t)p[k + 1],
                               c2 = (uint32_t)p[k + 2], d = (uint32_t)p[k + 3];
                const uint32_t w[3] = {(a & 0xFFFFFFu) | (b << 24),
                                       ((b >> 8) & 0xFFFFu) | (c2 << 16),
                                       ((c2 >> 16) & 0xFFu) | (d << 8)};
                memcpy(q, w, 12);
            }
            for (; k < m; ++k, q += 3) {
                const uint32_t v = (uint32_t)p[k];
                q[0] = (uint8_t)v;
                q[1] = (uint8_t)(v >> 8);
                q[2] = (uint8_t)(v >> 16);
            }
        } else if (bb == 2) {
            for (uint64_t k = 0; k < m; ++k, q += 2) {
                const uint32_t v = (uint32_t)p[k];
                q[0] = (uint8_t)v;
                q[1] = (uint8_t)(v >> 8);
            }
        } else if (bb == 1) {
            for (uint64_t k = 0; k < m; ++k)
                *q++ = (uint8_t)p[k];
        } else {
            memcpy(q, p, m * 4);
            q += m * 4;
        }
        c.update(tmp, (size_t)(q - tmp));
    }
    c.final(out);
}

// int16 containers: 16-bit samples are the byte stream itself, narrower
// ones keep their low byte
static inline void hash_s16(const int16_t *s, uint64_t n, uint32_t bb, uint8_t out[16])
{
    Ctx c;
    if (bb == 2) {
        c.update((const uint8_t *)s, (size_t)n * 2u);
    } else {
        uint8_t tmp[4096];
        for (uint64_t i = 0; i < n; i += sizeof(tmp)) {
            const uint64_t m = n - i < sizeof(tmp) ? n - i : sizeof(tmp);
            for (uint64_t k = 0; k < m; ++k)
                tmp[k] = (uint8_t)s[i + k];
            c.update(tmp, (size_t)m);
        }
    }
    c.final(out);
}

} // namespace md5cpu
