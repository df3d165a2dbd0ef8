/*
 * md5_host.h — RFC 1321 MD5 for the CPython extensions' host-side hashes:
 * the STREAMINFO MD5 of the PCM bytes a streaming encode_flac writes
 * (flac.c:187-188, 276-279) and the one a streaming FlacDecoder verifies
 * (flac.c:479-493).  Header-only, static functions.
 */
#ifndef ATG_MD5_HOST_H
#define ATG_MD5_HOST_H
#include <stdint.h>
#include <string.h>

typedef struct {
    uint32_t h[4];
    uint64_t len;
    uint8_t buf[64];
} md5_ctx;

static uint32_t rol(uint32_t x, int c) { return (x << c) | (x >> (32 - c)); }

static void md5_block(uint32_t h[4], const uint8_t *p)
{
    static const uint32_t K[64] = {
        0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613,
        0xfd469501, 0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193,
        0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d,
        0x02441453, 0xd8a1e681, 0xe7d3fbc8, 0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed,
        0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122,
        0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa,
        0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665, 0xf4292244,
        0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
        0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb,
        0xeb86d391};
    static const int S[64] = {7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
                              5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
                              4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
                              6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};
    uint32_t X[16];
    for (int i = 0; i < 16; ++i)
        X[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) |
               ((uint32_t)p[4 * i + 2] << 16) | ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; ++i) {
        uint32_t f;
        int g;
        if (i < 16) {
            f = (b & c) | (~b & d);
            g = i;
        } else if (i < 32) {
            f = (d & b) | (~d & c);
            g = (5 * i + 1) & 15;
        } else if (i < 48) {
            f = b ^ c ^ d;
            g = (3 * i + 5) & 15;
        } else {
            f = c ^ (b | ~d);
            g = (7 * i) & 15;
        }
        const uint32_t t = d;
        d = c;
        c = b;
        b = b + rol(a + f + K[i] + X[g], S[i]);
        a = t;
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

static void md5_init(md5_ctx *m)
{
    m->h[0] = 0x67452301u;
    m->h[1] = 0xefcdab89u;
    m->h[2] = 0x98badcfeu;
    m->h[3] = 0x10325476u;
    m->len = 0;
}

static void md5_update(md5_ctx *m, const uint8_t *p, size_t n)
{
    size_t have = (size_t)(m->len & 63u);
    m->len += n;
    if (have) {
        const size_t take = 64 - have < n ? 64 - have : n;
        memcpy(m->buf + have, p, take);
        p += take;
        n -= take;
        if (have + take < 64)
            return;
        md5_block(m->h, m->buf);
    }
    for (; n >= 64; p += 64, n -= 64)
        md5_block(m->h, p);
    memcpy(m->buf, p, n);
}

static void md5_final(md5_ctx *m, uint8_t out[16])
{
    const uint64_t bits = m->len * 8u;
    static const uint8_t pad[64] = {0x80};
    const size_t have = (size_t)(m->len & 63u);
    md5_update(m, pad, have < 56 ? 56 - have : 120 - have);
    uint8_t lb[8];
    for (int i = 0; i < 8; ++i)
        lb[i] = (uint8_t)(bits >> (8 * i));
    md5_update(m, lb, 8);
    for (int i = 0; i < 4; ++i)
        for (int k = 0; k < 4; ++k)
            out[4 * i + k] = (uint8_t)(m->h[i] >> (8 * k));
}

#endif
