// md5_cpu.h — RFC 1321 MD5 on host cores for the engine's host-hash mode
// (engine.hip, `md5_host`): the STREAMINFO MD5 of a track's little-endian
// PCM bytes (reference: src/encoders/flac.c:187-188, 1570-1576) computed
// from the int16 / int32 sample containers directly -- the packing of a
// group of samples into the byte stream is fused with the hash, so a host
// thread reads each container once and writes nothing.
//
// Few long tracks (config 5: 64 tracks of 8.6 MB of 24-bit 5.1 PCM) give the
// GPU one serial MD5 chain per track, ~0.8 us per 64-byte block on one wave
// (md5.hip), i.e. ~110 ms per batch whatever the GPU's width; a host core
// hashes one stream at ~0.6-1 GB/s, or sixteen side by side at ~6 GB/s
// (hash_bytes_multi, AVX-512; the engine packs the streams on the device).
#pragma once
#include <stdint.h>
#include <string.h>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

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

// ---- many streams at once: 16 MD5 chains in the 32-bit lanes of AVX-512
// registers (one chain per track, the tracks of a batch side by side).  A
// chain is serial -- each step needs the last -- so one core runs one
// scalar chain at ~1 GB/s whatever its width; sixteen side by side cost
// about what one does (the same dependent adds, rotates and `vpternlogd`
// F functions, one lane each).  The streams' common whole blocks run here;
// each stream's remaining bytes and padding finish on its own Ctx.

#if defined(__x86_64__)
// 16 x 16 32-bit transpose: row l (lane l's 16 words) -> register w holds
// word w of every lane
__attribute__((target("avx512f"))) static inline void transpose16(__m512i (&r)[16])
{
    __m512i t[16];
    for (int i = 0; i < 16; i += 2) {
        t[i] = _mm512_unpacklo_epi32(r[i], r[i + 1]);
        t[i + 1] = _mm512_unpackhi_epi32(r[i], r[i + 1]);
    }
    for (int i = 0; i < 16; i += 4) {
        r[i] = _mm512_unpacklo_epi64(t[i], t[i + 2]);
        r[i + 1] = _mm512_unpackhi_epi64(t[i], t[i + 2]);
        r[i + 2] = _mm512_unpacklo_epi64(t[i + 1], t[i + 3]);
        r[i + 3] = _mm512_unpackhi_epi64(t[i + 1], t[i + 3]);
    }
    for (int i = 0; i < 16; i += 8)
        for (int j = 0; j < 4; ++j) {
            t[i + j] = _mm512_shuffle_i32x4(r[i + j], r[i + j + 4], 0x88);
            t[i + j + 4] = _mm512_shuffle_i32x4(r[i + j], r[i + j + 4], 0xDD);
        }
    for (int j = 0; j < 8; ++j) {
        r[j] = _mm512_shuffle_i32x4(t[j], t[j + 8], 0x88);
        r[j + 8] = _mm512_shuffle_i32x4(t[j], t[j + 8], 0xDD);
    }
}

__attribute__((target("avx512f"))) static inline void mb16_blocks(uint32_t (&h)[4][16],
                                                                const uint8_t *const *p,
                                                                uint64_t nblocks)
{
    __m512i A = _mm512_loadu_si512(h[0]), B = _mm512_loadu_si512(h[1]);
    __m512i C = _mm512_loadu_si512(h[2]), D = _mm512_loadu_si512(h[3]);
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
    for (uint64_t j = 0; j < nblocks; ++j) {
        __m512i r[16];
        for (int l = 0; l < 16; ++l)
            r[l] = _mm512_loadu_si512(p[l] + 64 * j);
        transpose16(r); // r[w] = message word w of every lane
        const __m512i *X = r;
        const __m512i a0 = A, b0 = B, c0 = C, d0 = D;
#define MB_STEP(imm, a, b, c, d, x, i, s)                                                      \
    a = _mm512_add_epi32(                                                                   \
        b, _mm512_rol_epi32(_mm512_add_epi32(_mm512_add_epi32(                              \
                                a, _mm512_ternarylogic_epi32(b, c, d, imm)),                \
                                             _mm512_add_epi32(x, _mm512_set1_epi32((int)K[i]))), \
                            s))
        for (int i = 0; i < 16; i += 4) {
            MB_STEP(0xCA, A, B, C, D, X[i], i, 7);
            MB_STEP(0xCA, D, A, B, C, X[i + 1], i + 1, 12);
            MB_STEP(0xCA, C, D, A, B, X[i + 2], i + 2, 17);
            MB_STEP(0xCA, B, C, D, A, X[i + 3], i + 3, 22);
        }
        for (int i = 16; i < 32; i += 4) {
            MB_STEP(0xE4, A, B, C, D, X[(5 * i + 1) & 15], i, 5);
            MB_STEP(0xE4, D, A, B, C, X[(5 * (i + 1) + 1) & 15], i + 1, 9);
            MB_STEP(0xE4, C, D, A, B, X[(5 * (i + 2) + 1) & 15], i + 2, 14);
            MB_STEP(0xE4, B, C, D, A, X[(5 * (i + 3) + 1) & 15], i + 3, 20);
        }
        for (int i = 32; i < 48; i += 4) {
            MB_STEP(0x96, A, B, C, D, X[(3 * i + 5) & 15], i, 4);
            MB_STEP(0x96, D, A, B, C, X[(3 * (i + 1) + 5) & 15], i + 1, 11);
            MB_STEP(0x96, C, D, A, B, X[(3 * (i + 2) + 5) & 15], i + 2, 16);
            MB_STEP(0x96, B, C, D, A, X[(3 * (i + 3) + 5) & 15], i + 3, 23);
        }
        for (int i = 48; i < 64; i += 4) {
            MB_STEP(0x39, A, B, C, D, X[(7 * i) & 15], i, 6);
            MB_STEP(0x39, D, A, B, C, X[(7 * (i + 1)) & 15], i + 1, 10);
            MB_STEP(0x39, C, D, A, B, X[(7 * (i + 2)) & 15], i + 2, 15);
            MB_STEP(0x39, B, C, D, A, X[(7 * (i + 3)) & 15], i + 3, 21);
        }
#undef MB_STEP
        A = _mm512_add_epi32(A, a0);
        B = _mm512_add_epi32(B, b0);
        C = _mm512_add_epi32(C, c0);
        D = _mm512_add_epi32(D, d0);
    }
    _mm512_storeu_si512(h[0], A);
    _mm512_storeu_si512(h[1], B);
    _mm512_storeu_si512(h[2], C);
    _mm512_storeu_si512(h[3], D);
}

static inline bool have_avx512()
{
    static const bool ok = __builtin_cpu_supports("avx512f");
    return ok;
}
#endif

// streams hash_bytes_multi takes at once, and whether this CPU runs them
// side by side (otherwise one after another on the scalar path)
constexpr int kMultiLanes = 16;
static inline bool multi_simd()
{
#if defined(__x86_64__)
    return have_avx512();
#else
    return false;
#endif
}

// MD5 of n byte streams (n <= 16): p[i] / len[i] -> out[i]
static inline void hash_bytes_multi(const uint8_t *const *p, const uint64_t *len, int n,
                                    uint8_t (*out)[16], bool allow_simd = true)
{
    Ctx c[16];
    uint64_t common = 0;
#if defined(__x86_64__)
    if (allow_simd && n > 1 && have_avx512()) {
        common = ~0ull;
        for (int i = 0; i < n; ++i)
            common = len[i] / 64 < common ? len[i] / 64 : common;
        if (common) {
            uint32_t h[4][16];
            const uint8_t *q[16];
            for (int l = 0; l < 16; ++l) {
                const int i = l < n ? l : 0; // idle lanes repeat stream 0
                q[l] = p[i];
                for (int k = 0; k < 4; ++k)
                    h[k][l] = c[0].h[k];
            }
            mb16_blocks(h, q, common);
            for (int i = 0; i < n; ++i) {
                for (int k = 0; k < 4; ++k)
                    c[i].h[k] = h[k][i];
                c[i].len = common * 64;
            }
        }
    }
#endif
    for (int i = 0; i < n; ++i) {
        c[i].update(p[i] + common * 64, (size_t)(len[i] - common * 64));
        c[i].final(out[i]);
    }
}

} // namespace md5cpu
