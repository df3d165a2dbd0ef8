// md5.hip — STREAMINFO MD5 of each track's PCM (reference: MD5 of the
// little-endian signed sample bytes fed by the PCM reader callback,
// src/encoders/flac.c:187-188, 1570-1576; src/pcmconv.c:266-291).
//
// MD5 is one serial chain per track, so the kernel runs one lane per track
// and is launched on its own stream, concurrently with the encoder kernels
// (it occupies a handful of SIMDs).  Round functions use v_bfi/v_xor3 forms
// and v_alignbit rotates; message words are fetched 16 per block.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "flac_dev.h"
#include "launch.h"

#define MD5_D 4

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, 32 - s); }

#define MD5_STEP(f, a, b, c, d, x, t, s) \
    a = b + rotl(a + f(b, c, d) + x + t, s)
#define F1(x, y, z) (z ^ (x & (y ^ z)))
#define F2(x, y, z) (y ^ (z & (x ^ y)))
// x ^ y ^ z as one v_bitop3_b32 (truth table 0x96); the compiler emits two
// v_xor_b32 otherwise
__device__ __forceinline__ uint32_t xor3(uint32_t x, uint32_t y, uint32_t z)
{
    uint32_t r;
    asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x96" : "=v"(r) : "v"(x), "v"(y), "v"(z));
    return r;
}
#define F3(x, y, z) xor3(x, y, z)
#define F4(x, y, z) (y ^ (x | ~z))

__device__ __forceinline__ void md5_compress(uint32_t h[4], const uint32_t X[16])
{
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    MD5_STEP(F1, a, b, c, d, X[0], 0xd76aa478, 7);
    MD5_STEP(F1, d, a, b, c, X[1], 0xe8c7b756, 12);
    MD5_STEP(F1, c, d, a, b, X[2], 0x242070db, 17);
    MD5_STEP(F1, b, c, d, a, X[3], 0xc1bdceee, 22);
    MD5_STEP(F1, a, b, c, d, X[4], 0xf57c0faf, 7);
    MD5_STEP(F1, d, a, b, c, X[5], 0x4787c62a, 12);
    MD5_STEP(F1, c, d, a, b, X[6], 0xa8304613, 17);
    MD5_STEP(F1, b, c, d, a, X[7], 0xfd469501, 22);
    MD5_STEP(F1, a, b, c, d, X[8], 0x698098d8, 7);
    MD5_STEP(F1, d, a, b, c, X[9], 0x8b44f7af, 12);
    MD5_STEP(F1, c, d, a, b, X[10], 0xffff5bb1, 17);
    MD5_STEP(F1, b, c, d, a, X[11], 0x895cd7be, 22);
    MD5_STEP(F1, a, b, c, d, X[12], 0x6b901122, 7);
    MD5_STEP(F1, d, a, b, c, X[13], 0xfd987193, 12);
    MD5_STEP(F1, c, d, a, b, X[14], 0xa679438e, 17);
    MD5_STEP(F1, b, c, d, a, X[15], 0x49b40821, 22);
    MD5_STEP(F2, a, b, c, d, X[1], 0xf61e2562, 5);
    MD5_STEP(F2, d, a, b, c, X[6], 0xc040b340, 9);
    MD5_STEP(F2, c, d, a, b, X[11], 0x265e5a51, 14);
    MD5_STEP(F2, b, c, d, a, X[0], 0xe9b6c7aa, 20);
    MD5_STEP(F2, a, b, c, d, X[5], 0xd62f105d, 5);
    MD5_STEP(F2, d, a, b, c, X[10], 0x02441453, 9);
    MD5_STEP(F2, c, d, a, b, X[15], 0xd8a1e681, 14);
    MD5_STEP(F2, b, c, d, a, X[4], 0xe7d3fbc8, 20);
    MD5_STEP(F2, a, b, c, d, X[9], 0x21e1cde6, 5);
    MD5_STEP(F2, d, a, b, c, X[14], 0xc33707d6, 9);
    MD5_STEP(F2, c, d, a, b, X[3], 0xf4d50d87, 14);
    MD5_STEP(F2, b, c, d, a, X[8], 0x455a14ed, 20);
    MD5_STEP(F2, a, b, c, d, X[13], 0xa9e3e905, 5);
    MD5_STEP(F2, d, a, b, c, X[2], 0xfcefa3f8, 9);
    MD5_STEP(F2, c, d, a, b, X[7], 0x676f02d9, 14);
    MD5_STEP(F2, b, c, d, a, X[12], 0x8d2a4c8a, 20);
    MD5_STEP(F3, a, b, c, d, X[5], 0xfffa3942, 4);
    MD5_STEP(F3, d, a, b, c, X[8], 0x8771f681, 11);
    MD5_STEP(F3, c, d, a, b, X[11], 0x6d9d6122, 16);
    MD5_STEP(F3, b, c, d, a, X[14], 0xfde5380c, 23);
    MD5_STEP(F3, a, b, c, d, X[1], 0xa4beea44, 4);
    MD5_STEP(F3, d, a, b, c, X[4], 0x4bdecfa9, 11);
    MD5_STEP(F3, c, d, a, b, X[7], 0xf6bb4b60, 16);
    MD5_STEP(F3, b, c, d, a, X[10], 0xbebfbc70, 23);
    MD5_STEP(F3, a, b, c, d, X[13], 0x289b7ec6, 4);
    MD5_STEP(F3, d, a, b, c, X[0], 0xeaa127fa, 11);
    MD5_STEP(F3, c, d, a, b, X[3], 0xd4ef3085, 16);
    MD5_STEP(F3, b, c, d, a, X[6], 0x04881d05, 23);
    MD5_STEP(F3, a, b, c, d, X[9], 0xd9d4d039, 4);
    MD5_STEP(F3, d, a, b, c, X[12], 0xe6db99e5, 11);
    MD5_STEP(F3, c, d, a, b, X[15], 0x1fa27cf8, 16);
    MD5_STEP(F3, b, c, d, a, X[2], 0xc4ac5665, 23);
    MD5_STEP(F4, a, b, c, d, X[0], 0xf4292244, 6);
    MD5_STEP(F4, d, a, b, c, X[7], 0x432aff97, 10);
    MD5_STEP(F4, c, d, a, b, X[14], 0xab9423a7, 15);
    MD5_STEP(F4, b, c, d, a, X[5], 0xfc93a039, 21);
    MD5_STEP(F4, a, b, c, d, X[12], 0x655b59c3, 6);
    MD5_STEP(F4, d, a, b, c, X[3], 0x8f0ccc92, 10);
    MD5_STEP(F4, c, d, a, b, X[10], 0xffeff47d, 15);
    MD5_STEP(F4, b, c, d, a, X[1], 0x85845dd1, 21);
    MD5_STEP(F4, a, b, c, d, X[8], 0x6fa87e4f, 6);
    MD5_STEP(F4, d, a, b, c, X[15], 0xfe2ce6e0, 10);
    MD5_STEP(F4, c, d, a, b, X[6], 0xa3014314, 15);
    MD5_STEP(F4, b, c, d, a, X[13], 0x4e0811a1, 21);
    MD5_STEP(F4, a, b, c, d, X[4], 0xf7537e82, 6);
    MD5_STEP(F4, d, a, b, c, X[11], 0xbd3af235, 10);
    MD5_STEP(F4, c, d, a, b, X[2], 0x2ad7d2bb, 15);
    MD5_STEP(F4, b, c, d, a, X[9], 0xeb86d391, 21);
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

// byte j of the track's little-endian PCM byte stream (generic formats)
template <typename T>
__device__ __forceinline__ uint32_t pcm_byte(const T *s, uint64_t j, uint32_t bb)
{
    const uint64_t k = j / bb;
    const uint32_t r = (uint32_t)(j - k * bb);
    return ((uint32_t)(int32_t)s[k] >> (8u * r)) & 0xFFu;
}

// The little-endian byte stream of G int32 samples of BB bytes each, as
// MD5 words (v_perm_b32 picks the bytes): BB = 3 -> 64 samples, 48 words
// (3 blocks); BB = 2 -> 32 samples, 16 words; BB = 1 -> 64 samples, 16 words.
template <int BB>
struct S32Pack {
    static constexpr int G = BB == 2 ? 32 : 64;   // samples per group
    static constexpr int W = G * BB / 4;          // words per group
    static constexpr int Q = G / 4;               // uint4 loads per group
    __device__ static __forceinline__ void pack(const uint4 (&v)[Q], uint32_t (&w)[W])
    {
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            const uint32_t s0 = v[q].x, s1 = v[q].y, s2 = v[q].z, s3 = v[q].w;
            if constexpr (BB == 3) {
                w[3 * q] = __builtin_amdgcn_perm(s1, s0, 0x04020100u);
                w[3 * q + 1] = __builtin_amdgcn_perm(s2, s1, 0x05040201u);
                w[3 * q + 2] = __builtin_amdgcn_perm(s3, s2, 0x06050402u);
            } else if constexpr (BB == 2) {
                w[2 * q] = __builtin_amdgcn_perm(s1, s0, 0x05040100u);
                w[2 * q + 1] = __builtin_amdgcn_perm(s3, s2, 0x05040100u);
            } else {
                const uint32_t lo = __builtin_amdgcn_perm(s1, s0, 0x0C0C0400u);
                const uint32_t hi = __builtin_amdgcn_perm(s3, s2, 0x04000C0Cu);
                w[q] = lo | hi;
            }
        }
    }
};

// hash `groups` whole groups of int32 samples from q (16-byte aligned), one
// group's loads in flight while the previous group is hashed
template <int BB>
__device__ __forceinline__ void md5_s32_groups(uint32_t h[4], const uint4 *__restrict__ q,
                                               uint64_t groups)
{
    using P = S32Pack<BB>;
    if (!groups)
        return;
    uint4 cur[P::Q], nxt[P::Q];
#pragma unroll
    for (int i = 0; i < P::Q; ++i)
        cur[i] = q[i];
    for (uint64_t g = 0; g < groups; ++g) {
        const uint64_t ng = min(g + 1u, groups - 1u);
#pragma unroll
        for (int i = 0; i < P::Q; ++i)
            nxt[i] = q[ng * P::Q + i];
        uint32_t w[P::W];
        P::pack(cur, w);
#pragma unroll
        for (int b = 0; b < P::W / 16; ++b)
            md5_compress(h, &w[16 * b]);
#pragma unroll
        for (int i = 0; i < P::Q; ++i)
            cur[i] = nxt[i];
    }
}

template <typename T>
__global__ __launch_bounds__(64) void k_track_md5(FlacParams p, const T *__restrict__ pcm,
                                                  const TrackInfo *__restrict__ tracks,
                                                  TrackOut *__restrict__ tout)
{
    // the hash chains are the longest serial path of a batch: let their
    // waves issue ahead of the encoder kernels sharing the SIMD
    __builtin_amdgcn_s_setprio(3);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= p.n_tracks)
        return;
    const TrackInfo ti = tracks[t];
    const uint32_t bb = p.bps / 8u;
    const T *s = pcm + ti.pcm_start * p.channels;
    const uint64_t nbytes = ti.pcm_frames * p.channels * bb;
    // fast path: the sample container IS the byte stream (S16 at 16 bits)
    const bool raw = sizeof(T) == 2 && bb == 2 && (((uintptr_t)s) & 15u) == 0;
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    uint32_t X[16];
    const uint64_t full = nbytes / 64u;
    if (raw && full > 0) {
        // MD5_D blocks in flight per lane: the loads of block b + MD5_D are
        // issued before block b is hashed, so HBM latency hides behind
        // ~MD5_D x 320 dependent VALU ops (one chain per lane, 4 cyc each)
        const uint4 *q = (const uint4 *)s;
        uint4 buf[MD5_D][4];
#pragma unroll
        for (int j = 0; j < MD5_D; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                buf[j][i] = q[(uint64_t)min((uint64_t)j, full - 1u) * 4u + i];
        uint64_t blk = 0;
        for (; blk + MD5_D <= full; blk += MD5_D) {
#pragma unroll
            for (int j = 0; j < MD5_D; ++j) {
                // hash straight from the load registers, then refill them
                // (block blk + j + MD5_D, clamped) -- no message copies
                md5_compress(h, (const uint32_t *)&buf[j][0]);
                const uint64_t nb = min(blk + (uint64_t)(j + MD5_D), full - 1u);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    buf[j][i] = q[nb * 4u + i];
            }
        }
#pragma unroll
        for (int j = 0; j < MD5_D; ++j) {
            if (blk + (uint64_t)j < full) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    X[4 * i] = buf[j][i].x;
                    X[4 * i + 1] = buf[j][i].y;
                    X[4 * i + 2] = buf[j][i].z;
                    X[4 * i + 3] = buf[j][i].w;
                }
                md5_compress(h, X);
            }
        }
    } else if (!raw) {
        // int32 container, 16-byte aligned: whole sample groups by v_perm
        // packing; the bytes after the last whole group go the generic way
        uint64_t blk = 0;
        if (sizeof(T) == 4 && (((uintptr_t)s) & 15u) == 0 && bb >= 1 && bb <= 3) {
            const uint64_t samples = ti.pcm_frames * p.channels;
            const uint4 *q = (const uint4 *)s;
            if (bb == 3) {
                const uint64_t g = samples / S32Pack<3>::G;
                md5_s32_groups<3>(h, q, g);
                blk = g * 3u;
            } else if (bb == 2) {
                const uint64_t g = samples / S32Pack<2>::G;
                md5_s32_groups<2>(h, q, g);
                blk = g;
            } else {
                const uint64_t g = samples / S32Pack<1>::G;
                md5_s32_groups<1>(h, q, g);
                blk = g;
            }
        }
        for (; blk < full; ++blk) {
            for (int i = 0; i < 16; ++i) {
                const uint64_t j = blk * 64u + 4u * (uint32_t)i;
                X[i] = pcm_byte(s, j, bb) | (pcm_byte(s, j + 1, bb) << 8) |
                       (pcm_byte(s, j + 2, bb) << 16) | (pcm_byte(s, j + 3, bb) << 24);
            }
            md5_compress(h, X);
        }
    }
    // tail + padding (0x80, zeros, 64-bit little-endian bit length)
    uint8_t tail[128];
    const uint32_t rem = (uint32_t)(nbytes - full * 64u);
    for (uint32_t i = 0; i < rem; ++i)
        tail[i] = (uint8_t)pcm_byte(s, full * 64u + i, bb);
    tail[rem] = 0x80;
    const uint32_t tl = rem < 56u ? 64u : 128u;
    for (uint32_t i = rem + 1; i < tl - 8u; ++i)
        tail[i] = 0;
    const uint64_t bits = nbytes * 8u;
    for (int i = 0; i < 8; ++i)
        tail[tl - 8u + i] = (uint8_t)(bits >> (8 * i));
    for (uint32_t o = 0; o < tl; o += 64) {
        for (int i = 0; i < 16; ++i)
            X[i] = tail[o + 4 * i] | ((uint32_t)tail[o + 4 * i + 1] << 8) |
                   ((uint32_t)tail[o + 4 * i + 2] << 16) | ((uint32_t)tail[o + 4 * i + 3] << 24);
        md5_compress(h, X);
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            tout[t].md5[4 * i + j] = (uint8_t)(h[i] >> (8 * j));
}

// MD5 of a plain byte stream per lane (the decoder hashes the little-endian
// PCM bytes K5 of flac_decode.hip wrote; streams start 64-byte aligned)
__global__ __launch_bounds__(64) void k_bytes_md5(const uint8_t *__restrict__ base,
                                                  const uint64_t *__restrict__ off,
                                                  const uint64_t *__restrict__ len, uint32_t n,
                                                  uint8_t *__restrict__ md5)
{
    __builtin_amdgcn_s_setprio(3);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n)
        return;
    const uint8_t *s = base + off[t];
    const uint64_t nbytes = len[t];
    const uint64_t full = nbytes / 64u;
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    uint32_t X[16];
    if (full > 0) {
        const uint4 *q = (const uint4 *)s;
        uint4 buf[MD5_D][4];
#pragma unroll
        for (int j = 0; j < MD5_D; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                buf[j][i] = q[(uint64_t)min((uint64_t)j, full - 1u) * 4u + i];
        uint64_t blk = 0;
        for (; blk + MD5_D <= full; blk += MD5_D) {
#pragma unroll
            for (int j = 0; j < MD5_D; ++j) {
                md5_compress(h, (const uint32_t *)&buf[j][0]);
                const uint64_t nb = min(blk + (uint64_t)(j + MD5_D), full - 1u);
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    buf[j][i] = q[nb * 4u + i];
            }
        }
#pragma unroll
        for (int j = 0; j < MD5_D; ++j)
            if (blk + (uint64_t)j < full)
                md5_compress(h, (const uint32_t *)&buf[j][0]);
    }
    uint8_t tail[128];
    const uint32_t rem = (uint32_t)(nbytes - full * 64u);
    for (uint32_t i = 0; i < rem; ++i)
        tail[i] = s[full * 64u + i];
    tail[rem] = 0x80;
    const uint32_t tl = rem < 56u ? 64u : 128u;
    for (uint32_t i = rem + 1; i < tl - 8u; ++i)
        tail[i] = 0;
    const uint64_t bits = nbytes * 8u;
    for (int i = 0; i < 8; ++i)
        tail[tl - 8u + i] = (uint8_t)(bits >> (8 * i));
    for (uint32_t o = 0; o < tl; o += 64) {
        for (int i = 0; i < 16; ++i)
            X[i] = tail[o + 4 * i] | ((uint32_t)tail[o + 4 * i + 1] << 8) |
                   ((uint32_t)tail[o + 4 * i + 2] << 16) | ((uint32_t)tail[o + 4 * i + 3] << 24);
        md5_compress(h, X);
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            md5[16 * t + 4 * i + j] = (uint8_t)(h[i] >> (8 * j));
}

hipError_t launch_bytes_md5(const uint8_t *base, const uint64_t *off, const uint64_t *len,
                            uint32_t n, uint8_t *md5, hipStream_t s)
{
    if (!n)
        return hipSuccess;
    hipLaunchKernelGGL(k_bytes_md5, dim3((n + 63u) / 64u), dim3(64), 0, s, base, off, len, n,
                       md5);
    return hipGetLastError();
}

hipError_t launch_track_md5(const FlacParams &p, const void *pcm, int fmt,
                            const TrackInfo *tracks, TrackOut *tout, hipStream_t s)
{
    if (!p.n_tracks)
        return hipSuccess;
    dim3 grid((p.n_tracks + 63u) / 64u);
    if (fmt == 0)
        hipLaunchKernelGGL((k_track_md5<int16_t>), grid, dim3(64), 0, s, p,
                           (const int16_t *)pcm, tracks, tout);
    else
        hipLaunchKernelGGL((k_track_md5<int32_t>), grid, dim3(64), 0, s, p,
                           (const int32_t *)pcm, tracks, tout);
    return hipGetLastError();
}
