// md5.hip — STREAMINFO MD5 of each track's PCM (reference: MD5 of the
// little-endian signed sample bytes fed by the PCM reader callback,
// src/encoders/flac.c:187-188, 1570-1576; src/pcmconv.c:266-291).
//
// MD5 is one serial chain per track, so a lane hashes one track and the
// time of a batch is one lane's chain.  A lone wave issues one VALU op per
// ~2.2 ns (tools/md5_rate.hip, profiles/r02_int_rate.txt), so the chain is
// bound by its instruction count, not by dependent latency: a round is
// F (v_bitop3), a + F + (X[g] + T) (v_add3), the rotate (v_alignbit) and
// + b (v_add) once the message-plus-constant word X[g] + T is given.
// Whole 64-byte blocks therefore run on a wave PAIR per 64 streams: the
// helper wave loads the blocks, forms the 64 words X[g(i)] + T[i] in round
// order and stores them to an LDS ring; the hasher wave reads them with
// 16 ds_read_b128 and runs 4 VALU ops per round.  One s_barrier per block
// hands a ring slot over.  The encoder launches it on its own stream,
// concurrently with the encoder kernels (it occupies a handful of SIMDs).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "flac_dev.h"
#include "launch.h"
#include "wave.h"

// build-time tuning constants (see launch_track_md5 / launch_bytes_md5)
// the decoder's chains at raised wave priority; the encoder's split: part 0
// takes this share of every track's blocks
constexpr int kDecMd5Prio = 1;
constexpr uint32_t kMd5SplitPct = 60u;

#define MD5_D 4

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) { return __builtin_amdgcn_alignbit(x, x, 32 - s); }

#define MD5_STEP(f, a, b, c, d, x, t, s) \
    a = b + rotl(a + f(b, c, d) + x + t, s)
#define F1(x, y, z) (z ^ (x & (y ^ z)))
#define F2(x, y, z) (y ^ (z & (x ^ y)))
// x ^ y ^ z as one v_bitop3_b32 (truth table 0x96); the compiler emits two
// v_xor_b32 otherwise (the builtin, unlike inline asm, needs no hazard nop)
__device__ __forceinline__ uint32_t xor3(uint32_t x, uint32_t y, uint32_t z)
{
    return __builtin_amdgcn_bitop3_b32(x, y, z, 0x96);
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

// RFC 1321 round i: message word g(i), constant T[i], rotate s(i)
#define MD5_ROUNDS_LO(S) \
    S(0, 0, 0xd76aa478, 7) S(1, 1, 0xe8c7b756, 12) S(2, 2, 0x242070db, 17) \
    S(3, 3, 0xc1bdceee, 22) S(4, 4, 0xf57c0faf, 7) S(5, 5, 0x4787c62a, 12) \
    S(6, 6, 0xa8304613, 17) S(7, 7, 0xfd469501, 22) S(8, 8, 0x698098d8, 7) \
    S(9, 9, 0x8b44f7af, 12) S(10, 10, 0xffff5bb1, 17) S(11, 11, 0x895cd7be, 22) \
    S(12, 12, 0x6b901122, 7) S(13, 13, 0xfd987193, 12) S(14, 14, 0xa679438e, 17) \
    S(15, 15, 0x49b40821, 22) S(16, 1, 0xf61e2562, 5) S(17, 6, 0xc040b340, 9) \
    S(18, 11, 0x265e5a51, 14) S(19, 0, 0xe9b6c7aa, 20) S(20, 5, 0xd62f105d, 5) \
    S(21, 10, 0x02441453, 9) S(22, 15, 0xd8a1e681, 14) S(23, 4, 0xe7d3fbc8, 20) \
    S(24, 9, 0x21e1cde6, 5) S(25, 14, 0xc33707d6, 9) S(26, 3, 0xf4d50d87, 14) \
    S(27, 8, 0x455a14ed, 20) S(28, 13, 0xa9e3e905, 5) S(29, 2, 0xfcefa3f8, 9) \
    S(30, 7, 0x676f02d9, 14) S(31, 12, 0x8d2a4c8a, 20)
#define MD5_ROUNDS_HI(S) \
    S(32, 5, 0xfffa3942, 4) S(33, 8, 0x8771f681, 11) S(34, 11, 0x6d9d6122, 16) \
    S(35, 14, 0xfde5380c, 23) S(36, 1, 0xa4beea44, 4) S(37, 4, 0x4bdecfa9, 11) \
    S(38, 7, 0xf6bb4b60, 16) S(39, 10, 0xbebfbc70, 23) S(40, 13, 0x289b7ec6, 4) \
    S(41, 0, 0xeaa127fa, 11) S(42, 3, 0xd4ef3085, 16) S(43, 6, 0x04881d05, 23) \
    S(44, 9, 0xd9d4d039, 4) S(45, 12, 0xe6db99e5, 11) S(46, 15, 0x1fa27cf8, 16) \
    S(47, 2, 0xc4ac5665, 23) S(48, 0, 0xf4292244, 6) S(49, 7, 0x432aff97, 10) \
    S(50, 14, 0xab9423a7, 15) S(51, 5, 0xfc93a039, 21) S(52, 12, 0x655b59c3, 6) \
    S(53, 3, 0x8f0ccc92, 10) S(54, 10, 0xffeff47d, 15) S(55, 1, 0x85845dd1, 21) \
    S(56, 8, 0x6fa87e4f, 6) S(57, 15, 0xfe2ce6e0, 10) S(58, 6, 0xa3014314, 15) \
    S(59, 13, 0x4e0811a1, 21) S(60, 4, 0xf7537e82, 6) S(61, 11, 0xbd3af235, 10) \
    S(62, 2, 0x2ad7d2bb, 15) S(63, 9, 0xeb86d391, 21)
#define MD5_ROUNDS(S) MD5_ROUNDS_LO(S) MD5_ROUNDS_HI(S)

__device__ __forceinline__ uint32_t u4_at(const uint4 &v, int c)
{
    return c == 0 ? v.x : c == 1 ? v.y : c == 2 ? v.z : v.w;
}

// helper: the round-ordered words X[g(i)] + T[i] of half HALF of a block
template <int HALF>
__device__ __forceinline__ void md5_xt_half(const uint4 (&blk)[4], uint4 (&xt)[8])
{
    uint32_t w[32];
#define MD5_XT(i, g, t, s) w[(i) & 31] = u4_at(blk[(g) >> 2], (g) & 3) + (t);
    if constexpr (HALF == 0) {
        MD5_ROUNDS_LO(MD5_XT)
    } else {
        MD5_ROUNDS_HI(MD5_XT)
    }
#undef MD5_XT
#pragma unroll
    for (int q = 0; q < 8; ++q)
        xt[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
}

// hasher: rounds 32 * HALF .. 32 * HALF + 31 of a block on the state v =
// (a, b, c, d) from that half's X[g] + T words (F1 .. F4 by round)
template <int HALF>
__device__ __forceinline__ void md5_half_xt(uint32_t (&v)[4], const uint4 (&xt)[8])
{
#define MD5_F(i, x, y, z) ((i) < 16 ? F1(x, y, z) : (i) < 32 ? F2(x, y, z) : (i) < 48 ? F3(x, y, z) : F4(x, y, z))
#define MD5_HS(i, g, t, s)                                                                      \
    {                                                                                           \
        uint32_t &a = v[(64 - (i)) & 3];                                                        \
        const uint32_t b = v[(65 - (i)) & 3], c = v[(66 - (i)) & 3], d = v[(67 - (i)) & 3];   \
        a = b + rotl(a + MD5_F(i, b, c, d) + u4_at(xt[((i) >> 2) & 7], (i) & 3), s);            \
    }
    if constexpr (HALF == 0) {
        MD5_ROUNDS_LO(MD5_HS)
    } else {
        MD5_ROUNDS_HI(MD5_HS)
    }
#undef MD5_HS
#undef MD5_F
}

// LDS ring of the wave pair: 3 half-block slots x 8 round-quads x 64
// lanes = 24 KB (it fits beside four K2 frame workgroups on a CU), and the
// two progress counters.  Units are half blocks, u = 2 * block + half, in
// slot u % 3.  prod = units the helper has stored; cons = units whose ring
// reads the hasher has completed.  A wave's LDS instructions execute in
// issue order, so a counter store issued after the data stores (helper) or
// after the data loads (hasher) is seen only once those have executed; a
// hasher load issued after a counter load that showed unit u is ready sees
// unit u's data.  No s_barrier in the loop (one costs the pair ~130 ns).
struct Md5Pair {
    uint4 ring[3][8][64];
    uint32_t prod, cons;
};

#define MD5_SPIN_MAX (1u << 22) // bounded waits: a lost wake-up cannot hang the GPU

__device__ __forceinline__ uint32_t md5_ctr(const uint32_t *c)
{
    return __builtin_amdgcn_readfirstlane(__atomic_load_n(c, __ATOMIC_RELAXED));
}

__device__ __forceinline__ void md5_wait(const uint32_t *c, uint32_t need)
{
    for (uint32_t i = 0; i < MD5_SPIN_MAX && md5_ctr(c) < need; ++i)
        __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void md5_publish(uint32_t *c, uint32_t v)
{
    asm volatile("" ::: "memory");
    if ((threadIdx.x & 63u) == 0u)
        __atomic_store_n(c, v, __ATOMIC_RELAXED);
}

__device__ __forceinline__ void md5_load_unit(const Md5Pair &pr, uint32_t slot, int lane, uint4 (&x)[8])
{
#pragma unroll
    for (int k = 0; k < 8; ++k)
        x[k] = pr.ring[slot][k][lane];
}

// one block b = u / 2 of the hasher: half 0 from cur while unit u + 1 is
// loaded into nxt, half 1 from nxt while unit u + 2 (MORE) is loaded into
// cur; the prod counter is read before each speculative load and checked
// after the half it overlaps
template <bool ON_ALL, bool MORE>
__device__ __forceinline__ void md5_hasher_block(uint32_t b, uint32_t full, uint32_t h[4],
                                                 Md5Pair &pr, int lane, uint32_t &slot,
                                                 uint4 (&cur)[8], uint4 (&nxt)[8])
{
    const bool on = ON_ALL || b < full;
    const uint32_t u = 2u * b;
    const uint32_t s1 = slot == 2u ? 0u : slot + 1u, s2 = s1 == 2u ? 0u : s1 + 1u;
    uint32_t v[4] = {h[0], h[1], h[2], h[3]};
    uint32_t p = md5_ctr(&pr.prod);
    asm volatile("" ::: "memory");
    md5_load_unit(pr, s1, lane, nxt);
    if (on)
        md5_half_xt<0>(v, cur);
    if (p < u + 2u) {
        md5_wait(&pr.prod, u + 2u);
        md5_load_unit(pr, s1, lane, nxt);
    }
    md5_publish(&pr.cons, u + 2u); // units <= u + 1 read
    if (MORE) {
        p = md5_ctr(&pr.prod);
        asm volatile("" ::: "memory");
        md5_load_unit(pr, s2, lane, cur);
    }
    if (on) {
        md5_half_xt<1>(v, nxt);
        h[0] += v[0];
        h[1] += v[1];
        h[2] += v[2];
        h[3] += v[3];
    }
    if (MORE) {
        if (p < u + 3u) {
            md5_wait(&pr.prod, u + 3u);
            md5_load_unit(pr, s2, lane, cur);
        }
        md5_publish(&pr.cons, u + 3u);
    }
    slot = s2;
}

template <bool ON_ALL>
__device__ __forceinline__ void md5_hasher(uint32_t full, uint32_t nbmax, uint32_t h[4],
                                           Md5Pair &pr, int lane)
{
    uint4 cur[8], nxt[8];
    md5_wait(&pr.prod, 1u);
    md5_load_unit(pr, 0u, lane, cur);
    uint32_t slot = 0; // slot of unit 2b
    for (uint32_t b = 0; b + 1u < nbmax; ++b)
        md5_hasher_block<ON_ALL, true>(b, full, h, pr, lane, slot, cur, nxt);
    md5_hasher_block<ON_ALL, false>(nbmax - 1u, full, h, pr, lane, slot, cur, nxt);
}

// Whole blocks [0, full) of the lane's 16-byte aligned stream q, on the
// wave pair (threadIdx.x >> 6: 0 hasher, 1 helper; both call this with the
// same lane -> stream mapping and the same wave-uniform nbmax = max full,
// after pr's counters were zeroed and the pair met once).  The hasher's h
// advances over the lane's `full` blocks.  The hasher loads unit u + 1
// speculatively, with the prod counter, while it hashes unit u, and checks
// the counter after; the helper runs up to 2 units ahead.
__device__ __forceinline__ void md5_pair_blocks(const uint4 *__restrict__ q, uint32_t full,
                                                uint32_t nbmax, uint32_t h[4], Md5Pair &pr)
{
    const int lane = threadIdx.x & 63;
    const bool helper = (threadIdx.x >> 6) != 0;
    const uint32_t last = full ? full - 1u : 0u;
    if (helper) {
        uint4 buf[MD5_D][4]; // block k in buf[k % MD5_D]
        if (full) {
#pragma unroll
            for (int j = 0; j < MD5_D; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    buf[j][i] = q[(size_t)min((uint32_t)j, last) * 4u + i];
        }
        uint32_t slot = 0; // slot of unit 2b
        for (uint32_t b0 = 0; b0 < nbmax; b0 += MD5_D) {
#pragma unroll
            for (int j = 0; j < MD5_D; ++j) {
                const uint32_t b = b0 + (uint32_t)j;
                if (b < nbmax) {
#pragma unroll
                    for (int hf = 0; hf < 2; ++hf) {
                        const uint32_t u = 2u * b + (uint32_t)hf;
                        uint4 xt[8];
                        if (hf == 0)
                            md5_xt_half<0>(buf[j], xt);
                        else
                            md5_xt_half<1>(buf[j], xt);
                        if (hf == 1 && full) {
#pragma unroll
                            for (int i = 0; i < 4; ++i)
                                buf[j][i] = q[(size_t)min(b + MD5_D, last) * 4u + i];
                        }
                        if (u >= 3u)
                            md5_wait(&pr.cons, u - 2u); // unit u - 3 left the slot
#pragma unroll
                        for (int k = 0; k < 8; ++k)
                            pr.ring[slot][k][lane] = xt[k];
                        md5_publish(&pr.prod, u + 1u);
                        slot = slot == 2u ? 0u : slot + 1u;
                    }
                }
            }
        }
    } else if (wave_all(full == nbmax)) {
        md5_hasher<true>(full, nbmax, h, pr, lane); // every lane hashes every block
    } else {
        md5_hasher<false>(full, nbmax, h, pr, lane);
    }
}

// int32 containers (16-byte aligned tracks of 1..3-byte samples): the same
// wave pair, the helper packing whole sample groups into the little-endian
// byte stream with v_perm (S32Pack, defined below) -- a group of G samples is
// W / 16 blocks (3 for 24-bit) -- and feeding the same ring; `full` blocks
// are whole groups.
template <int BB>
struct S32Pack;

template <int BB>
__device__ __forceinline__ void md5_pair_blocks_s32(const uint4 *__restrict__ q, uint32_t full,
                                                    uint32_t nbmax, uint32_t h[4], Md5Pair &pr)
{
    using P = S32Pack<BB>;
    constexpr uint32_t BPG = P::W / 16; // blocks per group
    const int lane = threadIdx.x & 63;
    const bool helper = (threadIdx.x >> 6) != 0;
    if (helper) {
        const uint32_t groups = full / BPG;
        const uint32_t lastg = groups ? groups - 1u : 0u;
        uint4 cur[P::Q], nxt[P::Q];
        if (groups) {
#pragma unroll
            for (int i = 0; i < P::Q; ++i)
                cur[i] = q[i];
        }
        uint32_t slot = 0;
        for (uint32_t g = 0; g * BPG < nbmax; ++g) {
            if (groups) {
#pragma unroll
                for (int i = 0; i < P::Q; ++i)
                    nxt[i] = q[(size_t)min(g + 1u, lastg) * P::Q + i];
            }
            uint32_t w[P::W];
            P::pack(cur, w);
#pragma unroll
            for (uint32_t k = 0; k < BPG; ++k) {
                const uint32_t b = g * BPG + k;
                if (b < nbmax) {
                    uint4 bl[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i)
                        bl[i] = make_uint4(w[16 * k + 4 * i], w[16 * k + 4 * i + 1],
                                           w[16 * k + 4 * i + 2], w[16 * k + 4 * i + 3]);
#pragma unroll
                    for (int hf = 0; hf < 2; ++hf) {
                        const uint32_t u = 2u * b + (uint32_t)hf;
                        uint4 xt[8];
                        if (hf == 0)
                            md5_xt_half<0>(bl, xt);
                        else
                            md5_xt_half<1>(bl, xt);
                        if (u >= 3u)
                            md5_wait(&pr.cons, u - 2u);
#pragma unroll
                        for (int m = 0; m < 8; ++m)
                            pr.ring[slot][m][lane] = xt[m];
                        md5_publish(&pr.prod, u + 1u);
                        slot = slot == 2u ? 0u : slot + 1u;
                    }
                }
            }
#pragma unroll
            for (int i = 0; i < P::Q; ++i)
                cur[i] = nxt[i];
        }
    } else if (wave_all(full == nbmax)) {
        md5_hasher<true>(full, nbmax, h, pr, lane);
    } else {
        md5_hasher<false>(full, nbmax, h, pr, lane);
    }
}

// The pair's waves allocate 192 VGPRs.  A lone hash chain issues about as
// often as half a SIMD, so the waves beside it split the other half: at 192
// VGPRs at most one LPC wave (184), two search waves (120) or one pack wave
// (256) fit beside a chain -- each then gets the issue share it has on a
// SIMD of its own kernel, and none straggles.  At 128 VGPRs two LPC waves
// shared a chain's SIMD at a quarter of the issue each and the LPC kernel
// ran 2.2 ms instead of 1.3 ms beside the chains.
__device__ __forceinline__ void md5_vgpr_192()
{
    asm volatile("" ::: "v191");
}

// zero the pair's counters, then meet once
__device__ __forceinline__ void md5_pair_init(Md5Pair &pr)
{
    if (threadIdx.x == 0) {
        pr.prod = 0;
        pr.cons = 0;
    }
    __syncthreads();
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

// the MD5 state as digest-order bytes: the hand-over from the pair kernel
// to the finishing kernel (and, after the padding block, the digest itself)
__device__ __forceinline__ void md5_put(uint8_t *d, const uint32_t h[4])
{
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            d[4 * i + j] = (uint8_t)(h[i] >> (8 * j));
}

__device__ __forceinline__ void md5_get(const uint8_t *d, uint32_t h[4])
{
    for (int i = 0; i < 4; ++i)
        h[i] = d[4 * i] | ((uint32_t)d[4 * i + 1] << 8) | ((uint32_t)d[4 * i + 2] << 16) |
               ((uint32_t)d[4 * i + 3] << 24);
}

// the last partial block + padding (0x80, zeros, 64-bit little-endian bit
// length) of an nbytes stream whose whole blocks are in h; byte(j) = byte j
template <typename B>
__device__ __forceinline__ void md5_pad(uint32_t h[4], uint64_t nbytes, B &&byte)
{
    const uint64_t full = nbytes / 64u;
    uint32_t X[16];
    uint8_t tail[128];
    const uint32_t rem = (uint32_t)(nbytes - full * 64u);
    for (uint32_t i = 0; i < rem; ++i)
        tail[i] = (uint8_t)byte(full * 64u + i);
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
}

// S16 PCM at 16 bits, 16-byte aligned: the sample container IS the byte
// stream, hashed block by block on the wave pair
__device__ __forceinline__ bool md5_track_raw(const FlacParams &p, const TrackInfo &ti,
                                              const int16_t *pcm, uint64_t &full)
{
    const uint64_t nbytes = ti.pcm_frames * p.channels * 2u;
    full = nbytes / 64u;
    const int16_t *s = pcm + ti.pcm_start * p.channels;
    return p.bps == 16u && (((uintptr_t)s) & 15u) == 0 && full < (1ull << 32);
}

// whole blocks of the raw tracks (a hasher + helper wave pair per 64
// tracks), in two parts: part 0 blocks [0, 3 full / 5) from the initial
// state, part 1 the rest from part 0's state; the state goes to tout[t].md5
// (for part 1, then k_track_md5).  The engine runs the parts one batch
// apart, beside the search and pack kernels of two batches, so no chain
// runs beside the LPC kernel (whose two-waves-per-SIMD grid straggles when
// a chain takes SIMD slots).  Part 0 (~7.3 ms) fits under a batch's search
// and pack (~9 ms) with room; part 1 is what a last batch adds when waited.
__global__ __launch_bounds__(128) void k_track_md5_pair(FlacParams p, const int16_t *__restrict__ pcm,
                                                        const TrackInfo *__restrict__ tracks,
                                                        TrackOut *__restrict__ tout, int prio, int part,
                                                        uint32_t split_pct)
{
    // prio: the chains' waves issue ahead of the kernels sharing their SIMDs
    if (prio)
        __builtin_amdgcn_s_setprio(3);
    __shared__ Md5Pair pair_lds;
    const uint32_t t = blockIdx.x * 64u + (threadIdx.x & 63u);
    const bool valid = t < p.n_tracks;
    const TrackInfo ti = tracks[valid ? t : 0u];
    uint64_t full = 0;
    const bool raw = valid && md5_track_raw(p, ti, pcm, full);
    // part 2: every block (an unsplit chain)
    const uint32_t split = part == 2 ? 0u : (uint32_t)(full * split_pct / 100u);
    const uint32_t b0 = part == 1 ? split : 0u;
    const uint32_t n = raw ? (part == 0 ? split : (uint32_t)full - split) : 0u;
    const uint32_t nbmax = wave_max_u32(n);
    if (!nbmax)
        return;
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    if (part == 1 && split && raw && threadIdx.x < 64u)
        md5_get(tout[t].md5, h); // part 0's state (written for every lane with split > 0)
    md5_vgpr_192();
    md5_pair_init(pair_lds);
    md5_pair_blocks((const uint4 *)(pcm + ti.pcm_start * p.channels) + (size_t)b0 * 4u, n, nbmax,
                    h, pair_lds);
    if (threadIdx.x < 64u && n)
        md5_put(tout[t].md5, h);
}

// k_track_md5_pair for int32 containers of BB-byte samples: whole sample
// groups on the wave pair, split in two parts at a group boundary as above
template <int BB>
__global__ __launch_bounds__(128) void k_track_md5_pair_s32(FlacParams p,
                                                            const int32_t *__restrict__ pcm,
                                                            const TrackInfo *__restrict__ tracks,
                                                            TrackOut *__restrict__ tout, int prio,
                                                            int part, uint32_t split_pct)
{
    using P = S32Pack<BB>;
    constexpr uint32_t BPG = P::W / 16;
    if (prio)
        __builtin_amdgcn_s_setprio(3);
    __shared__ Md5Pair pair_lds;
    const uint32_t t = blockIdx.x * 64u + (threadIdx.x & 63u);
    const bool valid = t < p.n_tracks;
    const TrackInfo ti = tracks[valid ? t : 0u];
    const int32_t *s = pcm + ti.pcm_start * p.channels;
    const uint64_t groups64 = valid && (((uintptr_t)s) & 15u) == 0
                                  ? ti.pcm_frames * p.channels / P::G : 0u;
    const uint32_t groups = groups64 * BPG < (1ull << 32) ? (uint32_t)groups64 : 0u;
    const uint32_t split = part == 2 ? 0u : (uint32_t)((uint64_t)groups * split_pct / 100u);
    const uint32_t g0 = part == 1 ? split : 0u;
    const uint32_t n = (part == 0 ? split : groups - split) * BPG;
    const uint32_t nbmax = wave_max_u32(n);
    if (!nbmax)
        return;
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    if (part == 1 && split && threadIdx.x < 64u)
        md5_get(tout[t].md5, h);
    md5_vgpr_192();
    md5_pair_init(pair_lds);
    md5_pair_blocks_s32<BB>((const uint4 *)s + (size_t)g0 * P::Q, n, nbmax, h, pair_lds);
    if (threadIdx.x < 64u && n)
        md5_put(tout[t].md5, h);
}

// lane per track: the tracks the pair kernel did not take (int32
// containers, other widths, unaligned starts) from the start, then every
// track's last partial block + padding, and the digest
template <typename T>
__global__ __launch_bounds__(64) void k_track_md5(FlacParams p, const T *__restrict__ pcm,
                                                  const TrackInfo *__restrict__ tracks,
                                                  TrackOut *__restrict__ tout, int paired)
{
    __builtin_amdgcn_s_setprio(3);
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= p.n_tracks)
        return;
    const TrackInfo ti = tracks[t];
    const uint32_t bb = p.bps / 8u;
    const T *s = pcm + ti.pcm_start * p.channels;
    const uint64_t nbytes = ti.pcm_frames * p.channels * bb;
    uint64_t full = nbytes / 64u;
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    uint64_t blk = 0;
    if (paired && sizeof(T) == 2 && md5_track_raw(p, ti, (const int16_t *)pcm, full)) {
        if (full) // (no whole block: the pair kernel left this lane alone)
            md5_get(tout[t].md5, h);
        blk = full;
    } else if (sizeof(T) == 4 && (((uintptr_t)s) & 15u) == 0 && bb >= 1 && bb <= 3) {
        // int32 container, 16-byte aligned: whole sample groups by v_perm
        // packing -- on the wave pair when `paired` (its state in tout.md5),
        // here otherwise; the bytes after the last whole group go the
        // generic way
        const uint64_t samples = ti.pcm_frames * p.channels;
        const uint4 *q = (const uint4 *)s;
        const uint64_t g = samples / (bb == 2 ? S32Pack<2>::G : S32Pack<3>::G);
        const uint32_t bpg = bb == 3 ? 3u : 1u;
        if (paired && g * bpg < (1ull << 32)) {
            if (g)
                md5_get(tout[t].md5, h);
        } else if (bb == 3) {
            md5_s32_groups<3>(h, q, g);
        } else if (bb == 2) {
            md5_s32_groups<2>(h, q, g);
        } else {
            md5_s32_groups<1>(h, q, g);
        }
        blk = g * bpg;
    }
    uint32_t X[16];
    for (; blk < full; ++blk) {
        for (int i = 0; i < 16; ++i) {
            const uint64_t j = blk * 64u + 4u * (uint32_t)i;
            X[i] = pcm_byte(s, j, bb) | (pcm_byte(s, j + 1, bb) << 8) |
                   (pcm_byte(s, j + 2, bb) << 16) | (pcm_byte(s, j + 3, bb) << 24);
        }
        md5_compress(h, X);
    }
    md5_pad(h, nbytes, [&](uint64_t j) { return pcm_byte(s, j, bb); });
    md5_put(tout[t].md5, h);
}

// Rolled chains (engine "rolled" mode, many narrow batches in flight): one
// launch advances the whole-block chains of up to kRollMax batches at once,
// each by its own slice [full * part / parts, full * part_end / parts) of
// every track's blocks (int32 containers: of its sample groups), from the
// state the previous slice left in tout[t].md5.  A batch's chain thus runs
// as `parts` slices, one per later batch's enqueue, and every batch in
// flight shares ONE launch per step on one stream -- instead of one long
// kernel per batch, each on a stream of its own, whose chains serialise
// once the batches in flight outnumber the hardware queues.  Workgroup w
// belongs to the batch whose [wg0, wg0 + ceil(n_tracks / 64)) holds it.
__global__ __launch_bounds__(128) void k_track_md5_roll(MdRollArgs a)
{
    uint32_t k = 0;
    while (k + 1u < a.n && blockIdx.x >= a.b[k + 1].wg0)
        ++k;
    const MdRollBatch &B = a.b[k];
    __shared__ Md5Pair pair_lds;
    const uint32_t t = (blockIdx.x - B.wg0) * 64u + (threadIdx.x & 63u);
    const bool valid = t < B.n_tracks;
    const TrackInfo ti = B.tracks[valid ? t : 0u];
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    if (B.fmt == 0) {
        // S16 at 16 bits, 16-byte aligned (md5_track_raw)
        const int16_t *s = (const int16_t *)B.pcm + ti.pcm_start * B.channels;
        const uint64_t full = ti.pcm_frames * B.channels * 2u / 64u;
        const bool raw = valid && B.bps == 16u && (((uintptr_t)s) & 15u) == 0 &&
                         full < (1ull << 32);
        const uint32_t b0 = raw ? (uint32_t)(full * B.part / B.parts) : 0u;
        const uint32_t b1 = raw ? (uint32_t)(full * B.part_end / B.parts) : 0u;
        const uint32_t n = b1 - b0;
        const uint32_t nbmax = wave_max_u32(n);
        if (!nbmax)
            return;
        if (b0 && threadIdx.x < 64u)
            md5_get(B.tout[t].md5, h);
        md5_vgpr_192();
        md5_pair_init(pair_lds);
        md5_pair_blocks((const uint4 *)s + (size_t)b0 * 4u, n, nbmax, h, pair_lds);
        if (threadIdx.x < 64u && n)
            md5_put(B.tout[t].md5, h);
        return;
    }
    const uint32_t bb = B.bps / 8u;
    const int32_t *s = (const int32_t *)B.pcm + ti.pcm_start * B.channels;
    const uint32_t G = bb == 2u ? 32u : 64u, BPG = bb == 3u ? 3u : 1u, Q = G / 4u;
    const uint64_t groups64 = valid && (((uintptr_t)s) & 15u) == 0
                                  ? ti.pcm_frames * B.channels / G : 0u;
    const uint32_t groups = groups64 * BPG < (1ull << 32) ? (uint32_t)groups64 : 0u;
    const uint32_t g0 = (uint32_t)((uint64_t)groups * B.part / B.parts);
    const uint32_t g1 = (uint32_t)((uint64_t)groups * B.part_end / B.parts);
    const uint32_t n = (g1 - g0) * BPG;
    const uint32_t nbmax = wave_max_u32(n);
    if (!nbmax)
        return;
    if (g0 && threadIdx.x < 64u)
        md5_get(B.tout[t].md5, h);
    md5_vgpr_192();
    md5_pair_init(pair_lds);
    const uint4 *q = (const uint4 *)s + (size_t)g0 * Q;
    if (bb == 3u)
        md5_pair_blocks_s32<3>(q, n, nbmax, h, pair_lds);
    else if (bb == 2u)
        md5_pair_blocks_s32<2>(q, n, nbmax, h, pair_lds);
    else
        md5_pair_blocks_s32<1>(q, n, nbmax, h, pair_lds);
    if (threadIdx.x < 64u && n)
        md5_put(B.tout[t].md5, h);
}

// true when launch_track_md5 would hash this batch's whole blocks on wave
// pairs (the formats the rolled mode takes)
bool track_md5_paired(const FlacParams &p, int fmt)
{
    const uint32_t bb = p.bps / 8u;
    return (fmt == 0 && p.bps == 16u) || (fmt == 1 && p.bps % 8u == 0u && bb >= 1u && bb <= 3u);
}

hipError_t launch_track_md5_roll(const MdRollArgs &a, hipStream_t s)
{
    uint32_t wgs = 0;
    for (uint32_t k = 0; k < a.n; ++k)
        wgs = a.b[k].wg0 + (a.b[k].n_tracks + 63u) / 64u;
    if (!wgs)
        return hipSuccess;
    hipLaunchKernelGGL(k_track_md5_roll, dim3(wgs), dim3(128), 0, s, a);
    return hipGetLastError();
}

// the finishing kernel alone: every track's tail + padding after its rolled
// whole-block chain (the lane-per-track path for what the pairs skipped)
hipError_t launch_track_md5_finish(const FlacParams &p, const void *pcm, int fmt,
                                   const TrackInfo *tracks, TrackOut *tout, hipStream_t s)
{
    if (!p.n_tracks)
        return hipSuccess;
    const dim3 grid((p.n_tracks + 63u) / 64u);
    const int paired = track_md5_paired(p, fmt);
    if (fmt == 0)
        hipLaunchKernelGGL((k_track_md5<int16_t>), grid, dim3(64), 0, s, p,
                           (const int16_t *)pcm, tracks, tout, paired);
    else
        hipLaunchKernelGGL((k_track_md5<int32_t>), grid, dim3(64), 0, s, p,
                           (const int32_t *)pcm, tracks, tout, paired);
    return hipGetLastError();
}

// MD5 of a plain byte stream per lane (the decoder hashes the little-endian
// PCM bytes K5 of flac_decode.hip wrote; streams start 64-byte aligned):
// whole blocks on the wave pair, state to md5[16 t]
__global__ __launch_bounds__(128) void k_bytes_md5_pair(const uint8_t *__restrict__ base,
                                                        const uint64_t *__restrict__ off,
                                                        const uint64_t *__restrict__ len, uint32_t n,
                                                        uint8_t *__restrict__ md5, int prio)
{
    if (prio)
        __builtin_amdgcn_s_setprio(3);
    __shared__ Md5Pair pair_lds;
    const uint32_t t = blockIdx.x * 64u + (threadIdx.x & 63u);
    const bool valid = t < n;
    const uint64_t full = valid ? len[t] / 64u : 0u;
    const bool pair = full < (1ull << 32);
    const uint32_t nbmax = wave_max_u32(pair ? (uint32_t)full : 0u);
    if (!nbmax)
        return;
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    // the decoder's kernels run few, long waves (a lane parses a whole frame):
    // a chain wave takes a SIMD to itself (256 VGPRs + 256 AGPRs) so none
    // of them shares its issue with a chain
    asm volatile("" ::: "v255", "a255");
    md5_pair_init(pair_lds);
    md5_pair_blocks((const uint4 *)(base + off[valid ? t : 0u]), pair ? (uint32_t)full : 0u, nbmax,
                    h, pair_lds);
    if (threadIdx.x < 64u && valid)
        md5_put(md5 + 16u * t, h);
}

// lane per stream: the blocks the pair kernel did not take, the padding,
// the digest
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
    uint64_t blk = 0;
    if (full < (1ull << 32)) {
        if (full)
            md5_get(md5 + 16u * t, h);
        blk = full;
    }
    uint32_t X[16];
    for (; blk < full; ++blk) {
        for (int i = 0; i < 16; ++i)
            X[i] = s[blk * 64u + 4 * i] | ((uint32_t)s[blk * 64u + 4 * i + 1] << 8) |
                   ((uint32_t)s[blk * 64u + 4 * i + 2] << 16) |
                   ((uint32_t)s[blk * 64u + 4 * i + 3] << 24);
        md5_compress(h, X);
    }
    md5_pad(h, nbytes, [&](uint64_t j) { return (uint32_t)s[j]; });
    md5_put(md5 + 16u * t, h);
}

// Rolled byte-stream chains (decoder rolled mode, atg_decoder_set_inflight):
// as k_track_md5_roll, one launch advances every batch in flight by its own
// slice [full * part / parts, full * part_end / parts) of each stream's
// whole blocks, from the state the previous slice left in md5[16 t]
__global__ __launch_bounds__(128) void k_bytes_md5_roll(MdBytesRollArgs a)
{
    uint32_t k = 0;
    while (k + 1u < a.n && blockIdx.x >= a.b[k + 1].wg0)
        ++k;
    const MdBytesRoll &B = a.b[k];
    __shared__ Md5Pair pair_lds;
    const uint32_t t = (blockIdx.x - B.wg0) * 64u + (threadIdx.x & 63u);
    const bool valid = t < B.n;
    const uint64_t full = valid ? B.len[t] / 64u : 0u;
    const bool pair = full < (1ull << 32);
    const uint32_t b0 = pair ? (uint32_t)(full * B.part / B.parts) : 0u;
    const uint32_t b1 = pair ? (uint32_t)(full * B.part_end / B.parts) : 0u;
    const uint32_t n = b1 - b0;
    const uint32_t nbmax = wave_max_u32(n);
    if (!nbmax)
        return;
    uint32_t h[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    if (b0 && threadIdx.x < 64u)
        md5_get(B.md5 + 16u * t, h);
    // a SIMD to itself, as k_bytes_md5_pair (192 VGPRs, sharing SIMDs with
    // the parse and restore waves, measured the same: profiles/r05_dec_depth.json)
    asm volatile("" ::: "v255", "a255");
    md5_pair_init(pair_lds);
    md5_pair_blocks((const uint4 *)(B.base + B.off[valid ? t : 0u]) + (size_t)b0 * 4u, n, nbmax, h,
                    pair_lds);
    if (threadIdx.x < 64u && n)
        md5_put(B.md5 + 16u * t, h);
}

hipError_t launch_bytes_md5_roll(const MdBytesRollArgs &a, hipStream_t s)
{
    uint32_t wgs = 0;
    for (uint32_t k = 0; k < a.n; ++k)
        wgs = a.b[k].wg0 + (a.b[k].n + 63u) / 64u;
    if (!wgs)
        return hipSuccess;
    hipLaunchKernelGGL(k_bytes_md5_roll, dim3(wgs), dim3(128), 0, s, a);
    return hipGetLastError();
}

// the finishing kernel alone (tails, padding, streams the pairs skipped)
hipError_t launch_bytes_md5_finish(const uint8_t *base, const uint64_t *off, const uint64_t *len,
                                   uint32_t n, uint8_t *md5, hipStream_t s)
{
    if (!n)
        return hipSuccess;
    hipLaunchKernelGGL(k_bytes_md5, dim3((n + 63u) / 64u), dim3(64), 0, s, base, off, len, n, md5);
    return hipGetLastError();
}

hipError_t launch_bytes_md5(const uint8_t *base, const uint64_t *off, const uint64_t *len,
                            uint32_t n, uint8_t *md5, hipStream_t s)
{
    if (!n)
        return hipSuccess;
    const dim3 grid((n + 63u) / 64u);
    // the decoder's chains at raised wave priority (normal priority measured
    // no different)
    const int prio = kDecMd5Prio;
    hipLaunchKernelGGL(k_bytes_md5_pair, grid, dim3(128), 0, s, base, off, len, n, md5, prio);
    hipLaunchKernelGGL(k_bytes_md5, grid, dim3(64), 0, s, base, off, len, n, md5);
    return hipGetLastError();
}

// part 0 / 1: the two halves of a split chain (part 1 adds the finishing
// kernel); part 2: the whole chain and the finishing kernel
hipError_t launch_track_md5(const FlacParams &p, const void *pcm, int fmt,
                            const TrackInfo *tracks, TrackOut *tout, int part, hipStream_t s)
{
    if (!p.n_tracks)
        return hipSuccess;
    const dim3 grid((p.n_tracks + 63u) / 64u);
    const uint32_t bb = p.bps / 8u;
    const int paired = (fmt == 0 && p.bps == 16u) || (fmt == 1 && bb >= 1u && bb <= 3u);
    // the chains at normal wave priority (raised priority measured no
    // different: the engine keeps three batches in flight so the chains stay
    // off the critical path); part 0 takes kMd5SplitPct % of every track's
    // blocks (50/60/70 measured within 0.5 % of each other)
    const int prio = 0;
    const uint32_t split_pct = kMd5SplitPct;
    if (paired && fmt == 0)
        hipLaunchKernelGGL(k_track_md5_pair, grid, dim3(128), 0, s, p, (const int16_t *)pcm, tracks,
                           tout, prio, part, split_pct);
    else if (paired && bb == 3u)
        hipLaunchKernelGGL(k_track_md5_pair_s32<3>, grid, dim3(128), 0, s, p, (const int32_t *)pcm,
                           tracks, tout, prio, part, split_pct);
    else if (paired && bb == 2u)
        hipLaunchKernelGGL(k_track_md5_pair_s32<2>, grid, dim3(128), 0, s, p, (const int32_t *)pcm,
                           tracks, tout, prio, part, split_pct);
    else if (paired)
        hipLaunchKernelGGL(k_track_md5_pair_s32<1>, grid, dim3(128), 0, s, p, (const int32_t *)pcm,
                           tracks, tout, prio, part, split_pct);
    if (part == 0)
        return hipGetLastError();
    if (fmt == 0)
        hipLaunchKernelGGL((k_track_md5<int16_t>), grid, dim3(64), 0, s, p,
                           (const int16_t *)pcm, tracks, tout, paired);
    else
        hipLaunchKernelGGL((k_track_md5<int32_t>), grid, dim3(64), 0, s, p,
                           (const int32_t *)pcm, tracks, tout, paired);
    return hipGetLastError();
}

// host-hashed digests (engine host-MD5 mode) into the tracks' TrackOut, for
// the stream-header kernel that follows on the same stream
__global__ __launch_bounds__(64) void k_put_md5(TrackOut *__restrict__ tout,
                                                const uint8_t *__restrict__ md5, uint32_t n)
{
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n)
        return;
    for (int i = 0; i < 16; ++i)
        tout[t].md5[i] = md5[16u * t + i];
}

// engine host-MD5 mode: a track's MD5 byte stream -- the low bb bytes of
// each container, little-endian (FrameList.to_bytes, src/pcm.c) -- packed
// on the device, so the download carries only those bytes and the host
// threads hash them as they are (md5_cpu.h hash_bytes_multi).  A lane per
// four samples: 4 bb bytes, whole dwords (dst is 16-byte aligned).
template <typename T>
__global__ __launch_bounds__(256) void k_md5_pack(const T *__restrict__ src, uint64_t n, uint32_t bb,
                                                  uint8_t *__restrict__ dst)
{
    const uint64_t i = 4u * ((uint64_t)blockIdx.x * 256u + threadIdx.x);
    if (i >= n)
        return;
    if (i + 4u <= n) {
        const uint32_t v0 = (uint32_t)src[i], v1 = (uint32_t)src[i + 1];
        const uint32_t v2 = (uint32_t)src[i + 2], v3 = (uint32_t)src[i + 3];
        uint32_t *o = (uint32_t *)(dst + i * bb);
        if (bb == 1u) {
            o[0] = (v0 & 0xFFu) | ((v1 & 0xFFu) << 8) | ((v2 & 0xFFu) << 16) | (v3 << 24);
        } else if (bb == 2u) {
            *(uint2 *)o = make_uint2((v0 & 0xFFFFu) | (v1 << 16), (v2 & 0xFFFFu) | (v3 << 16));
        } else if (bb == 3u) {
            o[0] = (v0 & 0xFFFFFFu) | (v1 << 24);
            o[1] = ((v1 >> 8) & 0xFFFFu) | (v2 << 16);
            o[2] = ((v2 >> 16) & 0xFFu) | (v3 << 8);
        } else {
            *(uint4 *)o = make_uint4(v0, v1, v2, v3);
        }
    } else {
        for (uint64_t q = i; q < n; ++q) {
            const uint32_t v = (uint32_t)src[q];
            for (uint32_t b = 0; b < bb; ++b)
                dst[q * bb + b] = (uint8_t)(v >> (8u * b));
        }
    }
}

hipError_t launch_md5_pack(const void *src, int s16, uint64_t n, uint32_t bb, uint8_t *dst,
                           hipStream_t s)
{
    if (!n)
        return hipSuccess;
    const dim3 grid((unsigned)((n + 1023u) / 1024u));
    if (s16)
        hipLaunchKernelGGL((k_md5_pack<int16_t>), grid, dim3(256), 0, s, (const int16_t *)src, n,
                           bb, dst);
    else
        hipLaunchKernelGGL((k_md5_pack<int32_t>), grid, dim3(256), 0, s, (const int32_t *)src, n,
                           bb, dst);
    return hipGetLastError();
}

hipError_t launch_put_md5(TrackOut *tout, const uint8_t *md5, uint32_t n, hipStream_t s)
{
    if (!n)
        return hipSuccess;
    hipLaunchKernelGGL(k_put_md5, dim3((n + 63u) / 64u), dim3(64), 0, s, tout, md5, n);
    return hipGetLastError();
}
