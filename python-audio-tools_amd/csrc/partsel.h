// partsel.h — the reference's residual partition-order search
// (flacenc_encode_residuals, src/encoders/flac.c:1362-1402) over a wave whose
// lane l owns a contiguous run inside finest partition l >> (6 - P): Rice
// parameters and size estimates of every (order, partition), argmin with the
// reference's strict `<`.  Shared by both K2 variants (flac_search.hip,
// flac_search16.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "flac_dev.h"
#include "rice.h"
#include "wave.h"


struct RunCtx {
    int lane;
    int a;       // first sample of this lane's run
    int len;     // samples in the run
    uint32_t N;
    int P;       // deepest partition order usable (N % 2^P == 0, P <= max)
    uint32_t max_rice;
};

struct PartSel {
    uint32_t porder;
    uint32_t method;
    uint32_t k_lane;  // Rice parameter applied to this lane's residuals
    uint32_t k_own;   // Rice parameter of this lane's partition (for storage)
    uint32_t hdr_bits;
};

// Rice parameter and estimate of partition j at level lv (sum = its |r| sum)
template <typename S>
__device__ __forceinline__ void part_eval(uint32_t lv, uint32_t j, S Sj, S total,
                                          uint32_t order, const RunCtx &c, uint32_t &k, S &e)
{
    const uint32_t Sp = c.N >> lv;
    const bool degen = Sp < order; // partition 0 takes every residual
    const uint32_t plen = j == 0 ? Sp - order : Sp;
    const S sum = degen ? (j == 0 ? total : (S)0) : Sj;
    k = rice_param(plen, (uint64_t)sum, c.max_rice);
    e = part_estimate<S>(plen, sum, k);
}

// wave primitives on 32- or 64-bit values
__device__ __forceinline__ uint32_t wshfl_up(uint32_t v, int d)
{
    return (uint32_t)__shfl_up((int)v, d, 64);
}
__device__ __forceinline__ uint64_t wshfl_up(uint64_t v, int d) { return shfl_up_u64(v, d); }
__device__ __forceinline__ uint32_t wshfl(uint32_t v, int src)
{
    return (uint32_t)__shfl((int)v, src, 64);
}
__device__ __forceinline__ uint64_t wshfl(uint64_t v, int src) { return shfl_u64(v, src); }
__device__ __forceinline__ uint32_t wshfl_xor(uint32_t v, int m) { return shfl_xor_u32(v, m); }
__device__ __forceinline__ uint64_t wshfl_xor(uint64_t v, int m) { return shfl_xor_u64(v, m); }
__device__ __forceinline__ uint32_t wreadlane(uint32_t v, int l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t wreadlane(uint64_t v, int l) { return readlane_u64(v, l); }

// flacenc_encode_residuals' partition-order search (flac.c:1362-1402) from
// per-lane |r| sums; level lv partition of lane l is l >> (6 - lv).
// All 127 (level, partition) pairs are evaluated in two lane-parallel
// passes instead of seven:
//   pass A  level 6, partition = lane;
//   pass B  levels 5..0 packed into lanes [64 - 2^(lv+1), 64 - 2^lv):
//           lanes 0-31 level 5, 32-47 level 4, 48-55 level 3, 56-59 level 2,
//           60-61 level 1, 62 level 0 (63 idle).
// Partition sums come from one inclusive prefix scan of the lane sums; the
// level totals from a full butterfly (A) and a segmented one (B) whose
// segments are aligned to their power-of-two sizes.
template <typename S>
__device__ __forceinline__ PartSel select_partitions_t(S lane_sum, uint32_t order,
                                                       const RunCtx &c)
{
    const int lane = c.lane;
    S pre = lane_sum;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const S t = wshfl_up(pre, d);
        pre += lane >= d ? t : (S)0;
    }
    const S total = wreadlane(pre, 63);

    const uint32_t lvB = lane < 32 ? 5u : lane < 48 ? 4u : lane < 56 ? 3u
                       : lane < 60 ? 2u : lane < 62 ? 1u : 0u;
    const uint32_t offB = 64u - (2u << lvB);
    const uint32_t jB = (uint32_t)lane - offB;
    const uint32_t wB = 64u >> lvB; // lanes per partition at level lvB
    const int first = (int)((jB * wB) & 63u), last = (int)((jB * wB + wB - 1u) & 63u);
    const S p_last = wshfl(pre, last);
    const S p_prev = wshfl(pre, (first + 63) & 63);
    const S SB = p_last - (first ? p_prev : (S)0);

    uint32_t kA, kB;
    S eA, eB;
    part_eval<S>(6, (uint32_t)lane, lane_sum, total, order, c, kA, eA);
    part_eval<S>(lvB, jB, SB, total, order, c, kB, eB);
#pragma unroll
    for (int m = 1; m < 64; m <<= 1)
        eA += wshfl_xor(eA, m);
    const uint32_t segB = lane == 63 ? 1u : (1u << lvB);
#pragma unroll
    for (int m = 1; m < 32; m <<= 1) {
        const S o = wshfl_xor(eB, m);
        eB += (uint32_t)m < segB ? o : (S)0;
    }

    S best_tot = (S)~(S)0;
    uint32_t best_p = 0;
#pragma unroll
    for (int lv = 0; lv <= 6; ++lv) {
        const S T = lv == 6 ? wreadlane(eA, 0) : wreadlane(eB, 64 - (2 << lv));
        if (lv <= c.P && T < best_tot) {
            best_tot = T;
            best_p = (uint32_t)lv;
        }
    }
    PartSel r;
    r.porder = best_p;
    uint32_t ko;
    if (best_p == 6u)
        ko = kA;
    else
        ko = (uint32_t)__shfl((int)kB, (int)(64u - (2u << best_p) + ((uint32_t)lane >> (6u - best_p))), 64);
    r.k_own = ko;
    const bool degen_best = (c.N >> best_p) < order;
    const uint32_t k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)ko);
    r.k_lane = degen_best ? k0 : ko;
    r.method = 0;
    if (c.max_rice > 14u)
        r.method = wave_max_u32(ko) > 14u ? 1u : 0u;
    r.hdr_bits = 6u + (1u << best_p) * (r.method ? 5u : 4u);
    return r;
}


// `small`: the subframe's sum |r| is known to be < 2^31 (32-bit search)
__device__ __forceinline__ PartSel select_partitions(uint64_t lane_sum, uint32_t order,
                                                     const RunCtx &c, bool small = false)
{
    if (small)
        return select_partitions_t<uint32_t>((uint32_t)lane_sum, order, c);
    return select_partitions_t<uint64_t>(lane_sum, order, c);
}


// ---- N = 4096, 64 samples per lane, subframe sum |r| < 2^31 (the 16-bit
// searches, flac_search16.hip).  Same Rice parameters, estimates and argmin
// as select_partitions, in fewer vector instructions:
//   * partition sums from four DPP butterfly steps (levels 5..2), the four
//     row sums read into SGPRs (levels 1, 0 and the level-2 partitions are
//     evaluated on the scalar unit);
//   * levels 3..6 evaluated in every lane of each partition with a 32-bit
//     closed form of the reference's Rice loop (plen << k with plen < 2^13
//     and k <= 14 never overflows), the level total being the wave sum over
//     lanes divided by the lanes per partition (every lane of a partition
//     holds the same estimate).
// Estimate (flac.c:1437-1505): 4 + (k ? sum >> (k - 1) : 2 sum) + (k + 1)
// plen - plen / 2 = 4 + ((2 sum) >> k) + (k + 1) plen - plen / 2.
__device__ __forceinline__ uint32_t est32(uint32_t plen, uint32_t bl, uint32_t sum, uint32_t maxk,
                                          uint32_t &k)
{
    // smallest k with plen << k >= sum, capped at maxk (flac.c:1477-1484)
    const uint32_t a = 32u - (uint32_t)__clz((int)(sum - 1u)); // bit length of sum - 1
    int kk = (int)a - (int)bl;
    kk = kk < 0 ? 0 : kk;
    kk += (plen << kk) < sum ? 1 : 0;
    k = sum ? ((uint32_t)kk < maxk ? (uint32_t)kk : maxk) : 0u;
    return 4u + ((sum << 1) >> k) + (k + 1u) * plen - (plen >> 1);
}

// RICE2: the caller's samples may be wider than 16 bits (max_rice 30); the
// 16-bit searches (max_rice 14) leave the method test out
template <bool RICE2 = false>
__device__ __forceinline__ PartSel select_fast32(uint32_t lane_sum, uint32_t order, const RunCtx &c)
{
    const int lane = c.lane;
    const uint32_t maxk = c.max_rice;
    const uint32_t g6 = lane_sum;
    const uint32_t g5 = g6 + dpp_u32<DPP_QUAD_SWAP1>(g6);
    const uint32_t g4 = g5 + dpp_u32<DPP_QUAD_SWAP2>(g5);
    const uint32_t g3 = g4 + dpp_u32<DPP_ROW_HALF_MIRROR>(g4);
    const uint32_t g2 = g3 + dpp_u32<DPP_ROW_MIRROR>(g3);
    const uint32_t r0 = rd_lane(g2, 0), r1 = rd_lane(g2, 16), r2 = rd_lane(g2, 32),
                   r3 = rd_lane(g2, 48);
    const uint32_t h0 = r0 + r1, h1 = r2 + r3, total = h0 + h1;
    const uint32_t o1 = order ? 1u : 0u;

    // levels 0..2 on scalars: Sp = 4096, 2048, 1024 (bit lengths 13, 12, 11;
    // Sp - order with 1 <= order <= 12 one bit shorter)
    uint32_t k0, k1a, k1b, k2[4];
    uint32_t T[7];
    T[0] = est32(4096u - order, 13u - o1, total, maxk, k0);
    T[1] = est32(2048u - order, 12u - o1, h0, maxk, k1a) + est32(2048u, 12u, h1, maxk, k1b);
    T[2] = est32(1024u - order, 11u - o1, r0, maxk, k2[0]) + est32(1024u, 11u, r1, maxk, k2[1]) +
           est32(1024u, 11u, r2, maxk, k2[2]) + est32(1024u, 11u, r3, maxk, k2[3]);
    // levels 3..6 in the lanes: partition 0 = lanes [0, 2^(6 - lv))
    uint32_t k3, k4, k5, k6;
    const uint32_t p3 = lane < 8 ? order : 0u, p4 = lane < 4 ? order : 0u,
                   p5 = lane < 2 ? order : 0u, p6 = lane < 1 ? order : 0u;
    const uint32_t e3 = est32(512u - p3, 10u - (p3 ? 1u : 0u), g3, maxk, k3);
    const uint32_t e4 = est32(256u - p4, 9u - (p4 ? 1u : 0u), g4, maxk, k4);
    const uint32_t e5 = est32(128u - p5, 8u - (p5 ? 1u : 0u), g5, maxk, k5);
    const uint32_t e6 = est32(64u - p6, 7u - (p6 ? 1u : 0u), g6, maxk, k6);
    T[3] = dpp_wave_sum<uint32_t>(e3) >> 3;
    T[4] = dpp_wave_sum<uint32_t>(e4) >> 2;
    T[5] = dpp_wave_sum<uint32_t>(e5) >> 1;
    T[6] = dpp_wave_sum<uint32_t>(e6);

    uint32_t best_tot = 0xFFFFFFFFu, best_p = 0;
#pragma unroll
    for (int lv = 0; lv <= 6; ++lv) {
        if (lv <= c.P && T[lv] < best_tot) {
            best_tot = T[lv];
            best_p = (uint32_t)lv;
        }
    }
    PartSel r;
    r.porder = best_p;
    uint32_t ko;
    switch (best_p) {
    case 0: ko = k0; break;
    case 1: ko = lane < 32 ? k1a : k1b; break;
    case 2: ko = lane < 16 ? k2[0] : lane < 32 ? k2[1] : lane < 48 ? k2[2] : k2[3]; break;
    case 3: ko = k3; break;
    case 4: ko = k4; break;
    case 5: ko = k5; break;
    default: ko = k6; break;
    }
    r.k_own = ko;
    r.k_lane = ko; // N = 4096: no partition is shorter than the order
    // RICE2 (5-bit parameters) once a chosen k passes 14, after the choice,
    // as select_partitions_t
    r.method = 0;
    if (RICE2 && c.max_rice > 14u)
        r.method = wave_max_u32(ko) > 14u ? 1u : 0u;
    r.hdr_bits = 6u + (1u << best_p) * (r.method ? 5u : 4u);
    return r;
}
