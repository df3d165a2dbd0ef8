// rice.h — the reference's Rice-parameter choice and partition size
// estimate (src/encoders/flac.c:1437-1505), shared by the 4096-sample search
// (flac_search.hip) and the large-frame path (flac_big.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Rice parameter of one partition: the reference's loop
//   while ((uint64_t)(plength << Rice) < sum) if (Rice < max) Rice++; else break;
// including its 32-bit shift (flac.c:1477-1484).
__device__ __forceinline__ uint32_t rice_param(uint32_t plen, uint64_t sum, uint32_t maxk)
{
    const uint32_t bl = 32u - (uint32_t)__clz((int)plen);
    if (bl + maxk <= 32u) {
        if (sum == 0)
            return 0;
        if (plen == 0)
            return maxk;
        const int a = 64 - __clzll((long long)(sum - 1));
        int k = a - (int)bl;
        k = k < 0 ? 0 : k;
        if (((uint64_t)plen << k) < sum)
            k++;
        return (uint32_t)k < maxk ? (uint32_t)k : maxk;
    }
    uint32_t k = 0;
    while ((uint64_t)(uint32_t)(plen << k) < sum) {
        if (k < maxk)
            k++;
        else
            break;
    }
    return k;
}

// Estimated bits of one partition (flac.c:1437-1505).  S = uint64_t is the
// reference's accumulator; S = uint32_t gives the same values whenever the
// subframe's sum |r| < 2^31 (then no term or total reaches 2^32).
template <typename S>
__device__ __forceinline__ S part_estimate(uint32_t plen, S sum, uint32_t k)
{
    if (k > 0)
        return (S)4u + (sum >> (k - 1)) + (S)(uint32_t)((1u + k) * plen) - (S)(plen / 2u);
    return (S)4u + (sum << 1) + (S)plen - (S)(plen / 2u);
}

