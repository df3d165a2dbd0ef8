// alac_common.h — device helpers shared by the ALAC encoder and decoder
// kernels (alac_encode.hip, alac_decode.hip): the reference's integer
// primitives (src/encoders/alac.c:907-1017, src/decoders/alac.c:1006-1145).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define ALAC_MAX_ORDER 8 // MAX_LPC_ORDER (alac.c:25)
#define ALAC_SHIFT 2     // INTERLACING_SHIFT (alac.c:26)

// TRUNCATE_BITS (alac.c:918-930)
__device__ __forceinline__ int32_t alac_trunc(int32_t v, uint32_t bits)
{
    const uint32_t m = bits >= 32 ? 0xFFFFFFFFu : (1u << bits) - 1u;
    const uint32_t t = (uint32_t)v & m;
    const uint32_t sb = bits >= 1 && bits <= 32 ? 1u << (bits - 1) : 0u;
    return (t & sb) ? (int32_t)(t - (m + 1u)) : (int32_t)t;
}

// SIGN_ONLY (alac.c:907-916)
__device__ __forceinline__ int32_t alac_sgn(int32_t v) { return (v > 0) - (v < 0); }

// floor(log2(v)) for v > 0 (the encoder's LOG2, alac.c:1007-1017)
__device__ __forceinline__ uint32_t alac_log2(uint32_t v) { return 31u - (uint32_t)__clz(v); }

// bits write_residual (alac.c:1081-1100) emits for `value` with parameter k
__device__ __forceinline__ uint32_t alac_code_bits(uint32_t value, uint32_t k, uint32_t ss)
{
    const uint32_t m = (1u << k) - 1u;
    if (value >= 9u * m) // MSB = value / m > 8: escape
        return 9u + ss;
    uint32_t msb = 0;
#pragma unroll
    for (uint32_t t = 1; t <= 8; ++t)
        msb += value >= t * m ? 1u : 0u;
    const uint32_t lsb = value - msb * m;
    return msb + 1u + (k > 1u ? (lsb > 0u ? k : k - 1u) : 0u);
}
