// wave.h — wave64 helpers for gfx950 (64-lane wavefronts, no warp idioms).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ uint32_t shfl_xor_u32(uint32_t v, int m)
{
    return (uint32_t)__shfl_xor((int)v, m, 64);
}

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m)
{
    uint32_t lo = shfl_xor_u32((uint32_t)v, m);
    uint32_t hi = shfl_xor_u32((uint32_t)(v >> 32), m);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_u64(uint64_t v, int src)
{
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint64_t shfl_up_u64(uint64_t v, int d)
{
    const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, d, 64);
    const uint32_t hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), d, 64);
    return ((uint64_t)hi << 32) | lo;
}

// value of lane l (wave-uniform result, lands in SGPRs)
__device__ __forceinline__ uint64_t readlane_u64(uint64_t v, int l)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, l);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v >> 32), l);
    return ((uint64_t)hi << 32) | lo;
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v)
{
#pragma unroll
    for (int m = 1; m < 64; m <<= 1)
        v += shfl_xor_u32(v, m);
    return v;
}

__device__ __forceinline__ uint64_t wave_sum_u64(uint64_t v)
{
#pragma unroll
    for (int m = 1; m < 64; m <<= 1)
        v += shfl_xor_u64(v, m);
    return v;
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) {
        uint32_t o = shfl_xor_u32(v, m);
        v = o > v ? o : v;
    }
    return v;
}

__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v)
{
#pragma unroll
    for (int m = 1; m < 64; m <<= 1)
        v |= shfl_xor_u32(v, m);
    return v;
}

__device__ __forceinline__ bool wave_all(bool b)
{
    return __ballot(!b) == 0;
}

// exclusive prefix sum over the wave
__device__ __forceinline__ uint32_t wave_excl_scan_u32(uint32_t v, int lane)
{
    uint32_t x = v;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        uint32_t y = (uint32_t)__shfl_up((int)x, d, 64);
        if (lane >= d)
            x += y;
    }
    return x - v;
}

__device__ __forceinline__ int uniform_i32(int v)
{
    return __builtin_amdgcn_readfirstlane(v);
}

__device__ __forceinline__ uint32_t uniform_u32(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}

// v_mad_i32_i24: 24-bit signed multiply, 32-bit add (one full-rate VALU op)
__device__ __forceinline__ int mad24(int a, int b_uniform, int c)
{
    int d;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "s"(b_uniform), "v"(c));
    return d;
}

// XCD-aware block remap: blocks b and b+8 land on the same XCD under the
// observed round-robin dispatch (MI355X_MICROARCH.md, speed only).  Keep the
// `group` consecutive logical blocks of one unit (e.g. the subframe
// candidates of one frame) on one XCD so they share its L2.
__device__ __forceinline__ void xcd_unit_map(uint32_t b, uint32_t group,
                                             uint32_t *unit, uint32_t *member)
{
    const uint32_t xcd = b & 7u;
    const uint32_t slot = b >> 3;
    *member = slot % group;
    *unit = (slot / group) * 8u + xcd;
}
