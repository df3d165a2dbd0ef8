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

// ---- DPP (data-parallel primitive) forms: VALU lane exchanges with no LDS
// round trip.  EVERY LANE OF THE WAVE MUST BE ACTIVE.  Butterfly steps
// within 16-lane rows (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror) leave each 2/4/8/16-lane group's total in all of its lanes;
// the four row totals are then read into SGPRs.
enum : int {
    DPP_QUAD_SWAP1 = 0xB1, // quad_perm [1,0,3,2]
    DPP_QUAD_SWAP2 = 0x4E, // quad_perm [2,3,0,1]
    DPP_ROW_MIRROR = 0x140,
    DPP_ROW_HALF_MIRROR = 0x141
};

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v)
{
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, true);
}

template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v)
{
    const uint32_t lo = dpp_u32<CTRL>((uint32_t)v), hi = dpp_u32<CTRL>((uint32_t)(v >> 32));
    return ((uint64_t)hi << 32) | lo;
}

// v summed over its aligned group of 2^steps lanes (steps <= 4), in every
// lane of the group
template <int STEPS, typename T>
__device__ __forceinline__ T dpp_group_sum(T v)
{
    if constexpr (STEPS >= 1) {
        if constexpr (sizeof(T) == 8) v += dpp_u64<DPP_QUAD_SWAP1>(v); else v += dpp_u32<DPP_QUAD_SWAP1>(v);
    }
    if constexpr (STEPS >= 2) {
        if constexpr (sizeof(T) == 8) v += dpp_u64<DPP_QUAD_SWAP2>(v); else v += dpp_u32<DPP_QUAD_SWAP2>(v);
    }
    if constexpr (STEPS >= 3) {
        if constexpr (sizeof(T) == 8) v += dpp_u64<DPP_ROW_HALF_MIRROR>(v); else v += dpp_u32<DPP_ROW_HALF_MIRROR>(v);
    }
    if constexpr (STEPS >= 4) {
        if constexpr (sizeof(T) == 8) v += dpp_u64<DPP_ROW_MIRROR>(v); else v += dpp_u32<DPP_ROW_MIRROR>(v);
    }
    return v;
}

__device__ __forceinline__ uint32_t rd_lane(uint32_t v, int l)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ uint64_t rd_lane(uint64_t v, int l) { return readlane_u64(v, l); }

// wave total (uniform), all lanes active
template <typename T>
__device__ __forceinline__ T dpp_wave_sum(T v)
{
    v = dpp_group_sum<4>(v);
    return (rd_lane(v, 0) + rd_lane(v, 16)) + (rd_lane(v, 32) + rd_lane(v, 48));
}

__device__ __forceinline__ uint32_t dpp_wave_max_u32(uint32_t v)
{
    v = max(v, dpp_u32<DPP_QUAD_SWAP1>(v));
    v = max(v, dpp_u32<DPP_QUAD_SWAP2>(v));
    v = max(v, dpp_u32<DPP_ROW_HALF_MIRROR>(v));
    v = max(v, dpp_u32<DPP_ROW_MIRROR>(v));
    return max(max(rd_lane(v, 0), rd_lane(v, 16)), max(rd_lane(v, 32), rd_lane(v, 48)));
}

__device__ __forceinline__ uint32_t dpp_wave_or_u32(uint32_t v)
{
    v |= dpp_u32<DPP_QUAD_SWAP1>(v);
    v |= dpp_u32<DPP_QUAD_SWAP2>(v);
    v |= dpp_u32<DPP_ROW_HALF_MIRROR>(v);
    v |= dpp_u32<DPP_ROW_MIRROR>(v);
    return (rd_lane(v, 0) | rd_lane(v, 16)) | (rd_lane(v, 32) | rd_lane(v, 48));
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
