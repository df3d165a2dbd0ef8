// pcm_read.h — derive a subframe candidate's sample from interleaved PCM.
// Candidates for stereo with mid/side: 0 = left, 1 = right,
// 2 = average (l + r) >> 1, 3 = difference l - r  (reference
// flacenc_average_difference, src/encoders/flac.c:1507-1529).
// Otherwise candidate c is channel c.
//
// Branch-free in `cand` (lanes of one wave may hold different candidates):
// both stereo samples are loaded (one dword for 16-bit pairs) and the
// candidate is selected with v_cndmask.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

template <typename T>
__device__ __forceinline__ int32_t cand_sample(const T *__restrict__ pcm,
                                               uint64_t pcm_frame, uint32_t ch,
                                               uint32_t cand, bool ms)
{
    if (!ms)
        return (int32_t)pcm[pcm_frame * ch + cand];
    int32_t l, r;
    if (sizeof(T) == 2 && (((uintptr_t)pcm) & 3u) == 0u) {
        const uint32_t v = ((const uint32_t *)pcm)[pcm_frame];
        l = (int32_t)(int16_t)(v & 0xFFFFu);
        r = (int32_t)(int16_t)(v >> 16);
    } else {
        l = (int32_t)pcm[pcm_frame * 2u];
        r = (int32_t)pcm[pcm_frame * 2u + 1u];
    }
    const int32_t avg = (int32_t)((uint32_t)l + (uint32_t)r) >> 1;
    const int32_t dif = (int32_t)((uint32_t)l - (uint32_t)r);
    const int32_t lr = (cand & 1u) ? r : l;
    const int32_t ad = (cand & 1u) ? dif : avg;
    return (cand & 2u) ? ad : lr;
}

// Loader modes chosen once per kernel (uniform), so the per-sample code has
// no branches:  PCM_CH  candidate = channel;  PCM_MS  stereo candidates from
// two loads;  PCM_MS16  stereo candidates from one dword (16-bit pairs,
// 4-byte aligned PCM).
enum { PCM_CH = 0, PCM_MS = 1, PCM_MS16 = 2 };

template <typename T>
__device__ __forceinline__ int pcm_mode(const T *pcm, bool ms)
{
    if (!ms)
        return PCM_CH;
    return (sizeof(T) == 2 && (((uintptr_t)pcm) & 3u) == 0u) ? PCM_MS16 : PCM_MS;
}

// sample j of the candidate, src = first PCM frame of the subframe
template <int MODE, typename T>
__device__ __forceinline__ int32_t cand_at(const T *__restrict__ src, uint32_t j, uint32_t ch,
                                           uint32_t cand)
{
    if (MODE == PCM_CH)
        return (int32_t)src[j * ch + cand];
    int32_t l, r;
    if (MODE == PCM_MS16) {
        const uint32_t v = ((const uint32_t *)src)[j];
        l = (int32_t)(int16_t)(v & 0xFFFFu);
        r = (int32_t)(int16_t)(v >> 16);
    } else {
        l = (int32_t)src[2u * j];
        r = (int32_t)src[2u * j + 1u];
    }
    const int32_t avg = (int32_t)((uint32_t)l + (uint32_t)r) >> 1;
    const int32_t dif = (int32_t)((uint32_t)l - (uint32_t)r);
    const int32_t lr = (cand & 1u) ? r : l;
    const int32_t ad = (cand & 1u) ? dif : avg;
    return (cand & 2u) ? ad : lr;
}
