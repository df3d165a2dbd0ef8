// pcm_read.h — derive a subframe candidate's sample from interleaved PCM.
// Candidates for stereo with mid/side: 0 = left, 1 = right,
// 2 = average (l + r) >> 1, 3 = difference l - r  (reference
// flacenc_average_difference, src/encoders/flac.c:1507-1529).
// Otherwise candidate c is channel c.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

template <typename T>
__device__ __forceinline__ int32_t cand_sample(const T *__restrict__ pcm,
                                               uint64_t pcm_frame, uint32_t ch,
                                               uint32_t cand, bool ms)
{
    const T *p = pcm + pcm_frame * ch;
    if (!ms)
        return (int32_t)p[cand];
    const int32_t l = (int32_t)p[0];
    const int32_t r = (int32_t)p[1];
    switch (cand) {
    case 0:
        return l;
    case 1:
        return r;
    case 2:
        return (int32_t)((uint32_t)l + (uint32_t)r) >> 1;
    default:
        return (int32_t)((uint32_t)l - (uint32_t)r);
    }
}
