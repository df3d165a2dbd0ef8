// pcm_convert.hip — the integer PCM converters of the reference's
// pcmconverter module, elementwise over whole tracks:
//
//   BPS      BPSConverter_read (src/pcmconverter.c:667-747): fewer bits =
//            (x >> shift) ^ dither_bit, the bits read MSB first from a byte
//            stream (the reference's os.urandom reader, src/dither.c:73-89),
//            one per sample in the order the reference consumes them: per
//            4096-frame read(), channel by channel; more bits = x << shift.
//   DOWNMIX  Downmixer_read (:220-342): 6-channel layout from the channel
//            mask (missing channels silent), then
//            L = round(fL + 0.6·0.7·(bL+bR) + 0.7·fC), R likewise with −,
//            clamped to the sample range; fp64, no contraction.
//   AVERAGE  Averager_read (:64-97): int64 sum / channels (C truncation).
//
// Input and output are interleaved int32 (the FrameList layout).  The
// kernels are HBM streams (4-24 B in, 4-8 B out per frame): BPS runs 8
// groups of 4 samples per lane with 16-byte vector loads/stores (buffers
// 16-byte aligned), downmix/average a thread per frame.  The caller supplies the dither bytes, so a conversion is
// reproducible and testable; the reference draws them from os.urandom.
#include <hip/hip_runtime.h>

#include <cmath>
#include <string>

#include "../../include/atgpu.h"

#pragma clang fp contract(off)

namespace {

thread_local std::string g_conv_err;

atg_status cfail(atg_status s, const std::string &m)
{
    g_conv_err = m;
    return s;
}

#define CHIP(expr)                                                                         \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return cfail(ATG_ERR_DEVICE, std::string(#expr ": ") + hipGetErrorString(e_)); \
    } while (0)

__device__ __forceinline__ int32_t bps_one(int32_t x, uint64_t f, uint32_t c, uint64_t frames,
                                           uint32_t ch, uint32_t in_bps, uint32_t out_bps,
                                           const uint8_t *__restrict__ dither, uint64_t bit0)
{
    if (out_bps < in_bps) {
        const uint64_t chunk = f / 4096u * 4096u;
        const uint64_t clen = frames - chunk < 4096u ? frames - chunk : 4096u;
        const uint64_t b = bit0 + chunk * ch + (uint64_t)c * clen + (f - chunk);
        const int32_t bit = (dither[b >> 3] >> (7 - (uint32_t)(b & 7))) & 1;
        return (x >> (in_bps - out_bps)) ^ bit;
    }
    return (int32_t)((uint32_t)x << (out_bps - in_bps));
}

// kBpsGroups groups of 4 consecutive samples per lane, groups 1024 samples
// apart (each 16-byte load/store coalesced across the block), all loads
// issued before the first group is converted, stores non-temporal (the
// output is not read again here): 0.93 -> 0.83 ms for 537 M samples, 4.65
// -> 5.27 TB/s against one group per lane and cached stores
// (profiles/r05_zz_convert.txt); the frame/channel of a group's first
// sample costs one division
constexpr int kBpsGroups = 8;

__global__ __launch_bounds__(256) void k_pcm_bps(const int32_t *__restrict__ in,
                                                 int32_t *__restrict__ out, uint64_t frames,
                                                 uint32_t ch, uint32_t in_bps, uint32_t out_bps,
                                                 const uint8_t *__restrict__ dither,
                                                 uint64_t bit0)
{
    typedef int v4i __attribute__((ext_vector_type(4)));
    const uint64_t n = frames * ch;
    const uint64_t base = (uint64_t)blockIdx.x * 1024u * kBpsGroups + threadIdx.x * 4u;
    int4 v[kBpsGroups];
#pragma unroll
    for (int u = 0; u < kBpsGroups; ++u) {
        const uint64_t q0 = base + (uint64_t)u * 1024u;
        v[u] = q0 + 4 <= n ? *(const int4 *)(in + q0) : make_int4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < kBpsGroups; ++u) {
        const uint64_t q0 = base + (uint64_t)u * 1024u;
        if (q0 >= n)
            break;
        uint64_t f = q0 / ch;
        uint32_t c = (uint32_t)(q0 - f * ch);
        if (q0 + 4 <= n) {
            int32_t *e = (int32_t *)&v[u];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                e[k] = bps_one(e[k], f, c, frames, ch, in_bps, out_bps, dither, bit0);
                if (++c == ch) {
                    c = 0;
                    ++f;
                }
            }
            __builtin_nontemporal_store(*(const v4i *)&v[u], (v4i *)(out + q0));
        } else {
            for (uint64_t q = q0; q < n; ++q) {
                out[q] = bps_one(in[q], f, c, frames, ch, in_bps, out_bps, dither, bit0);
                if (++c == ch) {
                    c = 0;
                    ++f;
                }
            }
        }
    }
}

// ReplayGainReader_read (src/replaygain.c:886-925): lround(x * multiplier),
// clamp, XOR one dither bit; bits consumed per read(pcm_frames) chunk,
// channel by channel (chunk = the caller's pcm_frames)
__global__ __launch_bounds__(256) void k_pcm_gain(const int32_t *__restrict__ in,
                                                  int32_t *__restrict__ out, uint64_t frames,
                                                  uint32_t ch, uint32_t bps, double mult,
                                                  uint32_t chunk_frames,
                                                  const uint8_t *__restrict__ dither,
                                                  uint64_t bit0)
{
    const uint64_t q0 = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
    const uint64_t n = frames * ch;
    if (q0 >= n)
        return;
    const int32_t maxv = (1 << (bps - 1)) - 1, minv = -(1 << (bps - 1));
    uint64_t f = q0 / ch;
    uint32_t c = (uint32_t)(q0 - f * ch);
    const uint64_t qe = q0 + 4 < n ? q0 + 4 : n;
    for (uint64_t q = q0; q < qe; ++q) {
        const uint64_t chunk = f / chunk_frames * chunk_frames;
        const uint64_t clen = frames - chunk < chunk_frames ? frames - chunk : chunk_frames;
        const uint64_t b = bit0 + chunk * ch + (uint64_t)c * clen + (f - chunk);
        const int32_t bit = (dither[b >> 3] >> (7 - (uint32_t)(b & 7))) & 1;
        int32_t v = (int32_t)lround((double)in[q] * mult);
        v = v < minv ? minv : (v > maxv ? maxv : v);
        out[q] = v ^ bit;
        if (++c == ch) {
            c = 0;
            ++f;
        }
    }
}

__global__ __launch_bounds__(256) void k_pcm_downmix(const int32_t *__restrict__ in,
                                                     int32_t *__restrict__ out, uint64_t frames,
                                                     uint32_t ch, uint32_t mask, uint32_t bps)
{
    const uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= frames)
        return;
    int32_t six[6];
    uint32_t k = 0;
    for (uint32_t m = 0; m < 6; ++m) {
        if (mask & (1u << m))
            six[m] = in[f * ch + k++];
        else
            six[m] = 0;
    }
    const double REAR_GAIN = 0.6, CENTER_GAIN = 0.7;
    const int32_t smin = -(1 << (bps - 1)), smax = (1 << (bps - 1)) - 1;
    const double mono_rear = 0.7 * (double)(six[4] + six[5]);
    const int32_t l = (int32_t)round((double)six[0] + REAR_GAIN * mono_rear +
                                     CENTER_GAIN * (double)six[2]);
    const int32_t r = (int32_t)round((double)six[1] - REAR_GAIN * mono_rear +
                                     CENTER_GAIN * (double)six[2]);
    out[2 * f] = l > smax ? smax : (l < smin ? smin : l);
    out[2 * f + 1] = r > smax ? smax : (r < smin ? smin : r);
}

__global__ __launch_bounds__(256) void k_pcm_average(const int32_t *__restrict__ in,
                                                     int32_t *__restrict__ out, uint64_t frames,
                                                     uint32_t ch)
{
    const uint64_t f = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (f >= frames)
        return;
    int64_t acc = 0;
    for (uint32_t c = 0; c < ch; ++c)
        acc += in[f * ch + c];
    out[f] = (int32_t)(acc / (int64_t)ch);
}

uint32_t default_mask(uint32_t ch)
{
    // Downmixer_read's invented masks (pcmconverter.c:256-290)
    static const uint32_t m[7] = {0x0, 0x4, 0x3, 0x7, 0x33, 0x37, 0x3F};
    return ch <= 6 ? m[ch] : 0x3F;
}

} // namespace

extern "C" {

const char *atg_pcm_convert_last_error(void) { return g_conv_err.c_str(); }

uint32_t atg_pcm_convert_out_channels(int kind, uint32_t in_channels)
{
    return kind == ATG_CONV_DOWNMIX ? 2u : kind == ATG_CONV_AVERAGE ? 1u : in_channels;
}

atg_status atg_pcm_convert_device(int kind, const int32_t *d_in, int32_t *d_out,
                                  uint64_t frames, uint32_t channels, uint32_t channel_mask,
                                  uint32_t in_bps, uint32_t out_bps, const uint8_t *d_dither,
                                  uint64_t dither_bit0, void *stream)
{
    if ((!d_in || !d_out) && frames)
        return cfail(ATG_ERR_INVALID, "NULL buffer");
    if (channels < 1 || in_bps < 1 || in_bps > 32)
        return cfail(ATG_ERR_INVALID, "bad channels / bits per sample");
    hipStream_t s = (hipStream_t)stream;
    const dim3 grid((unsigned)((frames + 255) / 256)), blk(256);
    if (!frames)
        return ATG_OK;
    switch (kind) {
    case ATG_CONV_BPS:
        if (out_bps < 1 || out_bps > 32)
            return cfail(ATG_ERR_INVALID, "bad output bits per sample");
        if (out_bps < in_bps && !d_dither)
            return cfail(ATG_ERR_INVALID, "dither bytes required to reduce bits per sample");
        if (((uintptr_t)d_in | (uintptr_t)d_out) & 15)
            return cfail(ATG_ERR_INVALID, "PCM buffers must be 16-byte aligned");
        hipLaunchKernelGGL(k_pcm_bps,
                           dim3((unsigned)((frames * channels + 1024 * kBpsGroups - 1) /
                                           (1024 * kBpsGroups))),
                           blk, 0, s, d_in, d_out, frames, channels, in_bps, out_bps, d_dither,
                           dither_bit0);
        break;
    case ATG_CONV_DOWNMIX: {
        uint32_t mask = channel_mask ? channel_mask : default_mask(channels);
        // the reference links input channels to mask bits 0x1..0x20 in order
        uint32_t bits = 0;
        for (uint32_t m = mask & 0x3F; m; m >>= 1)
            bits += m & 1u;
        if (bits > channels)
            return cfail(ATG_ERR_INVALID, "channel mask names more channels than present");
        hipLaunchKernelGGL(k_pcm_downmix, grid, blk, 0, s, d_in, d_out, frames, channels,
                           mask & 0x3Fu, in_bps);
        break;
    }
    case ATG_CONV_AVERAGE:
        hipLaunchKernelGGL(k_pcm_average, grid, blk, 0, s, d_in, d_out, frames, channels);
        break;
    default:
        return cfail(ATG_ERR_INVALID, "unknown conversion");
    }
    CHIP(hipGetLastError());
    return ATG_OK;
}

atg_status atg_pcm_convert_host(int device, int kind, const int32_t *in, int32_t *out,
                                uint64_t frames, uint32_t channels, uint32_t channel_mask,
                                uint32_t in_bps, uint32_t out_bps, const uint8_t *dither,
                                uint64_t dither_bytes, uint64_t dither_bit0)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return cfail(ATG_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= n)
        return cfail(ATG_ERR_INVALID, "device index out of range");
    CHIP(hipSetDevice(device));
    const uint32_t oc = atg_pcm_convert_out_channels(kind, channels);
    const uint64_t need_bits = frames * channels;
    if (kind == ATG_CONV_BPS && out_bps < in_bps && dither_bytes * 8 < need_bits + dither_bit0)
        return cfail(ATG_ERR_INVALID, "not enough dither bytes");
    void *di = nullptr, *dout = nullptr, *dd = nullptr;
    const size_t ib = sizeof(int32_t) * (frames * channels ? frames * channels : 1);
    const size_t ob = sizeof(int32_t) * (frames * oc ? frames * oc : 1);
    if (hipMalloc(&di, ib) != hipSuccess || hipMalloc(&dout, ob) != hipSuccess ||
        hipMalloc(&dd, dither_bytes ? dither_bytes : 1) != hipSuccess) {
        (void)hipFree(di);
        (void)hipFree(dout);
        (void)hipFree(dd);
        return cfail(ATG_ERR_NOMEM, "device allocation failed");
    }
    atg_status st = ATG_OK;
    if (hipMemcpy(di, in, sizeof(int32_t) * frames * channels, hipMemcpyHostToDevice) !=
            hipSuccess ||
        (dither_bytes && hipMemcpy(dd, dither, dither_bytes, hipMemcpyHostToDevice) != hipSuccess))
        st = cfail(ATG_ERR_DEVICE, "copy to device failed");
    if (st == ATG_OK)
        st = atg_pcm_convert_device(kind, (const int32_t *)di, (int32_t *)dout, frames, channels,
                                    channel_mask, in_bps, out_bps,
                                    dither_bytes ? (const uint8_t *)dd : nullptr, dither_bit0,
                                    nullptr);
    if (st == ATG_OK &&
        (hipDeviceSynchronize() != hipSuccess ||
         hipMemcpy(out, dout, sizeof(int32_t) * frames * oc, hipMemcpyDeviceToHost) != hipSuccess))
        st = cfail(ATG_ERR_DEVICE, "conversion failed on the device");
    (void)hipFree(di);
    (void)hipFree(dout);
    (void)hipFree(dd);
    return st;
}

double atg_replaygain_multiplier(double replaygain, double peak)
{
    // ReplayGainReader_init (replaygain.c:838-842): long double pow, stored
    // in a double; gains above unity are replaced by 1 / peak
    double m = (double)powl(10.0L, (long double)replaygain / 20.0L);
    if (m > 1.0)
        m = (double)(1.0L / (long double)peak);
    return m;
}

atg_status atg_pcm_apply_gain_device(const int32_t *d_in, int32_t *d_out, uint64_t frames,
                                     uint32_t channels, uint32_t bps, double multiplier,
                                     uint32_t chunk_frames, const uint8_t *d_dither,
                                     uint64_t dither_bit0, void *stream)
{
    if (((!d_in || !d_out) && frames) || !d_dither)
        return cfail(ATG_ERR_INVALID, "NULL buffer");
    if (channels < 1 || bps < 1 || bps > 32 || chunk_frames < 1)
        return cfail(ATG_ERR_INVALID, "bad channels / bits per sample / chunk");
    if (!frames)
        return ATG_OK;
    hipLaunchKernelGGL(k_pcm_gain, dim3((unsigned)((frames * channels + 1023) / 1024)),
                       dim3(256), 0, (hipStream_t)stream, d_in, d_out, frames, channels, bps,
                       multiplier, chunk_frames, d_dither, dither_bit0);
    CHIP(hipGetLastError());
    return ATG_OK;
}

atg_status atg_pcm_apply_gain_host(int device, const int32_t *in, int32_t *out, uint64_t frames,
                                   uint32_t channels, uint32_t bps, double multiplier,
                                   uint32_t chunk_frames, const uint8_t *dither,
                                   uint64_t dither_bytes, uint64_t dither_bit0)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0)
        return cfail(ATG_ERR_DEVICE, "no HIP device available");
    if (device < 0 || device >= n)
        return cfail(ATG_ERR_INVALID, "device index out of range");
    CHIP(hipSetDevice(device));
    if (dither_bytes * 8 < frames * channels + dither_bit0)
        return cfail(ATG_ERR_INVALID, "not enough dither bytes");
    void *di = nullptr, *dout = nullptr, *dd = nullptr;
    const size_t nb = sizeof(int32_t) * (frames * channels ? frames * channels : 1);
    if (hipMalloc(&di, nb) != hipSuccess || hipMalloc(&dout, nb) != hipSuccess ||
        hipMalloc(&dd, dither_bytes ? dither_bytes : 1) != hipSuccess) {
        (void)hipFree(di);
        (void)hipFree(dout);
        (void)hipFree(dd);
        return cfail(ATG_ERR_NOMEM, "device allocation failed");
    }
    atg_status st = ATG_OK;
    if (hipMemcpy(di, in, sizeof(int32_t) * frames * channels, hipMemcpyHostToDevice) !=
            hipSuccess ||
        (dither_bytes && hipMemcpy(dd, dither, dither_bytes, hipMemcpyHostToDevice) != hipSuccess))
        st = cfail(ATG_ERR_DEVICE, "copy to device failed");
    if (st == ATG_OK)
        st = atg_pcm_apply_gain_device((const int32_t *)di, (int32_t *)dout, frames, channels,
                                       bps, multiplier, chunk_frames, (const uint8_t *)dd,
                                       dither_bit0, nullptr);
    if (st == ATG_OK &&
        (hipDeviceSynchronize() != hipSuccess ||
         hipMemcpy(out, dout, sizeof(int32_t) * frames * channels, hipMemcpyDeviceToHost) !=
             hipSuccess))
        st = cfail(ATG_ERR_DEVICE, "gain application failed on the device");
    (void)hipFree(di);
    (void)hipFree(dout);
    (void)hipFree(dd);
    return st;
}

} // extern "C"
