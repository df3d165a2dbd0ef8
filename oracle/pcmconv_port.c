/*
 * pcmconv_port.c — CPU restatement of the integer PCM converters of the
 * reference's pcmconverter module (src/pcmconverter.c), over whole tracks.
 *
 * TEST INFRASTRUCTURE ONLY (see flac_port.h): the checker for
 * python-audio-tools_amd/csrc/pcm_convert.hip; never linked by the product.
 *
 * Parity unpinned: the reference has no tests or fixtures that pin these
 * converters, and their bodies live inside Python-2
 * type methods, so they cannot be built here.  Each function restates the
 * cited reference lines; the dither bits, which the reference draws from
 * os.urandom (src/dither.c:73-89), are an input here.
 */
#include <math.h>
#include <stdint.h>

/* BPSConverter_read (pcmconverter.c:667-747): the reference reads 4096
   frames per call and walks them channel by channel, taking one dither bit
   per sample from a big-endian bit reader (src/dither.c). */
void pcmconvport_bps(const int32_t *in, int32_t *out, uint64_t frames, uint32_t ch,
                     uint32_t in_bps, uint32_t out_bps, const uint8_t *dither)
{
    uint64_t bit = 0;
    for (uint64_t f0 = 0; f0 < frames; f0 += 4096) {
        const uint64_t n = frames - f0 < 4096 ? frames - f0 : 4096;
        for (uint32_t c = 0; c < ch; c++) {
            for (uint64_t i = 0; i < n; i++) {
                const int32_t x = in[(f0 + i) * ch + c];
                int32_t y;
                if (out_bps < in_bps) {
                    const int b = (dither[bit >> 3] >> (7 - (bit & 7))) & 1;
                    bit++;
                    y = (x >> (in_bps - out_bps)) ^ b;
                } else if (out_bps > in_bps) {
                    y = (int32_t)((uint32_t)x << (out_bps - in_bps));
                } else {
                    y = x;
                }
                out[(f0 + i) * ch + c] = y;
            }
        }
    }
}

/* Downmixer_read (pcmconverter.c:220-342) */
void pcmconvport_downmix(const int32_t *in, int32_t *out, uint64_t frames, uint32_t ch,
                         uint32_t mask, uint32_t bps)
{
    static const uint32_t inv[7] = {0x0, 0x4, 0x3, 0x7, 0x33, 0x37, 0x3F};
    const uint32_t m = mask ? mask : (ch <= 6 ? inv[ch] : 0x3F);
    const double REAR_GAIN = 0.6, CENTER_GAIN = 0.7;
    const int SAMPLE_MIN = -(1 << (bps - 1)), SAMPLE_MAX = (1 << (bps - 1)) - 1;
    for (uint64_t f = 0; f < frames; f++) {
        int six[6];
        uint32_t k = 0;
        for (uint32_t b = 0; b < 6; b++)
            six[b] = (m & (1u << b)) ? in[f * ch + k++] : 0;
        const double mono_rear = 0.7 * (six[4] + six[5]);
        const int left_i = (int)round(six[0] + REAR_GAIN * mono_rear + CENTER_GAIN * six[2]);
        const int right_i = (int)round(six[1] - REAR_GAIN * mono_rear + CENTER_GAIN * six[2]);
        out[2 * f] = left_i > SAMPLE_MAX ? SAMPLE_MAX : (left_i < SAMPLE_MIN ? SAMPLE_MIN : left_i);
        out[2 * f + 1] =
            right_i > SAMPLE_MAX ? SAMPLE_MAX : (right_i < SAMPLE_MIN ? SAMPLE_MIN : right_i);
    }
}

/* Averager_read (pcmconverter.c:64-97) */
void pcmconvport_average(const int32_t *in, int32_t *out, uint64_t frames, uint32_t ch)
{
    for (uint64_t f = 0; f < frames; f++) {
        int64_t acc = 0;
        for (uint32_t c = 0; c < ch; c++)
            acc += in[f * ch + c];
        out[f] = (int)(acc / ch);
    }
}

/* ReplayGainReader_init / _read (src/replaygain.c:820-925) over a track read
   in chunks of chunk_frames (the caller's read(pcm_frames) size) */
double pcmconvport_rg_multiplier(double replaygain, double peak)
{
    double m = (double)powl(10.0L, (long double)replaygain / 20.0L);
    if (m > 1.0)
        m = (double)(1.0L / (long double)peak);
    return m;
}

void pcmconvport_apply_gain(const int32_t *in, int32_t *out, uint64_t frames, uint32_t ch,
                            uint32_t bps, double multiplier, uint32_t chunk_frames,
                            const uint8_t *dither)
{
    const int max_value = (1 << (bps - 1)) - 1, min_value = -(1 << (bps - 1));
    uint64_t bit = 0;
    for (uint64_t f0 = 0; f0 < frames; f0 += chunk_frames) {
        const uint64_t n = frames - f0 < chunk_frames ? frames - f0 : chunk_frames;
        for (uint32_t c = 0; c < ch; c++)
            for (uint64_t i = 0; i < n; i++) {
                int v = (int)lround(in[(f0 + i) * ch + c] * multiplier);
                v = v < min_value ? min_value : (v > max_value ? max_value : v);
                const int b = (dither[bit >> 3] >> (7 - (bit & 7))) & 1;
                bit++;
                out[(f0 + i) * ch + c] = v ^ b;
            }
    }
}
