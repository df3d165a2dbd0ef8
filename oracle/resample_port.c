/*
 * resample_port.c — CPU restatement of python-audio-tools' Resampler
 * (src/pcmconverter.c:370-495 with its float buffers :533-629) over the
 * vendored libsamplerate 0.1.8 sinc converter (src/samplerate/samplerate.c
 * src_process :122-183; src/samplerate/src_sinc.c: sinc_set_converter
 * :154-251, sinc_reset :253-270, calc_output_* :277-326, 423-475,
 * 908-1036, sinc_*_vari_process :329-420, 478-568, 1039-1128,
 * prepare_data :1135-1205).
 *
 * TEST INFRASTRUCTURE ONLY (see flac_port.h): the checker for
 * python-audio-tools_amd/csrc/resample.hip; never linked by the product.
 *
 * This restatement keeps the reference's own mechanics — the circular
 * float buffer with its memmoves and end padding, src_process per read()
 * with the output buffer that doubles when input is left over, and the
 * termination test on the buffer-relative index — so it checks both the
 * samples and the read() frame counts of the GPU path, which computes
 * every output from its absolute input position instead.
 *
 * PARITY UNPINNED.  The reference selects SRC_SINC_BEST_QUALITY
 * (pcmconverter.c:395), whose table high_qual_coeffs.h is absent from the
 * reference tree, so the reference resampler cannot be built here (and no
 * stand-in header may be written).  This restatement and the GPU kernel use
 * the MEDIUM table the tree does hold (tools/gen_src_coeffs.py ->
 * csrc/src_coeffs.h); no reference output pins them.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../python-audio-tools_amd/csrc/src_coeffs.h"

#define SHIFT_BITS 12
#define FP_ONE ((double)(1 << SHIFT_BITS))
#define INV_FP_ONE (1.0 / FP_ONE)
#define MAX_RATIO 256
#define BLOCK 4096 /* RESAMPLER_BLOCK_SIZE */

static double fmod_one(double x)
{
    double r = x - (double)lrint(x);
    return r < 0.0 ? r + 1.0 : r;
}

typedef struct {
    int ch;
    long b_len, b_current, b_end, b_real_end;
    float *buffer;
    const float *coeffs;
    int half_len, index_inc;
    double last_position, last_ratio;
    long in_count, in_used, out_count, out_gen;
} sinc_state;

static int sinc_open(sinc_state *f, int ch)
{
    memset(f, 0, sizeof *f);
    f->ch = ch;
    f->coeffs = (const float *)(const void *)SRC_MEDIUM_BITS;
    f->half_len = SRC_MEDIUM_HALF_LEN;
    f->index_inc = SRC_MEDIUM_INCREMENT;
    f->b_len = lrint(2.5 * f->half_len / (f->index_inc * 1.0) * MAX_RATIO);
    if (f->b_len < 4096)
        f->b_len = 4096;
    f->b_len *= ch;
    f->buffer = calloc((size_t)(f->b_len + ch), sizeof(float));
    f->b_real_end = -1;
    return f->buffer != NULL;
}

static void prepare(sinc_state *f, const float *data_in, int eoi, long half)
{
    long len = 0;
    if (f->b_real_end >= 0)
        return;
    if (f->b_current == 0) {
        len = f->b_len - 2 * half;
        f->b_current = f->b_end = half;
    } else if (f->b_end + half + f->ch < f->b_len) {
        len = f->b_len - f->b_current - half;
        if (len < 0)
            len = 0;
    } else {
        len = f->b_end - f->b_current;
        memmove(f->buffer, f->buffer + f->b_current - half, (size_t)(half + len) * sizeof(float));
        f->b_current = half;
        f->b_end = f->b_current + len;
        len = f->b_len - f->b_current - half;
        if (len < 0)
            len = 0;
    }
    if (f->in_count - f->in_used < len)
        len = f->in_count - f->in_used;
    len -= len % f->ch;
    memcpy(f->buffer + f->b_end, data_in + f->in_used, (size_t)len * sizeof(float));
    f->b_end += len;
    f->in_used += len;
    if (f->in_used == f->in_count && f->b_end - f->b_current < 2 * half && eoi) {
        if (f->b_len - f->b_end < half + 5) {
            len = f->b_end - f->b_current;
            memmove(f->buffer, f->buffer + f->b_current - half,
                    (size_t)(half + len) * sizeof(float));
            f->b_current = half;
            f->b_end = f->b_current + len;
        }
        f->b_real_end = f->b_end;
        len = half + 5;
        if (f->b_end + len > f->b_len)
            len = f->b_len - f->b_end;
        memset(f->buffer + f->b_end, 0, (size_t)len * sizeof(float));
        f->b_end += len;
    }
}

/* one output frame: left half from the farthest tap in, right half from the
   farthest tap in, per channel, fp64 */
static void calc_output(const sinc_state *f, int32_t increment, int32_t start, double scale,
                        float *out)
{
    double left[8], right[8];
    const int32_t max_fi = f->half_len << SHIFT_BITS;
    int k;
    for (k = 0; k < f->ch; k++)
        left[k] = right[k] = 0.0;
    int32_t fi = start;
    int32_t cc = (max_fi - fi) / increment;
    fi += cc * increment;
    long di = f->b_current - (long)f->ch * cc;
    do {
        const double fraction = (fi & ((1 << SHIFT_BITS) - 1)) * INV_FP_ONE;
        const int ix = fi >> SHIFT_BITS;
        const double icoeff = f->coeffs[ix] + fraction * (f->coeffs[ix + 1] - f->coeffs[ix]);
        for (k = 0; k < f->ch; k++)
            left[k] += icoeff * f->buffer[di + k];
        fi -= increment;
        di += f->ch;
    } while (fi >= 0);
    fi = increment - start;
    cc = (max_fi - fi) / increment;
    fi += cc * increment;
    di = f->b_current + (long)f->ch * (1 + cc);
    do {
        const double fraction = (fi & ((1 << SHIFT_BITS) - 1)) * INV_FP_ONE;
        const int ix = fi >> SHIFT_BITS;
        const double icoeff = f->coeffs[ix] + fraction * (f->coeffs[ix + 1] - f->coeffs[ix]);
        for (k = 0; k < f->ch; k++)
            right[k] += icoeff * f->buffer[di + k];
        fi -= increment;
        di -= f->ch;
    } while (fi > 0);
    for (k = 0; k < f->ch; k++)
        out[k] = (float)(scale * (left[k] + right[k]));
}

/* src_process + sinc_*_vari_process at a constant ratio */
static void process(sinc_state *f, const float *in, long in_frames, float *out, long out_frames,
                    int eoi, double ratio, long *used, long *gen)
{
    if (f->last_ratio < 1.0 / MAX_RATIO)
        f->last_ratio = ratio;
    f->in_count = in_frames * f->ch;
    f->out_count = out_frames * f->ch;
    f->in_used = f->out_gen = 0;
    const double src_ratio = f->last_ratio;
    double count = (f->half_len + 2.0) / f->index_inc;
    if (src_ratio < 1.0)
        count /= src_ratio;
    const long half = (long)(f->ch * (lrint(count) + 1));
    double input_index = f->last_position;
    double rem = fmod_one(input_index);
    f->b_current = (f->b_current + f->ch * lrint(input_index - rem)) % f->b_len;
    input_index = rem;
    const double terminate = 1.0 / src_ratio + 1e-20;
    while (f->out_gen < f->out_count) {
        long sih = (f->b_end - f->b_current + f->b_len) % f->b_len;
        if (sih <= half) {
            prepare(f, in, eoi, half);
            sih = (f->b_end - f->b_current + f->b_len) % f->b_len;
            if (sih <= half)
                break;
        }
        if (f->b_real_end >= 0 && f->b_current + input_index + terminate >= f->b_real_end)
            break;
        double float_increment = f->index_inc * 1.0;
        if (src_ratio < 1.0)
            float_increment = f->index_inc * src_ratio;
        const int32_t increment = (int32_t)lrint(float_increment * FP_ONE);
        const int32_t start = (int32_t)lrint((input_index * float_increment) * FP_ONE);
        calc_output(f, increment, start, float_increment / f->index_inc, out + f->out_gen);
        f->out_gen += f->ch;
        input_index += 1.0 / src_ratio;
        rem = fmod_one(input_index);
        f->b_current = (f->b_current + f->ch * lrint(input_index - rem)) % f->b_len;
        input_index = rem;
    }
    f->last_position = input_index;
    f->last_ratio = src_ratio;
    *used = f->in_used / f->ch;
    *gen = f->out_gen / f->ch;
}

/*
 * Resampler(reader, rate) read until the empty FrameList.  The wrapped
 * reader's read(4096) calls return reads[0..n_reads) frames of `in`
 * (reads == NULL: 4096-frame reads).  Output samples go to out (cap
 * frames); the frame count of every read() to sizes (sizes_cap entries,
 * the final 0 included; *n_sizes = how many there were).  Returns the
 * total output frames, or -1 on allocation failure.
 */
long rsport_resample(const int32_t *in, long frames, int ch, int bps, double ratio,
                     const uint32_t *reads, long n_reads, int32_t *out, long cap,
                     uint32_t *sizes, long sizes_cap, long *n_sizes)
{
    sinc_state f;
    if (ch < 1 || ch > 8 || !sinc_open(&f, ch))
        return -1;
    const unsigned q = 1u << (bps - 1);
    const int lo = -(1 << (bps - 1)), hi = (1 << (bps - 1)) - 1;
    long in_max = BLOCK, out_max = (unsigned)ceil(BLOCK * ratio);
    float *inb = malloc(sizeof(float) * (size_t)in_max * ch);
    float *outb = malloc(sizeof(float) * (size_t)out_max * ch);
    long in_frames = 0, fed = 0, r = 0, total = 0, k = 0;
    if (!inb || !outb)
        return -1;
    for (;;) {
        long out_frames = 0;
        int eoi;
        do {
            long got;
            if (reads)
                got = r < n_reads ? (long)reads[r++] : 0;
            else
                got = frames - fed < BLOCK ? frames - fed : BLOCK;
            if (in_frames + got > in_max) {
                in_max = in_frames + got;
                inb = realloc(inb, sizeof(float) * (size_t)in_max * ch);
            }
            for (long i = 0; i < got; i++)
                for (int c = 0; c < ch; c++)
                    inb[(in_frames + i) * ch + c] = (float)in[(fed + i) * ch + c] / q;
            fed += got;
            in_frames += got;
            eoi = in_frames == 0;
            long used, gen;
            process(&f, inb, in_frames, outb, out_max, eoi, ratio, &used, &gen);
            memmove(inb, inb + used * ch, sizeof(float) * (size_t)(in_frames - used) * ch);
            in_frames -= used;
            if (in_frames > 0) {
                out_max += out_max;
                outb = realloc(outb, sizeof(float) * (size_t)out_max * ch);
            }
            out_frames += gen;
        } while (out_frames == 0 && !eoi);
        for (long i = 0; i < out_frames * ch; i++) {
            const int s = (int)(outb[i] * q);
            if (total * ch + i < cap * ch)
                out[total * ch + i] = s > hi ? hi : (s < lo ? lo : s);
        }
        if (sizes && k < sizes_cap)
            sizes[k] = (uint32_t)out_frames;
        k++;
        total += out_frames;
        if (out_frames == 0)
            break;
    }
    if (n_sizes)
        *n_sizes = k;
    free(inb);
    free(outb);
    free(f.buffer);
    return total;
}

/* c_n and start_filter_index of every output frame from the absolute
   position recurrence (no buffer), for position tests */
uint64_t rsport_positions(uint64_t n_out, double ratio, uint32_t *center, int32_t *sfi)
{
    double float_increment = SRC_MEDIUM_INCREMENT * 1.0;
    if (ratio < 1.0)
        float_increment = SRC_MEDIUM_INCREMENT * ratio;
    double input_index = 0.0;
    uint64_t c = 0, n;
    for (n = 0; n < n_out; n++) {
        center[n] = (uint32_t)c;
        sfi[n] = (int32_t)lrint((input_index * float_increment) * FP_ONE);
        input_index += 1.0 / ratio;
        const double rem = fmod_one(input_index);
        c += (uint64_t)lrint(input_index - rem);
        input_index = rem;
    }
    return n;
}
