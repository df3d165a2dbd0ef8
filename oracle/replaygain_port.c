/*
 * replaygain_port.c — CPU restatement of the reference's ReplayGain title /
 * album analysis (src/replaygain.c: ReplayGain_init :115-182, title_gain
 * :186-322, filterYule/filterButter :566-610, analyze_samples :620-750,
 * analyzeResult / get_title_gain / get_album_gain :754-807).
 *
 * TEST INFRASTRUCTURE ONLY (see flac_port.h): the checker for
 * python-audio-tools_amd/csrc/replaygain.hip; never linked by the product.
 *
 * Parity unpinned: the reference has no ReplayGain fixtures (SURVEY.md
 * section 4) and replaygain.c is a Python-2 extension module, so it is not
 * built here.  The filters are a continuous IIR from zero state per track;
 * the summation of squared outputs follows the reference's batches exactly
 * (one ReplayGain_analyze_samples call per pcmreader.read(4096) result --
 * 4096-frame reads by default, or the chunk sizes the reader actually
 * returned -- the first 10 samples of each read as their own batch, 50 ms
 * window boundaries; singles for batch % 16, then 16-term groups).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../python-audio-tools_amd/csrc/rg_coeffs.h"

#define RG_BINS 12000
#define RG_ORDER 10

int rgport_freqindex(unsigned rate)
{
    static const unsigned rates[20] = {48000, 44100, 32000, 24000, 22050, 16000, 12000,
                                       11025, 8000,  18900, 37800, 56000, 64000, 88200,
                                       96000, 112000, 128000, 144000, 176400, 192000};
    for (int i = 0; i < 20; i++)
        if (rates[i] == rate)
            return i;
    return -1;
}

typedef struct {
    double in[RG_ORDER], yo[RG_ORDER], bo[2]; /* newest first */
} chan_state;

static double filter_one(chan_state *s, double x, const double *ky, const double *kb)
{
    /* filterYule then filterButter for one sample, same operation order */
    double y = 1e-10 + x * ky[0];
    for (int k = 1; k <= 10; k++) {
        y = y - s->yo[k - 1] * ky[2 * k - 1];
        y = y + s->in[k - 1] * ky[2 * k];
    }
    double b = y * kb[0] - s->bo[0] * kb[1] + s->yo[0] * kb[2] - s->bo[1] * kb[3] +
               s->yo[1] * kb[4];
    memmove(s->in + 1, s->in, sizeof(double) * (RG_ORDER - 1));
    s->in[0] = x;
    s->bo[1] = s->bo[0];
    s->bo[0] = b;
    memmove(s->yo + 1, s->yo, sizeof(double) * (RG_ORDER - 1));
    s->yo[0] = y;
    return b;
}

/* title analysis of one track: pcm interleaved int32, channels 1 or 2,
   read in chunks of chunk[0..n_chunks) frames (NULL: 4096-frame reads).
   Writes the track's window histogram A[12000] and returns the title peak
   (max |x| / 2^(bps-1)).  Returns -1 for unsupported rate / bps / channels
   or chunk sizes that do not add up to frames. */
static double title_impl(const int32_t *pcm, uint64_t frames, uint32_t channels, uint32_t bps,
                         uint32_t rate, const uint32_t *chunk, uint64_t n_chunks, uint32_t *A,
                         double *vals, uint64_t vcap, uint64_t *nvals);

double rgport_title_chunks(const int32_t *pcm, uint64_t frames, uint32_t channels,
                           uint32_t bps, uint32_t rate, const uint32_t *chunk,
                           uint64_t n_chunks, uint32_t *A)
{
    return title_impl(pcm, frames, channels, bps, rate, chunk, n_chunks, A, NULL, 0, NULL);
}

/* the value 1000 log10(...) of every closed window, in order (the number the
   histogram bins; tests use it to place a window next to a bin edge):
   returns the window count, -1 as rgport_title_chunks */
int64_t rgport_window_vals(const int32_t *pcm, uint64_t frames, uint32_t channels,
                           uint32_t bps, uint32_t rate, double *vals, uint64_t cap)
{
    uint32_t *A = (uint32_t *)malloc(sizeof(uint32_t) * RG_BINS);
    uint64_t n = 0;
    const double r = title_impl(pcm, frames, channels, bps, rate, NULL, 0, A, vals, cap, &n);
    free(A);
    return r < 0 ? -1 : (int64_t)n;
}

static double title_impl(const int32_t *pcm, uint64_t frames, uint32_t channels, uint32_t bps,
                         uint32_t rate, const uint32_t *chunk, uint64_t n_chunks, uint32_t *A,
                         double *vals, uint64_t vcap, uint64_t *nvals)
{
    const int fi = rgport_freqindex(rate);
    if (fi < 0 || (channels != 1 && channels != 2) || (bps != 8 && bps != 16 && bps != 24))
        return -1.0;
    const double *ky = RG_YULE[fi], *kb = RG_BUTTER[fi];
    const long window = (long)ceil(rate * 0.050);
    const int32_t peak_shift = 1 << (bps - 1);
    chan_state L, R;
    memset(&L, 0, sizeof(L));
    memset(&R, 0, sizeof(R));
    memset(A, 0, sizeof(uint32_t) * RG_BINS);
    double lsum = 0, rsum = 0, peak = 0;
    long totsamp = 0;
    if (chunk) {
        uint64_t tot = 0;
        for (uint64_t i = 0; i < n_chunks; i++)
            tot += chunk[i];
        if (tot != frames)
            return -1.0;
    }
    uint64_t ci = 0;
    for (uint64_t c0 = 0; c0 < frames;) {
        const long n = chunk ? (long)chunk[ci++]
                             : (long)(frames - c0 < 4096 ? frames - c0 : 4096);
        long pos = 0, batch = n;
        while (batch > 0) {
            long cur = batch > window - totsamp ? window - totsamp : batch;
            if (pos < RG_ORDER && cur > RG_ORDER - pos)
                cur = RG_ORDER - pos;
            const long singles = cur % 16;
            double gl = 0, gr = 0;
            for (long k = 0; k < cur; k++) {
                const uint64_t f = c0 + (uint64_t)(pos + k);
                const int32_t il = pcm[f * channels];
                const int32_t ir = channels == 2 ? pcm[f * channels + 1] : il;
                double xl, xr;
                if (bps == 8) {
                    xl = (double)(il << 8);
                    xr = (double)(ir << 8);
                } else if (bps == 16) {
                    xl = (double)il;
                    xr = (double)ir;
                } else {
                    xl = (double)(il >> 8);
                    xr = (double)(ir >> 8);
                }
                const double pl = (double)abs(il) / peak_shift, pr = (double)abs(ir) / peak_shift;
                peak = pl > peak ? pl : peak;
                peak = pr > peak ? pr : peak;
                const double ol = filter_one(&L, xl, ky, kb), orr = filter_one(&R, xr, ky, kb);
                if (k < singles) {
                    lsum += ol * ol;
                    rsum += orr * orr;
                } else {
                    const long g = (k - singles) % 16;
                    gl = g == 0 ? ol * ol : gl + ol * ol;
                    gr = g == 0 ? orr * orr : gr + orr * orr;
                    if (g == 15) {
                        lsum += gl;
                        rsum += gr;
                    }
                }
            }
            batch -= cur;
            pos += cur;
            totsamp += cur;
            if (totsamp == window) {
                const double val = 100. * 10. * log10((lsum + rsum) / totsamp * 0.5 + 1.e-37);
                if (nvals) {
                    if (*nvals < vcap)
                        vals[*nvals] = val;
                    ++*nvals;
                }
                int ival = (int)val;
                if (ival < 0)
                    ival = 0;
                if (ival >= RG_BINS)
                    ival = RG_BINS - 1;
                A[ival]++;
                lsum = rsum = 0.;
                totsamp = 0;
            }
        }
        c0 += (uint64_t)n;
    }
    return peak;
}

double rgport_title(const int32_t *pcm, uint64_t frames, uint32_t channels, uint32_t bps,
                    uint32_t rate, uint32_t *A)
{
    return rgport_title_chunks(pcm, frames, channels, bps, rate, NULL, 0, A);
}

/* analyzeResult (replaygain.c:754-776); NAN for "not enough samples" */
double rgport_gain(const uint32_t *A)
{
    uint32_t elems = 0;
    for (int i = 0; i < RG_BINS; i++)
        elems += A[i];
    if (elems == 0)
        return NAN;
    int32_t upper = (int32_t)ceil(elems * (1. - 0.95));
    size_t i;
    for (i = RG_BINS; i-- > 0;)
        if ((upper -= A[i]) <= 0)
            break;
    return (double)(64.82 - (double)i / 100.);
}
