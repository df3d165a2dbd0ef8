/*
 * alac_port.c — CPU restatement of python-audio-tools' ALAC encoder
 * (src/encoders/alac.c) and ALAC decoder (src/decoders/alac.c).
 *
 * TEST INFRASTRUCTURE ONLY (see flac_port.h): the parity checker for
 * python-audio-tools_amd/csrc/alac_encode.hip / alac_decode.hip and the CPU
 * "port" baseline; the product never links, loads or calls it.
 *
 * Pinning: byte-identical mdat output to the reference encoder and identical
 * PCM / error status to the reference decoder, both built from
 * /root/reference/src by oracle/Makefile (`make ref` -> oracle/_ref/alacenc,
 * alacdec), on the committed vectors of tests/golden/alac_vectors.json
 * (generator tests/golden/make_alac_golden.py) and on the reference's own
 * fixture test/alac-allframes.m4a.
 *
 * Encoder (alac.c:292-1116): a frameset per block of PCM frames, channels
 * grouped into frames as write_frameset does (:299-366), each frame
 * compressed -- mono, or stereo with the best of interlacing leftweights
 * 0..4 (:459-481, strict <) -- or written uncompressed when shorter than 10
 * samples or when any residual of the frame overflows (:384-399, the
 * longjmp); per channel: Tukey window, 9-lag autocorrelation, Levinson,
 * order 4 and 8 coefficients quantised at shift 9 (:698-905), sign-LMS
 * adaptive residuals (:933-1005), adaptive Golomb coding with zero runs
 * (:1021-1100); order 4 when bits4 < bits8 + 64.
 * Decoder (decoders/alac.c:183-254, 439-1259): atoms -> "alac" / "mdhd",
 * framesets from the start of "mdat" until remaining_frames is 0.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "alac_port.h"

#define MAX_ORDER 8
#define SHIFT 2 /* INTERLACING_SHIFT */

/* ------------------------------------------------------------- bit writer */
typedef struct {
    uint8_t *buf;
    size_t cap;
    uint64_t bits; /* bits written (counted even past cap) */
} bw;

static void bw_put(bw *w, unsigned n, uint32_t v)
{
    for (unsigned i = n; i-- > 0;) {
        const unsigned bit = (v >> i) & 1u;
        const uint64_t p = w->bits++;
        if (w->buf && (p >> 3) < w->cap) {
            if (bit)
                w->buf[p >> 3] |= (uint8_t)(0x80u >> (p & 7));
            else
                w->buf[p >> 3] &= (uint8_t)~(0x80u >> (p & 7));
        }
    }
}

static void bw_signed(bw *w, unsigned n, int32_t v)
{
    bw_put(w, n, (uint32_t)v & (n >= 32 ? 0xFFFFFFFFu : ((1u << n) - 1u)));
}

/* ------------------------------------------------------------- encoder */
static int trunc_bits(int v, unsigned bits)
{
    const int t = v & ((1 << bits) - 1);
    return (t & (1 << (bits - 1))) ? t - (1 << bits) : t;
}

static int sgn(int v) { return v > 0 ? 1 : (v < 0 ? -1 : 0); }

static unsigned ilog2u(unsigned v) /* floor(log2(v)), v > 0 */
{
    unsigned b = 0;
    while (v >>= 1)
        b++;
    return b;
}

/* Tukey(0.5) window exactly as window_signal (alac.c:778-816) */
static void tukey(unsigned N, double *w)
{
    const double alpha = 0.5;
    const unsigned w1 = (unsigned)(alpha * (N - 1)) / 2;
    const unsigned w2 = (unsigned)((N - 1) * (1.0 - (alpha / 2.0)));
    for (unsigned n = 0; n < N; n++) {
        if (n <= w1)
            w[n] = 0.5 * (1.0 + cos(M_PI * (((2 * n) / (alpha * (N - 1))) - 1.0)));
        else if (n <= w2)
            w[n] = 1.0;
        else
            w[n] = 0.5 * (1.0 + cos(M_PI * (((2.0 * n) / (alpha * (N - 1))) - (2.0 / alpha) +
                                            1.0)));
    }
}

/* window + autocorrelation + Levinson + quantisation at orders 4 and 8
   (alac.c:714-733, 818-905); returns 0 when R[0] == 0 (all-zero case) */
static int lpc_coeffs(const int32_t *s, unsigned N, const double *win, int32_t q4[4],
                      int32_t q8[8])
{
    double *x = malloc(sizeof(double) * N);
    double R[MAX_ORDER + 1];
    for (unsigned n = 0; n < N; n++)
        x[n] = s[n] * win[n];
    for (unsigned lag = 0; lag <= MAX_ORDER; lag++) {
        double acc = 0.0;
        for (unsigned i = 0; i < N - lag; i++)
            acc += x[i] * x[i + lag];
        R[lag] = acc;
    }
    free(x);
    if (R[0] == 0.0)
        return 0;
    double lp[MAX_ORDER][MAX_ORDER], err[MAX_ORDER];
    double k = R[1] / R[0];
    lp[0][0] = k;
    err[0] = R[0] * (1.0 - (k * k));
    for (unsigned i = 1; i < MAX_ORDER; i++) {
        double q = R[i + 1];
        for (unsigned j = 0; j < i; j++)
            q -= (lp[i - 1][j] * R[i - j]);
        k = q / err[i - 1];
        for (unsigned j = 0; j < i; j++)
            lp[i][j] = lp[i - 1][j] - (k * lp[i - 1][i - j - 1]);
        lp[i][i] = k;
        err[i] = err[i - 1] * (1.0 - (k * k));
    }
    for (int pass = 0; pass < 2; pass++) {
        const unsigned order = pass ? 8 : 4;
        int32_t *q = pass ? q8 : q4;
        double e = 0.0;
        for (unsigned i = 0; i < order; i++) {
            e += (lp[order - 1][i] * (1 << 9));
            const int ei = (int)round(e);
            q[i] = ei < -(1 << 15) ? -(1 << 15) : (ei > (1 << 15) - 1 ? (1 << 15) - 1 : ei);
            e -= (double)ei;
        }
    }
    return 1;
}

/* calculate_residuals (alac.c:932-1005): sign-LMS adaptive predictor */
static void lms_residuals(const int32_t *s, unsigned N, unsigned sample_size,
                          const int32_t *coef_in, unsigned order, int32_t *r)
{
    int c[32];
    for (unsigned j = 0; j < order; j++)
        c[j] = coef_in[j];
    unsigned i = 0;
    r[i] = s[i];
    i++;
    for (; i < order + 1 && i < N; i++)
        r[i] = trunc_bits(s[i] - s[i - 1], sample_size);
    for (; i < N; i++) {
        const int base = s[i - order - 1];
        int64_t sum = 1 << 8;
        for (unsigned j = 0; j < order; j++)
            sum += (int64_t)c[j] * (int64_t)(s[i - j - 1] - base);
        sum >>= 9;
        int e = trunc_bits(s[i] - base - (int)sum, sample_size);
        r[i] = e;
        if (e > 0) {
            for (unsigned j = 0; j < order; j++) {
                const int diff = base - s[i - order + j];
                const int sg = sgn(diff);
                c[order - j - 1] -= sg;
                e -= ((diff * sg) >> 9) * (int)(j + 1);
                if (e <= 0)
                    break;
            }
        } else if (e < 0) {
            for (unsigned j = 0; j < order; j++) {
                const int diff = base - s[i - order + j];
                const int sg = sgn(diff);
                c[order - j - 1] += sg;
                e -= ((diff * -sg) >> 9) * (int)(j + 1);
                if (e >= 0)
                    break;
            }
        }
    }
}

/* write_residual (alac.c:1081-1100) */
static void put_residual(bw *w, unsigned value, unsigned k, unsigned sample_size)
{
    const unsigned m = (1u << k) - 1u;
    const unsigned msb = value / m, lsb = value % m;
    if (msb > 8) {
        bw_put(w, 9, 0x1FF);
        bw_put(w, sample_size, value);
    } else {
        for (unsigned u = 0; u < msb; u++)
            bw_put(w, 1, 1);
        bw_put(w, 1, 0);
        if (k > 1) {
            if (lsb > 0)
                bw_put(w, k, lsb + 1);
            else
                bw_put(w, k - 1, 0);
        }
    }
}

/* encode_residuals (alac.c:1020-1079); returns 1 on residual overflow */
static int golomb(bw *w, const alacport_options *o, unsigned sample_size, const int32_t *r,
                  unsigned N)
{
    int history = (int)o->initial_history;
    unsigned sign_modifier = 0, i = 0;
    const unsigned max_unsigned = 1u << sample_size;
    while (i < N) {
        const unsigned u = r[i] >= 0 ? (unsigned)(r[i] << 1) : (unsigned)(-r[i] << 1) - 1;
        if (u >= max_unsigned)
            return 1;
        unsigned k = ilog2u((unsigned)(history >> 9) + 3);
        if (k > o->maximum_k)
            k = o->maximum_k;
        put_residual(w, u - sign_modifier, k, sample_size);
        sign_modifier = 0;
        if (u <= 0xFFFF) {
            history += ((int)(u * o->history_multiplier) -
                        ((history * (int)o->history_multiplier) >> 9));
            i++;
            if (history < 128 && i < N) {
                /* LOG2(0) would be UINT_MAX (NDEBUG build): k = 8; the
                   history here is never 0 for encoder-made residuals */
                unsigned kz = 7 - (history ? ilog2u((unsigned)history) : 0xFFFFFFFFu) +
                              (unsigned)((history + 16) >> 6);
                if (kz > o->maximum_k)
                    kz = o->maximum_k;
                unsigned zeros = 0;
                while (i < N && r[i] == 0) {
                    zeros++;
                    i++;
                }
                put_residual(w, zeros, kz, 16);
                if (zeros < 0xFFFF)
                    sign_modifier = 1;
                history = 0;
            }
        } else {
            i++;
            history = 0xFFFF;
        }
    }
    return 0;
}

/* compute_coefficients (alac.c:697-776) for one channel: the chosen
   coefficients and their residual block appended to `out`.  Returns 1 on
   residual overflow. */
static int encode_channel(const alacport_options *o, const int32_t *s, unsigned N,
                          const double *win, unsigned sample_size, int32_t *coef,
                          unsigned *order, bw *out, int32_t *scratch)
{
    int32_t q4[4], q8[8];
    if (!lpc_coeffs(s, N, win, q4, q8)) {
        memset(coef, 0, sizeof(int32_t) * 4);
        *order = 4;
        lms_residuals(s, N, sample_size, coef, 4, scratch);
        return golomb(out, o, sample_size, scratch, N);
    }
    bw b4 = {NULL, 0, 0}, b8 = {NULL, 0, 0};
    int32_t *r8 = scratch + N;
    lms_residuals(s, N, sample_size, q4, 4, scratch);
    lms_residuals(s, N, sample_size, q8, 8, r8);
    if (golomb(&b4, o, sample_size, scratch, N) || golomb(&b8, o, sample_size, r8, N))
        return 1;
    if (b4.bits < b8.bits + 64) {
        memcpy(coef, q4, sizeof(q4));
        *order = 4;
        return golomb(out, o, sample_size, scratch, N);
    }
    memcpy(coef, q8, sizeof(q8));
    *order = 8;
    return golomb(out, o, sample_size, r8, N);
}

static void sub_header(bw *w, const int32_t *coef, unsigned order)
{
    bw_put(w, 4, 0); /* prediction type */
    bw_put(w, 4, 9); /* QLP shift */
    bw_put(w, 3, 4); /* Rice modifier */
    bw_put(w, 5, order);
    for (unsigned i = 0; i < order; i++)
        bw_signed(w, 16, coef[i]);
}

static void frame_head(bw *w, const alacport_options *o, unsigned N, unsigned lsbs,
                       unsigned not_compressed)
{
    bw_put(w, 16, 0);
    bw_put(w, 1, N == o->block_size ? 0 : 1);
    bw_put(w, 2, lsbs);
    bw_put(w, 1, not_compressed);
    if (N != o->block_size)
        bw_put(w, 32, N);
}

/* one frame of 1 or 2 channels (write_frame, alac.c:373-654) appended to w */
static void write_frame(bw *w, const alacport_options *o, uint32_t bps, const int32_t *const *ch,
                        unsigned nch, unsigned N, const double *win)
{
    bw_put(w, 3, nch - 1);
    int compressed_ok = 0;
    if (N >= 10) {
        const unsigned lsbs = bps <= 16 ? 0 : (bps - 16) / 8;
        const unsigned lshift = lsbs * 8;
        int32_t *msb[2] = {NULL, NULL};
        for (unsigned c = 0; c < nch; c++) {
            msb[c] = malloc(sizeof(int32_t) * N);
            for (unsigned i = 0; i < N; i++)
                msb[c][i] = lshift ? ch[c][i] >> lshift : ch[c][i];
        }
        int32_t *scratch = malloc(sizeof(int32_t) * 2 * N);
        const size_t fcap = (size_t)N * nch * 4 + 64;
        if (nch == 1) {
            bw f = {calloc(fcap, 1), fcap, 0};
            frame_head(&f, o, N, lsbs, 0);
            bw_put(&f, 8, 0);
            bw_put(&f, 8, 0);
            int32_t coef[8];
            unsigned order;
            bw res = {calloc(fcap, 1), fcap, 0};
            if (!encode_channel(o, msb[0], N, win, bps - lshift, coef, &order, &res, scratch)) {
                sub_header(&f, coef, order);
                for (unsigned i = 0; lsbs && i < N; i++)
                    bw_put(&f, lshift, (uint32_t)ch[0][i] & ((1u << lshift) - 1u));
                for (uint64_t b = 0; b < res.bits; b++)
                    bw_put(&f, 1, (res.buf[b >> 3] >> (7 - (b & 7))) & 1);
                for (uint64_t b = 0; b < f.bits; b++)
                    bw_put(w, 1, (f.buf[b >> 3] >> (7 - (b & 7))) & 1);
                compressed_ok = 1;
            }
            free(f.buf);
            free(res.buf);
        } else {
            int32_t *c0 = malloc(sizeof(int32_t) * N), *c1 = malloc(sizeof(int32_t) * N);
            bw best = {NULL, 0, 0};
            uint64_t best_bits = UINT32_MAX; /* unsigned best_interlaced_frame_bits */
            int overflow = 0;
            /* write_compressed_frame's leftweight loop (alac.c:459-481) */
            for (unsigned lw = o->min_leftweight; lw <= o->max_leftweight && !overflow; lw++) {
                for (unsigned i = 0; i < N; i++) {
                    if (lw) {
                        int64_t t = msb[0][i] - msb[1][i];
                        t *= lw;
                        t >>= SHIFT;
                        c0[i] = msb[1][i] + (int)t;
                        c1[i] = msb[0][i] - msb[1][i];
                    } else {
                        c0[i] = msb[0][i];
                        c1[i] = msb[1][i];
                    }
                }
                bw f = {calloc(fcap, 1), fcap, 0};
                frame_head(&f, o, N, lsbs, 0);
                bw_put(&f, 8, SHIFT);
                bw_put(&f, 8, lw);
                int32_t k0[8], k1[8];
                unsigned o0, o1;
                bw r0 = {calloc(fcap, 1), fcap, 0}, r1 = {calloc(fcap, 1), fcap, 0};
                const unsigned ss = bps - lshift + 1;
                if (encode_channel(o, c0, N, win, ss, k0, &o0, &r0, scratch) ||
                    encode_channel(o, c1, N, win, ss, k1, &o1, &r1, scratch)) {
                    overflow = 1;
                } else {
                    sub_header(&f, k0, o0);
                    sub_header(&f, k1, o1);
                    for (unsigned i = 0; lsbs && i < N; i++)
                        for (unsigned c = 0; c < 2; c++)
                            bw_put(&f, lshift, (uint32_t)ch[c][i] & ((1u << lshift) - 1u));
                    for (uint64_t b = 0; b < r0.bits; b++)
                        bw_put(&f, 1, (r0.buf[b >> 3] >> (7 - (b & 7))) & 1);
                    for (uint64_t b = 0; b < r1.bits; b++)
                        bw_put(&f, 1, (r1.buf[b >> 3] >> (7 - (b & 7))) & 1);
                    if (f.bits < best_bits) {
                        best_bits = f.bits;
                        free(best.buf);
                        best = f;
                        f.buf = NULL;
                    }
                }
                free(f.buf);
                free(r0.buf);
                free(r1.buf);
            }
            if (!overflow) {
                for (uint64_t b = 0; b < best.bits; b++)
                    bw_put(w, 1, (best.buf[b >> 3] >> (7 - (b & 7))) & 1);
                compressed_ok = 1;
            }
            free(best.buf);
            free(c0);
            free(c1);
        }
        free(scratch);
        for (unsigned c = 0; c < nch; c++)
            free(msb[c]);
    }
    if (!compressed_ok) { /* write_uncompressed_frame (alac.c:402-430) */
        frame_head(w, o, N, 0, 1);
        for (unsigned i = 0; i < N; i++)
            for (unsigned c = 0; c < nch; c++)
                bw_signed(w, bps, ch[c][i]);
    }
}

/* channel grouping of write_frameset (alac.c:299-366): groups of 1 or 2
   channel indices, in frame order */
static unsigned frameset_groups(unsigned nch, int g[8][2])
{
    static const int T[9][6][2] = {
        {{0}},
        {{0, -1}},
        {{0, 1}},
        {{2, -1}, {0, 1}},
        {{2, -1}, {0, 1}, {3, -1}},
        {{2, -1}, {0, 1}, {3, 4}},
        {{2, -1}, {0, 1}, {4, 5}, {3, -1}},
        {{2, -1}, {0, 1}, {4, 5}, {6, -1}, {3, -1}},
        {{2, -1}, {6, 7}, {0, 1}, {4, 5}, {3, -1}},
    };
    static const unsigned n[9] = {0, 1, 1, 2, 3, 3, 4, 5, 5};
    if (nch <= 8) {
        for (unsigned i = 0; i < n[nch]; i++) {
            g[i][0] = T[nch][i][0];
            g[i][1] = T[nch][i][1];
        }
        return n[nch];
    }
    return 0;
}

unsigned alacport_frameset_groups(unsigned channels, int32_t *groups)
{
    int g[8][2];
    unsigned n = frameset_groups(channels, g);
    for (unsigned i = 0; i < n; i++) {
        groups[2 * i] = g[i][0];
        groups[2 * i + 1] = g[i][1];
    }
    return n;
}

size_t alacport_max_mdat_bytes(uint64_t frames, uint32_t channels, uint32_t bps,
                               uint32_t block_size)
{
    const uint64_t nfs = block_size ? (frames + block_size - 1) / block_size : 0;
    /* uncompressed frames: 3 + 20 + 32 bits + samples, per frame */
    return (size_t)(8 + frames * channels * ((bps + 7) / 8 + 1) + nfs * (channels * 8 + 16) + 64);
}

int alacport_encode(const int32_t *pcm, uint64_t frames, uint32_t channels, uint32_t bps,
                    const alacport_options *o, uint8_t *out, size_t cap, size_t *out_len,
                    uint32_t *frame_sizes, size_t fs_cap, size_t *n_framesets)
{
    if (!o || channels < 1 || channels > 8 || (bps != 16 && bps != 24) || o->block_size < 1)
        return 1;
    memset(out, 0, cap);
    bw w = {out, cap, 0};
    bw_put(&w, 32, 0);
    bw_put(&w, 8, 'm');
    bw_put(&w, 8, 'd');
    bw_put(&w, 8, 'a');
    bw_put(&w, 8, 't');
    int g[8][2];
    const unsigned ng = frameset_groups(channels, g);
    double *win = malloc(sizeof(double) * o->block_size);
    unsigned win_n = 0;
    int32_t *deint = malloc(sizeof(int32_t) * o->block_size * channels);
    size_t nfs = 0;
    for (uint64_t f0 = 0; f0 < frames; f0 += o->block_size) {
        const unsigned N = (unsigned)(frames - f0 < o->block_size ? frames - f0 : o->block_size);
        if (N != win_n) {
            tukey(N, win);
            win_n = N;
        }
        for (unsigned c = 0; c < channels; c++)
            for (unsigned i = 0; i < N; i++)
                deint[c * N + i] = pcm[(f0 + i) * channels + c];
        const uint64_t start = w.bits;
        for (unsigned k = 0; k < ng; k++) {
            const int32_t *chp[2] = {deint + (size_t)g[k][0] * N,
                                     g[k][1] >= 0 ? deint + (size_t)g[k][1] * N : NULL};
            write_frame(&w, o, bps, chp, g[k][1] >= 0 ? 2 : 1, N, win);
        }
        bw_put(&w, 3, 7);
        if (w.bits & 7)
            bw_put(&w, 8 - (unsigned)(w.bits & 7), 0);
        if (nfs < fs_cap && frame_sizes)
            frame_sizes[nfs] = (uint32_t)((w.bits - start) >> 3);
        nfs++;
    }
    free(win);
    free(deint);
    const uint64_t total = w.bits >> 3;
    if (total > cap)
        return 2;
    out[0] = (uint8_t)(total >> 24);
    out[1] = (uint8_t)(total >> 16);
    out[2] = (uint8_t)(total >> 8);
    out[3] = (uint8_t)total;
    *out_len = (size_t)total;
    if (n_framesets)
        *n_framesets = nfs;
    return 0;
}

/* ------------------------------------------------------------- decoder */
typedef struct {
    const uint8_t *d;
    uint64_t len_bits, pos;
    int eof;
} br;

static uint32_t br_get(br *r, unsigned n)
{
    uint32_t v = 0;
    for (unsigned i = 0; i < n; i++) {
        if (r->pos >= r->len_bits) {
            r->eof = 1;
            return 0;
        }
        v = (v << 1) | ((r->d[r->pos >> 3] >> (7 - (r->pos & 7))) & 1u);
        r->pos++;
    }
    return v;
}

static int32_t br_signed(br *r, unsigned n)
{
    const uint32_t v = br_get(r, n);
    if (n == 0)
        return 0;
    if (n >= 32)
        return (int32_t)v;
    return (v & (1u << (n - 1))) ? (int32_t)(v - (1u << n)) : (int32_t)v;
}

static uint32_t be32(const uint8_t *p)
{
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

/* find_atom over [off, end): the first atom named `name` ->
   body [*b0, *b1); 1 = not found (I/O error in the walk) */
static int find_atom(const uint8_t *d, uint64_t off, uint64_t end, const char *name,
                     uint64_t *b0, uint64_t *b1)
{
    for (;;) {
        if (off + 8 > end)
            return 1;
        const uint32_t size = be32(d + off);
        if (!memcmp(d + off + 4, name, 4)) {
            if (size < 8 || off + size > end)
                return 1; /* substream_append past the end: I/O error */
            *b0 = off + 8;
            *b1 = off + size;
            return 0;
        }
        /* skip_bytes(size - 8): unsigned wrap for size < 8 */
        const uint64_t skip = (uint32_t)(size - 8u);
        off = off + 8 + skip;
    }
}

static int find_path(const uint8_t *d, uint64_t off, uint64_t end, const char *const *names,
                     uint64_t *b0, uint64_t *b1)
{
    for (; *names; names++) {
        if (find_atom(d, off, end, *names, b0, b1))
            return 1;
        off = *b0;
        end = *b1;
    }
    return 0;
}

/* read_stts / read_stsc / read_stco + populate_seektable (alac.c:500-672) */
static int seektable(const uint8_t *d, uint64_t m0, uint64_t m1, uint32_t total,
                     alacport_seekpoint *sp, size_t sp_cap, uint32_t *n_sp)
{
    static const char *const stts[] = {"minf", "stbl", "stts", NULL};
    static const char *const stsc[] = {"minf", "stbl", "stsc", NULL};
    static const char *const stco[] = {"minf", "stbl", "stco", NULL};
    uint64_t t0, t1, c0, c1, o0, o1;
    *n_sp = 0;
    int have = !find_path(d, m0, m1, stts, &t0, &t1) && !find_path(d, m0, m1, stsc, &c0, &c1) &&
               !find_path(d, m0, m1, stco, &o0, &o1);
    /* each table must parse completely (else it counts as not found) */
    uint32_t nt = 0, nc = 0, no = 0;
    if (have) {
        nt = t1 - t0 >= 8 ? be32(d + t0 + 4) : 0;
        nc = c1 - c0 >= 8 ? be32(d + c0 + 4) : 0;
        no = o1 - o0 >= 8 ? be32(d + o0 + 4) : 0;
        have = t1 - t0 >= 8 && (t1 - t0 - 8) / 8 >= nt && c1 - c0 >= 8 &&
               (c1 - c0 - 8) / 12 >= nc && o1 - o0 >= 8 && (o1 - o0 - 8) / 4 >= no;
    }
    if (!have)
        return 0;
    uint32_t sum = 0;
    uint64_t nframes = 0;
    for (uint32_t i = 0; i < nt; i++) {
        const uint32_t cnt = be32(d + t0 + 8 + 8 * i), dur = be32(d + t0 + 12 + 8 * i);
        sum += cnt * dur;
        nframes += cnt;
    }
    if (sum != total)
        return ALACPORT_INVALID_SEEKTABLE;
    if (nframes == 0 || nc == 0)
        return ALACPORT_INVALID_SEEKTABLE;
    /* walk the frame durations chunk by chunk */
    uint32_t ti = 0, tleft = nt ? be32(d + t0 + 8) : 0;
    uint64_t left = nframes, pcm = 0;
    size_t nchunks = 0;
    for (uint32_t i = 0; i < nc; i++) {
        const uint32_t first = be32(d + c0 + 8 + 12 * i), per = be32(d + c0 + 12 + 12 * i);
        if (per == 0)
            return ALACPORT_INVALID_SEEKTABLE;
        const int last = i + 1 >= nc;
        const uint32_t next_first = last ? 0 : be32(d + c0 + 8 + 12 * (i + 1));
        for (uint32_t j = first; last ? left > 0 : j < next_first; j++) {
            if (left < per)
                return ALACPORT_INVALID_SEEKTABLE;
            uint64_t chunk = 0;
            for (uint32_t k = 0; k < per; k++) {
                while (tleft == 0) {
                    ti++;
                    tleft = be32(d + t0 + 8 + 8 * ti);
                }
                chunk += be32(d + t0 + 12 + 8 * ti);
                tleft--;
            }
            left -= per;
            if (nchunks < no && nchunks < sp_cap) {
                sp[nchunks].pcm_frames_offset = (uint32_t)pcm;
                sp[nchunks].file_offset = be32(d + o0 + 8 + 4 * nchunks);
            }
            pcm += (uint32_t)chunk;
            nchunks++;
        }
    }
    if (nchunks != no)
        return ALACPORT_INVALID_SEEKTABLE;
    *n_sp = (uint32_t)nchunks;
    return 0;
}

int alacport_read_info(const uint8_t *d, size_t len, alacport_info *info,
                       alacport_seekpoint *sp, size_t sp_cap)
{
    memset(info, 0, sizeof(*info));
    uint64_t m0, m1, a0, a1;
    static const char *const mdia[] = {"moov", "trak", "mdia", NULL};
    static const char *const stsd[] = {"minf", "stbl", "stsd", NULL};
    static const char *const mdhd[] = {"mdhd", NULL};
    if (find_path(d, 0, len, mdia, &m0, &m1))
        return ALACPORT_MDIA_NOT_FOUND;
    if (find_path(d, m0, m1, stsd, &a0, &a1))
        return ALACPORT_STSD_NOT_FOUND;
    /* read_alac_atom (alac.c:1354-1395):
       "8u 24p 32u" "32p 4b 6P 16p 16p 16p 4P 16p 16p 16p 16p 4P"
       "32p 4b 4P 32u 8p 8u 8u 8u 8u 8u 16p 32p 32p 32u" = 80 bytes */
    if (a1 - a0 < 80)
        return ALACPORT_IO_ERROR;
    const uint8_t *p = d + a0 + 8;
    const uint8_t *alac1 = p + 4;
    p += 36;
    const uint8_t *alac2 = p + 4;
    p += 12;
    info->max_samples_per_frame = be32(p);
    p += 5;
    info->bits_per_sample = p[0];
    info->history_multiplier = p[1];
    info->initial_history = p[2];
    info->maximum_k = p[3];
    info->channels = p[4];
    p += 5 + 2 + 8;
    info->sample_rate = be32(p);
    if (memcmp(alac1, "alac", 4) || memcmp(alac2, "alac", 4))
        return ALACPORT_INVALID_ALAC_ATOM;
    if (find_path(d, m0, m1, mdhd, &a0, &a1))
        return ALACPORT_MDHD_NOT_FOUND;
    if (a1 - a0 < 4)
        return ALACPORT_IO_ERROR;
    if (d[a0] != 0)
        return ALACPORT_INVALID_MDHD_ATOM;
    if (a1 - a0 < 24)
        return ALACPORT_IO_ERROR;
    info->total_frames = be32(d + a0 + 16);
    int st = seektable(d, m0, m1, info->total_frames, sp, sp_cap, &info->n_seekpoints);
    if (st)
        return st;
    /* seek_mdat (alac.c:953-971): top-level walk from the file start */
    uint64_t off = 0;
    for (;;) {
        if (off + 8 > len)
            return ALACPORT_NO_MDAT;
        const uint32_t size = be32(d + off);
        if (!memcmp(d + off + 4, "mdat", 4))
            break;
        off = off + 8 + (uint32_t)(size - 8u);
    }
    info->mdat_offset = off + 8;
    return 0;
}

static int log2i(int v)
{
    int b = -1;
    while (v) {
        b++;
        v >>= 1;
    }
    return b;
}

/* read_residual (alac.c:1089-1120) */
static unsigned get_residual(br *r, unsigned k, unsigned sample_size)
{
    int msb = 0;
    while (msb < 9) {
        const uint32_t b = br_get(r, 1);
        if (r->eof)
            return 0;
        if (!b)
            break;
        msb++;
    }
    if (msb == 9)
        return br_get(r, sample_size);
    if (k == 0)
        return (unsigned)msb;
    const uint32_t lsb = br_get(r, k);
    if (lsb > 1)
        return msb * ((1u << k) - 1) + (lsb - 1);
    r->pos -= 1; /* unread the last bit */
    return msb * ((1u << k) - 1);
}

/* read_residuals (alac.c:1017-1085); returns the residual count produced */
static unsigned get_residuals(br *r, int32_t *res, unsigned count, unsigned sample_size,
                              const alacport_info *in)
{
    int history = (int)in->initial_history;
    unsigned sign_modifier = 0, n = 0;
    for (int i = 0; i < (int)count; i++) {
        int kk = log2i((history >> 9) + 3);
        unsigned k = (unsigned)kk < in->maximum_k ? (unsigned)kk : in->maximum_k;
        const unsigned u = get_residual(r, k, sample_size) + sign_modifier;
        if (r->eof)
            return n;
        sign_modifier = 0;
        res[n++] = (u & 1) ? -(int32_t)((u + 1) >> 1) : (int32_t)(u >> 1);
        if (u > 0xFFFF)
            history = 0xFFFF;
        else
            history += (int)((u * in->history_multiplier) -
                             (((unsigned)history * in->history_multiplier) >> 9));
        if (history < 128 && (i + 1) < (int)count) {
            int kz = 7 - log2i(history) + ((history + 16) / 64);
            unsigned k2 = (unsigned)kz < in->maximum_k ? (unsigned)kz : in->maximum_k;
            unsigned z = get_residual(r, k2, 16);
            if (r->eof)
                return n;
            if (z > 0) {
                if (z > count - (unsigned)i)
                    z = count - (unsigned)i;
                for (unsigned j = 0; j < z; j++) {
                    res[n++] = 0;
                    i++;
                }
            }
            history = 0;
            if (z <= 0xFFFF)
                sign_modifier = 1;
        }
    }
    return n;
}

/* decode_subframe (alac.c:1147-1235) */
static void restore(int32_t *s, unsigned sample_size, const int32_t *res, unsigned n,
                    int32_t *coef, unsigned order, unsigned shift)
{
    unsigned i = 0;
    if (n == 0)
        return;
    s[i] = res[i];
    i++;
    if (order < 31) {
        for (unsigned j = 0; j < order && i < n; j++, i++)
            s[i] = trunc_bits(res[i] + s[i - 1], sample_size);
        for (; i < n; i++) {
            const int base = s[i - (order + 1)];
            int residual = res[i];
            /* 1 << (shift - 1) as an int shift on x86 (count masked to 5
               bits): shift 0 gives INT_MIN, as the reference build does */
            int64_t sum = (int64_t)(int32_t)(1u << ((shift - 1u) & 31u));
            for (unsigned j = 0; j < order; j++)
                sum += (int64_t)coef[j] * (int64_t)(s[i - j - 1] - base);
            sum >>= shift;
            sum += base;
            s[i] = trunc_bits((int)(residual + sum), sample_size);
            if (residual > 0) {
                for (unsigned j = 0; j < order; j++) {
                    const int diff = base - s[i - order + j];
                    const int sg = sgn(diff);
                    coef[order - j - 1] -= sg;
                    residual -= ((diff * sg) >> shift) * (int)(j + 1);
                    if (residual <= 0)
                        break;
                }
            } else if (residual < 0) {
                for (unsigned j = 0; j < order; j++) {
                    const int diff = base - s[i - order + j];
                    const int sg = sgn(diff);
                    coef[order - j - 1] += sg;
                    residual -= ((diff * -sg) >> shift) * (int)(j + 1);
                    if (residual >= 0)
                        break;
                }
            }
        }
    } else { /* the reference's verbatim branch advances i twice per sample */
        for (; i < n; i++) {
            s[i] = trunc_bits(res[i] + s[i - 1], sample_size);
            i++;
        }
    }
}

/* ALAC channel order -> wave order (alac_order_to_wave_order, alac.c:709-816):
   out channel c takes decoded channel map[c] */
static void wave_order(unsigned n, unsigned *map)
{
    static const unsigned M[9][8] = {{0}, {0}, {0, 1}, {1, 2, 0}, {1, 2, 0, 3},
                                     {1, 2, 0, 3, 4}, {1, 2, 0, 5, 3, 4},
                                     {1, 2, 0, 6, 3, 4, 5}, {3, 4, 0, 7, 5, 6, 1, 2}};
    for (unsigned c = 0; c < n; c++)
        map[c] = n <= 8 ? M[n][c] : c;
}

int alacport_decode(const uint8_t *d, size_t len, const alacport_info *in, uint64_t start,
                    uint64_t remaining, int32_t *pcm, size_t pcm_cap, uint64_t *pcm_frames,
                    uint32_t *fs_frames, uint64_t *fs_offsets, size_t fs_cap,
                    size_t *n_framesets)
{
    br r = {d, (uint64_t)len * 8, start * 8, 0};
    uint64_t out_frames = 0;
    size_t nfs = 0;
    int status = 0;
    const unsigned maxn = in->max_samples_per_frame;
    while (remaining) {
        const uint64_t fs_start = r.pos >> 3;
        /* frameset: frames until the 3-bit channel count reads 8 */
        int32_t *chan[8];
        unsigned nchan = 0, frames_n[8];
        unsigned cc = br_get(&r, 3) + 1;
        while (!r.eof && cc != 8) {
            if (br_get(&r, 16) != 0) {
                status = r.eof ? ALACPORT_IO_ERROR : ALACPORT_INVALID_UNUSED_BITS;
                goto done;
            }
            const unsigned has_size = br_get(&r, 1);
            const unsigned lsbs = br_get(&r, 2);
            const unsigned not_compressed = br_get(&r, 1);
            const unsigned N = has_size ? br_get(&r, 32) : maxn;
            if (r.eof)
                break;
            if (nchan + cc > 8 || N > (1u << 24)) { /* beyond any encoder output */
                status = ALACPORT_IO_ERROR;
                goto done;
            }
            for (unsigned c = 0; c < cc; c++)
                chan[nchan + c] = calloc((size_t)N + 1, sizeof(int32_t));
            if (not_compressed) {
                for (unsigned i = 0; i < N && !r.eof; i++)
                    for (unsigned c = 0; c < cc; c++)
                        chan[nchan + c][i] = br_signed(&r, in->bits_per_sample);
                for (unsigned c = 0; c < cc; c++)
                    frames_n[nchan + c] = N;
            } else {
                const unsigned shift = br_get(&r, 8), lw = br_get(&r, 8);
                int32_t coef[8][32];
                unsigned order[8], qshift[8];
                for (unsigned c = 0; c < cc; c++) {
                    br_get(&r, 4);
                    qshift[c] = br_get(&r, 4);
                    br_get(&r, 3);
                    order[c] = br_get(&r, 5);
                    for (unsigned j = 0; j < order[c]; j++)
                        coef[c][j] = br_signed(&r, 16);
                }
                int32_t *L = NULL;
                if (lsbs) {
                    L = malloc(sizeof(int32_t) * ((size_t)cc * N + 1));
                    for (unsigned i = 0; i < cc * N && !r.eof; i++)
                        L[i] = (int32_t)br_get(&r, lsbs * 8);
                }
                const unsigned ss = in->bits_per_sample - lsbs * 8 + (cc - 1);
                int32_t *res = malloc(sizeof(int32_t) * ((size_t)N + 2));
                for (unsigned c = 0; c < cc && !r.eof; c++) {
                    const unsigned n = get_residuals(&r, res, N, ss, in);
                    if (r.eof)
                        break;
                    const unsigned outn = order[c] > n ? order[c] : n;
                    free(chan[nchan + c]);
                    chan[nchan + c] = calloc((size_t)outn + 1, sizeof(int32_t));
                    restore(chan[nchan + c], ss, res, n, coef[c], order[c], qshift[c]);
                    frames_n[nchan + c] = n;
                }
                free(res);
                if (!r.eof && cc == 2 && lw > 0) {
                    int32_t *a = chan[nchan], *b = chan[nchan + 1];
                    for (unsigned i = 0; i < frames_n[nchan]; i++) {
                        const int c0 = a[i], c1 = b[i];
                        int64_t t = (int64_t)(c1 * (int)lw);
                        t >>= (shift & 63u);
                        const int rs = c0 - (int)t;
                        a[i] = c1 + rs;
                        b[i] = rs;
                    }
                }
                if (!r.eof && lsbs) {
                    for (unsigned c = 0; c < cc; c++)
                        for (unsigned i = 0; i < frames_n[nchan + c] && i < N; i++)
                            chan[nchan + c][i] =
                                (chan[nchan + c][i] << (lsbs * 8)) | L[i * cc + c];
                }
                free(L);
            }
            nchan += cc;
            if (r.eof)
                break;
            cc = br_get(&r, 3) + 1;
        }
        if (r.eof) {
            status = ALACPORT_IO_ERROR;
            for (unsigned c = 0; c < nchan; c++)
                free(chan[c]);
            goto done;
        }
        if (r.pos & 7)
            r.pos += 8 - (r.pos & 7);
        const unsigned n0 = nchan ? frames_n[0] : 0;
        remaining -= remaining < n0 ? remaining : n0;
        int mismatch = nchan != in->channels;
        for (unsigned c = 1; c < nchan; c++)
            mismatch |= frames_n[c] != n0;
        if (!mismatch) {
            unsigned map[8];
            wave_order(nchan, map);
            if ((out_frames + n0) * nchan > pcm_cap) {
                status = -1;
            } else {
                for (unsigned i = 0; i < n0; i++)
                    for (unsigned c = 0; c < nchan; c++)
                        pcm[(out_frames + i) * nchan + c] = chan[map[c]][i];
                out_frames += n0;
            }
            if (nfs < fs_cap) {
                if (fs_frames)
                    fs_frames[nfs] = n0;
                if (fs_offsets)
                    fs_offsets[nfs] = fs_start;
            }
            nfs++;
        }
        for (unsigned c = 0; c < nchan; c++)
            free(chan[c]);
        if (mismatch) {
            status = ALACPORT_CHANNEL_MISMATCH;
            goto done;
        }
        if (status)
            goto done;
    }
done:
    *pcm_frames = out_frames;
    if (n_framesets)
        *n_framesets = nfs;
    return status;
}
