/*
 * flac_port.c — clean-room CPU restatement of the python-audio-tools 2.22alpha1
 * FLAC encoder (reference src/encoders/flac.c) plus a FLAC decoder.
 *
 * TEST INFRASTRUCTURE ONLY (see flac_port.h).  Never linked into the product.
 *
 * The encoder is restated as "plan, then emit": every subframe candidate is
 * sized analytically with exactly the arithmetic the reference's bit
 * accumulator performs (uint32 bit counts, strict-< tie breaking), the winner
 * is recorded as a plan and only the winner is serialised.  This is the same
 * decomposition the GPU engine uses, so a disagreement points at one stage.
 *
 * Reference anchors (file:line in /root/reference):
 *   stream driver / STREAMINFO      src/encoders/flac.c:164-279, 376-409
 *   frame header + UTF-8 number     src/encoders/flac.c:412-518, 1531-1566
 *   stereo decorrelation choice     src/encoders/flac.c:520-671, 1507-1529
 *   subframe choice                 src/encoders/flac.c:673-811
 *   FIXED                           src/encoders/flac.c:856-930
 *   LPC (window/autocorr/Levinson/quantise/exhaustive search)
 *                                   src/encoders/flac.c:932-1324
 *   residual partitions / Rice      src/encoders/flac.c:1326-1505
 *   wasted bits / constant test     src/encoders/flac.c:1578-1631
 *   bit writer semantics            src/bitstream.c:1904-2058, 2234-2313
 *   CRC-8 / CRC-16                  src/common/flac_crc.c:23,63
 *   decoder                         src/decoders/flac.c:174-285, 710-1269
 */
#include "flac_port.h"

#include <ctype.h>
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif
#ifndef M_LN2
#define M_LN2 0.69314718055994530942
#endif

#define VENDOR_STRING "Python Audio Tools 2.22alpha1"

/* ------------------------------------------------------------------ */
/* CRC-8 (poly 0x07) and CRC-16 (poly 0x8005), MSB-first, init 0.      */
/* ------------------------------------------------------------------ */
static uint8_t crc8_tab[256];
static uint16_t crc16_tab[256];
static int crc_ready;

static void crc_init(void)
{
    if (crc_ready)
        return;
    for (unsigned b = 0; b < 256; b++) {
        unsigned c8 = b;
        unsigned c16 = b << 8;
        for (int i = 0; i < 8; i++) {
            c8 = (c8 & 0x80) ? ((c8 << 1) ^ 0x07) : (c8 << 1);
            c16 = (c16 & 0x8000) ? ((c16 << 1) ^ 0x8005) : (c16 << 1);
        }
        crc8_tab[b] = (uint8_t)c8;
        crc16_tab[b] = (uint16_t)c16;
    }
    crc_ready = 1;
}

static uint8_t crc8_bytes(const uint8_t *p, size_t n)
{
    uint8_t c = 0;
    for (size_t i = 0; i < n; i++)
        c = crc8_tab[c ^ p[i]];
    return c;
}

static uint16_t crc16_bytes(const uint8_t *p, size_t n)
{
    uint16_t c = 0;
    for (size_t i = 0; i < n; i++)
        c = (uint16_t)((c << 8) ^ crc16_tab[(c >> 8) ^ p[i]]);
    return c;
}

/* ------------------------------------------------------------------ */
/* MD5 (RFC 1321)                                                      */
/* ------------------------------------------------------------------ */
typedef struct {
    uint32_t h[4];
    uint64_t len;
    uint8_t buf[64];
    unsigned fill;
} md5_state;

static const uint32_t md5_K[64] = {
    0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a,
    0xa8304613, 0xfd469501, 0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be,
    0x6b901122, 0xfd987193, 0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340,
    0x265e5a51, 0xe9b6c7aa, 0xd62f105d, 0x02441453, 0xd8a1e681, 0xe7d3fbc8,
    0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed, 0xa9e3e905, 0xfcefa3f8,
    0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122, 0xfde5380c,
    0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa,
    0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665,
    0xf4292244, 0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92,
    0xffeff47d, 0x85845dd1, 0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1,
    0xf7537e82, 0xbd3af235, 0x2ad7d2bb, 0xeb86d391};
static const uint8_t md5_R[64] = {
    7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22, 7, 12, 17, 22,
    5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20, 5, 9,  14, 20,
    4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23, 4, 11, 16, 23,
    6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21, 6, 10, 15, 21};

static void md5_block(uint32_t h[4], const uint8_t *p)
{
    uint32_t w[16];
    for (int i = 0; i < 16; i++)
        w[i] = (uint32_t)p[4 * i] | ((uint32_t)p[4 * i + 1] << 8) |
               ((uint32_t)p[4 * i + 2] << 16) | ((uint32_t)p[4 * i + 3] << 24);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    for (int i = 0; i < 64; i++) {
        uint32_t f;
        int g;
        if (i < 16) {
            f = (b & c) | (~b & d);
            g = i;
        } else if (i < 32) {
            f = (d & b) | (~d & c);
            g = (5 * i + 1) & 15;
        } else if (i < 48) {
            f = b ^ c ^ d;
            g = (3 * i + 5) & 15;
        } else {
            f = c ^ (b | ~d);
            g = (7 * i) & 15;
        }
        uint32_t t = a + f + md5_K[i] + w[g];
        a = d;
        d = c;
        c = b;
        b = b + ((t << md5_R[i]) | (t >> (32 - md5_R[i])));
    }
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

static void md5_begin(md5_state *s)
{
    s->h[0] = 0x67452301;
    s->h[1] = 0xefcdab89;
    s->h[2] = 0x98badcfe;
    s->h[3] = 0x10325476;
    s->len = 0;
    s->fill = 0;
}

static void md5_feed(md5_state *s, const uint8_t *p, size_t n)
{
    s->len += n;
    while (n) {
        unsigned take = 64 - s->fill;
        if (take > n)
            take = (unsigned)n;
        memcpy(s->buf + s->fill, p, take);
        s->fill += take;
        p += take;
        n -= take;
        if (s->fill == 64) {
            md5_block(s->h, s->buf);
            s->fill = 0;
        }
    }
}

static void md5_end(md5_state *s, uint8_t out[16])
{
    uint64_t bits = s->len * 8;
    uint8_t pad = 0x80;
    md5_feed(s, &pad, 1);
    pad = 0;
    while (s->fill != 56)
        md5_feed(s, &pad, 1);
    uint8_t lenle[8];
    for (int i = 0; i < 8; i++)
        lenle[i] = (uint8_t)(bits >> (8 * i));
    md5_feed(s, lenle, 8);
    for (int i = 0; i < 4; i++)
        for (int j = 0; j < 4; j++)
            out[4 * i + j] = (uint8_t)(s->h[i] >> (8 * j));
}

static void md5_pcm(md5_state *s, const int32_t *pcm, size_t nsamples,
                    unsigned bps)
{
    uint8_t tmp[4096];
    unsigned bytes = bps / 8;
    size_t fill = 0;
    /* FrameList.to_bytes saturates out-of-range samples (src/pcm.c:1826-1948) */
    const int32_t hi = bps >= 1 && bps <= 31 ? (int32_t)((1u << (bps - 1)) - 1u) : INT32_MAX;
    const int32_t lo = -hi - 1;
    for (size_t i = 0; i < nsamples; i++) {
        uint32_t v = (uint32_t)(pcm[i] > hi ? hi : (pcm[i] < lo ? lo : pcm[i]));
        for (unsigned b = 0; b < bytes; b++)
            tmp[fill++] = (uint8_t)(v >> (8 * b));
        if (fill + 4 > sizeof(tmp)) {
            md5_feed(s, tmp, fill);
            fill = 0;
        }
    }
    md5_feed(s, tmp, fill);
}

void flacport_pcm_md5(const int32_t *pcm, uint64_t pcm_frames,
                      uint32_t channels, uint32_t bits_per_sample,
                      uint8_t digest[16])
{
    md5_state s;
    md5_begin(&s);
    md5_pcm(&s, pcm, (size_t)(pcm_frames * channels), bits_per_sample);
    md5_end(&s, digest);
}

/* ------------------------------------------------------------------ */
/* MSB-first bit writer over a caller buffer                           */
/* ------------------------------------------------------------------ */
typedef struct {
    uint8_t *buf;
    size_t cap;  /* bytes */
    uint64_t pos; /* bits written */
    int overflow;
} bitw;

static void bw_put(bitw *w, unsigned count, uint32_t value)
{
    /* count <= 32; value's low `count` bits are written MSB first */
    for (unsigned i = count; i-- > 0;) {
        uint64_t byte = w->pos >> 3;
        if (byte >= w->cap) {
            w->overflow = 1;
            return;
        }
        if ((w->pos & 7) == 0)
            w->buf[byte] = 0;
        if ((value >> i) & 1u)
            w->buf[byte] |= (uint8_t)(0x80u >> (w->pos & 7));
        w->pos++;
    }
}

static void bw_put_signed(bitw *w, unsigned count, int32_t value)
{
    /* two's complement in `count` bits (bitstream.c:2021-2035) */
    uint32_t mask = count >= 32 ? 0xFFFFFFFFu : ((1u << count) - 1u);
    bw_put(w, count, (uint32_t)value & mask);
}

static void bw_put_zeros(bitw *w, uint64_t n)
{
    while (n > 32) {
        bw_put(w, 32, 0);
        n -= 32;
    }
    bw_put(w, (unsigned)n, 0);
}

static void bw_align(bitw *w)
{
    if (w->pos & 7)
        bw_put(w, 8 - (unsigned)(w->pos & 7), 0);
}

/* ------------------------------------------------------------------ */
/* Encoder                                                             */
/* ------------------------------------------------------------------ */
enum { SF_CONSTANT = 0, SF_VERBATIM = 1, SF_FIXED = 2, SF_LPC = 3 };

#define MAX_LPC 32
#define MAX_PART_ORDER 15

typedef struct {
    unsigned porder;
    unsigned method;
    uint8_t rice[1u << MAX_PART_ORDER];
    uint32_t bits; /* exact bits of the whole residual section */
} resid_plan;

typedef struct {
    int type;
    unsigned bps;    /* subframe bits per sample (bps or bps+1 for side) */
    unsigned wasted;
    unsigned order;
    unsigned precision;
    int shift;
    int32_t coef[MAX_LPC];
    resid_plan res;
    uint32_t bits;   /* exact bits of the whole subframe */
} subframe_plan;

typedef struct {
    const flacport_options *o;
    unsigned qlp_precision;
    unsigned max_rice;
    /* window cache (reference caches per block length, flac.c:1139) */
    unsigned win_len;
    double *win;
    double *xw;
    int32_t *shifted;
    int32_t *resid;
    int32_t *tmp_resid;
    uint8_t rice_tmp[1u << MAX_PART_ORDER];
    uint8_t rice_best[1u << MAX_PART_ORDER];
    resid_plan cand_res;
} enc_ctx;

static void copy_res(resid_plan *d, const resid_plan *s)
{
    d->porder = s->porder;
    d->method = s->method;
    d->bits = s->bits;
    memcpy(d->rice, s->rice, 1u << s->porder);
}

static void copy_plan(subframe_plan *d, const subframe_plan *s)
{
    d->type = s->type;
    d->bps = s->bps;
    d->wasted = s->wasted;
    d->order = s->order;
    d->precision = s->precision;
    d->shift = s->shift;
    memcpy(d->coef, s->coef, sizeof(d->coef));
    d->bits = s->bits;
    copy_res(&d->res, &s->res);
}

static unsigned wasted_field_bits(unsigned w)
{
    return w ? w + 1 : 1;
}

static uint32_t zigzag(int32_t v)
{
    return ((uint32_t)v << 1) ^ (uint32_t)(v >> 31);
}

/* flacenc_encode_residuals + flacenc_encode_residual_partitions
   (flac.c:1326-1505): estimate every partition order, keep the smallest
   estimate (strict <), then count the exact bits the writer would emit. */
static void plan_residuals(enc_ctx *e, const int32_t *r, unsigned n_res,
                           unsigned block_size, unsigned order,
                           resid_plan *out)
{
    const unsigned max_po = e->o->max_residual_partition_order;
    uint64_t best_total = UINT64_MAX;
    unsigned best_p = 0;

    for (unsigned p = 0; p <= max_po && p <= MAX_PART_ORDER; p++) {
        if (block_size % (1u << p))
            break;
        uint64_t total = 0;
        unsigned pos = 0;
        for (unsigned part = 0; part < (1u << p); part++) {
            uint32_t plen = (part == 0) ? (block_size >> p) - order
                                        : (block_size >> p);
            unsigned take = plen < n_res - pos ? plen : n_res - pos;
            uint64_t sum = 0;
            for (unsigned i = 0; i < take; i++) {
                int32_t v = r[pos + i];
                if (v >= 0)
                    sum += (uint64_t)v;
                else
                    sum -= (uint64_t)(int64_t)v;
            }
            pos += take;
            unsigned k = 0;
            while ((uint64_t)(uint32_t)(plen << k) < sum) {
                if (k < e->max_rice)
                    k++;
                else
                    break;
            }
            if (k > 0)
                total += 4 + (sum >> (k - 1)) +
                         (uint64_t)(uint32_t)((1 + k) * plen) -
                         (uint64_t)(plen / 2);
            else
                total += 4 + (sum << 1) + (uint64_t)plen - (uint64_t)(plen / 2);
            e->rice_tmp[part] = (uint8_t)k;
        }
        if (total < best_total) {
            best_total = total;
            best_p = p;
            memcpy(e->rice_best, e->rice_tmp, 1u << p);
        }
    }

    unsigned maxk = 0;
    for (unsigned part = 0; part < (1u << best_p); part++)
        if (e->rice_best[part] > maxk)
            maxk = e->rice_best[part];

    out->porder = best_p;
    out->method = maxk > 14 ? 1 : 0;
    memcpy(out->rice, e->rice_best, 1u << best_p);

    uint32_t bits = 2 + 4;
    unsigned pos = 0;
    for (unsigned part = 0; part < (1u << best_p); part++) {
        uint32_t plen = (part == 0) ? (block_size >> best_p) - order
                                    : (block_size >> best_p);
        unsigned take = plen < n_res - pos ? plen : n_res - pos;
        unsigned k = out->rice[part];
        bits += out->method ? 5 : 4;
        for (unsigned i = 0; i < take; i++)
            bits += (zigzag(r[pos + i]) >> k) + 1 + k;
        pos += take;
    }
    out->bits = bits;
}

static void emit_residuals(bitw *w, const resid_plan *rp, const int32_t *r,
                           unsigned n_res, unsigned block_size,
                           unsigned order)
{
    bw_put(w, 2, rp->method);
    bw_put(w, 4, rp->porder);
    unsigned pos = 0;
    for (unsigned part = 0; part < (1u << rp->porder); part++) {
        uint32_t plen = (part == 0) ? (block_size >> rp->porder) - order
                                    : (block_size >> rp->porder);
        unsigned take = plen < n_res - pos ? plen : n_res - pos;
        unsigned k = rp->rice[part];
        bw_put(w, rp->method ? 5 : 4, k);
        for (unsigned i = 0; i < take; i++) {
            uint32_t u = zigzag(r[pos + i]);
            uint32_t msb = u >> k;
            bw_put_zeros(w, msb);
            bw_put(w, 1, 1);
            if (k)
                bw_put(w, k, u & ((1u << k) - 1u));
        }
        pos += take;
    }
}

/* residual of an integer predictor: r[i] = s[i+o] - (sum_j c_j s[i+o-j-1]) >> shift
   with a 64-bit accumulator (flac.c:999-1008) */
static void lpc_residual(const int32_t *s, unsigned n, unsigned order,
                         const int32_t *coef, int shift, int32_t *r)
{
    for (unsigned i = order; i < n; i++) {
        int64_t acc = 0;
        for (unsigned j = 0; j < order; j++)
            acc += (int64_t)coef[j] * (int64_t)s[i - j - 1];
        acc >>= shift;
        r[i - order] = (int32_t)((uint32_t)s[i] - (uint32_t)(int32_t)acc);
    }
}

/* k-th order fixed difference of s at position i (int wrap arithmetic,
   equals the iterated differences of flacenc_next_fixed_order) */
static int32_t fixed_diff(const int32_t *s, unsigned i, unsigned k)
{
    uint32_t a = (uint32_t)s[i];
    switch (k) {
    case 0:
        return (int32_t)a;
    case 1:
        return (int32_t)(a - (uint32_t)s[i - 1]);
    case 2:
        return (int32_t)(a - 2u * (uint32_t)s[i - 1] + (uint32_t)s[i - 2]);
    case 3:
        return (int32_t)(a - 3u * (uint32_t)s[i - 1] + 3u * (uint32_t)s[i - 2] -
                         (uint32_t)s[i - 3]);
    default:
        return (int32_t)(a - 4u * (uint32_t)s[i - 1] + 6u * (uint32_t)s[i - 2] -
                         4u * (uint32_t)s[i - 3] + (uint32_t)s[i - 4]);
    }
}

static uint64_t int_abs_u64(int32_t v)
{
    /* accumulator += abs(int) : abs(INT_MIN) stays negative (flac.c:1628) */
    int32_t a = (int32_t)(v < 0 ? 0u - (uint32_t)v : (uint32_t)v);
    return (uint64_t)(int64_t)a;
}

static void plan_fixed(enc_ctx *e, const int32_t *s, unsigned n, unsigned bps,
                       unsigned wasted, subframe_plan *sp)
{
    unsigned best = 0;
    uint64_t best_sum = 0;
    for (unsigned i = 4; i < n; i++)
        best_sum += int_abs_u64(s[i]);
    if (n > 4) {
        for (unsigned k = 1; k <= 4; k++) {
            uint64_t sum = 0;
            for (unsigned i = 4; i < n; i++)
                sum += int_abs_u64(fixed_diff(s, i, k));
            if (sum < best_sum) {
                best_sum = sum;
                best = k;
            }
        }
    }
    for (unsigned i = best; i < n; i++)
        e->resid[i - best] = fixed_diff(s, i, best);

    sp->type = SF_FIXED;
    sp->order = best;
    plan_residuals(e, e->resid, n - best, n, best, &sp->res);
    sp->bits = 7 + wasted_field_bits(wasted) + best * (bps - wasted) +
               sp->res.bits;
}

static void tukey_window(enc_ctx *e, unsigned N)
{
    if (e->win_len == N)
        return;
    const double alpha = 0.5;
    const unsigned window1 = (unsigned)(alpha * (N - 1)) / 2;
    const unsigned window2 = (unsigned)((N - 1) * (1.0 - (alpha / 2.0)));
    for (unsigned n = 0; n < N; n++) {
        if (n <= window1)
            e->win[n] = 0.5 * (1.0 + cos(M_PI * (((2 * n) / (alpha * (N - 1))) -
                                                 1.0)));
        else if (n <= window2)
            e->win[n] = 1.0;
        else
            e->win[n] = 0.5 * (1.0 + cos(M_PI * (((2.0 * n) / (alpha * (N - 1))) -
                                                 (2.0 / alpha) + 1.0)));
    }
    e->win_len = N;
}

/* x86 cvttsd2si semantics for (int)double: NaN / out of range -> INT_MIN */
static int32_t d2i_x86(double x)
{
    if (!(x > -2147483649.0 && x < 2147483648.0))
        return INT32_MIN;
    return (int32_t)x;
}

static void quantize(const double *lp, unsigned order, unsigned prec,
                     int32_t *q, int *shift_out)
{
    double l = DBL_MIN;
    int log2cmax;
    for (unsigned i = 0; i < order; i++) {
        double a = fabs(lp[i]);
        l = a > l ? a : l;
    }
    frexp(l, &log2cmax);
    int shift = (int)(prec - 1) - (log2cmax - 1) - 1;
    if (shift < -16)
        shift = -16;
    if (shift > 15)
        shift = 15;
    const int qmax = (1 << (prec - 1)) - 1;
    const int qmin = -(1 << (prec - 1));
    double err = 0.0;
    for (unsigned i = 0; i < order; i++) {
        if (shift >= 0)
            err += lp[i] * (1 << shift);
        else
            err += lp[i] / (1 << -shift);
        int32_t ei = d2i_x86(round(err));
        q[i] = ei < qmin ? qmin : (ei > qmax ? qmax : ei);
        err -= (double)ei;
    }
    *shift_out = shift >= 0 ? shift : 0;
}

static unsigned estimate_order(unsigned bps, unsigned prec, unsigned max_order,
                               unsigned N, const double *err)
{
    const double error_scale = (M_LN2 * M_LN2) / ((double)N * 2.0);
    unsigned best = 0;
    double best_bits = DBL_MAX;
    for (unsigned i = 0; i < max_order; i++) {
        unsigned order = i + 1;
        if (err[i] > 0.0) {
            unsigned header = order * (bps + prec);
            double bpr = log(err[i] * error_scale) / (M_LN2 * 2);
            bpr = bpr > 0.0 ? bpr : 0.0;
            double est = header + bpr * (N - order);
            if (est < best_bits) {
                best = order;
                best_bits = est;
            }
        } else {
            return order;
        }
    }
    return best;
}

static uint32_t lpc_header_bits(unsigned order, unsigned bps, unsigned wasted,
                                unsigned prec)
{
    return 7 + wasted_field_bits(wasted) + order * (bps - wasted) + 4 + 5 +
           order * prec;
}

static void plan_lpc(enc_ctx *e, const int32_t *s, unsigned N, unsigned bps,
                     unsigned wasted, subframe_plan *sp)
{
    const unsigned maxo = e->o->max_lpc_order;
    sp->type = SF_LPC;

    if (N > maxo + 1) {
        double R[MAX_LPC + 1];
        double lp[MAX_LPC][MAX_LPC];
        double err[MAX_LPC];

        tukey_window(e, N);
        for (unsigned n = 0; n < N; n++)
            e->xw[n] = s[n] * e->win[n];
        for (unsigned lag = 0; lag <= maxo; lag++) {
            double acc = 0.0;
            for (unsigned i = 0; i < N - lag; i++)
                acc += e->xw[i] * e->xw[i + lag];
            R[lag] = acc;
        }
        /* Levinson-Durbin (flac.c:1190-1231) */
        double k = R[1] / R[0];
        lp[0][0] = k;
        err[0] = R[0] * (1.0 - (k * k));
        for (unsigned i = 1; i < maxo; i++) {
            double q = R[i + 1];
            for (unsigned j = 0; j < i; j++)
                q -= (lp[i - 1][j] * R[i - j]);
            k = q / err[i - 1];
            for (unsigned j = 0; j < i; j++)
                lp[i][j] = lp[i - 1][j] - (k * lp[i - 1][i - j - 1]);
            lp[i][i] = k;
            err[i] = err[i - 1] * (1.0 - (k * k));
        }

        sp->precision = e->qlp_precision;
        if (!e->o->exhaustive_model_search) {
            unsigned order = estimate_order(bps, e->qlp_precision, maxo, N, err);
            sp->order = order;
            quantize(lp[order - 1], order, e->qlp_precision, sp->coef,
                     &sp->shift);
            lpc_residual(s, N, order, sp->coef, sp->shift, e->resid);
            plan_residuals(e, e->resid, N - order, N, order, &sp->res);
        } else {
            uint32_t best_bits = UINT32_MAX;
            int32_t cq[MAX_LPC];
            int cshift;
            for (unsigned order = 1; order <= maxo; order++) {
                quantize(lp[order - 1], order, e->qlp_precision, cq, &cshift);
                lpc_residual(s, N, order, cq, cshift, e->tmp_resid);
                plan_residuals(e, e->tmp_resid, N - order, N, order,
                               &e->cand_res);
                uint32_t bits = lpc_header_bits(order, bps, wasted,
                                                e->qlp_precision) +
                                e->cand_res.bits;
                if (bits < best_bits) {
                    best_bits = bits;
                    sp->order = order;
                    sp->shift = cshift;
                    memcpy(sp->coef, cq, sizeof(int32_t) * order);
                    copy_res(&sp->res, &e->cand_res);
                }
            }
        }
    } else {
        sp->order = 1;
        sp->coef[0] = 1;
        sp->precision = 2;
        sp->shift = 0;
        lpc_residual(s, N, 1, sp->coef, 0, e->resid);
        plan_residuals(e, e->resid, N - 1, N, 1, &sp->res);
    }
    sp->bits = lpc_header_bits(sp->order, bps, wasted, sp->precision) +
               sp->res.bits;
}

static int all_identical(const int32_t *s, unsigned n)
{
    for (unsigned i = 1; i < n; i++)
        if (s[i] != s[0])
            return 0;
    return 1;
}

static unsigned wasted_bits(const int32_t *s, unsigned n)
{
    uint32_t acc = 0;
    for (unsigned i = 0; i < n; i++)
        acc |= (uint32_t)s[i];
    if (!acc)
        return 0;
    unsigned w = 0;
    while (!(acc & 1u)) {
        acc >>= 1;
        w++;
    }
    return w;
}

/* flacenc_write_subframe (flac.c:673-811) as a plan */
static void plan_subframe(enc_ctx *e, const int32_t *samples, unsigned N,
                          unsigned bps, subframe_plan *out,
                          int32_t *shifted_out)
{
    const flacport_options *o = e->o;
    const int try_verbatim = !o->disable_verbatim_subframes;
    const int try_constant = !o->disable_constant_subframes;
    const int try_fixed = !o->disable_fixed_subframes;
    const int try_lpc = !(o->disable_lpc_subframes || o->max_lpc_order == 0);

    out->bps = bps;
    if (try_constant && all_identical(samples, N)) {
        out->type = SF_CONSTANT;
        out->wasted = 0;
        out->bits = 8 + bps;
        shifted_out[0] = samples[0];
        return;
    }
    unsigned w = wasted_bits(samples, N);
    for (unsigned i = 0; i < N; i++)
        shifted_out[i] = samples[i] >> w;
    out->wasted = w;

    static __thread subframe_plan fixed, lpc;
    uint32_t verbatim_bits = INT_MAX;
    if (try_fixed)
        plan_fixed(e, shifted_out, N, bps, w, &fixed);
    if (try_lpc)
        plan_lpc(e, shifted_out, N, bps, w, &lpc);
    if (try_verbatim)
        verbatim_bits = (bps - w) * N;

    int pick; /* SF_FIXED / SF_LPC / SF_VERBATIM */
    if (try_fixed && try_lpc && try_verbatim) {
        uint32_t m = lpc.bits < verbatim_bits ? lpc.bits : verbatim_bits;
        if (fixed.bits < m)
            pick = SF_FIXED;
        else if (lpc.bits < verbatim_bits)
            pick = SF_LPC;
        else
            pick = SF_VERBATIM;
    } else if (!try_fixed && !try_lpc) {
        pick = SF_VERBATIM;
    } else if (try_fixed && !try_lpc && !try_verbatim) {
        pick = SF_FIXED;
    } else if (!try_fixed && try_lpc && !try_verbatim) {
        pick = SF_LPC;
    } else if (try_fixed && try_lpc && !try_verbatim) {
        pick = fixed.bits < lpc.bits ? SF_FIXED : SF_LPC;
    } else if (try_fixed && !try_lpc && try_verbatim) {
        pick = fixed.bits < verbatim_bits ? SF_FIXED : SF_VERBATIM;
    } else {
        pick = lpc.bits < verbatim_bits ? SF_LPC : SF_VERBATIM;
    }

    if (pick == SF_FIXED) {
        copy_plan(out, &fixed);
    } else if (pick == SF_LPC) {
        copy_plan(out, &lpc);
    } else {
        out->type = SF_VERBATIM;
        out->bits = 7 + wasted_field_bits(w) + (bps - w) * N;
    }
    out->bps = bps;
    out->wasted = w;
}

static void emit_subframe_header(bitw *w, unsigned type_code, unsigned wasted)
{
    bw_put(w, 1, 0);
    bw_put(w, 6, type_code);
    if (wasted) {
        bw_put(w, 1, 1);
        bw_put_zeros(w, wasted - 1);
        bw_put(w, 1, 1);
    } else {
        bw_put(w, 1, 0);
    }
}

static void emit_subframe(enc_ctx *e, bitw *w, const subframe_plan *sp,
                          const int32_t *s, unsigned N)
{
    const unsigned sbps = sp->bps - sp->wasted;
    switch (sp->type) {
    case SF_CONSTANT:
        emit_subframe_header(w, 0, 0);
        bw_put_signed(w, sp->bps, s[0]);
        break;
    case SF_VERBATIM:
        emit_subframe_header(w, 1, sp->wasted);
        for (unsigned i = 0; i < N; i++)
            bw_put_signed(w, sbps, s[i]);
        break;
    case SF_FIXED:
        emit_subframe_header(w, 8 | sp->order, sp->wasted);
        for (unsigned i = 0; i < sp->order; i++)
            bw_put_signed(w, sbps, s[i]);
        for (unsigned i = sp->order; i < N; i++)
            e->resid[i - sp->order] = fixed_diff(s, i, sp->order);
        emit_residuals(w, &sp->res, e->resid, N - sp->order, N, sp->order);
        break;
    default:
        emit_subframe_header(w, 32 | (sp->order - 1), sp->wasted);
        for (unsigned i = 0; i < sp->order; i++)
            bw_put_signed(w, sbps, s[i]);
        bw_put(w, 4, sp->precision - 1);
        bw_put_signed(w, 5, sp->shift);
        for (unsigned i = 0; i < sp->order; i++)
            bw_put_signed(w, sp->precision, sp->coef[i]);
        lpc_residual(s, N, sp->order, sp->coef, sp->shift, e->resid);
        emit_residuals(w, &sp->res, e->resid, N - sp->order, N, sp->order);
        break;
    }
}

static void emit_utf8(bitw *w, uint32_t v)
{
    if (v <= 0x7F) {
        bw_put(w, 8, v);
        return;
    }
    unsigned nbytes = v <= 0x7FF ? 2 : v <= 0xFFFF ? 3 : v <= 0x1FFFFF ? 4
                    : v <= 0x3FFFFFF ? 5 : 6;
    int shift = (int)(nbytes - 1) * 6;
    /* nbytes ones, a zero, then the leading value bits */
    bw_put(w, nbytes + 1, ((1u << nbytes) - 1u) << 1);
    bw_put(w, 7 - nbytes, v >> shift);
    for (shift -= 6; shift >= 0; shift -= 6) {
        bw_put(w, 2, 2);
        bw_put(w, 6, (v >> shift) & 0x3F);
    }
}

static void emit_frame_header(bitw *w, unsigned block_size, unsigned rate,
                              unsigned bps, unsigned assignment,
                              uint32_t frame_number)
{
    unsigned bs_code, sr_code, bps_code;
    switch (block_size) {
    case 192: bs_code = 1; break;
    case 576: bs_code = 2; break;
    case 1152: bs_code = 3; break;
    case 2304: bs_code = 4; break;
    case 4608: bs_code = 5; break;
    case 256: bs_code = 8; break;
    case 512: bs_code = 9; break;
    case 1024: bs_code = 10; break;
    case 2048: bs_code = 11; break;
    case 4096: bs_code = 12; break;
    case 8192: bs_code = 13; break;
    case 16384: bs_code = 14; break;
    case 32768: bs_code = 15; break;
    default:
        bs_code = block_size <= 0xFF ? 6 : (block_size <= 0xFFFF ? 7 : 0);
    }
    switch (rate) {
    case 88200: sr_code = 1; break;
    case 176400: sr_code = 2; break;
    case 192000: sr_code = 3; break;
    case 8000: sr_code = 4; break;
    case 16000: sr_code = 5; break;
    case 22050: sr_code = 6; break;
    case 24000: sr_code = 7; break;
    case 32000: sr_code = 8; break;
    case 44100: sr_code = 9; break;
    case 48000: sr_code = 10; break;
    case 96000: sr_code = 11; break;
    default:
        if (rate <= 255000 && rate % 1000 == 0)
            sr_code = 12;
        else if (rate <= 655350 && rate % 10 == 0)
            sr_code = 14;
        else if (rate <= 0xFFFF)
            sr_code = 13;
        else
            sr_code = 0;
    }
    switch (bps) {
    case 8: bps_code = 1; break;
    case 12: bps_code = 2; break;
    case 16: bps_code = 4; break;
    case 20: bps_code = 5; break;
    case 24: bps_code = 6; break;
    default: bps_code = 0;
    }
    uint64_t start = w->pos;
    bw_put(w, 14, 0x3FFE);
    bw_put(w, 2, 0);
    bw_put(w, 4, bs_code);
    bw_put(w, 4, sr_code);
    bw_put(w, 4, assignment);
    bw_put(w, 3, bps_code);
    bw_put(w, 1, 0);
    emit_utf8(w, frame_number);
    if (bs_code == 6)
        bw_put(w, 8, block_size - 1);
    else if (bs_code == 7)
        bw_put(w, 16, block_size - 1);
    if (sr_code == 12)
        bw_put(w, 8, rate / 1000);
    else if (sr_code == 13)
        bw_put(w, 16, rate);
    else if (sr_code == 14)
        bw_put(w, 16, rate / 10);
    /* header is always byte aligned here */
    bw_put(w, 8, w->overflow ? 0 : crc8_bytes(w->buf + (start >> 3),
                                              (size_t)((w->pos - start) >> 3)));
}

/* one frame; returns frame byte count */
static int encode_frame(enc_ctx *e, bitw *w, const int32_t *pcm, unsigned N,
                        unsigned channels, unsigned bps, unsigned rate,
                        uint32_t frame_number, int32_t **chan, int32_t **shifted,
                        subframe_plan *plans)
{
    const flacport_options *o = e->o;
    uint64_t start = w->pos;
    for (unsigned c = 0; c < channels; c++)
        for (unsigned i = 0; i < N; i++)
            chan[c][i] = pcm[(size_t)i * channels + c];

    if (channels == 2 && (o->mid_side || o->adaptive_mid_side)) {
        /* chan[2] = average, chan[3] = difference (flac.c:1507-1529) */
        for (unsigned i = 0; i < N; i++) {
            chan[2][i] = (int32_t)((int64_t)chan[0][i] + chan[1][i]) >> 1;
            chan[3][i] = (int32_t)((uint32_t)chan[0][i] - (uint32_t)chan[1][i]);
        }
        for (unsigned c = 0; c < 4; c++)
            plan_subframe(e, chan[c], N, c == 3 ? bps + 1 : bps, &plans[c],
                          shifted[c]);
        const uint32_t L = plans[0].bits, R = plans[1].bits, A = plans[2].bits,
                       D = plans[3].bits;
        unsigned assign, s0, s1;
        if (o->mid_side) {
            uint32_t m = L + D < D + R ? L + D : D + R;
            m = m < A + D ? m : A + D;
            if (L + R < m) {
                assign = 1; s0 = 0; s1 = 1;
            } else if (L < (R < A ? R : A)) {
                assign = 8; s0 = 0; s1 = 3;
            } else if (R < A) {
                assign = 9; s0 = 3; s1 = 1;
            } else {
                assign = 10; s0 = 2; s1 = 3;
            }
        } else if (L + R < A + D) {
            assign = 1; s0 = 0; s1 = 1;
        } else {
            assign = 10; s0 = 2; s1 = 3;
        }
        emit_frame_header(w, N, rate, bps, assign, frame_number);
        emit_subframe(e, w, &plans[s0], shifted[s0], N);
        emit_subframe(e, w, &plans[s1], shifted[s1], N);
    } else {
        emit_frame_header(w, N, rate, bps, channels - 1, frame_number);
        for (unsigned c = 0; c < channels; c++) {
            plan_subframe(e, chan[c], N, bps, &plans[0], shifted[0]);
            emit_subframe(e, w, &plans[0], shifted[0], N);
        }
    }
    bw_align(w);
    if (w->overflow)
        return -1;
    uint16_t crc = crc16_bytes(w->buf + (start >> 3),
                               (size_t)((w->pos - start) >> 3));
    bw_put(w, 16, crc);
    return w->overflow ? -1 : (int)((w->pos - start) >> 3);
}

size_t flacport_max_stream_bytes(uint64_t pcm_frames, uint32_t channels,
                                 uint32_t bits_per_sample, uint32_t block_size,
                                 uint32_t padding_size)
{
    uint64_t nframes = block_size ? (pcm_frames + block_size - 1) / block_size : 0;
    /* verbatim worst case (+1 bit side channel) plus headers */
    uint64_t per_frame = 32 + (uint64_t)channels *
                         (8 + ((uint64_t)block_size * (bits_per_sample + 1) + 7) / 8 + 4);
    return (size_t)(4 + 4 + 34 + 4 + 8 + sizeof(VENDOR_STRING) + 4 + padding_size +
                    nframes * per_frame + 64);
}

static void put_u24(uint8_t *p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 16);
    p[1] = (uint8_t)(v >> 8);
    p[2] = (uint8_t)v;
}

static void write_streaminfo(uint8_t *p, uint32_t block_size, uint32_t min_fs,
                             uint32_t max_fs, uint32_t rate, uint32_t channels,
                             uint32_t bps, uint64_t total, const uint8_t md5[16])
{
    bitw w = {p, 34, 0, 0};
    uint32_t bs = block_size > 0xFFFF ? 0xFFFF : block_size;
    bw_put(&w, 16, bs);
    bw_put(&w, 16, bs);
    bw_put(&w, 24, min_fs > 0xFFFFFF ? 0xFFFFFF : min_fs);
    bw_put(&w, 24, max_fs > 0xFFFFFF ? 0xFFFFFF : max_fs);
    bw_put(&w, 20, rate > 0xFFFFF ? 0xFFFFF : rate);
    bw_put(&w, 3, channels - 1 > 7 ? 7 : channels - 1);
    bw_put(&w, 5, bps - 1 > 31 ? 31 : bps - 1);
    bw_put(&w, 4, (uint32_t)(total >> 32) & 0xF);
    bw_put(&w, 32, (uint32_t)total);
    memcpy(p + 18, md5, 16);
}

int flacport_encode(const int32_t *pcm, uint64_t pcm_frames,
                    uint32_t channels, uint32_t bits_per_sample,
                    uint32_t sample_rate, const flacport_options *opts,
                    uint8_t *out, size_t out_cap, size_t *out_len,
                    uint64_t *frame_offsets, uint32_t *frame_lengths,
                    size_t max_frames, size_t *n_frames)
{
    return flacport_encode_sizes(pcm, pcm_frames, channels, bits_per_sample,
                                 sample_rate, opts, NULL, 0, out, out_cap, out_len,
                                 frame_offsets, frame_lengths, max_frames, n_frames);
}

int flacport_encode_sizes(const int32_t *pcm, uint64_t pcm_frames,
                          uint32_t channels, uint32_t bits_per_sample,
                          uint32_t sample_rate, const flacport_options *opts,
                          const uint32_t *read_sizes, size_t n_read_sizes,
                          uint8_t *out, size_t out_cap, size_t *out_len,
                          uint64_t *frame_offsets, uint32_t *frame_lengths,
                          size_t max_frames, size_t *n_frames)
{
    crc_init();
    if (!opts || channels < 1 || channels > 8 || opts->block_size == 0 ||
        opts->max_lpc_order > MAX_LPC ||
        opts->max_residual_partition_order > MAX_PART_ORDER)
        return -1;
    /* N = the block_size option: it derives qlp precision and STREAMINFO's
       min/max block size (flac.c:164-178, 193-194).  A frame holds whatever
       one read() returned (flac.c:244-274), so the scratch buffers are sized
       for the largest listed read; a listed 0 is an empty read and ends the
       stream, as the reference's `while (samples->_[0]->len > 0)`. */
    const unsigned N = opts->block_size;
    unsigned NA = N;
    for (size_t i = 0; i < n_read_sizes; i++) {
        if (read_sizes[i] > 0xFFFF)
            return -1;  /* a frame header holds at most a 16-bit size */
        if (read_sizes[i] > NA)
            NA = read_sizes[i];
    }
    const size_t vlen = strlen(VENDOR_STRING);
    const size_t head = 4 + 4 + 34 + 4 + 4 + vlen + 4 + 4 + opts->padding_size;
    if (out_cap < head)
        return -2;

    enc_ctx e;
    memset(&e, 0, sizeof(e));
    e.o = opts;
    e.qlp_precision = N <= 192 ? 7 : N <= 384 ? 8 : N <= 576 ? 9 : N <= 1152 ? 10
                    : N <= 2304 ? 11 : N <= 4608 ? 12 : 13;
    e.max_rice = bits_per_sample <= 16 ? 14 : 30;
    e.win = malloc(sizeof(double) * NA);
    e.xw = malloc(sizeof(double) * NA);
    e.resid = malloc(sizeof(int32_t) * (NA + 1));
    e.tmp_resid = malloc(sizeof(int32_t) * (NA + 1));
    int32_t *chan_mem = malloc(sizeof(int32_t) * NA * (channels + 4));
    int32_t *shift_mem = malloc(sizeof(int32_t) * NA * 4);
    subframe_plan *plans = malloc(sizeof(subframe_plan) * 4);
    int32_t *chan[12], *shifted[4];
    for (unsigned c = 0; c < channels + 4 && c < 12; c++)
        chan[c] = chan_mem + (size_t)c * NA;
    for (unsigned c = 0; c < 4; c++)
        shifted[c] = shift_mem + (size_t)c * NA;

    /* stream header: fLaC, STREAMINFO, VORBIS_COMMENT, PADDING
       (flac.c:208-238) */
    uint8_t *p = out;
    memcpy(p, "fLaC", 4);
    p += 4;
    p[0] = 0x00;
    put_u24(p + 1, 34);
    p += 4;
    uint8_t *streaminfo = p;
    p += 34;
    p[0] = 0x04;
    put_u24(p + 1, (uint32_t)(4 + vlen + 4));
    p += 4;
    p[0] = (uint8_t)vlen; p[1] = (uint8_t)(vlen >> 8);
    p[2] = (uint8_t)(vlen >> 16); p[3] = (uint8_t)(vlen >> 24);
    p += 4;
    memcpy(p, VENDOR_STRING, vlen);
    p += vlen;
    memset(p, 0, 4);
    p += 4;
    p[0] = 0x81;
    put_u24(p + 1, opts->padding_size);
    p += 4;
    memset(p, 0, opts->padding_size);
    p += opts->padding_size;

    bitw w = {p, out_cap - (size_t)(p - out), 0, 0};
    uint32_t min_fs = 0xFFFFFF, max_fs = 0;
    uint64_t done = 0;
    size_t nf = 0;
    int rc = 0;
    md5_state md5;
    md5_begin(&md5);
    while (done < pcm_frames) {
        unsigned want = nf < n_read_sizes ? read_sizes[nf] : N;
        if (want == 0)
            break;
        unsigned n = (pcm_frames - done) < want ? (unsigned)(pcm_frames - done) : want;
        const int32_t *fp = pcm + done * channels;
        md5_pcm(&md5, fp, (size_t)n * channels, bits_per_sample);
        uint64_t off = w.pos >> 3;
        int bytes = encode_frame(&e, &w, fp, n, channels, bits_per_sample,
                                 sample_rate, (uint32_t)nf, chan, shifted, plans);
        if (bytes < 0) {
            rc = -3;
            break;
        }
        if (nf < max_frames) {
            if (frame_offsets)
                frame_offsets[nf] = off;
            if (frame_lengths)
                frame_lengths[nf] = n;
        }
        if ((uint32_t)bytes < min_fs)
            min_fs = (uint32_t)bytes;
        if ((uint32_t)bytes > max_fs)
            max_fs = (uint32_t)bytes;
        nf++;
        done += n;
    }
    uint8_t digest[16];
    md5_end(&md5, digest);
    write_streaminfo(streaminfo, N, min_fs, max_fs, sample_rate, channels,
                     bits_per_sample, done, digest);
    if (out_len)
        *out_len = (size_t)(p - out) + (size_t)(w.pos >> 3);
    if (n_frames)
        *n_frames = nf;

    free(e.win);
    free(e.xw);
    free(e.resid);
    free(e.tmp_resid);
    free(chan_mem);
    free(shift_mem);
    free(plans);
    return rc;
}

/* ------------------------------------------------------------------ */
/* Decoder: restatement of src/decoders/flac.c (python-audio-tools     */
/* 2.22alpha1), error for error.  Codes (FD_*) are the reference's     */
/* flac_status values (src/decoders/flac.h:68-81) extended with the    */
/* conditions FlacDecoder.read() raises itself (flac.c:204-265).       */
/* ------------------------------------------------------------------ */
typedef struct {
    const uint8_t *p;
    uint64_t len_bits;
    uint64_t pos; /* bits */
    int eof;      /* a read went past the end (br_abort -> IOError) */
} bitr;

static uint32_t br_get(bitr *r, unsigned n)
{
    /* bitstream->read(n) for n <= 32 (src/bitstream.c FUNC_READ_BITS) */
    uint32_t v = 0;
    for (unsigned i = 0; i < n; i++) {
        if (r->pos >= r->len_bits) {
            r->eof = 1;
            return 0;
        }
        v = (v << 1) | ((r->p[r->pos >> 3] >> (7 - (r->pos & 7))) & 1u);
        r->pos++;
    }
    return v;
}

static int32_t br_get_signed(bitr *r, unsigned n)
{
    /* br_read_signed_bits_be (src/bitstream.c:418-425): sign bit, then
       count-1 magnitude bits; count 0 asks for 2^32-1 bits -> EOF */
    if (n == 0) {
        br_get(r, 1);
        r->pos = r->len_bits;
        r->eof = 1;
        return 0;
    }
    if (n > 33) { /* reads beyond 32 bits keep the low 32: only EOF matters */
        r->pos += n;
        if (r->pos > r->len_bits) { r->pos = r->len_bits; r->eof = 1; }
        return 0;
    }
    uint32_t sign = br_get(r, 1);
    uint32_t v = n > 1 ? br_get(r, n - 1) : 0;
    return sign ? (int32_t)(v - (1u << (n - 1))) : (int32_t)v;
}

/* read_unary(stop): count bits != stop until a stop bit */
static uint32_t br_unary(bitr *r, unsigned stop)
{
    uint32_t n = 0;
    while (!r->eof && br_get(r, 1) != stop)
        n++;
    return n;
}

enum {
    FD_OK = 0, FD_ERROR = 1, FD_SYNC = 2, FD_RESERVED = 3, FD_BPS = 4, FD_RATE = 5,
    FD_HDR_CRC = 6, FD_RATE_MISMATCH = 7, FD_CH_MISMATCH = 8, FD_BPS_MISMATCH = 9,
    FD_MAXBS = 10, FD_CODING = 11, FD_FIXED_ORDER = 12, FD_SUBFRAME_TYPE = 13,
    FD_FRAME_CRC = 14, FD_EOF = 15, FD_MD5 = 16
};

#define FD_RET(r, code) return (r)->eof ? FD_EOF : (code)

typedef struct {
    unsigned block_size, sample_rate, assign, channels, bps;
    uint32_t frame_number;
} fd_header;

/* flacdec_read_frame_header (src/decoders/flac.c:710-851) */
static int fd_frame_header(bitr *r, const flacport_streaminfo *si, fd_header *h)
{
    const uint64_t start = r->pos;
    if (br_get(r, 14) != 0x3FFE) FD_RET(r, FD_SYNC);
    if (br_get(r, 1) != 0) FD_RET(r, FD_RESERVED);
    br_get(r, 1); /* blocking strategy */
    unsigned bs_bits = br_get(r, 4), sr_bits = br_get(r, 4);
    h->assign = br_get(r, 4);
    h->channels = (h->assign >= 8 && h->assign <= 10) ? 2 : h->assign + 1;
    switch (br_get(r, 3)) {
    case 0: h->bps = si->bits_per_sample; break;
    case 1: h->bps = 8; break;
    case 2: h->bps = 12; break;
    case 4: h->bps = 16; break;
    case 5: h->bps = 20; break;
    case 6: h->bps = 24; break;
    default: FD_RET(r, FD_BPS);
    }
    br_get(r, 1);
    /* read_utf8 (flac.c:1310-1320) */
    unsigned nbytes = br_unary(r, 0);
    if (nbytes > 7) { r->pos = r->len_bits; r->eof = 1; return FD_EOF; }
    uint32_t num = br_get(r, 7 - nbytes);
    for (; nbytes > 1; nbytes--)
        num = (num << 6) | (br_get(r, 8) & 0x3F);
    h->frame_number = num;
    static const unsigned bs_tab[16] = {0, 192, 576, 1152, 2304, 4608, 0, 0,
                                        256, 512, 1024, 2048, 4096, 8192, 16384, 32768};
    if (bs_bits == 0) h->block_size = si->max_block_size;
    else if (bs_bits == 6) h->block_size = br_get(r, 8) + 1;
    else if (bs_bits == 7) h->block_size = br_get(r, 16) + 1;
    else h->block_size = bs_tab[bs_bits];
    static const unsigned sr_tab[12] = {0, 88200, 176400, 192000, 8000, 16000,
                                        22050, 24000, 32000, 44100, 48000, 96000};
    if (sr_bits == 0) h->sample_rate = si->sample_rate;
    else if (sr_bits < 12) h->sample_rate = sr_tab[sr_bits];
    else if (sr_bits == 12) h->sample_rate = br_get(r, 8) * 1000;
    else if (sr_bits == 13) h->sample_rate = br_get(r, 16);
    else if (sr_bits == 14) h->sample_rate = br_get(r, 16) * 10;
    else FD_RET(r, FD_RATE);
    br_get(r, 8);
    if (r->eof) return FD_EOF;
    if (crc8_bytes(r->p + (start >> 3), (size_t)((r->pos - start) >> 3)) != 0)
        return FD_HDR_CRC;
    if (si->sample_rate != h->sample_rate) return FD_RATE_MISMATCH;
    if (si->channels != h->channels) return FD_CH_MISMATCH;
    if (si->bits_per_sample != h->bps) return FD_BPS_MISMATCH;
    if (h->block_size > si->max_block_size) return FD_MAXBS;
    return FD_OK;
}

/* flacdec_read_residual (flac.c:1135-1209): res[0 .. N-order) */
static int fd_residual(bitr *r, unsigned order, unsigned N, int32_t *res)
{
    const unsigned method = br_get(r, 2);
    const unsigned porder = br_get(r, 4);
    unsigned idx = 0;
    /* a partition order that does not divide the block leaves residuals the
       reference never reads (it would predict from a stale buffer); both
       engines reject such streams (decoder limits) */
    if (!r->eof && method <= 1 && ((N >> porder) << porder) != N)
        return FD_ERROR;
    for (unsigned part = 0; part < (1u << porder); part++) {
        int plen;
        if (part == 0) {
            plen = (int)(N / (1u << porder)) - (int)order;
            if (plen < 0) plen = 0;
        } else {
            plen = (int)(N / (1u << porder));
        }
        unsigned rice, esc;
        if (method == 0) {
            rice = br_get(r, 4);
            esc = rice == 0xF ? br_get(r, 5) : 0;
        } else if (method == 1) {
            rice = br_get(r, 5);
            esc = rice == 0x1F ? br_get(r, 5) : 0;
        } else {
            FD_RET(r, FD_CODING);
        }
        if (r->eof) return FD_EOF;
        if (!esc) {
            for (; plen; plen--) {
                const uint32_t msb = br_unary(r, 1);
                const uint32_t lsb = br_get(r, rice);
                const uint32_t value = (msb << rice) | lsb;
                const int32_t sv = (int32_t)value >> 1;
                res[idx++] = (value & 1u) ? -sv - 1 : sv;
                if (r->eof) return FD_EOF;
            }
        } else {
            for (; plen; plen--)
                res[idx++] = br_get_signed(r, esc);
        }
        if (r->eof) return FD_EOF;
    }
    return FD_OK;
}

/* flacdec_read_subframe and friends (flac.c:854-1132) */
static int fd_subframe(bitr *r, unsigned N, unsigned bps, int32_t *s, int32_t *res)
{
    br_get(r, 1); /* padding, unchecked */
    const unsigned t = br_get(r, 6);
    unsigned kind, order;
    if (t == 0) { kind = 0; order = 0; }
    else if (t == 1) { kind = 1; order = 0; }
    else if ((t & 0x38) == 0x08) { kind = 2; order = t & 7; }
    else if ((t & 0x20) == 0x20) { kind = 3; order = (t & 0x1F) + 1; }
    else FD_RET(r, FD_SUBFRAME_TYPE);
    unsigned wasted = 0;
    if (br_get(r, 1))
        wasted = br_unary(r, 1) + 1;
    if (r->eof) return FD_EOF;
    bps -= wasted; /* unsigned, as the reference */
    if (kind == 0) {
        const int32_t v = br_get_signed(r, bps);
        for (unsigned i = 0; i < N; i++) s[i] = v;
    } else if (kind == 1) {
        for (unsigned i = 0; i < N; i++) s[i] = br_get_signed(r, bps);
    } else if (kind == 2) {
        for (unsigned i = 0; i < order; i++) s[i] = br_get_signed(r, bps);
        int rc = fd_residual(r, order, N, res);
        if (rc) return rc;
        if (order > 4) return FD_FIXED_ORDER;
        for (unsigned i = order; i < N; i++) {
            const uint32_t *u = (const uint32_t *)s; /* int arithmetic wraps */
            uint32_t v;
            switch (order) {
            case 0: v = 0; break;
            case 1: v = u[i - 1]; break;
            case 2: v = 2u * u[i - 1] - u[i - 2]; break;
            case 3: v = 3u * u[i - 1] - 3u * u[i - 2] + u[i - 3]; break;
            default: v = 4u * u[i - 1] - 6u * u[i - 2] + 4u * u[i - 3] - u[i - 4];
            }
            s[i] = (int32_t)(v + (uint32_t)res[i - order]);
        }
    } else {
        int32_t coef[32];
        for (unsigned i = 0; i < order; i++) s[i] = br_get_signed(r, bps);
        const unsigned prec = br_get(r, 4) + 1;
        /* qlp_shift_needed is unsigned: MAX(x, 0) keeps a negative shift as a
           huge count, and x86's 64-bit sar masks the count to 6 bits */
        const unsigned shift = (unsigned)br_get_signed(r, 5) & 63u;
        for (unsigned i = 0; i < order; i++) coef[i] = br_get_signed(r, prec);
        int rc = fd_residual(r, order, N, res);
        if (rc) return rc;
        for (unsigned i = order; i < N; i++) {
            int64_t acc = 0;
            for (unsigned j = 0; j < order; j++)
                acc += (int64_t)coef[j] * (int64_t)s[i - j - 1];
            s[i] = (int32_t)((uint32_t)(int32_t)(acc >> shift) + (uint32_t)res[i - order]);
        }
    }
    if (r->eof) return FD_EOF;
    if (wasted)
        for (unsigned i = 0; i < N; i++) s[i] = (int32_t)((uint32_t)s[i] << wasted);
    return FD_OK;
}

int flacport_read_metadata(const uint8_t *data, size_t len, flacport_streaminfo *si,
                           flacport_seekpoint *sp, size_t sp_cap)
{
    /* flacdec_read_metadata (flac.c:568-707) */
    static const uint32_t masks[9] = {0, 0x4, 0x3, 0x7, 0x33, 0x37, 0x3F, 0x70F, 0x63F};
    memset(si, 0, sizeof(*si));
    bitr r = {data, (uint64_t)len * 8, 0, 0};
    uint32_t magic = br_get(&r, 32);
    if (r.eof) return 2;
    if (magic != 0x664C6143u) return 1;
    unsigned last;
    do {
        last = br_get(&r, 1);
        const unsigned type = br_get(&r, 7);
        const uint32_t blen = br_get(&r, 24);
        if (r.eof) return 2;
        const uint64_t body = r.pos;
        if (type == 0) {
            si->min_block_size = br_get(&r, 16);
            si->max_block_size = br_get(&r, 16);
            si->min_frame_size = br_get(&r, 24);
            si->max_frame_size = br_get(&r, 24);
            si->sample_rate = br_get(&r, 20);
            si->channels = br_get(&r, 3) + 1;
            si->bits_per_sample = br_get(&r, 5) + 1;
            si->total_samples = ((uint64_t)br_get(&r, 4) << 32) | br_get(&r, 32);
            for (int i = 0; i < 16; i++) si->md5[i] = (uint8_t)br_get(&r, 8);
            si->channel_mask = si->channels <= 8 ? masks[si->channels] : 0;
            /* the reference reads exactly 34 bytes whatever the length says */
        } else if (type == 3) {
            const unsigned n = blen / 18;
            for (unsigned k = 0; k < n; k++) {
                flacport_seekpoint p;
                p.sample_number = ((uint64_t)br_get(&r, 32) << 32) | br_get(&r, 32);
                p.byte_offset = ((uint64_t)br_get(&r, 32) << 32) | br_get(&r, 32);
                p.samples = br_get(&r, 16);
                if (sp && k < sp_cap) sp[k] = p;
            }
            si->n_seekpoints = n;
        } else if (type == 4) {
            /* flacdec_read_vorbis_comment (flac.c:508-566): little-endian
               lengths; a read error inside the block is swallowed */
            if (body + (uint64_t)blen * 8 > r.len_bits) { r.eof = 1; return 2; }
            const uint8_t *c = data + (body >> 3);
            size_t cl = blen, i = 0;
#define LE32(q) ((uint32_t)(q)[0] | ((uint32_t)(q)[1] << 8) | ((uint32_t)(q)[2] << 16) | ((uint32_t)(q)[3] << 24))
            if (i + 4 <= cl) {
                uint32_t vl = LE32(c + i);
                i += 4;
                if (vl <= cl - i) {
                    i += vl;
                    if (i + 4 <= cl) {
                        uint32_t lines = LE32(c + i);
                        i += 4;
                        static const char pre[] = "WAVEFORMATEXTENSIBLE_CHANNEL_MASK=";
                        for (; lines > 0; lines--) {
                            if (i + 4 > cl) break;
                            uint32_t ll = LE32(c + i);
                            i += 4;
                            if (ll > cl - i) break;
                            char buf[256];
                            size_t keep = ll < 255 ? ll : 255;
                            for (size_t k = 0; k < keep; k++)
                                buf[k] = (char)toupper(c[i + k]);
                            buf[keep] = 0;
                            /* the reference uppercases the line into a
                               NUL-terminated buffer: strstr prefix test, then
                               strtoul base 16 on the rest */
                            if (strncmp(buf, pre, sizeof(pre) - 1) == 0) {
                                unsigned long m = strtoul(buf + sizeof(pre) - 1, NULL, 16);
                                unsigned mask = (unsigned)m, bits = 0;
                                for (unsigned mm = mask; mm; mm >>= 1) bits += mm & 1u;
                                if (bits == si->channels) si->channel_mask = mask;
                            }
                            i += ll;
                        }
                    }
                }
            }
#undef LE32
        }
        if (type != 0 && type != 3) r.pos = body + (uint64_t)blen * 8;
        if (r.pos > r.len_bits) { r.pos = r.len_bits; r.eof = 1; }
        if (r.eof) return 2;
    } while (!last);
    si->frames_offset = r.pos >> 3;
    return 0;
}

int flacport_decode_frames(const uint8_t *data, size_t len, const flacport_streaminfo *si,
                           uint64_t remaining, int check_crc, int32_t *pcm, size_t pcm_cap,
                           uint64_t *frame_offsets, uint32_t *frame_block_sizes,
                           size_t frame_cap, size_t *n_frames, uint64_t *pcm_frames)
{
    /* the frame loop of FlacDecoder_read / offsets (flac.c:174-285, 365-443) */
    crc_init();
    const unsigned ch = si->channels;
    const unsigned alloc = si->max_block_size ? si->max_block_size : 1;
    const size_t stride = (size_t)alloc + 32; /* warm-up samples may exceed a tiny block */
    int32_t *sub = malloc(sizeof(int32_t) * stride * 16);
    int32_t *res = malloc(sizeof(int32_t) * stride);
    bitr r = {data, (uint64_t)len * 8, 0, 0};
    size_t nf = 0;
    uint64_t done = 0;
    int rc = FD_OK;
    while (remaining != 0) {
        const uint64_t fstart = r.pos;
        fd_header h;
        rc = fd_frame_header(&r, si, &h);
        if (rc) break;
        const unsigned N = (unsigned)(h.block_size < remaining ? h.block_size : remaining);
        for (unsigned c = 0; c < h.channels && !rc; c++) {
            unsigned sbps = h.bps;
            if ((h.assign == 8 && c == 1) || (h.assign == 9 && c == 0) ||
                (h.assign == 10 && c == 1))
                sbps = h.bps + 1;
            rc = fd_subframe(&r, N, sbps, sub + (size_t)c * stride, res);
        }
        if (rc) break;
        if (r.pos & 7) br_get(&r, 8 - (unsigned)(r.pos & 7));
        br_get(&r, 16);
        if (r.eof) { rc = FD_EOF; break; }
        if (check_crc && crc16_bytes(data + (fstart >> 3), (size_t)((r.pos - fstart) >> 3)) != 0) {
            rc = FD_FRAME_CRC;
            break;
        }
        if (nf >= frame_cap || (done + N) * ch > pcm_cap) { rc = -1; break; } /* capacity */
        frame_offsets[nf] = fstart >> 3;
        frame_block_sizes[nf] = h.block_size;
        nf++;
        /* flacdec_decorrelate_channels (flac.c:1212-1269) */
        int32_t *a = sub, *b = sub + stride;
        int32_t *o = pcm + done * ch;
        for (unsigned k = 0; k < N; k++) {
            if (h.assign == 8) {
                o[2 * k] = a[k];
                o[2 * k + 1] = (int32_t)((uint32_t)a[k] - (uint32_t)b[k]);
            } else if (h.assign == 9) {
                o[2 * k] = (int32_t)((uint32_t)a[k] + (uint32_t)b[k]);
                o[2 * k + 1] = b[k];
            } else if (h.assign == 10) {
                int64_t mid = a[k];
                int32_t side = b[k];
                mid = (int64_t)((uint64_t)mid << 1) | (side & 1);
                o[2 * k] = (int32_t)((mid + side) >> 1);
                o[2 * k + 1] = (int32_t)((mid - side) >> 1);
            } else {
                for (unsigned c = 0; c < ch; c++)
                    o[(size_t)k * ch + c] = sub[(size_t)c * stride + k];
            }
        }
        done += N;
        remaining -= h.block_size; /* uint64, wraps as the reference's */
    }
    free(sub);
    free(res);
    *n_frames = nf;
    *pcm_frames = done;
    return rc;
}

int flacport_decode(const uint8_t *flac, size_t len, uint32_t *channels,
                    uint32_t *bits_per_sample, uint32_t *sample_rate,
                    uint64_t *total_frames, int32_t *pcm, size_t pcm_cap)
{
    crc_init();
    size_t i = 0;
    /* skip an ID3v2 prefix (flac.py:1682-1683 __stream_offset__) */
    if (len >= 10 && memcmp(flac, "ID3", 3) == 0) {
        size_t sz = ((size_t)(flac[6] & 0x7F) << 21) | ((size_t)(flac[7] & 0x7F) << 14) |
                    ((size_t)(flac[8] & 0x7F) << 7) | (flac[9] & 0x7F);
        i = 10 + sz;
    }
    if (i > len)
        return -1;
    flacport_streaminfo si;
    if (flacport_read_metadata(flac + i, len - i, &si, NULL, 0))
        return -1;
    if (channels) *channels = si.channels;
    if (bits_per_sample) *bits_per_sample = si.bits_per_sample;
    if (sample_rate) *sample_rate = si.sample_rate;
    if (total_frames) *total_frames = si.total_samples;
    if (!pcm)
        return 0;
    if (pcm_cap < si.total_samples * si.channels)
        return -2;
    /* frames cut at the writer's read sizes may be shorter than the
       STREAMINFO minimum block: every frame holds >= 1 sample */
    size_t cap = (size_t)si.total_samples + 2;
    uint64_t *offs = malloc(sizeof(uint64_t) * cap);
    uint32_t *bss = malloc(sizeof(uint32_t) * cap);
    size_t nf;
    uint64_t got;
    const size_t start = i + si.frames_offset;
    int rc = flacport_decode_frames(flac + start, len - start, &si, si.total_samples, 1, pcm,
                                    pcm_cap, offs, bss, cap, &nf, &got);
    free(offs);
    free(bss);
    if (rc)
        return rc == FD_EOF ? -4 : -3;
    static const uint8_t zero[16] = {0};
    if (memcmp(si.md5, zero, 16) != 0) {
        uint8_t d[16];
        flacport_pcm_md5(pcm, got, si.channels, si.bits_per_sample, d);
        if (memcmp(d, si.md5, 16) != 0)
            return -5;
    }
    return 0;
}
