/*
 * rg_converge.c -- why ReplayGain's time split is certified, not exact.
 *
 * Runs the reference's Yule + Butterworth pair (src/replaygain.c:566-610,
 * fp64, its operation order, coefficients from csrc/rg_coeffs.h) over a
 * synthetic 44.1 kHz signal twice: the serial trajectory from frame 0, and a
 * trajectory started at frame P from zero filter state with the exact input
 * history (what a warm segment of k_rg_seg does).  Prints the largest
 * difference of the Yule output history and the Butterworth output at
 * growing distances from P: it falls to the filter's rounding-noise floor
 * (~1e-10 on samples of ~1e4) within ~2 k frames and then stays there --
 * the two fp64 trajectories never coalesce bit for bit.
 *
 *   gcc -O2 -ffp-contract=off -o /tmp/rg_converge tools/rg_converge.c -lm
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../python-audio-tools_amd/csrc/rg_coeffs.h"

typedef struct {
    double in[10], yo[10], bo[2];
} cs;

static double step(cs *s, double x, const double *ky, const double *kb)
{
    double y = 1e-10 + x * ky[0];
    for (int k = 1; k <= 10; k++) {
        y = y - s->yo[k - 1] * ky[2 * k - 1];
        y = y + s->in[k - 1] * ky[2 * k];
    }
    double b = y * kb[0] - s->bo[0] * kb[1] + s->yo[0] * kb[2] - s->bo[1] * kb[3] +
               s->yo[1] * kb[4];
    memmove(s->in + 1, s->in, 9 * sizeof(double));
    s->in[0] = x;
    s->bo[1] = s->bo[0];
    s->bo[0] = b;
    memmove(s->yo + 1, s->yo, 9 * sizeof(double));
    s->yo[0] = y;
    return b;
}

int main(void)
{
    const int fi = 1, rate = 44100; /* RG_YULE/RG_BUTTER row of 44.1 kHz */
    const long N = 400000, P = 20000;
    const double *ky = RG_YULE[fi], *kb = RG_BUTTER[fi];
    double *x = malloc(sizeof(double) * N);
    uint64_t r = 1;
    for (long i = 0; i < N; i++) {
        r ^= r << 13;
        r ^= r >> 7;
        r ^= r << 17;
        const double t = (double)i / rate;
        x[i] = round(8000 * sin(2 * M_PI * 440 * t) +
                     ((r >> 11) * (1.0 / 9007199254740992.0) - 0.5) * 200);
    }
    cs a, b;
    memset(&a, 0, sizeof(a));
    for (long i = 0; i < P; i++)
        step(&a, x[i], ky, kb);
    memset(&b, 0, sizeof(b));
    for (int k = 0; k < 10; k++)
        b.in[k] = x[P - 1 - k];
    long identical = 0;
    for (long n = 0; n < N - P; n++) {
        step(&a, x[P + n], ky, kb);
        step(&b, x[P + n], ky, kb);
        if (!memcmp(a.yo, b.yo, sizeof(a.yo)) && !memcmp(a.bo, b.bo, sizeof(a.bo)))
            identical++;
        if ((n & (n - 1)) == 0 || n % 50000 == 0) {
            double m = 0;
            for (int k = 0; k < 10; k++)
                m = fmax(m, fabs(a.yo[k] - b.yo[k]));
            printf("frames after the warm start %7ld: max |dYule| %.3g  |dButter| %.3g\n", n, m,
                   fabs(a.bo[0] - b.bo[0]));
        }
    }
    printf("frames with bit-identical filter state: %ld of %ld\n", identical, N - P);
    free(x);
    return 0;
}
