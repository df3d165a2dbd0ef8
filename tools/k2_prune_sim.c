/* k2_prune_sim.c — development tool: how often K2's LPC jobs survive the
 * residual lower-bound pruning (flac_search16.hip residual_lb) on config-2
 * shaped frames, i.e. how many predictors per candidate pay for pass 2
 * (the exact bit count) and the partition search; and how many a bound
 * checked after 16, 32 or 48 of a lane's 64 samples would prune there
 * (what ending pass 1 early could save).  Jobs are simulated in
 * the kernel's order: FIXED always evaluated, LPC orders 12 .. 1, a job
 * pruned when its lane-sum bound exceeds (best finished LPC total - hdr).
 *
 * Build: gcc -O2 -ffp-contract=off -o tools/bin/k2_prune_sim tools/k2_prune_sim.c -lm
 * (includes the CPU restatement oracle/flac_port.c for the LPC analysis).
 */
#include "../oracle/flac_port.c"

#include <stdio.h>

static uint64_t xs = 88172645463325252ull;
static double urand(void)
{
    xs ^= xs << 13;
    xs ^= xs >> 7;
    xs ^= xs << 17;
    return (double)(xs >> 11) / 9007199254740992.0;
}
static double grand(void)
{
    double u = urand() + 1e-300, v = urand();
    return sqrt(-2.0 * log(u)) * cos(2 * M_PI * v);
}

static float lb_lane(uint32_t lane_sum, uint32_t cnt)
{
    const float cf = (float)cnt;
    float U = 2.0f * (float)lane_sum - cf;
    U = U > 0.f ? U : 0.f;
    const float x = (U + cf) * 0.69314718f / cf;
    const float lb = x >= 1.0f ? cf * log2f(x) + cf * 1.44269504f : U + cf;
    const float l4 = lb - 4.0f;
    return l4 > 0.f ? (float)(uint32_t)l4 : 0.f;
}

int main(int argc, char **argv)
{
    const int n_frames = argc > 1 ? atoi(argv[1]) : 400;
    flacport_options o = {4096, 12, 0, 6, 1, 0, 1, 0, 0, 0, 0, 4096};
    enc_ctx *e = calloc(1, sizeof(enc_ctx));
    e->o = &o;
    e->qlp_precision = 12;
    e->max_rice = 14;
    e->win = calloc(4096, sizeof(double));
    e->xw = calloc(4096, sizeof(double));
    static int32_t L[4096], R[4096], C[4][4096], res[4096];
    long jobs = 0, pass2 = 0, subfr = 0;
    long per_order_pass2[13] = {0};
    long early[3] = {0, 0, 0}; double cost_all = 0, cost_saved[3] = {0, 0, 0};
    for (int f = 0; f < n_frames; ++f) {
        const double f1 = 100 + 1900 * urand(), f2 = 2000 + 10000 * urand();
        const double a1 = 0.05 + 0.55 * urand(), a2 = 0.3 * urand();
        const int white = urand() < 0.05;
        for (int i = 0; i < 4096; ++i) {
            const double ph = 2 * M_PI * (i + 4096.0 * f) / 44100.0;
            double l = (a1 * sin(ph * f1) + a2 * sin(ph * f2)) * 32767.0 + grand() * 64.0;
            double r = (a1 * sin(ph * f1 * 1.3) + a2 * sin(ph * f2 * 1.3)) * 32767.0 +
                       grand() * 64.0;
            if (white) {
                l = (urand() * 65536.0) - 32768.0;
                r = (urand() * 65536.0) - 32768.0;
            }
            l = round(l);
            r = round(r);
            L[i] = (int32_t)(l < -32768 ? -32768 : l > 32767 ? 32767 : l);
            R[i] = (int32_t)(r < -32768 ? -32768 : r > 32767 ? 32767 : r);
        }
        for (int i = 0; i < 4096; ++i) {
            C[0][i] = L[i];
            C[1][i] = R[i];
            C[2][i] = (L[i] + R[i]) >> 1;
            C[3][i] = L[i] - R[i];
        }
        for (int c = 0; c < 4; ++c) {
            const int32_t *s = C[c];
            const unsigned bps = c == 3 ? 17 : 16;
            /* LPC analysis as plan_lpc */
            double Rr[MAX_LPC + 1], lp[MAX_LPC][MAX_LPC], err[MAX_LPC];
            tukey_window(e, 4096);
            for (unsigned n = 0; n < 4096; n++)
                e->xw[n] = s[n] * e->win[n];
            for (unsigned lag = 0; lag <= 12; lag++) {
                double acc = 0.0;
                for (unsigned i = 0; i < 4096 - lag; i++)
                    acc += e->xw[i] * e->xw[i + lag];
                Rr[lag] = acc;
            }
            double k = Rr[1] / Rr[0];
            lp[0][0] = k;
            err[0] = Rr[0] * (1.0 - (k * k));
            for (unsigned i = 1; i < 12; i++) {
                double q = Rr[i + 1];
                for (unsigned j = 0; j < i; j++)
                    q -= (lp[i - 1][j] * Rr[i - j]);
                k = q / err[i - 1];
                for (unsigned j = 0; j < i; j++)
                    lp[i][j] = lp[i - 1][j] - (k * lp[i - 1][i - j - 1]);
                lp[i][i] = k;
                err[i] = err[i - 1] * (1.0 - (k * k));
            }
            uint32_t best = 0xFFFFFFFFu;
            subfr++;
            for (int order = 12; order >= 1; --order) {
                int32_t cq[MAX_LPC];
                int sh;
                quantize(lp[order - 1], order, 12, cq, &sh);
                lpc_residual(s, 4096, order, cq, sh, res);
                const uint32_t hdr = 7 + 1 + order * bps + 9 + order * 12;
                uint32_t thr = best == 0xFFFFFFFFu ? 0xFFFFFFFFu : (best > hdr ? best - hdr : 0);
                /* lane sums over the lane's 64 samples (lane 0 has 64 - order residuals) */
                float lb = 0;
                for (int lane = 0; lane < 64; ++lane) {
                    uint32_t sum = 0;
                    int a = lane * 64 - order, b = a + 64;
                    if (a < 0)
                        a = 0;
                    for (int i = a; i < b; ++i)
                        sum += (uint32_t)abs(res[i]);
                    lb += lb_lane(sum, lane ? 64 : 64 - order);
                }
                jobs++;
                {
                    const int D = order / 2 + 1;
                    const double cpl = (double)(D + 3) * 64; /* pass-1 VALU per lane-run */
                    cost_all += cpl;
                    const int cuts[3] = {16, 32, 48};
                    for (int q = 0; q < 3; ++q) {
                        float lbp = 0;
                        for (int lane = 0; lane < 64; ++lane) {
                            uint32_t sum = 0;
                            int a = lane * 64 - order, b = lane * 64 - order + cuts[q];
                            int cnt = cuts[q];
                            if (a < 0) { cnt += a; a = 0; }
                            for (int i = a; i < b; ++i)
                                sum += (uint32_t)abs(res[i]);
                            lbp += lb_lane(sum, cnt);
                        }
                        if (thr != 0xFFFFFFFFu && (uint32_t)lbp > thr) {
                            early[q]++;
                            cost_saved[q] += cpl * (64 - cuts[q]) / 64.0;
                        }
                    }
                }
                if (thr != 0xFFFFFFFFu && (uint32_t)lb > thr)
                    continue;
                pass2++;
                per_order_pass2[order]++;
                plan_residuals(e, res, 4096 - order, 4096, order, &e->cand_res);
                const uint32_t tot = hdr + e->cand_res.bits;
                if (tot < best)
                    best = tot;
            }
        }
    }
    printf("subframes %ld  LPC jobs %ld  pass2 %ld (%.2f per subframe, %.1f %%)\n", subfr, jobs,
           pass2, (double)pass2 / subfr, 100.0 * pass2 / jobs);
    for (int q = 0; q < 3; ++q)
        printf("check after %d of 64: %.1f %% of jobs pruned there, pass-1 cost saved %.1f %%\n",
               16 * (q + 1), 100.0 * early[q] / jobs, 100.0 * cost_saved[q] / cost_all);
    for (int o2 = 12; o2 >= 1; --o2)
        printf("order %2d: pass2 in %.1f %% of subframes\n", o2, 100.0 * per_order_pass2[o2] / subfr);
    return 0;
}
