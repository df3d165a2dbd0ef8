// k2_mfma_probe.hip — measured answer to "can K2's LPC evaluation run on
// MFMA?" (DESIGN 4a'').  Standalone: hipcc --offload-arch=gfx950 -O3
// tools/k2_mfma_probe.hip -o /tmp/k2_mfma_probe && /tmp/k2_mfma_probe
//
// K2 evaluates, per (frame, candidate channel), the 12 LPC predictors (and
// the FIXED orders) over 4096 16-bit samples and needs every residual's
// code v = n ^ (n >> 31), n = ~r, summed per 64-sample partition (the
// partition search and the pruning bound start from these sums).  Here the
// whole evaluation is one integer product per 16-sample tile:
//
//   A [16 samples x 64 k]  the raw little-endian bytes of s[t-7..t] and
//                          s[t-15..t-8] (k = byte: lo/hi limb of one lag),
//                          lo bytes offset by -128 (x ^ 0x80) so every limb
//                          is a signed i8
//   B [64 k x 16 columns]  per column (12 LPC orders + FIXED 1..4) the
//                          coefficient limbs c = 256 ch + cl (cl balanced),
//                          the fold tap -2^sh at lag -1 (s[t] itself), so
//                          acc >> sh = ~r with the seed below
//   three v_mfma_i32_16x16x64_i8: D1 = sum ch*hi, D2 = sum (cl*hi + ch*lo'),
//   D3 = seed + sum cl*lo', seed = 128 * sum c - 2^sh;
//   acc = (D1 << 16) + (D2 << 8) + D3 (wrapping int32: exact whenever the
//   true sum fits, which K2's bound check guarantees)
//
// then per output: acc >> sh, v = n ^ (n >> 31), partition sums.  The probe
// (1) checks the i8 fragment maps with exact data, (2) checks the MFMA
// kernel against a scalar int64 reference on a subset, (3) times it at K2's
// size (65,536 frames x 4 candidates x 4,096 samples), and (4) times a
// v_dot2 kernel computing the same sums the way K2 does (O_t pair words,
// one v_dot2 per tap pair with the fold tap, alignbit for even t), so the
// two evaluations are compared on the same outputs.  One JSON line.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));          \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

typedef int v4i __attribute__((ext_vector_type(4)));
typedef short s2v __attribute__((ext_vector_type(2)));

constexpr int kN = 4096;       // samples per frame
constexpr int kPre = 16;       // history samples before t = 0
constexpr int kCols = 16;      // 12 LPC orders + FIXED 1..4
constexpr int kParts = kN / 64;

struct Pred {                  // one frame-candidate's 16 columns
    int16_t c[kCols][12];      // coefficient of lag j (j < order)
    uint8_t order[kCols];
    uint8_t sh[kCols];
};

// ---- (1) fragment map check: D = A B with the lane maps the kernels assume
// (lane l: A[row l & 15][k of (l >> 4, j)], B[k of (l >> 4, j)][col l & 15],
// D reg r = [row 4 (l >> 4) + r][col l & 15])
__global__ void k_layout(const int8_t *a, const int8_t *b, int *d)
{
    const int l = threadIdx.x;
    v4i av, bv;
    std::memcpy(&av, a + 16 * l, 16);
    std::memcpy(&bv, b + 16 * l, 16);
    v4i c = {0, 0, 0, 0};
    c = __builtin_amdgcn_mfma_i32_16x16x64_i8(av, bv, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r)
        d[4 * l + r] = c[r];
}

// ---- scalar reference: S[fc][col][part] (int64 arithmetic)
__global__ void k_ref(const int16_t *pcm, const Pred *pred, uint32_t nfc, uint32_t *S)
{
    const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
    if (g >= nfc * kCols * kParts)
        return;
    const uint32_t fc = g / (kCols * kParts), col = (g / kParts) % kCols, q = g % kParts;
    const int16_t *s = pcm + (uint64_t)fc * (kPre + kN) + kPre;
    const Pred &P = pred[fc];
    uint32_t sum = 0;
    for (int t = 64 * q; t < 64 * q + 64; ++t) {
        int64_t acc = -((int64_t)1 << P.sh[col]) * s[t] - ((int64_t)1 << P.sh[col]);
        for (int j = 0; j < P.order[col]; ++j)
            acc += (int64_t)P.c[col][j] * s[t - 1 - j];
        const int32_t n = (int32_t)(acc >> P.sh[col]);
        sum += (uint32_t)(n ^ (n >> 31));
    }
    S[g] = sum;
}

// ---- (2)/(3) MFMA kernel: workgroup per frame-candidate, wave w takes
// samples [1024 w, 1024 w + 1024) = 64 tiles of 16
__global__ __launch_bounds__(256) void k_mfma(const int16_t *__restrict__ pcm,
                                              const Pred *__restrict__ pred,
                                              uint32_t *__restrict__ S)
{
    // two byte images of the frame (lo bytes ^ 0x80): copy 1 starts one
    // sample later, so every lane reads 4-byte aligned dwords
    __shared__ uint32_t img[2][(kPre + kN) / 2 + 4];
    const uint32_t fc = blockIdx.x;
    const uint32_t *src = (const uint32_t *)(pcm + (uint64_t)fc * (kPre + kN));
    for (uint32_t i = threadIdx.x; i < (kPre + kN) / 2; i += 256) {
        const uint32_t x = src[i] ^ 0x00800080u;
        img[0][i] = x;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < (kPre + kN) / 2 - 1; i += 256)
        img[1][i] = __builtin_amdgcn_alignbyte(img[0][i + 1], img[0][i], 2);
    __syncthreads();
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int g = l >> 4, n = l & 15;
    // B fragments of column n for this lane's k group (constant per frame)
    const Pred &P = pred[fc];
    const int order = P.order[n], sh = P.sh[n];
    int8_t b1[16], b2[16], b3[16];
    int32_t csum = 0;
    for (int j = 0; j < 12; ++j)
        csum += j < order ? P.c[n][j] : 0;
    csum -= 1 << sh;
    for (int j = 0; j < 16; ++j) {
        const int idx = j >> 1, limb = j & 1;
        const int lag = g < 2 ? 6 + 8 * g - idx : 99;
        int coef = 0;
        if (lag == -1)
            coef = -(1 << sh);
        else if (lag >= 0 && lag < order)
            coef = P.c[n][lag];
        const int cl = ((coef + 128) & 255) - 128, ch = (coef - cl) >> 8;
        b1[j] = (int8_t)(limb ? ch : 0);
        b2[j] = (int8_t)(limb ? cl : ch);
        b3[j] = (int8_t)(limb ? 0 : cl);
    }
    v4i B1, B2, B3;
    std::memcpy(&B1, b1, 16);
    std::memcpy(&B2, b2, 16);
    std::memcpy(&B3, b3, 16);
    const int32_t seed = 128 * csum - (1 << sh);
    const v4i C3 = {seed, seed, seed, seed}, Z = {0, 0, 0, 0};
    const int ga = g < 2 ? g : 1; // groups 2, 3 read valid (ignored) bytes
    uint32_t part = 0;
    for (int tile = 0; tile < 64; ++tile) {
        const int t0 = 1024 * w + 16 * tile;
        // A: row m = l & 15 -> sample t; 16 bytes of s[t - 7 - 8 ga ..]
        const int u = t0 + n + kPre - 7 - 8 * ga;
        const uint32_t *p = (u & 1) ? &img[1][(u - 1) >> 1] : &img[0][u >> 1];
        v4i A;
        A[0] = (int)p[0];
        A[1] = (int)p[1];
        A[2] = (int)p[2];
        A[3] = (int)p[3];
        const v4i D1 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B1, Z, 0, 0, 0);
        const v4i D2 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B2, Z, 0, 0, 0);
        const v4i D3 = __builtin_amdgcn_mfma_i32_16x16x64_i8(A, B3, C3, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            // (D1 << 16) + (D2 << 8) + D3 as two shift-adds
            uint32_t acc = ((uint32_t)D1[r] << 8) + (uint32_t)D2[r];
            acc = (acc << 8) + (uint32_t)D3[r];
            const int32_t nn = (int32_t)acc >> sh;
            part += (uint32_t)(nn ^ (nn >> 31));
        }
        if ((tile & 3) == 3) { // a 64-sample partition: the 4 row groups' sums
            part += (uint32_t)__shfl_xor((int)part, 16, 64);
            part += (uint32_t)__shfl_xor((int)part, 32, 64);
            if (g == 0)
                S[((uint64_t)fc * kCols + n) * kParts + (1024 * w + 16 * tile) / 64] = part;
            part = 0;
        }
    }
}

// ---- (4) the v_dot2 evaluation the way K2 runs it: workgroup per
// frame-candidate, packed int16 pair words in LDS; a wave takes columns
// (jobs) in turn, lane = 64 consecutive samples = one partition; per sample
// O_t = (s[t-1], s[t]) (an LDS word for odd t, one alignbit for even t) and
// floor(order/2)+1 v_dot2 with tap pairs (c0, -2^sh), (c2, c1), ...
__global__ __launch_bounds__(256) void k_dot2(const int16_t *__restrict__ pcm,
                                              const Pred *__restrict__ pred,
                                              uint32_t *__restrict__ S)
{
    __shared__ uint32_t wd[(kPre + kN) / 2 + 4];
    const uint32_t fc = blockIdx.x;
    const uint32_t *src = (const uint32_t *)(pcm + (uint64_t)fc * (kPre + kN));
    for (uint32_t i = threadIdx.x; i < (kPre + kN) / 2; i += 256)
        wd[i] = src[i];
    __syncthreads();
    const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
    const Pred &P = pred[fc];
    for (int col = w; col < kCols; col += 4) {
        const int order = P.order[col], sh = P.sh[col];
        // tap pairs on (lo = s[t-1-2i], hi = s[t-2i]) words: pair 0 = (c0, -2^sh)
        int32_t tp[7];
        for (int i = 0; i < 7; ++i) {
            const int jl = 2 * i, jh = 2 * i - 1; // lag of the lo / hi element
            const int lo = jl < order ? P.c[col][jl] : 0;
            const int hi = i == 0 ? -(1 << sh) : (jh < order ? P.c[col][jh] : 0);
            tp[i] = (int32_t)(((uint32_t)(uint16_t)hi << 16) | (uint16_t)lo);
        }
        const int npair = order / 2 + 1;
        const int32_t seed = -(1 << sh);
        uint32_t sum = 0;
        const int t0 = 64 * l;
        for (int t = t0; t < t0 + 64; ++t) {
            int32_t acc = seed;
            for (int i = 0; i < 7; ++i) {
                if (i >= npair)
                    break;
                // O_{t-2i} = (s[t-1-2i], s[t-2i]), sample index + kPre
                const int u = t - 2 * i - 1 + kPre; // index of the lo element
                const uint32_t word = (u & 1) ? __builtin_amdgcn_alignbyte(wd[(u >> 1) + 1],
                                                                           wd[u >> 1], 2)
                                              : wd[u >> 1];
                acc = __builtin_amdgcn_sdot2(__builtin_bit_cast(s2v, word),
                                             __builtin_bit_cast(s2v, tp[i]), acc, false);
            }
            const int32_t nn = acc >> sh;
            sum += (uint32_t)(nn ^ (nn >> 31));
        }
        S[((uint64_t)fc * kCols + col) * kParts + (t0 >> 6)] = sum;
    }
}

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint32_t rnd()
{
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return (uint32_t)(rng >> 11);
}

int main(int argc, char **argv)
{
    const uint32_t nfc = argc > 1 ? (uint32_t)atoi(argv[1]) : 65536u * 4u;
    const uint32_t ncheck = 256;
    // (1) fragment maps
    std::vector<int8_t> ha(64 * 16), hb(64 * 16);
    for (auto &x : ha) x = (int8_t)(rnd() % 255 - 127);
    for (auto &x : hb) x = (int8_t)(rnd() % 255 - 127);
    int8_t *da, *db;
    int *dd;
    CK(hipMalloc(&da, 1024));
    CK(hipMalloc(&db, 1024));
    CK(hipMalloc(&dd, 1024));
    CK(hipMemcpy(da, ha.data(), 1024, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, hb.data(), 1024, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_layout, dim3(1), dim3(64), 0, 0, da, db, dd);
    std::vector<int> hd(256);
    CK(hipMemcpy(hd.data(), dd, 1024, hipMemcpyDeviceToHost));
    int layout_bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int r = 0; r < 4; ++r) {
            const int row = 4 * (l >> 4) + r, col = l & 15;
            int want = 0;
            for (int g = 0; g < 4; ++g)
                for (int j = 0; j < 16; ++j)
                    want += ha[16 * (16 * g + row) + j] * hb[16 * (16 * g + col) + j];
            layout_bad += want != hd[4 * l + r];
        }
    // data: random-walk PCM with noise, per frame-candidate
    std::vector<int16_t> pcm((uint64_t)nfc * (kPre + kN));
    for (uint32_t f = 0; f < nfc; ++f) {
        int x = (int)(rnd() % 20000) - 10000;
        const int amp = 1 + (int)(rnd() % 3000);
        for (int i = 0; i < kPre + kN; ++i) {
            x += (int)(rnd() % (2 * amp + 1)) - amp;
            x = x > 32000 ? 32000 : (x < -32000 ? -32000 : x);
            pcm[(uint64_t)f * (kPre + kN) + i] = (int16_t)x;
        }
    }
    std::vector<Pred> pred(nfc);
    for (uint32_t f = 0; f < nfc; ++f) {
        Pred &P = pred[f];
        std::memset(&P, 0, sizeof(P));
        for (int col = 0; col < 12; ++col) {
            P.order[col] = (uint8_t)(col + 1);
            P.sh[col] = (uint8_t)(9 + rnd() % 6); // 9..14
            // sum |c| <= 2^15: |sum c s| < 2^30, plus the fold 2^29
            const int lim = (1 << 15) / (col + 1);
            for (int j = 0; j <= col; ++j)
                P.c[col][j] = (int16_t)((int)(rnd() % (2 * lim - 1)) - (lim - 1));
        }
        static const int fx[4][4] = {{1, 0, 0, 0}, {2, -1, 0, 0}, {3, -3, 1, 0}, {4, -6, 4, -1}};
        for (int o = 0; o < 4; ++o) {
            P.order[12 + o] = (uint8_t)(o + 1);
            P.sh[12 + o] = 0;
            for (int j = 0; j < 4; ++j)
                P.c[12 + o][j] = (int16_t)fx[o][j];
        }
    }
    int16_t *dp;
    Pred *dpr;
    uint32_t *dS, *dR, *dT;
    const uint64_t nS = (uint64_t)nfc * kCols * kParts;
    CK(hipMalloc(&dp, pcm.size() * 2));
    CK(hipMalloc(&dpr, sizeof(Pred) * nfc));
    CK(hipMalloc(&dS, nS * 4));
    CK(hipMalloc(&dT, nS * 4));
    CK(hipMalloc(&dR, (uint64_t)ncheck * kCols * kParts * 4));
    CK(hipMemcpy(dp, pcm.data(), pcm.size() * 2, hipMemcpyHostToDevice));
    CK(hipMemcpy(dpr, pred.data(), sizeof(Pred) * nfc, hipMemcpyHostToDevice));
    // (2) parity on the first ncheck frame-candidates
    const uint32_t nref = ncheck * kCols * kParts;
    hipLaunchKernelGGL(k_ref, dim3((nref + 255) / 256), dim3(256), 0, 0, dp, dpr, ncheck, dR);
    hipLaunchKernelGGL(k_mfma, dim3(nfc), dim3(256), 0, 0, dp, dpr, dS);
    hipLaunchKernelGGL(k_dot2, dim3(nfc), dim3(256), 0, 0, dp, dpr, dT);
    CK(hipDeviceSynchronize());
    std::vector<uint32_t> hr(nref), hs(nref), ht(nref);
    CK(hipMemcpy(hr.data(), dR, nref * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hs.data(), dS, nref * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(ht.data(), dT, nref * 4, hipMemcpyDeviceToHost));
    uint32_t bad_mfma = 0, bad_dot2 = 0;
    for (uint32_t i = 0; i < nref; ++i) {
        bad_mfma += hr[i] != hs[i];
        bad_dot2 += hr[i] != ht[i];
    }
    // (3)/(4) timing: 5 launches each
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float ms_mfma = 0, ms_dot2 = 0;
    for (int rep = 0; rep < 2; ++rep) {
        CK(hipEventRecord(e0, 0));
        for (int k = 0; k < 5; ++k)
            hipLaunchKernelGGL(k_mfma, dim3(nfc), dim3(256), 0, 0, dp, dpr, dS);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms_mfma, e0, e1));
        CK(hipEventRecord(e0, 0));
        for (int k = 0; k < 5; ++k)
            hipLaunchKernelGGL(k_dot2, dim3(nfc), dim3(256), 0, 0, dp, dpr, dT);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms_dot2, e0, e1));
    }
    // whole-size agreement of the two fast kernels
    std::vector<uint32_t> as(nS), at(nS);
    CK(hipMemcpy(as.data(), dS, nS * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(at.data(), dT, nS * 4, hipMemcpyDeviceToHost));
    uint64_t diff_full = 0;
    for (uint64_t i = 0; i < nS; ++i)
        diff_full += as[i] != at[i];
    const double outputs = (double)nfc * kCols * kN;
    printf("{\"frame_candidates\": %u, \"columns\": %d, \"layout_mismatches\": %d, "
           "\"mfma_vs_ref_mismatches\": %u, \"dot2_vs_ref_mismatches\": %u, "
           "\"mfma_vs_dot2_mismatches_full\": %llu, \"ms_mfma\": %.4f, \"ms_dot2\": %.4f, "
           "\"ns_per_1k_outputs_mfma\": %.4f, \"ns_per_1k_outputs_dot2\": %.4f}\n",
           nfc, kCols, layout_bad, bad_mfma, bad_dot2, (unsigned long long)diff_full,
           ms_mfma / 5, ms_dot2 / 5, ms_mfma / 5 * 1e6 / outputs * 1e3,
           ms_dot2 / 5 * 1e6 / outputs * 1e3);
    return 0;
}
