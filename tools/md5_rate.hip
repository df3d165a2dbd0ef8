// md5_rate.hip — what bounds one MD5 chain per lane on MI355X.  The
// STREAMINFO MD5 of a track is one serial chain of 64-round compressions
// (16384 of them per 1 MiB track in the bench batch), so the per-round
// dependent latency sets a floor on the encode step.  Variants:
//   0  md5_compress as shipped (md5.hip)
//   1  a + x + T precomputed off the chain (v_add3 with an SGPR constant),
//      chain = bitop3 -> v_add -> v_alignbit -> v_add
//   2  as 1, rotate as v_lshlrev + v_lshrrev + v_or (fast ops only)
//   3  as 1, two tracks interleaved per lane (issue vs latency bound)
// Launch modes: 64 lanes per wave (T/64 waves) or 1 live lane per wave.
// Build: hipcc --offload-arch=gfx950 -O3 -I python-audio-tools_amd/csrc -o tools/bin/md5_rate tools/md5_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <vector>

#include "md5.hip"

// a + x + T as its own value (an empty asm fences the sum so the compiler
// cannot re-associate F into it and put the add3 back on the chain)
__device__ __forceinline__ uint32_t add3_s(uint32_t a, uint32_t x, uint32_t t)
{
    uint32_t r = a + x + t;
    asm("" : "+v"(r));
    return r;
}
__device__ __forceinline__ uint32_t vadd(uint32_t a, uint32_t b) { return a + b; }
template <int S>
__device__ __forceinline__ uint32_t rot_v(uint32_t y)
{
    return __builtin_amdgcn_alignbit(y, y, 32 - S);
}
template <int S>
__device__ __forceinline__ uint32_t rot_f(uint32_t y)
{
    uint32_t lo = y << S, hi = y >> (32 - S);
    asm("" : "+v"(lo), "+v"(hi));
    return lo | hi;
}

#define G1(x, y, z) (z ^ (x & (y ^ z)))
#define G2(x, y, z) (y ^ (z & (x ^ y)))
#define G3(x, y, z) (x ^ y ^ z)
#define G4(x, y, z) (y ^ (x | ~z))

template <bool FAST>
struct Md5Asm {
    template <int S>
    __device__ static __forceinline__ uint32_t rot(uint32_t y)
    {
        if constexpr (FAST)
            return rot_f<S>(y);
        else
            return rot_v<S>(y);
    }
};

#define ST(R, F, a, b, c, d, x, t, s) a = vadd(R::template rot<s>(vadd(add3_s(a, x, t), F(b, c, d))), b)

template <bool FAST>
__device__ __forceinline__ void md5_asm(uint32_t h[4], const uint32_t X[16])
{
    using R = Md5Asm<FAST>;
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3];
    ST(R, G1, a, b, c, d, X[0], 0xd76aa478, 7);
    ST(R, G1, d, a, b, c, X[1], 0xe8c7b756, 12);
    ST(R, G1, c, d, a, b, X[2], 0x242070db, 17);
    ST(R, G1, b, c, d, a, X[3], 0xc1bdceee, 22);
    ST(R, G1, a, b, c, d, X[4], 0xf57c0faf, 7);
    ST(R, G1, d, a, b, c, X[5], 0x4787c62a, 12);
    ST(R, G1, c, d, a, b, X[6], 0xa8304613, 17);
    ST(R, G1, b, c, d, a, X[7], 0xfd469501, 22);
    ST(R, G1, a, b, c, d, X[8], 0x698098d8, 7);
    ST(R, G1, d, a, b, c, X[9], 0x8b44f7af, 12);
    ST(R, G1, c, d, a, b, X[10], 0xffff5bb1, 17);
    ST(R, G1, b, c, d, a, X[11], 0x895cd7be, 22);
    ST(R, G1, a, b, c, d, X[12], 0x6b901122, 7);
    ST(R, G1, d, a, b, c, X[13], 0xfd987193, 12);
    ST(R, G1, c, d, a, b, X[14], 0xa679438e, 17);
    ST(R, G1, b, c, d, a, X[15], 0x49b40821, 22);
    ST(R, G2, a, b, c, d, X[1], 0xf61e2562, 5);
    ST(R, G2, d, a, b, c, X[6], 0xc040b340, 9);
    ST(R, G2, c, d, a, b, X[11], 0x265e5a51, 14);
    ST(R, G2, b, c, d, a, X[0], 0xe9b6c7aa, 20);
    ST(R, G2, a, b, c, d, X[5], 0xd62f105d, 5);
    ST(R, G2, d, a, b, c, X[10], 0x02441453, 9);
    ST(R, G2, c, d, a, b, X[15], 0xd8a1e681, 14);
    ST(R, G2, b, c, d, a, X[4], 0xe7d3fbc8, 20);
    ST(R, G2, a, b, c, d, X[9], 0x21e1cde6, 5);
    ST(R, G2, d, a, b, c, X[14], 0xc33707d6, 9);
    ST(R, G2, c, d, a, b, X[3], 0xf4d50d87, 14);
    ST(R, G2, b, c, d, a, X[8], 0x455a14ed, 20);
    ST(R, G2, a, b, c, d, X[13], 0xa9e3e905, 5);
    ST(R, G2, d, a, b, c, X[2], 0xfcefa3f8, 9);
    ST(R, G2, c, d, a, b, X[7], 0x676f02d9, 14);
    ST(R, G2, b, c, d, a, X[12], 0x8d2a4c8a, 20);
    ST(R, G3, a, b, c, d, X[5], 0xfffa3942, 4);
    ST(R, G3, d, a, b, c, X[8], 0x8771f681, 11);
    ST(R, G3, c, d, a, b, X[11], 0x6d9d6122, 16);
    ST(R, G3, b, c, d, a, X[14], 0xfde5380c, 23);
    ST(R, G3, a, b, c, d, X[1], 0xa4beea44, 4);
    ST(R, G3, d, a, b, c, X[4], 0x4bdecfa9, 11);
    ST(R, G3, c, d, a, b, X[7], 0xf6bb4b60, 16);
    ST(R, G3, b, c, d, a, X[10], 0xbebfbc70, 23);
    ST(R, G3, a, b, c, d, X[13], 0x289b7ec6, 4);
    ST(R, G3, d, a, b, c, X[0], 0xeaa127fa, 11);
    ST(R, G3, c, d, a, b, X[3], 0xd4ef3085, 16);
    ST(R, G3, b, c, d, a, X[6], 0x04881d05, 23);
    ST(R, G3, a, b, c, d, X[9], 0xd9d4d039, 4);
    ST(R, G3, d, a, b, c, X[12], 0xe6db99e5, 11);
    ST(R, G3, c, d, a, b, X[15], 0x1fa27cf8, 16);
    ST(R, G3, b, c, d, a, X[2], 0xc4ac5665, 23);
    ST(R, G4, a, b, c, d, X[0], 0xf4292244, 6);
    ST(R, G4, d, a, b, c, X[7], 0x432aff97, 10);
    ST(R, G4, c, d, a, b, X[14], 0xab9423a7, 15);
    ST(R, G4, b, c, d, a, X[5], 0xfc93a039, 21);
    ST(R, G4, a, b, c, d, X[12], 0x655b59c3, 6);
    ST(R, G4, d, a, b, c, X[3], 0x8f0ccc92, 10);
    ST(R, G4, c, d, a, b, X[10], 0xffeff47d, 15);
    ST(R, G4, b, c, d, a, X[1], 0x85845dd1, 21);
    ST(R, G4, a, b, c, d, X[8], 0x6fa87e4f, 6);
    ST(R, G4, d, a, b, c, X[15], 0xfe2ce6e0, 10);
    ST(R, G4, c, d, a, b, X[6], 0xa3014314, 15);
    ST(R, G4, b, c, d, a, X[13], 0x4e0811a1, 21);
    ST(R, G4, a, b, c, d, X[4], 0xf7537e82, 6);
    ST(R, G4, d, a, b, c, X[11], 0xbd3af235, 10);
    ST(R, G4, c, d, a, b, X[2], 0x2ad7d2bb, 15);
    ST(R, G4, b, c, d, a, X[9], 0xeb86d391, 21);
    h[0] += a;
    h[1] += b;
    h[2] += c;
    h[3] += d;
}

template <int V>
__device__ __forceinline__ void compress(uint32_t h[4], const uint32_t X[16])
{
    if constexpr (V == 0)
        md5_compress(h, X);
    else
        md5_asm<V == 2>(h, X);
}

// track t = blocks [t * nb, (t + 1) * nb) of 64 bytes; D blocks in flight
template <int V, bool ONE>
__global__ __launch_bounds__(64) void k_md5(const uint4 *__restrict__ data, uint32_t ntr,
                                            uint32_t nb, uint32_t *__restrict__ out)
{
    __builtin_amdgcn_s_setprio(3);
    uint32_t t = ONE ? blockIdx.x : blockIdx.x * 64u + threadIdx.x;
    if (ONE && threadIdx.x != 0)
        return;
    constexpr int TR = V == 3 ? 2 : 1;
    if (t * TR >= ntr)
        return;
    uint32_t h[TR][4];
    const uint4 *q[TR];
    for (int r = 0; r < TR; ++r) {
        h[r][0] = 0x67452301u;
        h[r][1] = 0xefcdab89u;
        h[r][2] = 0x98badcfeu;
        h[r][3] = 0x10325476u;
        q[r] = data + (size_t)(t * TR + r) * nb * 4u;
    }
    uint4 buf[TR][MD5_D][4];
#pragma unroll
    for (int r = 0; r < TR; ++r)
#pragma unroll
        for (int j = 0; j < MD5_D; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i)
                buf[r][j][i] = q[r][j * 4 + i];
    for (uint32_t blk = 0; blk + MD5_D <= nb; blk += MD5_D) {
#pragma unroll
        for (int j = 0; j < MD5_D; ++j) {
            if constexpr (TR == 2) {
                // both chains in one instruction stream (the compiler
                // interleaves the two independent compressions)
                md5_asm<false>(h[0], (const uint32_t *)&buf[0][j][0]);
                md5_asm<false>(h[1], (const uint32_t *)&buf[1][j][0]);
            } else {
                compress<V>(h[0], (const uint32_t *)&buf[0][j][0]);
            }
            const uint32_t nbk = min(blk + (uint32_t)(j + MD5_D), nb - 1u);
#pragma unroll
            for (int r = 0; r < TR; ++r)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    buf[r][j][i] = q[r][nbk * 4u + i];
        }
    }
    for (int r = 0; r < TR; ++r)
        for (int i = 0; i < 4; ++i)
            out[(t * TR + r) * 4 + i] = h[r][i];
}

typedef short bg_short2 __attribute__((ext_vector_type(2)));
// background load shaped like K2: 256-thread workgroups with 33 KB of LDS,
// a v_dot2 chain per ds_read_b128 (VALU-bound, LDS ~40% busy), `iters` long
__global__ __launch_bounds__(256) void k_busy(uint32_t *out, uint32_t iters, int lds_reads)
{
    __shared__ uint4 lds[33 * 1024 / 16];
    const int tid = threadIdx.x;
    for (int i = tid; i < 33 * 1024 / 16; i += 256)
        lds[i] = make_uint4(i, i + 1, i + 2, i + 3);
    __syncthreads();
    int acc[8] = {tid, tid + 1, tid + 2, tid + 3, tid + 4, tid + 5, tid + 6, tid + 7};
    for (uint32_t it = 0; it < iters; ++it) {
        uint4 w = lds_reads ? lds[(tid + it * 64) & (33 * 1024 / 16 - 1)] : make_uint4(it, it, it, it);
#pragma unroll
        for (int r = 0; r < 9; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k)
                acc[k] = __builtin_amdgcn_sdot2(__builtin_bit_cast(bg_short2, w.x ^ (uint32_t)k),
                                                __builtin_bit_cast(bg_short2, w.y + (uint32_t)r), acc[k], false);
    }
    int s = 0;
    for (int k = 0; k < 8; ++k)
        s += acc[k];
    if (s == 0x7fffffff)
        out[0] = s;
}

template <int V, bool ONE>
static float run(const uint4 *d, uint32_t ntr, uint32_t nb, uint32_t *out)
{
    const uint32_t tr = V == 3 ? ntr / 2 : ntr;
    dim3 grid = ONE ? dim3(tr) : dim3((tr + 63) / 64);
    hipLaunchKernelGGL((k_md5<V, ONE>), grid, dim3(64), 0, 0, d, ntr, nb, out);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k_md5<V, ONE>), grid, dim3(64), 0, 0, d, ntr, nb, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

// shader clock (s_memtime ticks per s_memrealtime 100 MHz tick) while the
// rest of the GPU is idle or busy: one wave spinning ~2 ms
__global__ void k_clock(unsigned long long *out)
{
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long r = r0;
    while (r - r0 < 200000ull)
        r = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) {
        out[0] = t1 - t0;
        out[1] = r - r0;
    }
}

static hipStream_t g_bg = nullptr, g_fg = nullptr;

static void clock_probe(const char *what)
{
    unsigned long long *d, h[2];
    hipMalloc(&d, 16);
    hipLaunchKernelGGL(k_clock, dim3(1), dim3(64), 0, g_fg, d);
    hipStreamSynchronize(g_fg);
    hipMemcpy(h, d, 16, hipMemcpyDeviceToHost);
    printf("shader clock %-28s %.0f MHz\n", what, 100.0 * (double)h[0] / (double)h[1]);
    hipFree(d);
}
static uint32_t *g_sink = nullptr;

// MD5 variant V timed on its own stream while k_busy fills the GPU
template <int V>
static float run_loaded(const uint4 *d, uint32_t ntr, uint32_t nb, uint32_t *out, int lds_reads)
{
    const uint32_t tr = V == 3 ? ntr / 2 : ntr;
    dim3 grid((tr + 63) / 64);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_busy, dim3(256 * 8 * 4), dim3(256), 0, g_bg, g_sink, 4000u, lds_reads);
    hipEventRecord(e0, g_fg);
    hipLaunchKernelGGL((k_md5<V, false>), grid, dim3(64), 0, g_fg, d, ntr, nb, out);
    hipEventRecord(e1, g_fg);
    hipEventSynchronize(e1);
    hipDeviceSynchronize();
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main(int argc, char **argv)
{
    const uint32_t ntr = argc > 1 ? (uint32_t)atoi(argv[1]) : 1024;
    const uint32_t nb = argc > 2 ? (uint32_t)atoi(argv[2]) : 16384;
    const size_t bytes = (size_t)ntr * nb * 64;
    std::vector<uint32_t> host(bytes / 4);
    uint32_t s = 12345;
    for (auto &v : host) {
        s = s * 1664525u + 1013904223u;
        v = s;
    }
    uint4 *d;
    uint32_t *out;
    hipMalloc(&d, bytes);
    hipMalloc(&out, ntr * 16);
    hipMemcpy(d, host.data(), bytes, hipMemcpyHostToDevice);
    std::vector<uint32_t> ref(ntr * 4), got(ntr * 4);
    struct R {
        const char *name;
        float (*fn)(const uint4 *, uint32_t, uint32_t, uint32_t *);
    } runs[] = {
        {"v0 shipped, 64 lanes", run<0, false>},     {"v1 add3 off-chain, 64 lanes", run<1, false>},
        {"v2 fast rotate, 64 lanes", run<2, false>}, {"v3 2 tracks/lane", run<3, false>},
        {"v0 shipped, 1 lane/wave", run<0, true>},   {"v1 add3 off-chain, 1 lane/wave", run<1, true>},
    };
    {
        // the shipped wave-pair kernel (md5.hip k_bytes_md5: whole blocks on a
        // hasher + helper pair, then the padding block)
        std::vector<uint64_t> off(ntr), len(ntr);
        for (uint32_t t = 0; t < ntr; ++t) {
            off[t] = (uint64_t)t * nb * 64u;
            len[t] = (uint64_t)nb * 64u;
        }
        uint64_t *doff, *dlen;
        uint8_t *dmd5;
        hipMalloc(&doff, ntr * 8);
        hipMalloc(&dlen, ntr * 8);
        hipMalloc(&dmd5, ntr * 16);
        hipMemcpy(doff, off.data(), ntr * 8, hipMemcpyHostToDevice);
        hipMemcpy(dlen, len.data(), ntr * 8, hipMemcpyHostToDevice);
        launch_bytes_md5((const uint8_t *)d, doff, dlen, ntr, dmd5, 0);
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        hipEventRecord(e0);
        launch_bytes_md5((const uint8_t *)d, doff, dlen, ntr, dmd5, 0);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        printf("%-34s %8.3f ms  %7.1f ns/block\n", "k_bytes_md5 wave pair (shipped)", ms, ms * 1e6 / nb);
    }
    hipStreamCreateWithFlags(&g_bg, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&g_fg, hipStreamNonBlocking);
    hipMalloc(&g_sink, 64);
    {
        // under a K2-shaped background load (launched first on its own stream)
        std::vector<uint64_t> off(ntr), len(ntr);
        for (uint32_t t = 0; t < ntr; ++t) {
            off[t] = (uint64_t)t * nb * 64u;
            len[t] = (uint64_t)nb * 64u;
        }
        uint64_t *doff, *dlen;
        uint8_t *dmd5;
        hipMalloc(&doff, ntr * 8);
        hipMalloc(&dlen, ntr * 8);
        hipMalloc(&dmd5, ntr * 16);
        hipMemcpy(doff, off.data(), ntr * 8, hipMemcpyHostToDevice);
        hipMemcpy(dlen, len.data(), ntr * 8, hipMemcpyHostToDevice);
        clock_probe("(GPU idle)");
        hipLaunchKernelGGL(k_busy, dim3(256 * 8 * 4), dim3(256), 0, g_bg, g_sink, 4000u, 1);
        clock_probe("(K2-shaped load)");
        hipDeviceSynchronize();
        for (int lr = 0; lr < 2; ++lr) {
            hipEvent_t e0, e1;
            hipEventCreate(&e0);
            hipEventCreate(&e1);
            hipEvent_t b0, b1;
            hipEventCreate(&b0);
            hipEventCreate(&b1);
            hipEventRecord(b0, g_bg);
            hipLaunchKernelGGL(k_busy, dim3(256 * 8 * 4), dim3(256), 0, g_bg, g_sink, 4000u, lr);
            hipEventRecord(b1, g_bg);
            hipEventRecord(e0, g_fg);
            launch_bytes_md5((const uint8_t *)d, doff, dlen, ntr, dmd5, g_fg);
            hipEventRecord(e1, g_fg);
            hipDeviceSynchronize();
            float ms = 0, bms = 0;
            hipEventElapsedTime(&ms, e0, e1);
            hipEventElapsedTime(&bms, b0, b1);
            printf("loaded(lds=%d, busy %.1f ms) %-20s %8.3f ms  %7.1f ns/block\n", lr, bms,
                   "wave pair (shipped)", ms, ms * 1e6 / nb);
            const float m0 = run_loaded<0>(d, ntr, nb, out, lr);
            printf("loaded(lds=%d) %-35s %8.3f ms  %7.1f ns/block\n", lr, "v0 single wave", m0,
                   m0 * 1e6 / nb);
        }
    }
    for (size_t i = 0; i < sizeof(runs) / sizeof(runs[0]); ++i) {
        hipMemset(out, 0, ntr * 16);
        const float ms = runs[i].fn(d, ntr, nb, out);
        hipMemcpy(got.data(), out, ntr * 16, hipMemcpyDeviceToHost);
        if (i == 0)
            ref = got;
        const bool ok = memcmp(ref.data(), got.data(), ntr * 16) == 0;
        printf("%-34s %8.3f ms  %7.1f ns/block  %s\n", runs[i].name, ms, ms * 1e6 / nb,
               ok ? "digests match v0" : "DIGEST MISMATCH");
    }
    return 0;
}
