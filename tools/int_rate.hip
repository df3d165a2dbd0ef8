// int_rate.hip — measures the MI355X vector issue cost of the integer
// instructions the FLAC subframe search is built from (v_add_u32, v_xor,
// v_ashrrev, v_add3, v_dot2_i32_i16, v_alignbit, v_perm, v_mad_i32_i24,
// v_pk_* 16-bit) against v_fma_f32 (2 cycles per wave64 instruction with two
// or more waves per SIMD, MI355X_MICROARCH.md): 8 independent chains per
// lane, W waves per SIMD, timed with HIP events.  A development tool: it
// says whether K2 is bound by instruction count or by issue latency.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/int_rate tools/int_rate.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 2048;

#define CHAINS8(BODY)                                                                  \
    _Pragma("unroll") for (int k = 0; k < 8; ++k) { BODY; }

template <int OP>
__global__ __launch_bounds__(256) void k_op(unsigned *out, unsigned a, unsigned b)
{
    unsigned x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        x[k] = a + threadIdx.x * 7u + k;
    float f[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        f[k] = (float)x[k];
    for (int i = 0; i < kIters; ++i) {
        if constexpr (OP == 0)
            CHAINS8(asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f[k]) : "v"(f[(k + 1) & 7])))
        else if constexpr (OP == 1)
            CHAINS8(asm volatile("v_add_u32 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 2)
            CHAINS8(asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 3)
            CHAINS8(asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(x[k]) : "s"(b)))
        else if constexpr (OP == 4)
            CHAINS8(asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "v"(x[(k + 2) & 7])))
        else if constexpr (OP == 5)
            CHAINS8(asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "s"(b)))
        else if constexpr (OP == 6)
            CHAINS8(asm volatile("v_dot2c_i32_i16 %0, %2, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "s"(b)))
        else if constexpr (OP == 7)
            CHAINS8(asm volatile("v_alignbit_b32 %0, %0, %1, 16" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 8)
            CHAINS8(asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "s"(b)))
        else if constexpr (OP == 9)
            CHAINS8(asm volatile("v_mad_i32_i24 %0, %1, %2, %0" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "s"(b)))
        else if constexpr (OP == 10)
            CHAINS8(asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 11)
            CHAINS8(asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 12)
            CHAINS8(asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 13)
            CHAINS8(asm volatile("v_max_u32 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 14)
            CHAINS8(asm volatile("v_dot2_u32_u16 %0, %1, %2, %0" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "s"(b)))
        else if constexpr (OP == 15)
            CHAINS8(asm volatile("v_pk_lshrrev_b16 %0, %1, %0" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 16)
            CHAINS8(asm volatile("v_sad_u32 %0, %0, %1, %0" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 17)
            CHAINS8(asm volatile("v_mov_b32 %0, %1" : "=v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 18) // dependent chain of one op per lane (latency)
            asm volatile("v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n"
                         "v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1\n v_add_u32 %0, %0, %1"
                         : "+v"(x[0]) : "v"(x[1]));
        else if constexpr (OP == 19) // dependent dot2 chain
            asm volatile("v_dot2_i32_i16 %0, %1, %2, %0\n v_dot2_i32_i16 %0, %1, %2, %0\n v_dot2_i32_i16 %0, %1, %2, %0\n v_dot2_i32_i16 %0, %1, %2, %0\n"
                         "v_dot2_i32_i16 %0, %1, %2, %0\n v_dot2_i32_i16 %0, %1, %2, %0\n v_dot2_i32_i16 %0, %1, %2, %0\n v_dot2_i32_i16 %0, %1, %2, %0"
                         : "+v"(x[0]) : "v"(x[1]), "s"(b));
        else if constexpr (OP == 20)
            CHAINS8(asm volatile("v_ashrrev_i32 %0, %1, %0" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 21)
            CHAINS8(asm volatile("v_ashrrev_i32 %0, 31, %0" : "+v"(x[k])))
        else if constexpr (OP == 22)
            CHAINS8(asm volatile("v_lshrrev_b32 %0, %1, %0" : "+v"(x[k]) : "s"(b)))
        else if constexpr (OP == 23)
            CHAINS8(asm volatile("v_add_u32 %0, %1, %0" : "+v"(x[k]) : "s"(b)))
        else if constexpr (OP == 24)
            CHAINS8(asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 25)
            CHAINS8(asm volatile("v_max_i32 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 26)
            CHAINS8(asm volatile("v_and_b32 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 27)
            CHAINS8(asm volatile("v_or_b32 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 28)
            CHAINS8(asm volatile("v_lshlrev_b32 %0, %1, %0" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 29)
            CHAINS8(asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "s"(0ull)))
        else if constexpr (OP == 30)
            CHAINS8(asm volatile("v_bfe_u32 %0, %0, %1, 5" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 31)
            CHAINS8(asm volatile("v_xad_u32 %0, %0, %1, %0" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 32)
            CHAINS8(asm volatile("v_cvt_pk_u16_u32 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 33)
            CHAINS8(asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 34)
            CHAINS8(asm volatile("v_add_co_u32 %0, vcc, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7]) : "vcc"))
        else if constexpr (OP == 35)
            CHAINS8(asm volatile("v_not_b32 %0, %0" : "+v"(x[k])))
        else if constexpr (OP == 36)
            CHAINS8(asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 37)
            CHAINS8(asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "v"(x[(k + 2) & 7])))
        else if constexpr (OP == 38)
            CHAINS8(asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 39)
            CHAINS8(asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "v"(x[(k + 2) & 7])))
        else if constexpr (OP == 40)
            CHAINS8(asm volatile("v_dot2_i32_i16 %0, %1, %2, %0" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "v"(x[(k + 2) & 7])))
        else if constexpr (OP == 41)
            CHAINS8(asm volatile("v_dot2c_i32_i16 %0, %1, %2" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "v"(x[(k + 2) & 7])))
        else if constexpr (OP == 42)
            CHAINS8(asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x[k])))
        else if constexpr (OP == 43)
            CHAINS8(asm volatile("s_mov_b64 vcc, -1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x[k]) : "v"(x[(k + 1) & 7]) : "vcc"))
        else if constexpr (OP == 44)
            CHAINS8(asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "v"(x[(k + 2) & 7])))
        else if constexpr (OP == 45)
            CHAINS8(asm volatile("v_mad_i32_i24 %0, %1, %2, %0" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "v"(x[(k + 2) & 7])))
        else if constexpr (OP == 46)
            CHAINS8(asm volatile("v_max_i32 %0, 0, %0" : "+v"(x[k])))
        else if constexpr (OP == 47)
            CHAINS8(asm volatile("v_min_u32 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 48)
            CHAINS8(asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 49)
            CHAINS8(asm volatile("v_dot4_i32_i8 %0, %1, %2, %0" : "+v"(x[k]) : "v"(x[(k + 1) & 7]), "v"(x[(k + 2) & 7])))
        else if constexpr (OP == 50)
            CHAINS8(asm volatile("v_add_i32 %0, %0, %1" : "+v"(x[k]) : "v"(x[(k + 1) & 7])))
        else if constexpr (OP == 51)
            CHAINS8(asm volatile("v_pk_fma_f32 %0, %1, %2, %0" : "+v"(*(double*)&x[k & 6]) : "v"(*(double*)&x[(k+2) & 6]), "v"(*(double*)&x[(k+4) & 6])))
    }
    unsigned s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        s += x[k] + (unsigned)f[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static const char *kNames[] = {"v_fma_f32",      "v_add_u32",      "v_xor_b32",     "v_ashrrev_i32",
                               "v_add3_u32",     "v_dot2_i32_i16", "v_dot2c_i32_i16", "v_alignbit_b32",
                               "v_perm_b32",     "v_mad_i32_i24",  "v_pk_add_u16",  "v_lshrrev_b32",
                               "v_cndmask_b32",  "v_max_u32",      "v_dot2_u32_u16", "v_pk_lshrrev_b16",
                               "v_sad_u32",      "v_mov_b32",      "dep v_add_u32", "dep v_dot2", "v_ashrrev_i32 v-sh", "v_ashrrev_i32 31", "v_lshrrev_b32 s-sh", "v_add_u32 sgpr", "v_sub_u32", "v_max_i32", "v_and_b32", "v_or_b32", "v_lshlrev_b32", "v_cndmask_e64 s", "v_bfe_u32", "v_xad_u32", "v_cvt_pk_u16_u32", "v_add_u32_e64", "v_add_co_u32", "v_not_b32", "v_mul_u32_u24", "v_min3_u32", "v_lshl_add_u32", "v_bitop3_b32", "v_dot2_i32_i16 vv", "v_dot2c_i32_i16 vv", "v_lshlrev_b32 c", "v_cndmask vcc set", "v_perm vvv", "v_mad_i32_i24 vv", "v_max_i32 c", "v_min_u32", "v_mul_lo_u32", "v_dot4_i32_i8 vv", "v_add_i32 (sat?)", "v_pk_fma_f32"};

template <int OP>
static void run(unsigned *d, int cus, int waves_per_simd)
{
    const int blocks = cus * waves_per_simd; // 256 threads = 4 waves = one per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, d, 3u, 1u);
    hipEventRecord(e0);
    const int reps = 5;
    for (int r = 0; r < reps; ++r)
        hipLaunchKernelGGL(k_op<OP>, dim3(blocks), dim3(256), 0, 0, d, 3u, 1u);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    // wave-instructions issued per SIMD
    const double per_simd = (double)waves_per_simd * kIters * 8.0 * reps;
    printf("%-18s waves/SIMD %d  %.3f ns per wave-instruction per SIMD\n", kNames[OP], waves_per_simd,
           ms * 1e6 / per_simd);
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

template <int OP>
static void sweep(unsigned *d, int cus)
{
    for (int w : {4})
        run<OP>(d, cus, w);
}

int main()
{
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    printf("CUs %d, clock %d kHz\n", cus, prop.clockRate);
    unsigned *d;
    hipMalloc(&d, (size_t)cus * 8 * 256 * sizeof(unsigned));
    sweep<40>(d, cus);
    sweep<41>(d, cus);
    sweep<42>(d, cus);
    sweep<43>(d, cus);
    sweep<44>(d, cus);
    sweep<45>(d, cus);
    sweep<46>(d, cus);
    sweep<47>(d, cus);
    sweep<48>(d, cus);
    sweep<49>(d, cus);
    sweep<50>(d, cus);
    sweep<51>(d, cus);
    hipFree(d);
    return 0;
}
