// f64_rate.hip — measures the MI355X vector issue rate of the fp64
// operations the resampler's filter is built from (v_mul_f64, v_add_f64,
// v_cvt_f64_f32, v_fma_f64) and of v_fma_f32 for reference: 8 independent
// chains per lane, 256 threads x 4 blocks per CU, timed with HIP events.
// A development tool: the measured rates are the roofline peak the bench's
// fp64 figures are quoted against.  Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 4096;

__global__ __launch_bounds__(256) void k_mul(double *out, double a, double b)
{
    double x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        x[k] = a + threadIdx.x + k;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            x[k] = x[k] * b;
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_add(double *out, double a, double b)
{
    double x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        x[k] = a + threadIdx.x + k;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            x[k] = x[k] + b;
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fma64(double *out, double a, double b)
{
    double x[8];
#pragma unroll
    for (int k = 0; k < 8; ++k)
        x[k] = a + threadIdx.x + k;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            x[k] = __builtin_fma(x[k], b, a);
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_cvt(double *out, double a, double b)
{
    float x[8];
    double acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        x[k] = (float)(a + threadIdx.x + k);
        acc[k] = 0;
    }
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const double d = (double)x[k];
            asm volatile("" : "+v"(x[k]));
            acc[k] = d; // one cvt per element per iteration
        }
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        s += acc[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s + b;
}

__global__ __launch_bounds__(256) void k_fma32(double *out, double a, double b)
{
    float x[8];
    const float bf = (float)b, af = (float)a;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        x[k] = af + threadIdx.x + k;
    for (int i = 0; i < kIters; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k)
            x[k] = __builtin_fmaf(x[k], bf, af);
    }
    float s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k)
        s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class K>
static void run(const char *name, K kern, double *d, int blocks)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, nullptr, d, 1.0000001, 0.9999999);
    (void)hipEventRecord(e0, nullptr);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, nullptr, d, 1.0000001, 0.9999999);
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double wave_insts = (double)blocks * 4 /* waves per block */ * kIters * 8;
    const int simds = 256 * 4;
    const double cyc = ms * 1e-3 * 2.4e9; // at the 2.4 GHz engine clock
    printf("%-8s %8.3f ms  %.3e wave-instr/s  %.2f cycles per wave64 instr per SIMD "
           "(at 2.4 GHz)  %.1f T lane-ops/s\n",
           name, ms, wave_insts / (ms * 1e-3), cyc * simds / wave_insts,
           wave_insts * 64 / (ms * 1e-3) / 1e12);
}

int main()
{
    const int blocks = 256 * 8;
    double *d = nullptr;
    if (hipMalloc(&d, sizeof(double) * blocks * 256) != hipSuccess)
        return 1;
    run("mul_f64", k_mul, d, blocks);
    run("add_f64", k_add, d, blocks);
    run("fma_f64", k_fma64, d, blocks);
    run("cvt_f64", k_cvt, d, blocks);
    run("fma_f32", k_fma32, d, blocks);
    (void)hipFree(d);
    return 0;
}
