// PCIe duplex probe, kernel side: device -> pinned host memory written by a
// kernel (16-byte stores, grid-stride) alone and beside an SDMA host ->
// device copy on another stream; also the SDMA device -> host copy for
// comparison.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/duplex_kernel
// tools/duplex_kernel.hip; run: tools/bin/duplex_kernel [MiB] [blocks]
// [normal streams] [high-priority streams] [copy stream priority: 0 normal,
// 1 least, -1 greatest]: the extra streams (each given one empty kernel
// first) stand in for the engine's, to see whether the copy streams still
// run both directions at once beside them
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                              \
        }                                                                              \
    } while (0)

__global__ void k_store(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static double now()
{
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

int main(int argc, char **argv)
{
    const size_t mib = argc > 1 ? std::atoi(argv[1]) : 512;
    const unsigned blocks = argc > 2 ? std::atoi(argv[2]) : 1024;
    const int n_norm = argc > 3 ? std::atoi(argv[3]) : 0;
    const int n_high = argc > 4 ? std::atoi(argv[4]) : 0;
    const int cprio = argc > 5 ? std::atoi(argv[5]) : 0;
    int least = 0, greatest = 0;
    CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
    for (int k = 0; k < n_norm + n_high; ++k) {
        hipStream_t x;
        CK(hipStreamCreateWithPriority(&x, hipStreamNonBlocking, k < n_norm ? 0 : greatest));
        hipLaunchKernelGGL(k_store, dim3(1), dim3(64), 0, x, (const uint4 *)nullptr, (uint4 *)nullptr,
                           (size_t)0);
    }
    const size_t n = mib << 20;
    void *h_up, *h_dn, *d_up, *d_dn;
    CK(hipHostMalloc(&h_up, n, hipHostMallocDefault));
    CK(hipHostMalloc(&h_dn, n, hipHostMallocDefault));
    CK(hipMalloc(&d_up, n));
    CK(hipMalloc(&d_dn, n));
    CK(hipMemset(d_dn, 1, n));
    hipStream_t s1, s2;
    const int pc = cprio == 0 ? 0 : (cprio > 0 ? least : greatest);
    CK(hipStreamCreateWithPriority(&s1, hipStreamNonBlocking, pc));
    CK(hipStreamCreateWithPriority(&s2, hipStreamNonBlocking, pc));
    auto kd2h = [&]() {
        hipLaunchKernelGGL(k_store, dim3(blocks), dim3(256), 0, s2, (const uint4 *)d_dn,
                           (uint4 *)h_dn, n / 16);
    };
    auto sd2h = [&]() { CK(hipMemcpyAsync(h_dn, d_dn, n, hipMemcpyDeviceToHost, s2)); };
    auto h2d = [&]() { CK(hipMemcpyAsync(d_up, h_up, n, hipMemcpyHostToDevice, s1)); };
    auto best = [&](auto fn) {
        double b = 1e9;
        for (int r = 0; r < 5; ++r) {
            CK(hipDeviceSynchronize());
            const double t0 = now();
            fn();
            CK(hipDeviceSynchronize());
            b = std::min(b, now() - t0);
        }
        return b;
    };
    const double t_h2d = best([&] { h2d(); });
    const double t_kd = best([&] { kd2h(); });
    const double t_sd = best([&] { sd2h(); });
    const double t_both_k = best([&] { h2d(); kd2h(); });
    const double t_both_s = best([&] { h2d(); sd2h(); });
    std::printf("{\"extra_normal\": %d, \"extra_high\": %d, \"copy_prio\": %d, \"range\": [%d, %d], ", n_norm, n_high, pc, least, greatest);
    std::printf("\"bytes\": %zu, \"blocks\": %u, \"h2d_sdma_GBps\": %.1f, \"d2h_kernel_GBps\": %.1f, "
                "\"d2h_sdma_GBps\": %.1f, \"h2d_sdma+d2h_kernel_ms\": %.2f, \"aggregate_kernel_GBps\": %.1f, "
                "\"h2d_sdma+d2h_sdma_ms\": %.2f, \"aggregate_sdma_GBps\": %.1f}\n",
                n, blocks, n / t_h2d / 1e9, n / t_kd / 1e9, n / t_sd / 1e9, t_both_k * 1e3,
                2 * n / t_both_k / 1e9, t_both_s * 1e3, 2 * n / t_both_s / 1e9);
    // the bytes the kernel wrote arrived
    const unsigned char *p = (const unsigned char *)h_dn;
    if (p[0] != 1 || p[n - 1] != 1) {
        std::fprintf(stderr, "kernel-written host bytes wrong\n");
        return 1;
    }
    return 0;
}
