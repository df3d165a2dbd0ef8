// cu_probe.hip — which physical CUs (XCC, SE, SH, CU from the HW_ID and
// XCC_ID registers) a CU-masked stream's workgroups run on: checks how
// hipExtStreamCreateWithCUMask's bit i maps onto MI355X's 8 XCDs.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/cu_probe tools/cu_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void k_where(uint32_t *out)
{
    // HW_ID (reg 4): cu_id [11:8], sh_id [12], se_id [15:13]; XCC_ID (reg 20) [3:0]
    const uint32_t hw = __builtin_amdgcn_s_getreg((31 << 11) | (0 << 6) | 4);
    const uint32_t xcc = __builtin_amdgcn_s_getreg((3 << 11) | (0 << 6) | 20);
    // keep the workgroup resident a while so the grid spreads over the CUs
    long long t0 = clock64();
    while (clock64() - t0 < 200000)
        ;
    if (threadIdx.x == 0)
        out[blockIdx.x] = (xcc << 16) | (((hw >> 13) & 7u) << 8) | (((hw >> 12) & 1u) << 4) |
                          ((hw >> 8) & 15u);
}

static void probe(const char *name, const uint32_t *mask)
{
    hipStream_t s;
    if (mask) {
        if (hipExtStreamCreateWithCUMask(&s, 8, mask) != hipSuccess) {
            printf("%s: mask stream failed\n", name);
            return;
        }
    } else {
        (void)hipStreamCreate(&s);
    }
    const int n = 8192;
    uint32_t *d;
    (void)hipMalloc(&d, n * 4);
    hipLaunchKernelGGL(k_where, dim3(n), dim3(64), 0, s, d);
    (void)hipStreamSynchronize(s);
    std::vector<uint32_t> h(n);
    (void)hipMemcpy(h.data(), d, n * 4, hipMemcpyDeviceToHost);
    std::set<uint32_t> cus;
    int per_xcc[16] = {0};
    for (uint32_t v : h)
        cus.insert(v);
    for (uint32_t v : cus)
        per_xcc[(v >> 16) & 15]++;
    printf("%-8s %3zu CUs; per XCC:", name, cus.size());
    for (int x = 0; x < 8; ++x)
        printf(" %d", per_xcc[x]);
    printf("\n");
    if (cus.size() <= 16) {
        for (uint32_t v : cus)
            printf("   xcc %u se %u sh %u cu %u\n", v >> 16, (v >> 8) & 7, (v >> 4) & 1, v & 15);
    }
    (void)hipFree(d);
    (void)hipStreamDestroy(s);
}

int main()
{
    uint32_t m_md5[8] = {0}, m_main[8], m_lo[8] = {0};
    for (int k = 0; k < 8; ++k)
        m_main[k] = 0xFFFFFFFFu;
    for (int k = 0; k < 8; ++k) {
        const int cu = 33 * k;
        m_md5[cu >> 5] |= 1u << (cu & 31);
        m_main[cu >> 5] &= ~(1u << (cu & 31));
    }
    m_lo[0] = 0xFFu; // bits 0..7
    probe("all", nullptr);
    probe("main", m_main);
    probe("md5", m_md5);
    probe("bits0-7", m_lo);
    return 0;
}
