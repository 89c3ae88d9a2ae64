// Micro-benchmark (profiling aid): read bandwidth of the tile access patterns of the fast kernel.
// A: lane = row, ten 16-byte loads per row (what pe_fast does)
// B: coalesced, consecutive lanes take consecutive 16-byte pieces of the tile's block
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

__global__ void __launch_bounds__(512) rows_kernel(const uint8_t* __restrict__ p0, const uint8_t* __restrict__ p1,
                                                   const uint8_t* __restrict__ p2, const uint8_t* __restrict__ p3,
                                                   int n, uint32_t* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t acc = 0;
    const int ntiles = (n + 31) / 32;
    for (int t = blockIdx.x * 8 + wave; t < ntiles; t += gridDim.x * 8) {
        const int row = min(t * 32 + (lane & 31), n - 1);
        const uint8_t* s = (lane < 32 ? p0 : p2) + (size_t)row * 160;
        const uint8_t* q = (lane < 32 ? p1 : p3) + (size_t)row * 160;
#pragma unroll
        for (int k = 0; k < 10; ++k) {
            const uint4 a = *reinterpret_cast<const uint4*>(s + 16 * k);
            const uint4 b = *reinterpret_cast<const uint4*>(q + 16 * k);
            acc += a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void __launch_bounds__(512) coal_kernel(const uint8_t* __restrict__ p0, const uint8_t* __restrict__ p1,
                                                   const uint8_t* __restrict__ p2, const uint8_t* __restrict__ p3,
                                                   int n, uint32_t* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t acc = 0;
    const int ntiles = (n + 31) / 32;
    for (int t = blockIdx.x * 8 + wave; t < ntiles; t += gridDim.x * 8) {
        const size_t base = (size_t)t * 32 * 160;
#pragma unroll
        for (int i = 0; i < 5; ++i) {
            const size_t off = base + (size_t)(i * 64 + lane) * 16;
            const uint4 a = *reinterpret_cast<const uint4*>(p0 + off);
            const uint4 b = *reinterpret_cast<const uint4*>(p1 + off);
            const uint4 c = *reinterpret_cast<const uint4*>(p2 + off);
            const uint4 d = *reinterpret_cast<const uint4*>(p3 + off);
            acc += a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w ^ c.x ^ c.w ^ d.y ^ d.z;
        }
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const int n = 20000000;
    uint8_t* p[4];
    for (int i = 0; i < 4; ++i) {
        if (hipMalloc(&p[i], (size_t)n * 160) != hipSuccess) return 1;
        (void)hipMemset(p[i], 0x41 + i, (size_t)n * 160);
    }
    uint32_t* out;
    (void)hipMalloc(&out, 4);
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const double bytes = 4.0 * n * 160;
    for (int bpc = 1; bpc <= 4; bpc *= 2) {
        for (int pass = 0; pass < 2; ++pass) {
            float best = 1e9f;
            for (int rep = 0; rep < 5; ++rep) {
                (void)hipEventRecord(e0);
                if (pass == 0)
                    hipLaunchKernelGGL(rows_kernel, dim3(cus * bpc), dim3(512), 0, 0, p[0], p[1], p[2], p[3], n, out);
                else
                    hipLaunchKernelGGL(coal_kernel, dim3(cus * bpc), dim3(512), 0, 0, p[0], p[1], p[2], p[3], n, out);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                float ms;
                (void)hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
            }
            printf("%s blocks/CU=%d  %.3f ms  %.0f GB/s\n", pass ? "coalesced" : "lane-rows", bpc, best,
                   bytes / (best / 1e3) / 1e9);
        }
    }
    return 0;
}
