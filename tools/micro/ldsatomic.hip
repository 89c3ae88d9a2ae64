// Micro-benchmark (profiling aid): LDS atomic add throughput per CU for the stats histogram
// pattern (64 lanes, distinct bank pairs), u64 vs u32, full vs partial exec masks.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int MODE>
__global__ void __launch_bounds__(512) k_atomic(uint32_t* out, int iters) {
    __shared__ unsigned long long h64[4096];
    __shared__ uint32_t h32[8192];
    for (int i = threadIdx.x; i < 4096; i += 512) h64[i] = 0;
    for (int i = threadIdx.x; i < 8192; i += 512) h32[i] = 0;
    __syncthreads();
    const int lane = threadIdx.x & 63;
    int a = (lane & 15) * 2 + (lane >> 4) * 512;  // distinct bank pairs per 16-lane group
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 16; ++u) {
            const int idx = (a + u * 32) & 4095;
            if (MODE == 0) atomicAdd(&h64[idx >> 1 << 1 >> 1], 1ull);
            if (MODE == 1) atomicAdd(&h32[idx], 1u);
            if (MODE == 2 && lane < 16) atomicAdd(&h64[idx >> 1], 1ull);
            if (MODE == 3) { atomicAdd(&h32[idx], 1u); atomicAdd(&h32[(idx + 4096) & 8191], 3u); }
        }
        a += 7;
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = (uint32_t)h64[5] + h32[9];
}

int main() {
    int cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    uint32_t* out;
    (void)hipMalloc(&out, 4 * 4096);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 2000;
    const char* names[] = {"ds_add_u64 64 lanes", "ds_add_u32 64 lanes", "ds_add_u64 16 lanes", "2x ds_add_u32"};
    for (int mode = 0; mode < 4; ++mode) {
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
            (void)hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(k_atomic<0>, dim3(cus * 2), dim3(512), 0, 0, out, iters);
            if (mode == 1) hipLaunchKernelGGL(k_atomic<1>, dim3(cus * 2), dim3(512), 0, 0, out, iters);
            if (mode == 2) hipLaunchKernelGGL(k_atomic<2>, dim3(cus * 2), dim3(512), 0, 0, out, iters);
            if (mode == 3) hipLaunchKernelGGL(k_atomic<3>, dim3(cus * 2), dim3(512), 0, 0, out, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (ms < best) best = ms;
        }
        // wave-instructions per CU: 16 waves x iters x 16 (x2 for mode 3)
        const double winst = 16.0 * iters * 16 * (mode == 3 ? 2 : 1);
        printf("%-22s %.3f ms  %.2f cycles per wave-instruction per CU (2.4 GHz)\n", names[mode], best,
               best * 1e-3 * 2.4e9 / winst);
    }
    return 0;
}
