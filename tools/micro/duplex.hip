// Micro-benchmark (profiling aid): H2D alone, D2H alone, and both at once on two streams, from/to
// page-locked host memory (hipHostMalloc and registered THP mappings), to see whether the
// copies overlap (full-duplex PCIe) or share one path.
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static double now() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x)                                                       \
    do {                                                            \
        hipError_t e_ = (x);                                        \
        if (e_ != hipSuccess) {                                     \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
            exit(1);                                                \
        }                                                           \
    } while (0)

static char* thp(size_t n) {
    char* m = (char*)mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    madvise(m, n, MADV_HUGEPAGE);
    memset(m, 1, n);
    CK(hipHostRegister(m, n, hipHostRegisterPortable));
    return m;
}

int main(int argc, char** argv) {
    const size_t chunk = (size_t)(argc > 1 ? atoi(argv[1]) : 128) << 20;
    const int reps = argc > 2 ? atoi(argv[2]) : 16;
    for (int kind = 0; kind < 2; ++kind) {
        char *hin, *hout, *din, *dout;
        if (kind == 0) {
            CK(hipHostMalloc((void**)&hin, chunk, hipHostMallocDefault));
            CK(hipHostMalloc((void**)&hout, chunk, hipHostMallocDefault));
        } else {
            hin = thp(chunk);
            hout = thp(chunk);
        }
        CK(hipMalloc(&din, chunk));
        CK(hipMalloc(&dout, chunk));
        CK(hipMemset(dout, 2, chunk));
        hipStream_t a, b;
        CK(hipStreamCreateWithFlags(&a, hipStreamNonBlocking));
        CK(hipStreamCreateWithFlags(&b, hipStreamNonBlocking));
        for (int mode = 0; mode < 3; ++mode) {
            CK(hipDeviceSynchronize());
            const double t0 = now();
            for (int r = 0; r < reps; ++r) {
                if (mode != 1) CK(hipMemcpyAsync(din, hin, chunk, hipMemcpyHostToDevice, a));
                if (mode != 0) CK(hipMemcpyAsync(hout, dout, chunk, hipMemcpyDeviceToHost, b));
            }
            CK(hipDeviceSynchronize());
            const double t = now() - t0;
            const double gb = (double)chunk * reps * (mode == 2 ? 2 : 1) / 1e9;
            printf("%s %-10s %6.1f GB/s total (%.3f s)\n", kind ? "thp-registered" : "hipHostMalloc ",
                   mode == 0 ? "H2D" : mode == 1 ? "D2H" : "H2D+D2H", gb / t, t);
        }
    }
    return 0;
}
